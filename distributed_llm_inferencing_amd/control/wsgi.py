"""Module-level WSGI application of the master (reference: ``master/master/wsgi.py:4-5``,
served by ``gunicorn master.wsgi:application --workers 3``, ``master/Dockerfile:44``).

Any WSGI server can import ``application``; settings come from the environment (same names
as the reference: ``SECRET_KEY``, ``DEBUG``, ``REDIS_*``, ``MODEL_CACHE_DIR`` ... plus
``QUEUE_BACKEND``, ``MASTER_DB``). Like Django's ``get_wsgi_application()``, importing it
builds the app, which starts the dispatcher pool and the heartbeat thread of this process.
Several server processes must share a queue backend across processes (``QUEUE_BACKEND=
sqlite`` or ``redis``); the in-process queue is for a single process.

    python -m distributed_llm_inferencing_amd.cli serve-master --server uvicorn
    uvicorn --interface wsgi distributed_llm_inferencing_amd.control.wsgi:application
"""
from ..utils.log import setup_logging
from .master import create_master_app

setup_logging("master")
application = create_master_app()
app = application
