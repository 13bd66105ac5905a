"""ASGI front of the master for high request rates (``serve-master --server uvicorn``).

The long poll of the status API (``GET /api/inference/status/<id>/?wait=<s>``) runs as a
coroutine on the server's event loop — hundreds of clients waiting for their requests hold
no thread each (in the threaded WSGI server every waiting client was a CPython thread, and
the master's Python threads, not the GPU, bounded end-to-end throughput). Everything else
(the reference's routes, pages, forms, session flash messages, admin) is the unchanged
Flask app, served through the WSGI adapter.

    uvicorn distributed_llm_inferencing_amd.control.asgi:application
"""
from __future__ import annotations

import json
import re
from urllib.parse import parse_qs

from .store import NotFound

_STATUS = re.compile(r"^/api/inference/status/(\d+)/$")


def create_asgi_app(flask_app):
    from uvicorn.middleware.wsgi import WSGIMiddleware
    wsgi = WSGIMiddleware(flask_app, workers=32)
    store = flask_app.extensions["dli"].store

    async def respond(send, status: int, body: dict):
        data = json.dumps(body).encode()
        await send({"type": "http.response.start", "status": status,
                    "headers": [(b"content-type", b"application/json"),
                                (b"content-length", str(len(data)).encode())]})
        await send({"type": "http.response.body", "body": data})

    async def app(scope, receive, send):
        if scope["type"] == "http" and scope["method"] == "GET":
            m = _STATUS.match(scope["path"])
            qs = parse_qs(scope.get("query_string", b"").decode())
            if m and qs.get("wait"):
                try:
                    wait = min(float(qs["wait"][0] or 0), 60.0)
                    r = await store.wait_final_async(int(m.group(1)), wait)
                    await respond(send, 200, {
                        "id": r["id"], "status": r["status"], "model_name": r["model_name"],
                        "prompt": r["prompt"], "result": r["result"], "error": r["error"],
                        "created_at": r["created_at"], "completed_at": r["completed_at"]})
                except Exception as e:  # noqa: BLE001 — same answer as the Flask route
                    msg = e.args[0] if isinstance(e, NotFound) else str(e)
                    await respond(send, 500, {"status": "error",
                                              "message": f"Error retrieving inference status: "
                                                         f"{msg}"})
                return
        await wsgi(scope, receive, send)

    return app


def _build():
    from ..utils.log import setup_logging
    from .master import create_master_app
    setup_logging("master")
    return create_asgi_app(create_master_app())


class _Lazy:
    """``application`` for ASGI servers, built on first use (importing must not start the
    dispatcher threads of a process that only wanted the factory)."""

    def __init__(self):
        self._app = None

    async def __call__(self, scope, receive, send):
        if self._app is None:
            self._app = _build()
        await self._app(scope, receive, send)


application = _Lazy()
