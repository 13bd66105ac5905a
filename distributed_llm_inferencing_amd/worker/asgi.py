"""ASGI front of a worker (``serve-worker --server uvicorn``).

``POST /inference`` for a model this worker serves from its engine (the common case: no
``shard_ids``) runs as a coroutine awaiting the engine thread's future: hundreds of
concurrent requests hold no thread each (the reference's worker served one request at a
time, ``worker/Dockerfile:45``; a threaded server holds one CPython thread per in-flight
request, which bounded a GPU worker at a few hundred requests/s). Same body, auth, status
codes, messages and JSON as the Flask route; every other request (and the rare paths:
model not loaded yet, shard_ids, pipeline heads) goes to the unchanged Flask app through
the WSGI adapter.
"""
from __future__ import annotations

import asyncio
import json
import time

from ..utils import faults
from .server import request_params, success_body


def create_asgi_app(flask_app):
    from uvicorn.middleware.wsgi import WSGIMiddleware
    wsgi = WSGIMiddleware(flask_app, workers=32)
    st = flask_app.extensions["dli_worker"]
    settings = st.settings

    async def respond(send, status: int, body: dict):
        data = json.dumps(body).encode()
        await send({"type": "http.response.start", "status": status,
                    "headers": [(b"content-type", b"application/json"),
                                (b"content-length", str(len(data)).encode())]})
        await send({"type": "http.response.body", "body": data})

    async def read_body(receive) -> bytes:
        chunks = []
        while True:
            msg = await receive()
            chunks.append(msg.get("body", b""))
            if not msg.get("more_body"):
                return b"".join(chunks)

    def replay(body: bytes):
        sent = False

        async def receive():
            nonlocal sent
            if not sent:
                sent = True
                return {"type": "http.request", "body": body, "more_body": False}
            return {"type": "http.disconnect"}
        return receive

    async def app(scope, receive, send):
        if scope["type"] == "lifespan":           # nothing to start: acknowledge
            while True:
                msg = await receive()
                if msg["type"] == "lifespan.startup":
                    await send({"type": "lifespan.startup.complete"})
                elif msg["type"] == "lifespan.shutdown":
                    await send({"type": "lifespan.shutdown.complete"})
                    return
        if not (scope["type"] == "http" and scope["method"] == "POST"
                and scope["path"] == "/inference"):
            await wsgi(scope, receive, send)
            return
        body = await read_body(receive)
        try:
            data = json.loads(body or b"{}")
        except ValueError:
            data = None
        name = data.get("model_name") if isinstance(data, dict) else None
        svc = st.services.get(name) if name else None
        if svc is None or data.get("shard_ids") or not data.get("prompt"):
            await wsgi(scope, replay(body), send)              # rare paths: Flask route
            return
        if settings.auth_enabled:
            hdr = dict(scope.get("headers") or []).get(b"authorization", b"").decode()
            if hdr != f"Bearer {settings.auth_key}":
                await respond(send, 401, {"status": "error", "message": "Unauthorized access"})
                return
        t0 = time.time()
        try:
            faults.check("worker.inference")
            params, timeout = request_params(data)
            fut = svc.submit(data["prompt"], params)
            out = await asyncio.wait_for(asyncio.wrap_future(fut), timeout + 30)
            if out.finish_reason == "timeout":
                raise TimeoutError("Inference generation timed out")
            await respond(send, 200, success_body(out, t0))
        except (TimeoutError, asyncio.TimeoutError) as e:
            await respond(send, 408, {"status": "error",
                                      "message": str(e) or "Inference generation timed out"})
        except Exception as e:  # noqa: BLE001
            await respond(send, 500, {"status": "error", "message": f"Inference failed: {e}"})

    return app
