"""ASGI front of the master for high request rates (``serve-master --server uvicorn``).

The long poll of the status API (``GET /api/inference/status/<id>/?wait=<s>``) runs as a
coroutine on the server's event loop — hundreds of clients waiting for their requests hold
no thread each (in the threaded WSGI server every waiting client was a CPython thread, and
the master's Python threads, not the GPU, bounded end-to-end throughput).

The submit API (``POST /api/inference/submit/``) of a client WITHOUT a session cookie (API
clients, the load generator) is served here too: same form fields and validation, same
JSON answers and status codes, one store insert awaited on the store's database thread.
Through Flask it cost ~2.3 ms of GIL time per request (WSGI thread hand-off, request and
session objects, and the signed + zlib-compressed session cookie that carries the flash
message), which capped the master at ~250 requests/s on 8 CPUs with an engine that never
saturates (scripts/bench_control_plane.py). A browser (it holds a session cookie) still
goes through Flask, so the dashboard's flash message is unchanged.

Everything else (the reference's routes, pages, forms, session flash messages, admin) is
the unchanged Flask app, served through the WSGI adapter.

    uvicorn distributed_llm_inferencing_amd.control.asgi:application
"""
from __future__ import annotations

import json
import os
import re
from urllib.parse import parse_qs

from .store import NotFound

_STATUS = re.compile(r"^/api/inference/status/(\d+)/$")
_SUBMIT = "/api/inference/submit/"


def create_asgi_app(flask_app):
    from uvicorn.middleware.wsgi import WSGIMiddleware
    wsgi = WSGIMiddleware(flask_app, workers=32)
    state = flask_app.extensions["dli"]
    store = state.store
    cookie_name = flask_app.config.get("SESSION_COOKIE_NAME", "session").encode() + b"="

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

    def submit_form(scope, body: bytes):
        """The submitted form as a dict (first value per field, as Flask's request.form
        .get), or None when this path does not take the request (a session cookie: keep
        the flash message; a content type other than urlencoded / JSON)."""
        ctype = b""
        for k, v in scope.get("headers", ()):
            if k == b"cookie" and cookie_name in v:
                return None
            if k == b"content-type":
                ctype = v.split(b";")[0].strip().lower()
        if ctype == b"application/x-www-form-urlencoded":
            return {k: v[0] for k, v in parse_qs(body.decode("utf-8", "replace"),
                                                  keep_blank_values=True).items()}
        if ctype == b"application/json":
            try:
                d = json.loads(body or b"{}")
            except ValueError:
                return None
            return d if isinstance(d, dict) else None
        return None

    async def submit(scope, body: bytes, send) -> bool:
        import asyncio
        from .master import validate_inference_form
        form = submit_form(scope, body)
        if form is None:
            return False
        data, errors = validate_inference_form(form)
        if errors:
            await respond(send, 400, {"status": "error",
                                      "message": "Form validation failed. Please correct the "
                                                 "errors and try again.", "errors": errors})
            return True
        rid = await asyncio.wrap_future(store.submit(
            lambda _c: store.create_request(data["model_name"], data["prompt"])))
        state.dispatcher.submit(rid)
        await respond(send, 200, {"status": "success", "message": "Inference request submitted "
                                  "successfully", "request_id": rid})
        return True

    def ensure_dispatch():
        # the async dispatcher runs on THIS (the server's) event loop when the master was
        # built for it (DLI_DISPATCH_ON_SERVER_LOOP=1, set by serve-master for ASGI servers)
        import asyncio
        d = state.dispatcher
        if (os.environ.get("DLI_DISPATCH_ON_SERVER_LOOP", "0") == "1"
                and hasattr(d, "start_on_loop") and not d._threads):
            d.start_on_loop(asyncio.get_running_loop())
        n = getattr(state, "notifier", None)
        if n is not None and not n._listening:          # peers' finished requests
            asyncio.get_running_loop().create_task(n.listen(store._notify_final))

    async def app(scope, receive, send):
        if scope["type"] == "lifespan":
            while True:
                msg = await receive()
                if msg["type"] == "lifespan.startup":
                    ensure_dispatch()
                    await send({"type": "lifespan.startup.complete"})
                elif msg["type"] == "lifespan.shutdown":
                    await send({"type": "lifespan.shutdown.complete"})
                    return
        ensure_dispatch()
        if (scope["type"] == "http" and scope["method"] == "POST"
                and scope["path"] == _SUBMIT):
            body = await read_body(receive)
            if not await submit(scope, body, send):
                await wsgi(scope, replay(body), send)
            return
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
                    if r["status"] in ("completed", "failed"):
                        store.answered(r["id"])
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
