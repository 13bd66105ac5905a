"""Serve an ASGI application on aiohttp's HTTP server (``serve-master / serve-worker
--server aiohttp``).

uvicorn parses HTTP with h11 here (httptools is not installed), in pure Python: at the
request rates of the end-to-end config (two master requests and one worker request per
generation, ~500 generations/s) that parsing is a large share of the master's GIL time.
aiohttp ships a C HTTP parser; this adapter turns each aiohttp request into one ASGI
``http`` call of the same application (the masters' and workers' ASGI fronts, which serve
their hot routes as coroutines and everything else through the Flask app's WSGI adapter),
buffers the ASGI response and answers it. Same routes, bodies, status codes and headers as
under uvicorn; no streaming responses (none of the apps stream).
"""
from __future__ import annotations

from typing import Any, Callable


def asgi_handler(asgi_app: Callable, host: str, port: int):
    from aiohttp import web
    from multidict import CIMultiDict

    async def handler(request: "web.Request") -> "web.StreamResponse":
        body = await request.read()
        peer = request.transport.get_extra_info("peername") if request.transport else None
        scope = {
            "type": "http", "asgi": {"version": "3.0", "spec_version": "2.3"},
            "http_version": f"{request.version.major}.{request.version.minor}",
            "method": request.method, "scheme": "http", "path": request.path,
            "raw_path": request.raw_path.split("?", 1)[0].encode("latin-1"),
            "query_string": request.query_string.encode("latin-1"), "root_path": "",
            "headers": [(k.lower(), v) for k, v in request.raw_headers],
            "client": (peer[0], peer[1]) if peer else None, "server": (host, port),
        }
        delivered = False

        async def receive():
            nonlocal delivered
            if not delivered:
                delivered = True
                return {"type": "http.request", "body": body, "more_body": False}
            return {"type": "http.disconnect"}

        out: dict = {"status": 500, "headers": [], "body": []}

        async def send(msg):
            if msg["type"] == "http.response.start":
                out["status"] = msg["status"]
                out["headers"] = msg.get("headers", [])
            elif msg["type"] == "http.response.body":
                out["body"].append(msg.get("body", b""))

        await asgi_app(scope, receive, send)
        headers = CIMultiDict()
        for k, v in out["headers"]:
            name = k.decode("latin-1")
            if name.lower() in ("content-length", "transfer-encoding", "connection"):
                continue                     # aiohttp frames the buffered body itself
            headers.add(name, v.decode("latin-1"))
        return web.Response(status=out["status"], body=b"".join(out["body"]), headers=headers)

    return handler


def run_asgi(asgi_app: Any, host: str = "0.0.0.0", port: int = 8000,
             backlog: int = 4096, reuse_port: bool = False) -> None:
    from aiohttp import web
    app = web.Application(client_max_size=64 << 20)
    app.router.add_route("*", "/{tail:.*}", asgi_handler(asgi_app, host, port))

    async def lifespan_startup(_app):
        # the ASGI lifespan startup event (the master starts its dispatcher on this loop)
        msgs = [{"type": "lifespan.startup"}, {"type": "lifespan.shutdown"}]

        async def receive():
            return msgs.pop(0)

        async def send(_msg):
            return None
        try:
            await asgi_app({"type": "lifespan", "asgi": {"version": "3.0"}}, receive, send)
        except Exception:  # noqa: BLE001 — an app without lifespan support, as uvicorn's "auto"
            pass
    app.on_startup.append(lifespan_startup)
    web.run_app(app, host=host, port=port, backlog=backlog, access_log=None,
                print=None, keepalive_timeout=75, reuse_port=reuse_port or None)
