"""Slow path of the native HTTP server: run requests through the FastAPI ASGI app in-process.

Requests the native fast path does not take (validation errors, `/files/`, docs, 404/405, ...)
arrive from ``HttpServer.next_slow()`` on a pump thread, are executed by the ASGI app on a
dedicated asyncio loop, and the complete response goes back via ``HttpServer.respond()``.
This keeps every non-fast response byte-identical to what FastAPI itself produces.
"""
from __future__ import annotations

import asyncio
import http
import logging
import threading
from typing import Optional
from urllib.parse import unquote

log = logging.getLogger("mlapi_amd.bridge")


def _reason(status: int) -> str:
    try:
        return http.HTTPStatus(status).phrase
    except ValueError:
        return "Unknown"


class AsgiBridge:
    def __init__(self, app, server, workers: int = 1):
        self.app = app
        self.server = server
        self.workers = max(1, workers)
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self._loop_thread: Optional[threading.Thread] = None
        self._pumps: list = []
        self._stop = threading.Event()
        self._lifespan_q: Optional[asyncio.Queue] = None
        self._lifespan_task = None
        self._ready = threading.Event()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        self._loop_thread = threading.Thread(target=self._run_loop, name="mlapi-asgi", daemon=True)
        self._loop_thread.start()
        self._ready.wait(30)
        fut = asyncio.run_coroutine_threadsafe(self._lifespan("startup"), self.loop)
        fut.result(30)
        for i in range(self.workers):
            t = threading.Thread(target=self._pump, name=f"mlapi-slow-{i}", daemon=True)
            t.start()
            self._pumps.append(t)

    def stop(self) -> None:
        self._stop.set()
        for t in self._pumps:
            t.join(timeout=2)
        if self.loop is not None:
            try:
                asyncio.run_coroutine_threadsafe(self._lifespan("shutdown"), self.loop).result(10)
            except Exception:
                pass
            self.loop.call_soon_threadsafe(self.loop.stop)
        if self._loop_thread is not None:
            self._loop_thread.join(timeout=5)

    def _run_loop(self) -> None:
        self.loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self.loop)
        self._ready.set()
        self.loop.run_forever()

    async def _lifespan(self, phase: str) -> None:
        if self._lifespan_q is None:
            self._lifespan_q = asyncio.Queue()
            out_q: asyncio.Queue = asyncio.Queue()
            self._lifespan_out = out_q

            async def receive():
                return await self._lifespan_q.get()

            async def send(msg):
                await out_q.put(msg)

            scope = {"type": "lifespan", "asgi": {"version": "3.0", "spec_version": "2.0"}, "state": {}}

            async def runner():
                try:
                    await self.app(scope, receive, send)
                except Exception:  # app does not support lifespan
                    await out_q.put({"type": "lifespan.unsupported"})

            self._lifespan_task = asyncio.ensure_future(runner())
        await self._lifespan_q.put({"type": f"lifespan.{phase}"})
        try:
            msg = await asyncio.wait_for(self._lifespan_out.get(), 30)
        except asyncio.TimeoutError:
            return
        if msg["type"].endswith(".failed"):
            raise RuntimeError(f"ASGI lifespan {phase} failed: {msg.get('message')}")

    # ------------------------------------------------------------------ requests
    def _pump(self) -> None:
        while not self._stop.is_set():
            req = self.server.next_slow(100)
            if req is None:
                continue
            asyncio.run_coroutine_threadsafe(self._handle(req), self.loop)

    async def _handle(self, req: dict) -> None:
        target: bytes = req["target"]
        path_b, _, qs = target.partition(b"?")
        scope = {
            "type": "http",
            "asgi": {"version": "3.0", "spec_version": "2.3"},
            "http_version": req["http_version"],
            "method": req["method"],
            "scheme": "http",
            "path": unquote(path_b.decode("latin-1")),
            "raw_path": path_b,
            "query_string": qs,
            "root_path": "",
            "headers": req["headers"],
            "client": tuple(req["client"]),
            "server": tuple(req["server"]),
            "state": {},
        }
        body = req["body"]
        sent = False

        async def receive():
            nonlocal sent
            if not sent:
                sent = True
                return {"type": "http.request", "body": body, "more_body": False}
            await asyncio.sleep(3600)  # no disconnect notifications from the native side
            return {"type": "http.disconnect"}

        status = 500
        headers: list = []
        chunks: list = []

        async def send(msg):
            nonlocal status, headers
            if msg["type"] == "http.response.start":
                status = msg["status"]
                headers = [(k.decode("latin-1"), v.decode("latin-1")) for k, v in msg.get("headers", [])]
            elif msg["type"] == "http.response.body":
                chunks.append(msg.get("body", b""))

        try:
            await self.app(scope, receive, send)
        except Exception:
            # Mirror Starlette's ServerErrorMiddleware if the app raised past it.
            log.exception("unhandled error in ASGI app")
            status, chunks = 500, [b"Internal Server Error"]
            headers = [("content-length", "21"), ("content-type", "text/plain; charset=utf-8")]
        body_out = b"".join(chunks)
        self.server.respond(req["token"], status, _reason(status), headers, body_out, False)
