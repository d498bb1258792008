"""ASGI fast path for ``POST /predict`` under ``uvicorn main:app`` (the reference's own deploy
command, `/root/reference/README.md:16`).

The FastAPI route (`api/app.py`) validates the body with pydantic, routes through Starlette and
serialises the response with ``json.dumps``; with uvicorn's h11 parser in front that is
~0.6 ms of CPU per request, most of it not the model. This pure-ASGI
middleware answers the common case itself, exactly as the native server's fast path does
(`csrc/http/server.cpp`): a POST to the predict path with a JSON content type whose body the
native strict parser accepts (every feature a finite JSON number, any extra members valid JSON)
goes straight to the batching engine and back as the same bytes FastAPI would send. Everything
else - other routes, malformed or unusual bodies, a missing checkpoint, a failed prediction - is
replayed unchanged into the FastAPI app, so every error response keeps the reference's shape.
"""
from __future__ import annotations

import json
from typing import Callable, List


MAX_FAST_BODY = 1 << 20  # bytes buffered here before the request is handed to the route as is


def _json_ctype(ct: str) -> bool:
    """FastAPI's rule (routing.py): maintype 'application', subtype 'json' or '*+json'."""
    v = ct.split(";", 1)[0].strip().lower()
    if not v.startswith("application/"):
        return False
    sub = v[len("application/"):]
    return sub == "json" or (len(sub) > 5 and sub.endswith("+json"))


class PredictFastPath:
    """Pure ASGI middleware (no BaseHTTPMiddleware task / stream overhead)."""

    served = 0  # requests answered here, process-wide (tests / diagnostics)

    def __init__(self, app, names: List[str], runtime: Callable, path: str = "/predict"):
        from mlapi_amd._native import C

        self.app = app
        self.names = list(names)
        self.runtime = runtime  # () -> ServingRuntime (created lazily by the app)
        self.path = path
        self._parse = C().parse_predict_body

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http" or scope["method"] != "POST" or scope["path"] != self.path:
            return await self.app(scope, receive, send)
        ctype = ""
        for k, v in scope.get("headers", ()):
            if k == b"content-type":  # the first one, like Starlette's request.headers[...]
                ctype = v.decode("latin-1")
                break
        if not _json_ctype(ctype):
            return await self.app(scope, receive, send)
        messages = []
        size = 0
        complete = False
        while True:
            msg = await receive()
            messages.append(msg)
            if msg["type"] != "http.request":
                break  # client went away: let the app see the same messages
            size += len(msg.get("body", b""))
            if not msg.get("more_body", False):
                complete = True
                break
            if size > MAX_FAST_BODY:
                break  # not a plausible feature record: the route reads (and judges) the rest
        result = None
        if complete:
            body = b"".join(m.get("body", b"") for m in messages)
            x = self._parse(body, self.names) if body else None
            if x is not None:
                result = await self._predict(x)
        if result is None:
            pending = list(messages)

            async def replay():
                return pending.pop(0) if pending else await receive()

            return await self.app(scope, replay, send)
        payload = json.dumps({"prediction": result[0], "probability": result[1]}, ensure_ascii=False,
                             allow_nan=False, indent=None, separators=(",", ":")).encode("utf-8")
        await send({"type": "http.response.start", "status": 200,
                    "headers": [(b"content-length", str(len(payload)).encode()),
                                (b"content-type", b"application/json")]})
        await send({"type": "http.response.body", "body": payload})
        PredictFastPath.served += 1

    async def _predict(self, x):
        """(label, probability), or None to let the FastAPI route produce the (error) response."""
        try:
            r = self.runtime()
            if not r.store.check():  # per-request checkpoint semantics (main.py:19)
                return None
            label, p = await r.client.predict_one(x)
            json.dumps(label)  # the route would fail to serialise it: let it
            return label, p
        except Exception:  # noqa: BLE001 - the slow path reproduces the exact error response
            return None
