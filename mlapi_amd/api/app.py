"""The FastAPI application: the reference's HTTP surface on top of the native engine.

Route-for-route parity with `main.py`:

* ``POST /predict`` (`main.py:16-27`): body ``IrisSpecies`` (4 required floats), response
  ``{"prediction": <label>, "probability": <max class probability>}``. The reference unpickles
  the checkpoint and runs sklearn twice per request; here the request is awaited on the batching
  engine (HIP kernel on a GPU, or the C++ CPU backend) and the checkpoint is hot-reloaded only
  when the file changes.
* ``POST /files/`` (`main.py:29-39`): multipart ``file`` + ``token`` -> CSV parsed with pandas,
  ``print(df)``, echoed back as ``{"file": {col: {row: value}}, "token": token}``.
* ``/docs``, ``/redoc``, ``/openapi.json``: FastAPI defaults; the schema matches the reference's
  (title "FastAPI", version "0.1.0", same operation ids and component schemas).

Extra routes (excluded from the OpenAPI schema so it stays identical): ``/healthz``,
``/readyz``, ``/metrics``, ``POST /admin/reload``.

Error behaviour follows the reference: validation errors are FastAPI's 422 bodies, any failure
in the model path is an HTTP 500 ``Internal Server Error`` (text/plain).
"""
import contextlib
import io
import logging
import math
from typing import Optional

from fastapi import FastAPI, Request
from fastapi.exceptions import RequestValidationError
from fastapi.responses import JSONResponse, PlainTextResponse, Response
from pydantic import BaseModel, create_model

from mlapi_amd.api.multipart import MultipartError, parse_form
from mlapi_amd.utils.config import IRIS_FEATURES, Config

log = logging.getLogger("mlapi_amd.api")


# Request schema of `POST /predict` (`main.py:10-14`). No docstring on purpose: pydantic would
# publish it as the schema "description" and /openapi.json would no longer match the reference.
class IrisSpecies(BaseModel):
    sepal_length: float
    sepal_width: float
    petal_length: float
    petal_width: float


def request_model(feature_names) -> type:
    if list(feature_names) == IRIS_FEATURES:
        return IrisSpecies
    return create_model("FeatureRecord", **{n: (float, ...) for n in feature_names})


FILES_OPENAPI = {
    "requestBody": {
        "content": {"multipart/form-data": {"schema": {"$ref": "#/components/schemas/Body_create_file_files__post"}}},
        "required": True,
    },
    "responses": {
        "422": {
            "description": "Validation Error",
            "content": {"application/json": {"schema": {"$ref": "#/components/schemas/HTTPValidationError"}}},
        }
    },
}
FILES_BODY_SCHEMA = {
    "properties": {
        "file": {"contentMediaType": "application/octet-stream", "title": "File", "type": "string"},
        "token": {"title": "Token", "type": "string"},
    },
    "required": ["file", "token"],
    "title": "Body_create_file_files__post",
    "type": "object",
}


def _missing(name: str) -> dict:
    return {"type": "missing", "loc": ["body", name], "msg": "Field required", "input": None}


def dataframe_payload(df, strict_parity: bool = True):
    """``jsonable_encoder(df)`` as the reference sees it: ``dict(df)`` -> {col: dict(series)}.

    ``dict(series)`` yields numpy scalars, exactly what FastAPI's encoder receives in the reference:
    numpy ints / bools are not JSON-encodable and NaN is rejected by ``json.dumps(allow_nan=False)``,
    so with ``strict_parity`` (default) those cells raise -> HTTP 500 like the reference.
    Otherwise they are converted (ints/bools to JSON numbers/booleans, NaN to null).
    """
    import numpy as np

    out = {}
    for col, series in dict(df).items():
        colmap = {}
        for idx, v in dict(series).items():
            if isinstance(v, (np.bool_, np.integer)):
                if strict_parity:
                    raise ValueError(f"{type(v).__name__} is not JSON serializable")
                v = v.item()
            elif isinstance(v, float) and not math.isfinite(v):
                if strict_parity:
                    raise ValueError("Out of range float values are not JSON compliant")
                v = None
            elif isinstance(v, np.generic):
                v = v.item()
            colmap[idx.item() if isinstance(idx, np.generic) else idx] = v
        out[col.item() if isinstance(col, np.generic) else col] = colmap
    return out


def create_app(config: Optional[Config] = None, *, runtime=None) -> FastAPI:
    """Build the app. ``runtime`` is a :class:`mlapi_amd.serve.service.ServingRuntime`; when
    omitted one is created lazily from ``config`` on first use (so `uvicorn main:app` works)."""
    config = config or Config.from_env()
    @contextlib.asynccontextmanager
    async def lifespan(_app):
        yield
        r = _app.state.runtime
        if r is not None and getattr(r, "owned_by_app", False):  # uvicorn main:app owns its runtime
            r.close()
            _app.state.runtime = None

    # no title/version: OpenAPI info stays {"title": "FastAPI", "version": "0.1.0"} like the reference
    app = FastAPI(lifespan=lifespan)
    app.state.config = config
    app.state.runtime = runtime
    Record = request_model(config.feature_names)
    names = list(config.feature_names)

    def rt():
        if app.state.runtime is None:
            from mlapi_amd.serve.service import ServingRuntime

            app.state.runtime = ServingRuntime(config)
        return app.state.runtime

    if config.asgi_fast_path and names:
        from mlapi_amd.api.fastpath import PredictFastPath

        app.add_middleware(PredictFastPath, names=names, runtime=rt)

    from mlapi_amd.serve.runtime import EngineBusy

    @app.exception_handler(EngineBusy)
    async def _busy(request, exc):  # backpressure (not in the reference, which has no queue)
        return JSONResponse({"detail": str(exc)}, status_code=503, headers={"retry-after": "1"})

    @app.post("/predict")
    async def predict_species(iris: Record):  # type: ignore[valid-type]
        data = iris.model_dump()
        r = rt()
        if not r.store.check():  # per-request checkpoint semantics (main.py:19), via stat()
            raise RuntimeError(r.store.last_error or "no model loaded")
        label, probability = await r.client.predict_one([data[n] for n in names])
        return {"prediction": label, "probability": probability}

    @app.post("/files/", openapi_extra=FILES_OPENAPI)
    async def create_file(request: Request):
        body = await request.body()
        try:
            parts = parse_form(body, request.headers.get("content-type"))
        except MultipartError:  # Starlette: MultiPartException -> 400 (fastapi/routing.py)
            return JSONResponse({"detail": "There was an error parsing the body"}, status_code=400)
        fields = {}
        for p in parts:
            fields[p.name] = p  # last one wins, like FormData.get
        errors = []
        fpart, tpart = fields.get("file"), fields.get("token")
        if fpart is None or (not fpart.is_file and fpart.data == b""):
            errors.append(_missing("file"))
        if tpart is None or (not tpart.is_file and tpart.data == b""):
            errors.append(_missing("token"))
        if errors:
            raise RequestValidationError(errors)
        import pandas as pd

        s = str(fpart.data, "utf-8")  # main.py:31
        df = pd.read_csv(io.StringIO(s))  # main.py:32-33
        print(df)  # main.py:34
        token = tpart.data.decode("utf-8")
        return {"file": dataframe_payload(df, strict_parity=config.files_strict_parity), "token": token}

    # ---- operational endpoints (not part of the reference schema)
    @app.get("/healthz", include_in_schema=False)
    async def healthz():
        r = app.state.runtime
        ok = r is None or r.healthy()
        return JSONResponse({"status": "ok" if ok else "unhealthy"}, status_code=200 if ok else 503)

    @app.get("/readyz", include_in_schema=False)
    async def readyz():
        r = rt()
        ready = r.store.check() and r.healthy()
        return JSONResponse({"ready": bool(ready), "model_version": r.handle.version, "backend": r.handle.backend,
                             "error": r.store.last_error}, status_code=200 if ready else 503)

    @app.get("/metrics", include_in_schema=False)
    async def metrics():
        return PlainTextResponse(rt().metrics_text(), media_type="text/plain; version=0.0.4")

    def admin_allowed(request: Request) -> bool:
        mode = str(config.admin).lower()
        if mode == "on":
            return True
        if mode == "off":
            return False
        host = request.client.host if request.client else ""
        return host in ("127.0.0.1", "::1", "localhost", "testclient")  # loopback (default)

    @app.post("/admin/reload", include_in_schema=False)
    async def admin_reload(request: Request):
        if not admin_allowed(request):
            return JSONResponse({"detail": "Not Found"}, status_code=404)
        r = rt()
        r.store.invalidate()  # next check() re-reads the file
        ok = r.store.check()
        r.on_admin_reload()
        return JSONResponse({"reloaded": ok, "model_version": r.handle.version, "error": r.store.last_error},
                            status_code=200 if ok else 500)

    _orig_openapi = app.openapi

    def openapi():
        if app.openapi_schema:
            return app.openapi_schema
        schema = _orig_openapi()
        schema.setdefault("components", {}).setdefault("schemas", {})["Body_create_file_files__post"] = \
            FILES_BODY_SCHEMA
        schemas = schema["components"]["schemas"]
        schema["components"]["schemas"] = {k: schemas[k] for k in sorted(schemas)}
        app.openapi_schema = schema
        return schema

    app.openapi = openapi  # type: ignore[method-assign]

    return app
