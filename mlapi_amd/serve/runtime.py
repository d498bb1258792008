"""Python side of the serving runtime: native engine handle, model store (hot reload), async client.

* :class:`EngineHandle` owns one native ``_C.Engine`` (one GPU, or the C++ CPU backend) and the
  version -> :class:`LinearModel` map used to turn a returned class index into the label of the
  model that actually computed it (an in-flight batch may finish on the previous model).
* :class:`ModelStore` reproduces the reference's *de-facto hot swap*: the reference re-opens
  'LRClassifier.pkl' on every request (`main.py:19`), so replacing the file changes the served
  model and deleting it makes every request fail with 500. Here the file is
  stat()ed (cheap) instead of unpickled, and only a changed (mtime, size, inode) triggers a
  restricted unpickle + an atomic model swap in the engine.
* :class:`AsyncEngine` lets asyncio code ``await`` a single-row prediction: requests from all
  coroutines go into the engine's batcher; completions come back through an eventfd watched
  by the event loop (no thread hop per request).
"""
from __future__ import annotations

import asyncio
import logging
import math
import os
import threading
import time
from typing import Dict, Optional, Tuple

import numpy as np

from mlapi_amd._native import C
from mlapi_amd.models.linear import LinearModel
from mlapi_amd.utils.config import Config

log = logging.getLogger("mlapi_amd.serve")

DTYPES = {"f64": 0, "float64": 0, "f32": 1, "float32": 1, "bf16": 2, "bfloat16": 2}


class PredictionError(RuntimeError):
    """Maps to HTTP 500 Internal Server Error (the reference's behaviour for every failure)."""


class EngineBusy(PredictionError):
    """Backpressure: the engine queue is over ``max_queue`` -> HTTP 503 with Retry-After."""


class EngineHandle:
    def __init__(self, config: Config, device: Optional[int] = "config"):
        c = C()
        self.config = config
        self.device = config.device_index() if device == "config" else device
        ec = c.EngineConfig()
        ec.device = -1 if self.device is None else int(self.device)
        ec.max_batch = config.max_batch
        ec.max_wait_us = config.max_wait_us
        ec.slots = config.slots
        ec.dtype = DTYPES[config.dtype]
        ec.wide_dtype = DTYPES[config.wide_dtype]
        ec.split_max_rows = int(config.split_max_rows)
        ec.bar_rows = int(config.bar_rows)
        ec.host_merge_rows = int(config.host_merge_rows)
        ec.max_features = max(64, len(config.feature_names))
        ec.watchdog_ms = config.watchdog_ms
        ec.fail_every = config.fail_every
        ec.delay_us = config.delay_us
        ec.spin_us = config.spin_us
        ec.inline_args = bool(config.inline_args)
        ec.idle_inline_rows = int(config.idle_inline_rows)
        res = str(config.resident).strip().lower()
        # auto: on for a GPU of this rank's own and CPUs for its polling IO threads (resident_auto_ok)
        from mlapi_amd.parallel.comm import resident_auto_ok

        ec.resident = 1 if res == "on" or (res == "auto" and self.device is not None and resident_auto_ok()) else 0
        ec.resident_depth = int(config.resident_depth)
        ec.resident_idle_polls = int(config.resident_idle_polls)
        ec.resident_lease_ms = int(config.resident_lease_ms)
        ec.f32_gemv = bool(config.f32_gemv)
        ec.wide_host_merge_blocks = int(config.wide_host_merge_blocks)
        ec.completers = int(config.completers)
        ec.batchers = int(config.batchers)
        ec.gemv_record_rows = int(config.gemv_record_rows)
        ec.direct_wide = bool(config.direct_wide)
        ec.direct_wide_max_weight_bytes = int(config.direct_wide_max_weight_bytes)
        ec.record_completion = bool(config.record_completion)
        ec.stage_wide = bool(config.stage_wide)
        ec.max_queue = config.max_queue
        ec.direct_dispatch = bool(config.direct_dispatch)
        if ec.direct_dispatch:
            from mlapi_amd._build import hsaco_path

            hp = hsaco_path()
            ec.hsaco_path = str(hp) if hp.exists() else ""
        self.engine = c.Engine(ec)
        self._models: Dict[int, LinearModel] = {}
        self._lock = threading.Lock()
        self.version = 0

    @property
    def backend(self) -> str:
        return "cpu" if self.device is None else f"hip:{self.device}"

    def load(self, model: LinearModel) -> int:
        labels = model.label_json()
        if self.config.int_labels == "error" and model.classes.dtype.kind in "iub":
            labels = []  # reference parity (A17): integer labels are not JSON-encodable -> 500
        v = int(self.engine.load_model(int(model.kind), model.W, model.b, labels))
        with self._lock:
            self._models[v] = model
            for old in [k for k in self._models if k < v - 8]:  # keep a few for in-flight batches
                del self._models[old]
            self.version = v
        return v

    def unload(self) -> None:
        self.engine.unload_model()
        with self._lock:
            self.version = 0

    def model_for(self, version: int) -> Optional[LinearModel]:
        with self._lock:
            return self._models.get(version)

    def current_model(self) -> Optional[LinearModel]:
        with self._lock:
            return self._models.get(self.version) if self.version else None

    def stats(self) -> dict:
        return dict(self.engine.stats())

    def close(self) -> None:
        self.engine.stop()


class ModelStore:
    """Watches the checkpoint path and keeps the engine's model in sync with it."""

    def __init__(self, handle: EngineHandle, path: str, *, reload: str = "mtime", missing: str = "error"):
        self.handle = handle
        self.path = path
        self.reload = reload
        self.missing = missing
        self._key = ("unchecked",)  # sentinel: the first check() always looks at the file
        self._lock = threading.Lock()
        self._watcher: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.last_error: Optional[str] = None
        self.loads = 0

    def invalidate(self) -> None:
        """Forget the file's identity: the next :meth:`check` re-reads the checkpoint."""
        with self._lock:
            self._key = ("unchecked",)

    def _stat_key(self):
        try:
            st = os.stat(self.path)
        except OSError:
            return None
        return (st.st_mtime_ns, st.st_size, st.st_ino)

    def check(self) -> bool:
        """Sync with the file; returns True when a model is being served."""
        if self.reload == "off" and self._key != ("unchecked",):
            return self.handle.version != 0
        key = self._stat_key()
        if key == self._key:
            return self.handle.version != 0
        with self._lock:
            key = self._stat_key()
            if key == self._key:
                return self.handle.version != 0
            if key is None:
                self.last_error = f"checkpoint {self.path!r} not found"
                if self.missing == "error":
                    self.handle.unload()
                self._key = None
                return self.handle.version != 0
            try:
                from mlapi_amd.ckpt.native import load_model

                model = load_model(self.path)
                if model.n_features != len(self.handle.config.feature_names):
                    raise ValueError(f"checkpoint has {model.n_features} features, the API schema has "
                                     f"{len(self.handle.config.feature_names)}")
                self.handle.load(model)
                self.loads += 1
                self.last_error = None
                log.info("loaded %s (v%d, %s, %s)", self.path, self.handle.version, model.kind.name,
                         self.handle.backend)
            except Exception as e:  # corrupt / unsafe / truncated file: 500s like the reference
                self.last_error = f"{type(e).__name__}: {e}"
                log.error("failed to load %s: %s", self.path, self.last_error)
                if self.missing == "error":
                    self.handle.unload()
            self._key = key
            return self.handle.version != 0

    def start_watcher(self, interval_ms: int) -> None:
        if self._watcher is not None or self.reload == "off":
            return

        def run():
            while not self._stop.wait(interval_ms / 1000.0):
                try:
                    self.check()
                except Exception:  # pragma: no cover - never kill the watcher
                    log.exception("model watcher")

        self._watcher = threading.Thread(target=run, name="mlapi-model-watcher", daemon=True)
        self._watcher.start()

    def stop(self) -> None:
        self._stop.set()
        if self._watcher is not None:
            self._watcher.join(timeout=2)


class AsyncEngine:
    """asyncio front of an EngineHandle: ``await predict_one(row)`` -> (label, p_max)."""

    def __init__(self, handle: EngineHandle):
        self.handle = handle
        self._per_loop: Dict[int, Tuple[object, dict]] = {}
        self._tag = 0
        self._lock = threading.Lock()

    def _state(self):
        loop = asyncio.get_running_loop()
        st = self._per_loop.get(id(loop))
        if st is None or st[2] is not loop:  # a new loop may reuse a dead loop's id()
            sink = C().PySink()
            futures: dict = {}

            def on_ready():
                for tag, idx, status, p, _lat, version in sink.drain():
                    fut = futures.pop(tag, None)
                    if fut is not None and not fut.done():
                        fut.set_result((idx, status, p, version))

            loop.add_reader(sink.fd(), on_ready)
            st = (sink, futures, loop)
            self._per_loop[id(loop)] = st
        return st

    async def predict_raw(self, row) -> Tuple[int, int, float, int]:
        sink, futures, loop = self._state()
        with self._lock:
            self._tag += 1
            tag = self._tag
        fut = loop.create_future()
        futures[tag] = fut
        r = self.handle.engine.submit(np.asarray(row, dtype=np.float64), tag, sink)
        if r != 1:
            futures.pop(tag, None)
            if r < 0:
                raise EngineBusy("server overloaded, retry later")
            raise PredictionError("engine is not accepting requests")
        return await fut

    async def predict_one(self, row):
        x = [float(v) for v in row]
        if not all(math.isfinite(v) for v in x):
            # sklearn check_array: "Input X contains NaN or infinity." -> HTTP 500 (A12)
            raise PredictionError("Input X contains NaN or infinity.")
        idx, status, p, version = await self.predict_raw(x)
        if status != 0:
            raise PredictionError(f"prediction failed (status {status})")
        model = self.handle.model_for(version)
        if model is None:
            raise PredictionError("model version evicted")
        label = model.label_python(idx)
        if self.handle.config.int_labels == "error" and not isinstance(label, (str, float)):
            raise PredictionError("integer label is not JSON serializable")  # reference A17
        return label, float(p)

    def close(self) -> None:
        for sink, _f, loop in list(self._per_loop.values()):
            try:
                loop.remove_reader(sink.fd())
            except Exception:
                pass
        self._per_loop.clear()


def wait_for(pred, timeout_s: float = 5.0, interval_s: float = 0.005) -> bool:
    t = time.time() + timeout_s
    while time.time() < t:
        if pred():
            return True
        time.sleep(interval_s)
    return pred()
