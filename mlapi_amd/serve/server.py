"""NativeServer: the production front end (native HTTP fast path + ASGI slow path).

    python -m mlapi_amd.serve --port 8000                 # one process, one GPU (or CPU backend)
    torchrun --nproc-per-node 8 -m mlapi_amd.serve ...    # DP=8 replicas sharing one port

Compared with `uvicorn main:app` (which also works and serves the same app), the native server
parses/answers valid `/predict` requests in C++ IO threads and only hands the remaining traffic
to FastAPI; the model runs in the same batching engine either way.
"""
from __future__ import annotations

import atexit
import logging
import os
import signal
import threading
import weakref
from typing import Optional

from mlapi_amd._native import C
from mlapi_amd.api.app import create_app
from mlapi_amd.serve.asgi_bridge import AsgiBridge
from mlapi_amd.serve.service import ServingRuntime
from mlapi_amd.utils.config import Config

log = logging.getLogger("mlapi_amd.serve")

# Servers still running when the interpreter exits (e.g. an exception escaped between start() and
# stop()): their ASGI pump threads are daemon threads parked inside HttpServer.next_slow with the
# GIL released. During finalization such a thread is torn down by a forced unwind when it tries to
# take the GIL back, and that unwind through pybind11's noexcept gil_scoped_release ends the
# process in std::terminate ("terminate called without an active exception", rc 134). atexit
# handlers run before finalization, so stopping the servers there joins those threads cleanly.
_RUNNING: "weakref.WeakSet[NativeServer]" = weakref.WeakSet()


@atexit.register
def _stop_running_servers() -> None:
    for srv in list(_RUNNING):
        try:
            srv.stop()
        except Exception:  # pragma: no cover - best effort at exit
            log.exception("stopping server at exit")


class NativeServer:
    def __init__(self, config: Config, runtime: Optional[ServingRuntime] = None, app=None,
                 access_log_fd: int = 2):
        self.config = config
        self.runtime = runtime or ServingRuntime(config)
        self.runtime.owned_by_app = False
        self.app = app or create_app(config, runtime=self.runtime)
        c = C()
        sc = c.ServerConfig()
        sc.host = config.host
        sc.port = int(config.port)
        sc.io_threads = int(config.io_threads)
        sc.reuseport = bool(config.reuseport)
        sc.feature_names = list(config.feature_names)
        sc.server_header = config.server_header
        sc.fast_path = bool(config.fast_path)
        sc.access_log = bool(config.access_log)
        sc.io_spin_us = int(config.io_spin_us)
        sc.io_wait_spin_us = int(config.io_wait_spin_us)
        sc.io_ring_spin_us = int(config.io_ring_spin_us)
        sc.io_ring_sleep_us = int(config.io_ring_sleep_us)
        sc.idle_max_conns = int(config.idle_max_conns)
        sc.io_spin_lowload_us = int(config.io_spin_lowload_us)
        sc.io_spin_max_conns = int(config.io_spin_max_conns)
        sc.io_steer = int(config.io_steer)
        sc.steer_every = int(config.steer_every)
        sc.steer_stable = int(config.steer_stable)
        sc.io_cpus = [int(c) for c in str(config.io_cpus).split(",") if c.strip()]
        sc.access_log_fd = int(access_log_fd)
        sc.dispatch = str(config.dispatch)
        sc.dispatch_group = str(config.dispatch_group)
        sc.dispatch_claim = str(config.dispatch_claim)
        sc.dispatch_rank = int(os.environ.get("RANK", "0"))
        hd = str(config.health_dispatch).lower()
        sc.health_dispatch = hd == "on" or (hd == "auto" and int(os.environ.get("WORLD_SIZE", "1")) > 1)
        self.http = c.HttpServer(self.runtime.handle.engine, sc)
        self.runtime.http = self.http
        self.bridge = AsgiBridge(self.app, self.http, workers=config.slow_workers)
        self._started = False

    @property
    def port(self) -> int:
        return int(self.http.port())

    def start(self) -> "NativeServer":
        self.runtime.store.start_watcher(self.config.reload_interval_ms)
        self.http.start()
        self.bridge.start()
        self._started = True
        _RUNNING.add(self)
        log.info("serving on %s:%d (backend %s)", self.config.host, self.port, self.runtime.handle.backend)
        return self

    def stop(self) -> None:
        if not self._started:
            return
        self._started = False
        _RUNNING.discard(self)
        self.http.stop()
        self.bridge.stop()
        self.runtime.close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    def serve_forever(self) -> None:
        stop = threading.Event()
        for sig in (signal.SIGINT, signal.SIGTERM):
            try:
                signal.signal(sig, lambda *_: stop.set())
            except ValueError:  # not main thread
                pass
        self.start()
        try:
            while not stop.wait(0.5):
                pass
        finally:
            self.stop()
