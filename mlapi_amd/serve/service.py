"""ServingRuntime: everything one serving process (one GPU) needs, wired together."""
from __future__ import annotations

import logging
import os
from typing import Optional

from mlapi_amd.serve.runtime import AsyncEngine, EngineHandle, ModelStore
from mlapi_amd.utils.config import Config
from mlapi_amd.utils import metrics as metrics_mod

log = logging.getLogger("mlapi_amd.serve")


class ServingRuntime:
    """Engine (GPU or CPU backend) + checkpoint store + asyncio client + metrics for one process."""

    owned_by_app = True

    def __init__(self, config: Config, *, device="config", load: bool = True, watch: bool = False):
        self.config = config
        self.handle = EngineHandle(config, device=device)
        self.store = ModelStore(self.handle, config.model_path, reload=config.reload, missing=config.missing_model)
        self.client = AsyncEngine(self.handle)
        self.http = None  # set by NativeServer
        self.rank = int(os.environ.get("RANK", "0"))
        if load:
            self.store.check()
        if watch:
            self.store.start_watcher(config.reload_interval_ms)

    def healthy(self) -> bool:
        return bool(self.handle.engine.healthy())

    def on_admin_reload(self) -> None:
        """Hook: the data-parallel runtime re-broadcasts weights to the other replicas here."""

    def metrics_text(self) -> str:
        srv = self.http.stats() if self.http is not None else None
        return metrics_mod.render(self.handle.stats(), srv,
                                  labels={"rank": str(self.rank), "backend": self.handle.backend},
                                  extra=[("mlapi_model_loads_total", self.store.loads, None),
                                         ("mlapi_serving_dtype_info", 1, {"small": str(self.config.dtype),
                                                                          "wide": str(self.config.wide_dtype)})])

    def close(self) -> None:
        self.store.stop()
        self.client.close()
        self.handle.close()
