"""Data-parallel serving: one replica per GPU (BASELINE config 4: DP=8 over xGMI).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m mlapi_amd.serve --port 8000

* Rank 0 alone reads the checkpoint (restricted unpickler) and the weights reach every replica
  through one RCCL broadcast (collective C1, :func:`mlapi_amd.parallel.comm.broadcast_model`).
* Every rank runs the native HTTP server on the SAME port with SO_REUSEPORT, so the kernel
  spreads client connections over the 8 processes; each process feeds its own GPU's request
  queue/batcher (per-GPU queues). ``--port-stride 1`` gives each rank its own port instead
  (port + rank) for an external round-robin balancer.
* Hot reload keeps the reference's "replace the file, the served model changes" behaviour
  (main.py:19) cluster-wide: a control thread on every rank joins a tiny MAX all-reduce (gloo,
  host side) every ``reload_interval_ms``; when rank 0 has seen the file change (or any rank got
  ``POST /admin/reload``), all ranks enter the same RCCL broadcast and swap models atomically.
  A deleted checkpoint is broadcast as "no model" and every replica answers 500 (A16).
* Replica restart (``python -m mlapi_amd.launch --restart N``): a replica that dies is started
  again by the launcher with ``MLAPI_REPLICA_RESTART`` set. It cannot rejoin the survivors' RCCL /
  gloo groups, so it comes back as a standalone replica (:func:`serve_replica`): it reads the
  checkpoint itself, joins the same SO_REUSEPORT port and watches the file on its own. The
  survivors' reload controller sees its control group break at the next tick and falls back to
  per-rank file watching, so "replace the file, the served model changes" keeps holding.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from mlapi_amd.models.linear import LinearModel
from mlapi_amd.parallel.comm import DistInfo, broadcast_model, init_distributed, shutdown
from mlapi_amd.utils.config import Config

log = logging.getLogger("mlapi_amd.dp")


class DPReloadController:
    """Cluster-wide hot reload: rank 0 watches the file, every rank applies the same broadcast."""

    def __init__(self, runtime, info: DistInfo, interval_ms: int):
        self.rt = runtime
        self.info = info
        self.interval = max(5, interval_ms) / 1000.0
        self.ctrl = dist.new_group(backend="gloo") if info.world > 1 else None
        self.local_gen = 0       # rank 0: bumps on every file change
        self.applied_gen = 0
        self.request = threading.Event()
        self._stop = threading.Event()
        self._key = None
        self.degraded = False
        self._thread: Optional[threading.Thread] = None

    def _file_key(self):
        try:
            st = os.stat(self.rt.config.model_path)
            return (st.st_mtime_ns, st.st_size, st.st_ino)
        except OSError:
            return None

    def start(self, initial_key) -> None:
        self._key = initial_key
        self._thread = threading.Thread(target=self._run, name="mlapi-dp-reload", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            try:
                self.tick()
            except Exception as e:  # a peer left the control group (crashed / restarted replica)
                self.degrade(e)
                return

    def degrade(self, err: Exception) -> None:
        """The control group is broken: keep serving and reload from the file locally instead."""
        log.warning("rank %d: DP reload group failed (%s); falling back to per-rank file watching",
                    self.info.rank, err)
        self.degraded = True
        st = self.rt.store
        st.reload = self.rt.config.reload
        st._key = self._key if self._key is not None else ("unchecked",)
        st.start_watcher(self.rt.config.reload_interval_ms)

    def tick(self) -> None:
        req = 1 if self.request.is_set() else 0
        self.request.clear()
        if self.info.is_main and self.rt.config.reload != "off":
            key = self._file_key()
            if key != self._key:
                self._key = key
                self.local_gen += 1
        t = torch.tensor([self.local_gen, req], dtype=torch.int64)
        if self.ctrl is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctrl)
        gen, any_req = int(t[0]), int(t[1])
        if any_req and self.info.is_main:
            self.local_gen = gen + 1  # serviced on the next tick
        if gen > self.applied_gen:
            self.apply(gen)

    def apply(self, gen: int) -> None:
        """All ranks: rank 0 loads the file, RCCL-broadcasts (or broadcasts 'missing')."""
        model = None
        present = torch.tensor([0], dtype=torch.int64)
        if self.info.is_main:
            try:
                from mlapi_amd.ckpt.native import load_model

                model = load_model(self.rt.config.model_path)
                present[0] = 1
            except Exception as e:
                self.rt.store.last_error = f"{type(e).__name__}: {e}"
        if self.ctrl is not None:
            dist.broadcast(present, 0, group=self.ctrl)
        if int(present[0]) == 1:
            model = broadcast_model(model, self.info)  # C1 over RCCL
            self.rt.handle.load(model)
            self.rt.store.last_error = None
        elif self.rt.config.missing_model == "error":
            self.rt.handle.unload()
        self.applied_gen = gen
        log.info("rank %d applied model generation %d", self.info.rank, gen)


def start_dp_runtime(cfg: Config, info: Optional[DistInfo] = None):
    """Build this rank's ServingRuntime with the weights broadcast from rank 0 (no file I/O elsewhere)."""
    from mlapi_amd.serve.service import ServingRuntime

    info = info or init_distributed()
    local = int(os.environ.get("LOCAL_WORLD_SIZE", info.world))
    if cfg.pin == "on" or (cfg.pin == "auto" and local > 1 and not os.environ.get("MLAPI_LAUNCHER")):
        # before the engine / server threads exist: they inherit this rank's CPU slice
        from mlapi_amd.utils.affinity import pin_this_rank

        cpus = pin_this_rank(info.local_rank, local, None if info.device is None else info.device.index)
        log.info("rank %d pinned to %d CPUs", info.rank, len(cpus))
    model = None
    if info.is_main:
        from mlapi_amd.ckpt.native import load_model

        model = load_model(cfg.model_path)
    model = broadcast_model(model, info)
    device = "cpu" if info.device is None else f"cuda:{info.device.index}"
    rcfg = Config.from_env(**{**cfg.__dict__, "device": device})
    rt = ServingRuntime(rcfg, load=False)
    rt.handle.load(model)
    if cfg.fault_drop_rank == info.rank:  # fault injection: this replica fails every batch
        log.warning("rank %d: fault injection, dropping this replica", info.rank)
        rt.handle.engine.inject_drop(True)
    rt.store.reload = "off"  # the controller owns reloads in DP mode
    ctl = DPReloadController(rt, info, cfg.reload_interval_ms)
    rt.on_admin_reload = ctl.request.set  # POST /admin/reload on any rank
    try:
        st = os.stat(cfg.model_path)
        key = (st.st_mtime_ns, st.st_size, st.st_ino)
    except OSError:
        key = None
    return rt, ctl, key, info


def serve_replica(cfg: Config, port_stride: int = 0) -> int:
    """A restarted replica (``MLAPI_REPLICA_RESTART``): standalone on this rank's GPU and port."""
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.serve.service import ServingRuntime

    rank = int(os.environ.get("RANK", "0"))
    # device "auto" resolves to this rank's GPU through LOCAL_RANK (Config.device_index)
    rcfg = Config.from_env(**{**cfg.__dict__, "port": cfg.port + port_stride * rank, "reuseport": True})
    srv = NativeServer(rcfg, runtime=ServingRuntime(rcfg))
    log.warning("rank %d restarted (%s): standalone replica on port %d", rank,
                os.environ.get("MLAPI_REPLICA_RESTART"), srv.port)
    srv.serve_forever()
    return 0


def serve_dp(cfg: Config, port_stride: int = 0) -> int:
    from mlapi_amd.serve.server import NativeServer

    rt, ctl, key, info = start_dp_runtime(cfg)
    cfg_r = Config.from_env(**{**cfg.__dict__, "port": cfg.port + port_stride * info.rank, "reuseport": True})
    srv = NativeServer(cfg_r, runtime=rt)
    ctl.start(key)
    if cfg.fault_exit_rank == info.rank:  # fault injection: a replica process dies while serving
        log.warning("rank %d: fault injection, exiting in %d ms", info.rank, cfg.fault_exit_after_ms)
        threading.Timer(cfg.fault_exit_after_ms / 1000.0, lambda: os._exit(3)).start()
    log.info("rank %d/%d serving on port %d (%s)", info.rank, info.world, srv.port, rt.handle.backend)
    try:
        srv.serve_forever()
    finally:
        ctl.stop()
        shutdown(info)
    return 0
