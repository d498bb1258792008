"""Typed configuration from environment variables and CLI flags.

The reference has no configuration: the checkpoint path 'LRClassifier.pkl' is hard-coded and
resolved against the CWD on every request (`main.py:19`), the feature order is hard-coded
(`main.py:20`) and the only knobs are uvicorn's CLI flags (`README.md:16`). Defaults here keep
every one of those behaviours; everything else is opt-in.

Every field ``foo`` can be set with the environment variable ``MLAPI_FOO``.
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field
from typing import List, Optional

IRIS_FEATURES = ["sepal_length", "sepal_width", "petal_length", "petal_width"]  # main.py:11-14,20


@dataclass
class Config:
    # model / checkpoint
    model_path: str = "LRClassifier.pkl"      # main.py:19 (relative to the CWD, like the reference)
    reload: str = "mtime"                     # "mtime": hot-reload when the file changes; "off"
    reload_interval_ms: int = 50              # watcher period for the native fast path
    missing_model: str = "error"              # "error": HTTP 500 while the file is absent (A16); "keep"
    feature_names: List[str] = field(default_factory=lambda: list(IRIS_FEATURES))
    int_labels: str = "json"                  # "json": render int labels as numbers; "error": 500 like A17
    files_strict_parity: bool = True          # /files/: 500 on int/bool/NaN cells like the reference (R4d)
    # device / engine
    device: str = "auto"                      # "auto" | "cpu" | "cuda" | "cuda:N" | "N"
    dtype: str = "f64"                        # small-model (F<=32, K<=16) compute dtype: f64 (sklearn parity) | f32
    wide_dtype: str = "f64"                   # wider models: f64 storage on the f64-accumulating WIDE kernel (sklearn's
                                              # dtype: byte-exact bodies) | f32 (opt-in: f32 storage, same kernel)
                                              # | bf16 (opt-in: bf16 GEMV / MFMA GEMM)
    split_max_rows: int = 32                  # bf16 multiclass: batches <= this many rows take the class-split kernel
    bar_rows: int = 32                        # GPU wide paths: batches <= this many rows go to HBM through the BAR (0 = off)
    host_merge_rows: int = 16                 # GPU multiclass: class-split batches <= this many rows merge on the host
    max_batch: int = 256
    max_wait_us: int = 0                      # 0 = continuous batching
    slots: int = 4
    watchdog_ms: int = 2000
    fail_every: int = 0                       # fault injection (tests): fail every N-th batch
    delay_us: int = 0                         # fault injection: delay every batch
    spin_us: int = 0                          # batcher / completer spin before sleeping (0 = always sleep)
    io_spin_us: int = 0                       # IO threads busy-poll this long after activity (0 = block)
    io_wait_spin_us: int = 3                  # IO threads with rows in the engine watch for the hand-off this
                                              # long in user space before blocking (0 = off; 1-5 us measured
                                              # best, profiles/r4_waitspin/)
    idle_max_conns: int = 0                   # idle-engine path only while <= this many connections are open (0 = any)
    io_spin_lowload_us: int = 50              # ... only while <= io_spin_max_conns connections are open (batch=1 clients)
    io_spin_max_conns: int = 2
    io_steer: int = 1                         # group connections on IO threads by their SO_INCOMING_CPU (0 = off)
    steer_every: int = 32                     # ... sampled every this many requests per connection
    steer_stable: int = 3                     # ... moved only after this many samples in a row on one CPU
    io_cpus: str = ""                          # IO thread i pinned to the i-th CPU of this comma list (threads past it unpinned)
    max_queue: int = 1 << 20                  # backpressure: queued rows beyond this -> HTTP 503
    inline_args: bool = True                  # GPU: tiny batches travel in the kernel-argument block
    record_completion: bool = True            # GPU: kernel-argument batches complete through 16-B per-row records
    completers: int = 1                       # GPU: completer threads (done-word wait + delivery)
    batchers: int = 1                         # batcher threads (queue take + launch; launches serialised)
    gemv_record_rows: int = 2                 # GEMV batches >= this many rows complete via records (0 = never)
    idle_inline_rows: int = 8                 # GPU: idle engine -> the IO thread launches <= this many rows itself (0 = off)
    wide_host_merge_blocks: int = 0           # GPU: WIDE batches merge class blocks on the host up to this many blocks (0 = in-kernel)
    f32_gemv: bool = False                    # GPU: f32 binary F <= 2048 on the f32-accumulating GEMV (A/B)
    resident: str = "auto"                    # resident SMALL-path kernel (IO threads write rows into rings that GPU-
                                              # resident waves poll): auto (on for a GPU) | on (CPU backend: a host
                                              # thread plays the kernel, tests) | off (every row via the batcher)
    resident_depth: int = 2                   # host-memory polls in flight per resident wave (1, 2, 4)
    resident_idle_polls: int = 20000          # polls without a row before a resident wave slows its polling
    resident_lease_ms: int = 200              # a resident wave exits when its lease has not moved for this long
    io_ring_spin_us: int = 5                  # IO threads with rows on the resident kernel watch their records this
                                              # long in user space between epoll_wait(0) calls
    io_ring_sleep_us: int = 0                 # > 0: ... sleep that long in epoll_pwait2 instead of spinning (A/B)
    direct_dispatch: bool = True              # GPU: ... written as AQL packets into the engine's own HSA queue
    direct_wide: bool = True                  # GPU: class-split / record GEMV batches into that queue too ...
    direct_wide_max_weight_bytes: int = 256 << 10  # ... for models with at most this many bytes of W
    stage_wide: bool = False                  # GPU: copy wide models' rows H2D first (default: zero-copy reads)
    fault_drop_rank: int = -1                 # fault injection: this DP rank's engine fails every batch
    fault_exit_rank: int = -1                 # fault injection: this DP rank's process dies (exit 3) ...
    fault_exit_after_ms: int = 2000           # ... this long after it starts serving (not after a restart)
    pin: str = "auto"                         # CPU pinning per rank: auto (DP without launcher) | on | off
    # HTTP
    host: str = "127.0.0.1"
    port: int = 8000
    io_threads: int = 2
    reuseport: bool = True
    fast_path: bool = True
    asgi_fast_path: bool = True               # uvicorn main:app: POST /predict answered by an ASGI middleware
    server_header: str = "uvicorn"
    slow_workers: int = 1
    log_level: str = "warning"
    access_log: bool = False                  # uvicorn-format access log lines on stderr
    health_dispatch: str = "auto"             # auto (DP, world > 1) | on | off: unhealthy ranks leave the port
    dispatch: str = "acceptor"                # acceptor: one acceptor per port hands connections round robin to
                                              # the replicas / IO threads (csrc/http/dispatch.h) | source: the same,
                                              # a client address keeping its replica | reuseport: kernel hash
    dispatch_group: str = ""                  # acceptor group name ("" = named after host:port)
    dispatch_claim: str = ""                   # dispatch=source: client address this replica claims ("" = none)
    admin: str = "loopback"                   # POST /admin/*: loopback (local clients only) | on | off
    # observability
    metrics: bool = True

    @classmethod
    def from_env(cls, **overrides) -> "Config":
        cfg = cls()
        for f in dataclasses.fields(cls):
            env = os.environ.get("MLAPI_" + f.name.upper())
            if env is not None:
                setattr(cfg, f.name, _coerce(f, env))
        for k, v in overrides.items():
            if v is not None:
                setattr(cfg, k, v)
        return cfg

    @classmethod
    def add_arguments(cls, ap: argparse.ArgumentParser) -> None:
        for f in dataclasses.fields(cls):
            flag = "--" + f.name.replace("_", "-")
            if f.type in ("bool", bool):
                ap.add_argument(flag, dest=f.name, default=None, type=_parse_bool)
            elif f.name == "feature_names":
                ap.add_argument(flag, dest=f.name, default=None, type=lambda s: [x for x in s.split(",") if x])
            else:
                typ = int if f.type in ("int", int) else str
                ap.add_argument(flag, dest=f.name, default=None, type=typ)

    @classmethod
    def from_args(cls, ns: argparse.Namespace) -> "Config":
        return cls.from_env(**{f.name: getattr(ns, f.name, None) for f in dataclasses.fields(cls)})

    def device_index(self) -> Optional[int]:
        """None -> CPU backend; int -> HIP device ordinal."""
        d = str(self.device).strip().lower()
        if d == "cpu":
            return None
        if d in ("cuda", "gpu", "hip"):
            return int(os.environ.get("LOCAL_RANK", "0"))
        if d.startswith("cuda:"):
            return int(d.split(":", 1)[1])
        if d.isdigit():
            return int(d)
        # auto: a GPU if one is visible (LOCAL_RANK selects it under torchrun), else CPU
        from mlapi_amd._native import gpu_count

        n = gpu_count()
        if n == 0:
            return None
        return int(os.environ.get("LOCAL_RANK", "0")) % n


def _parse_bool(s: str) -> bool:
    return str(s).strip().lower() in ("1", "true", "yes", "on")


def _coerce(f: dataclasses.Field, s: str):
    if f.type in ("bool", bool):
        return _parse_bool(s)
    if f.type in ("int", int):
        return int(s)
    if f.name == "feature_names":
        return [x for x in s.split(",") if x]
    return s
