"""One-shot P2P all-reduce over IPC-mapped peer buffers (kernel and protocol:
``csrc/dist/p2p.h``).

Every DP collective of this framework is small (the fused ``[dW | b | loss | correct]`` gradient
buffer), so it is latency bound: RCCL's ring pays 2(N-1) sequential hops, while on
MI355X's full xGMI mesh each rank can read all N peers' buffers in one hop and reduce them itself.
The reduction order is the rank order on every rank, so DP replicas stay bitwise identical.

Handles are exchanged over the job's TCP store (the same host channel as RCCL's unique id). Ranks
sharing one GPU (the 1-GPU test box) use the same code path. :class:`NativeComm` routes sum
all-reduces of float32/bfloat16 tensors up to ``MLAPI_P2P_BYTES`` bytes here (0 = off).
"""
from __future__ import annotations

import datetime
from typing import Optional

import torch

_KEY = "mlapi/p2p/{gen}/{rank}/{what}"
_DT = {torch.float32: 7, torch.bfloat16: 9}


class P2PAllReduce:
    """In-place sum all-reduce of float32 / bfloat16 GPU tensors across ``world`` ranks."""

    def __init__(self, rank: int, world: int, device: torch.device, store=None, max_bytes: int = 4 << 20,
                 generation: int = 0, timeout_s: float = 300.0):
        from mlapi_amd._native import C

        if device is None or device.type != "cuda":
            raise ValueError("P2PAllReduce needs a GPU device")
        self.rank, self.world, self.device = rank, world, device
        self._p = C().P2PAllReduce(rank, world, device.index, int(max_bytes))
        if world > 1:
            if store is None:
                from mlapi_amd.parallel.rccl import default_store

                store = default_store()
            for what, h in (("data", self._p.data_handle()), ("flag", self._p.flag_handle())):
                store.set(_KEY.format(gen=generation, rank=rank, what=what), h)
            keys = [_KEY.format(gen=generation, rank=r, what=w) for r in range(world) for w in ("data", "flag")]
            store.wait(keys, datetime.timedelta(seconds=timeout_s))
            data = [bytes(store.get(_KEY.format(gen=generation, rank=r, what="data"))) for r in range(world)]
            flag = [bytes(store.get(_KEY.format(gen=generation, rank=r, what="flag"))) for r in range(world)]
            self._p.open_peers(data, flag)

    @property
    def max_bytes(self) -> int:
        return self._p.max_bytes

    @property
    def native(self):
        """The C++ object the fused DP kernels take (``p2p=`` of the train launchers)."""
        return self._p

    def supports(self, t: torch.Tensor, op: str = "sum") -> bool:
        return (op == "sum" and t.dtype in _DT and t.is_cuda and t.is_contiguous()
                and t.numel() * t.element_size() <= self.max_bytes and t.data_ptr() % 16 == 0)

    def all_reduce_(self, t: torch.Tensor, timeout_ms: int = 60_000) -> torch.Tensor:
        if not self.supports(t):
            raise ValueError("P2PAllReduce: contiguous, 16-byte aligned float32/bfloat16 GPU tensor "
                             f"of at most {self.max_bytes} bytes expected")
        self._p.all_reduce(t.data_ptr(), t.numel(), _DT[t.dtype], torch.cuda.current_stream(t.device).cuda_stream,
                           int(timeout_ms))
        return t

    def status(self) -> int:
        """0 = every call completed; 1 = a call timed out waiting for a peer (sticky). Synchronises."""
        return int(self._p.status())

    def check(self) -> None:
        if self.status() != 0:
            raise RuntimeError("P2PAllReduce: a peer did not arrive within the timeout")

    def status_now(self) -> int:
        """The sticky status word as the kernels have published it so far (host-mapped: no sync)."""
        return int(self._p.status_now())

    def check_now(self) -> None:
        """Raise at the first exchange a peer missed, without synchronising: a timed-out block skips
        its update while the others apply theirs, so the replicas are no longer identical and the
        step loop must stop (restore from the last checkpoint)."""
        if self._p.status_now() != 0:
            raise RuntimeError("P2P exchange: a peer did not arrive within the timeout; replicas may "
                               "have diverged in the last step (restore from a checkpoint)")

    def selftest(self, store=None, generation="", timeout_s: float = 120.0) -> int:
        """Start-up check that the IPC mappings carry data between these ranks: every rank writes a
        rank-tagged pattern into its buffer, a store barrier, then every rank reads every peer's
        pattern through the exchange's own load path. Returns this rank's count of wrong words
        (0 = ok). ``MLAPI_P2P_SELFTEST_CORRUPT=<rank>`` makes that rank write a wrong word (tests)."""
        import os

        corrupt = int(os.environ.get("MLAPI_P2P_SELFTEST_CORRUPT", "-1")) == self.rank
        self._p.selftest_write(1 if corrupt else 0)
        if self.world > 1:
            if store is None:
                from mlapi_amd.parallel.rccl import default_store

                store = default_store()
            key = f"mlapi/p2p-selftest/{generation}/{{}}"
            store.set(key.format(self.rank), "1")
            store.wait([key.format(r) for r in range(self.world)], datetime.timedelta(seconds=timeout_s))
        return int(self._p.selftest_verify())


def dp_exchange(info, nbytes: int, width: Optional[int] = None) -> Optional[P2PAllReduce]:
    """The rank's exchange for fused DP training steps (gradient reduction + all-reduce + update in
    one kernel, csrc/dist/p2p_device.h), or None when it does not apply: CPU ranks, ranks spread over
    several hosts (IPC peers must share a host), ``MLAPI_DP_FUSED=0``, and one replica (world = 1:
    the trainers' local step is the same kernels without the exchange arguments, so N = 1 pays
    nothing for DP). Collective: every rank calls it with the same ``nbytes``. Reuses the
    communicator's P2P buffers when they are big enough; otherwise a dedicated exchange is set up
    (its own store keys, ``dp<N>`` generation).

    Before first use an exchange proves itself (:func:`verify_exchange`, collective): the IPC
    pattern check, then the fused exchange kernel itself on a rank-tagged synthetic gradient of
    ``width`` floats (default: what ``nbytes`` holds), compared bitwise with the exact sum and - when
    the communicator is RCCL - with ncclAllReduce of the same buffer. Any failure on any rank and
    every rank gets None: the step uses the RCCL all-reduce (``info.p2p_verify`` = "ok" or
    "failed:<check>").
    """
    import os

    if info.device is None or os.environ.get("MLAPI_DP_FUSED", "1") == "0" or info.world == 1:
        return None
    if info.world > 1 and getattr(info, "local_world", info.world) != info.world:
        return None
    width = width if width is not None else max(4, (nbytes // 4 - 8) // 4 * 4)
    comm_p2p = getattr(info.comm, "p2p", None)
    if isinstance(comm_p2p, P2PAllReduce) and comm_p2p.max_bytes >= nbytes:
        return comm_p2p if _verified(comm_p2p, info, None, "comm", width) else None
    cache = info.__dict__.setdefault("_dp_exchanges", [])
    for ex in cache:
        if ex.max_bytes >= nbytes:
            return ex if _verified(ex, info, None, "cached", width) else None
    from mlapi_amd.parallel.rccl import default_store

    store = default_store()
    gen = f"dp{len(cache)}"
    ex = P2PAllReduce(info.rank, info.world, info.device, store=store, max_bytes=max(nbytes, 4096),
                      generation=gen)
    if not _verified(ex, info, store, gen, width):
        return None
    cache.append(ex)
    return ex


# verification checks, in order (the max over ranks names the first that failed anywhere)
VERIFY_CHECKS = {0: "ok", 1: "ipc-pattern", 2: "fused-timeout", 3: "fused-vs-exact", 4: "fused-vs-rccl"}


def synthetic_gradient(rank: int, nslabs: int, width: int, nstat: int):
    """Rank-tagged synthetic gradient slabs [nslabs][width] and stat slabs [nstat][2] whose values
    are small integers, so any summation order gives the same bits: the exact rank-order sum is
    known on every rank without communicating (:func:`synthetic_sum`)."""
    import numpy as np

    j = np.arange(width, dtype=np.int64)
    slabs = np.stack([((rank + 1) * 131 + s * 17 + j * 7) % 97 - 48 for s in range(nslabs)]).astype(np.float32)
    stats = np.array([[(rank + 1) * (i + 1), (rank + 2) * (i + 3) % 11] for i in range(nstat)], dtype=np.float32)
    return slabs, stats


def synthetic_sum(world: int, nslabs: int, width: int, nstat: int):
    import numpy as np

    g = np.zeros(width, dtype=np.float64)
    st = np.zeros(2, dtype=np.float64)
    for r in range(world):
        sl, ss = synthetic_gradient(r, nslabs, width, nstat)
        g += sl.astype(np.float64).sum(0)
        st += ss.astype(np.float64).sum(0)
    return g.astype(np.float32), st.astype(np.float32)


def check_allreduce(all_reduce, rank: int, world: int, width: int, nslabs: int = 2, nstat: int = 3) -> int:
    """The exchange check against an arbitrary all-reduce ``all_reduce(local_sums: np.ndarray) ->
    np.ndarray`` (the CPU FakeComm twin of :func:`verify_exchange`): 0 ok, 3 a wrong word."""
    import numpy as np

    sl, ss = synthetic_gradient(rank, nslabs, width, nstat)
    local = np.concatenate([sl.sum(0, dtype=np.float32), ss.sum(0, dtype=np.float32)])
    got = np.asarray(all_reduce(local), dtype=np.float32)
    g, st = synthetic_sum(world, nslabs, width, nstat)
    return 0 if np.array_equal(got.view(np.uint32), np.concatenate([g, st]).view(np.uint32)) else 3


def verify_exchange(ex: P2PAllReduce, info, width: int, timeout_ms: int = 5000) -> int:
    """This rank's verdict on the fused exchange (collective; every rank must call it at the same
    point of its exchange sequence): 0 ok, else the first failed check of VERIFY_CHECKS.

    Runs the exchange kernel the trainers use (gdw_reduce with the exchange: per-block publish,
    bounded flag wait, rank-order sum, two-shot when it would engage) on a rank-tagged synthetic
    gradient and compares every word bitwise with the exact sum; when the communicator is RCCL the
    same local sums also go through ncclAllReduce and must match bit for bit.
    ``MLAPI_P2P_VERIFY_FAULT=<rank>`` makes that rank skip one block's flag publish (tests: the
    peers see a stale flag, time out, and the job falls back to RCCL)."""
    import os

    import numpy as np

    from mlapi_amd._native import C
    from mlapi_amd.ops.linear import _stream

    width = max(4, (int(width) + 3) // 4 * 4)
    nslabs, nstat = 2, 3
    sl, ss = synthetic_gradient(info.rank, nslabs, width, nstat)
    dev = info.device
    slabs = torch.from_numpy(sl).to(dev)
    stat_slabs = torch.from_numpy(ss).to(dev)
    out = torch.zeros(width, dtype=torch.float32, device=dev)
    stats = torch.zeros(2, dtype=torch.float32, device=dev)
    if int(os.environ.get("MLAPI_P2P_VERIFY_FAULT", "-1")) == info.rank:
        ex.native.inject_skip_publish(0)
    timeout_ms = int(os.environ.get("MLAPI_P2P_VERIFY_TIMEOUT_MS", timeout_ms))
    C().gdw_reduce(slabs.data_ptr(), nslabs, 1, width, out.data_ptr(), stat_slabs.data_ptr(), nstat,
                   stats.data_ptr(), _stream(), p2p=ex.native, timeout_ms=int(timeout_ms))
    torch.cuda.synchronize(dev)
    if ex.status_now() != 0:
        return 2
    g, st = synthetic_sum(info.world, nslabs, width, nstat)
    fused = np.concatenate([out.cpu().numpy(), stats.cpu().numpy()])
    if not np.array_equal(fused.view(np.uint32), np.concatenate([g, st]).view(np.uint32)):
        return 3
    kind = getattr(info.comm, "kind", info.backend)
    if kind in ("native-rccl", "torch-rccl") or info.backend == "nccl":
        from mlapi_amd.parallel.comm import all_reduce_sum_

        local = torch.zeros(width + 2, dtype=torch.float32, device=dev)
        C().gdw_reduce(slabs.data_ptr(), nslabs, 1, width, local.data_ptr(), stat_slabs.data_ptr(), nstat,
                       local[width:].data_ptr(), _stream())
        all_reduce_sum_(local, info)
        if not np.array_equal(local.cpu().numpy().view(np.uint32), fused.view(np.uint32)):
            return 4
    return 0


def _verified(ex: P2PAllReduce, info, store, gen: str, width: int) -> bool:
    """Verify the exchange once (collective) and record the verdict in ``info.p2p_verify``."""
    if getattr(ex, "_verify_code", None) is None:
        from mlapi_amd.parallel.comm import all_reduce_max

        code = 1 if ex.selftest(store=store, generation=gen) != 0 else 0
        code = int(all_reduce_max(float(code), info))
        if code == 0:
            code = int(all_reduce_max(float(verify_exchange(ex, info, width)), info))
        ex._verify_code = code
        if code != 0:
            import logging

            logging.getLogger("mlapi_amd.parallel").warning(
                "P2P exchange verification failed (%s): DP steps use the RCCL all-reduce", VERIFY_CHECKS[code])
    code = ex._verify_code
    info.__dict__["p2p_verify"] = "ok" if code == 0 else "failed:" + VERIFY_CHECKS.get(code, str(code))
    info.__dict__["p2p_selftest"] = "failed" if code == 1 else "ok"
    return code == 0


def params_hash(t: torch.Tensor) -> float:
    """48-bit hash of a parameter tensor's bytes (exact in a float64 all-gather)."""
    import hashlib

    return float(int.from_bytes(hashlib.sha256(t.detach().cpu().numpy().tobytes()).digest()[:6], "little"))


def replicas_agree(params, info) -> bool:
    """All-gather a hash of every rank's parameters (collective): True if every replica is bitwise
    identical."""
    from mlapi_amd.parallel.comm import all_gather_floats

    h = params_hash(params) if isinstance(params, torch.Tensor) else sum(params_hash(p) for p in params) % (1 << 48)
    hs = all_gather_floats([h], info)[:, 0]
    return bool((hs == hs[0]).all())


def verify_every() -> int:
    """MLAPI_DP_VERIFY_EVERY: fused DP steps between replica checks (0 = never; default 1000)."""
    import os

    return int(os.environ.get("MLAPI_DP_VERIFY_EVERY", "1000"))


def from_env(rank: int, world: int, device: torch.device, store=None, generation: int = 0) -> Optional[P2PAllReduce]:
    """The P2P accelerator NativeComm uses when ``MLAPI_P2P_BYTES`` > 0 (and world > 1). The IPC
    handles are published under ``generation`` (the communicator's), so a communicator rebuilt after
    an abort never opens the previous generation's (freed) buffers."""
    import os

    n = int(os.environ.get("MLAPI_P2P_BYTES", "0"))
    if n <= 0 or world <= 1:
        return None
    return P2PAllReduce(rank, world, device, store=store, max_bytes=n, generation=generation)


class P2PComm:
    """Communicator (NativeComm's API) whose data plane is the one-shot P2P kernel: float32 /
    bfloat16 sum all-reduces stay on the GPU; the rare control-plane collectives (broadcast,
    gather, max) go through the host gloo group. Selected with ``MLAPI_COMM=p2p``; it is the GPU
    data plane that also works with several ranks on ONE device (RCCL refuses that), which is how
    multi-rank DP training is exercised on the 1-GPU test box."""

    kind = "p2p+gloo"

    def __init__(self, rank: int, world: int, device: torch.device, max_bytes: int = 4 << 20):
        from mlapi_amd.parallel.rccl import FakeComm

        self.rank, self.world, self.device = rank, world, device
        self.p2p = P2PAllReduce(rank, world, device, max_bytes=max_bytes) if world > 1 else None
        self._host = FakeComm(rank, world)
        self.aborted = False

    def _via_host(self, t: torch.Tensor, fn) -> torch.Tensor:
        h = t.detach().cpu()
        out = fn(h)
        return out.to(t.device) if out is not h else t.copy_(h)

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world == 1:
            return t
        # an exchange that once missed a peer (sticky status, e.g. a failed verification) is out of
        # step with its peers: the host group carries the rest of the job
        if self.p2p is not None and self.p2p.supports(t, op) and self.p2p.status_now() == 0:
            return self.p2p.all_reduce_(t)
        return self._via_host(t, lambda h: self._host.all_reduce_(h, op))

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return self._via_host(t, lambda h: self._host.broadcast_(h, src))

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        return self._host.all_gather(t.detach().cpu()).to(t.device)

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        return self._host.reduce_scatter(t.detach().cpu(), op).to(t.device)

    def barrier(self) -> None:
        torch.cuda.synchronize(self.device)
        self._host.barrier()

    def wait(self, timeout_ms: Optional[int] = None) -> None:
        if self.p2p is not None:
            self.p2p.check()

    def nranks(self) -> int:
        return self.world

    def abort(self) -> None:
        self.aborted = True
