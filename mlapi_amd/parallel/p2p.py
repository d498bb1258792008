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


def dp_exchange(info, nbytes: int) -> Optional[P2PAllReduce]:
    """The rank's exchange for fused DP training steps (gradient reduction + all-reduce + update in
    one kernel, csrc/dist/p2p_device.h), or None when it does not apply: CPU ranks, ranks spread over
    several hosts (IPC peers must share a host), ``MLAPI_DP_FUSED=0``, and one replica (world = 1:
    the trainers' local step is the same kernels without the exchange arguments, so N = 1 pays
    nothing for DP). Collective: every rank calls it with the same ``nbytes``. Reuses the
    communicator's P2P buffers when they are big enough; otherwise a dedicated exchange is set up
    (its own store keys, ``dp<N>`` generation). A new exchange is self-tested first
    (:meth:`P2PAllReduce.selftest`, max over ranks): if any rank reads a wrong word through the IPC
    mappings, every rank gets None and the step uses the RCCL all-reduce instead
    (``info.p2p_selftest`` = "ok" / "failed").
    """
    import os

    if info.device is None or os.environ.get("MLAPI_DP_FUSED", "1") == "0" or info.world == 1:
        return None
    if info.world > 1 and getattr(info, "local_world", info.world) != info.world:
        return None
    comm_p2p = getattr(info.comm, "p2p", None)
    if isinstance(comm_p2p, P2PAllReduce) and comm_p2p.max_bytes >= nbytes:
        return comm_p2p if _selftested(comm_p2p, info, None, "comm") else None
    cache = info.__dict__.setdefault("_dp_exchanges", [])
    for ex in cache:
        if ex.max_bytes >= nbytes:
            return ex
    from mlapi_amd.parallel.rccl import default_store

    store = default_store()
    gen = f"dp{len(cache)}"
    ex = P2PAllReduce(info.rank, info.world, info.device, store=store, max_bytes=max(nbytes, 4096),
                      generation=gen)
    if not _selftested(ex, info, store, gen):
        return None
    cache.append(ex)
    return ex


def _selftested(ex: P2PAllReduce, info, store, gen: str) -> bool:
    """Run the exchange's start-up self-test once (collective) and record the verdict."""
    if getattr(ex, "_selftest_ok", None) is None:
        from mlapi_amd.parallel.comm import all_reduce_max

        worst = all_reduce_max(float(ex.selftest(store=store, generation=gen)), info)
        ex._selftest_ok = worst == 0
        if worst != 0:
            import logging

            logging.getLogger("mlapi_amd.parallel").warning(
                "P2P self-test failed (%d wrong words on the worst rank): DP steps use the RCCL all-reduce",
                int(worst))
    info.__dict__["p2p_selftest"] = "ok" if ex._selftest_ok else "failed"
    return ex._selftest_ok


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
        if self.p2p is not None and self.p2p.supports(t, op):
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
