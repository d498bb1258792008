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


def dp_exchange(info, nbytes: int) -> Optional[P2PAllReduce]:
    """The rank's exchange for fused DP training steps (gradient reduction + all-reduce + update in
    one kernel, csrc/dist/p2p_device.h), or None when it does not apply: CPU ranks, ranks spread over
    several hosts (IPC peers must share a host), or ``MLAPI_DP_FUSED=0``. One replica (world = 1)
    gets one too, so the N = 1 step runs the same kernels as the N > 1 step. Collective: every rank
    calls it with the same ``nbytes``. Reuses the communicator's P2P buffers when they are big
    enough; otherwise a dedicated exchange is set up (its own store keys, ``dp<N>`` generation).
    """
    import os

    if info.device is None or os.environ.get("MLAPI_DP_FUSED", "1") == "0":
        return None
    if info.world > 1 and getattr(info, "local_world", info.world) != info.world:
        return None
    comm_p2p = getattr(info.comm, "p2p", None)
    if isinstance(comm_p2p, P2PAllReduce) and comm_p2p.max_bytes >= nbytes:
        return comm_p2p
    cache = info.__dict__.setdefault("_dp_exchanges", [])
    for ex in cache:
        if ex.max_bytes >= nbytes:
            return ex
    store = None
    if info.world > 1:
        from mlapi_amd.parallel.rccl import default_store

        store = default_store()
    ex = P2PAllReduce(info.rank, info.world, info.device, store=store, max_bytes=max(nbytes, 4096),
                      generation=f"dp{len(cache)}")
    cache.append(ex)
    return ex


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
