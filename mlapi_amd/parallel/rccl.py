"""Framework-owned communicators: native RCCL (C++) on GPUs, a gloo-backed stand-in on CPUs.

SURVEY 2.6 asks for RCCL "called directly from C++" with a unique-id bootstrap over a host
channel, plus a ``FakeComm`` with identical semantics for CPU-only multi-rank tests:

* :class:`NativeComm` wraps ``mlapi_amd._C.RcclComm`` (csrc/dist/comm.cpp): rank 0 draws the
  128-byte ``ncclUniqueId``, publishes it in the job's TCP key-value store (torchrun's agent store,
  or the default process group's store), every rank joins on its own GPU. Collectives run on the
  current HIP stream; ``wait``/``barrier`` take a deadline and abort the communicator instead of
  hanging on a dead peer.
* :class:`FakeComm` implements the same methods with torch.distributed (gloo) on CPU tensors.

Both speak in torch tensors. NativeComm is the default data plane of every GPU rank
(``MLAPI_COMM=auto``, see :func:`mlapi_amd.parallel.comm.init_distributed`); ``MLAPI_COMM=torch``
selects torch.distributed's own ``nccl`` backend (also RCCL) instead. With ``MLAPI_P2P_BYTES`` > 0,
small float32/bfloat16 sum all-reduces go through the one-shot P2P kernel (``parallel/p2p.py``).
"""
from __future__ import annotations

import os
import time
from typing import List, Optional

import torch

# RCCL enum values (rccl.h)
_DTYPE = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
          torch.float64: 8, torch.bfloat16: 9}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
_UID_KEY = "mlapi/rccl_unique_id/{}"


def exchange_unique_id(store, rank: int, make_id, generation: int = 0, timeout_s: float = 300.0) -> bytes:
    """Host-channel bootstrap: rank 0 publishes ``make_id()``, the others read it from the store."""
    key = _UID_KEY.format(generation)
    if rank == 0:
        uid = bytes(make_id())
        store.set(key, uid)
        return uid
    store.wait([key], __import__("datetime").timedelta(seconds=timeout_s))
    return bytes(store.get(key))


def default_store():
    """The job's TCP store: the default process group's, else torchrun's agent store."""
    import torch.distributed as dist

    if dist.is_initialized():
        return dist.distributed_c10d._get_default_store()
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    return dist.TCPStore(host, port, world, is_master=(rank == 0 and os.environ.get("TORCHELASTIC_USE_AGENT_STORE")
                                                         != "True"), use_libuv=True)


class NativeComm:
    """Device collectives through the framework's C++ RCCL communicator."""

    kind = "native-rccl"

    def __init__(self, rank: int, world: int, device: torch.device, store=None, timeout_ms: int = 120_000,
                 generation: int = 0):
        from mlapi_amd._native import C

        self._C = C()
        self.rank, self.world, self.device = rank, world, device
        self.timeout_ms = timeout_ms
        store = store if store is not None else (default_store() if world > 1 else None)
        uid = (exchange_unique_id(store, rank, self._C.RcclComm.unique_id, generation) if world > 1
               else self._C.RcclComm.unique_id())
        self.comm = self._C.RcclComm(uid, rank, world, device.index)
        n = self.comm.comm_count()
        if n != world:  # RCCL's own view of the job must match the launcher's
            raise RuntimeError(f"rank {rank}: ncclCommCount reports {n} ranks, expected {world}")
        # small sum all-reduces through the one-shot P2P kernel when MLAPI_P2P_BYTES > 0 (parallel/p2p.py);
        # its IPC handles are versioned by the same generation as the RCCL unique id
        from mlapi_amd.parallel.p2p import from_env

        self.generation = generation
        self.p2p = from_env(rank, world, device, store=store, generation=generation)

    def nranks(self) -> int:
        """Ranks in the RCCL communicator as RCCL reports them (ncclCommCount)."""
        return int(self.comm.comm_count())

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    def _check(self, t: torch.Tensor) -> None:
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("NativeComm: tensors must be contiguous GPU tensors")

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        self._check(t)
        if self.p2p is not None and self.p2p.supports(t, op):
            return self.p2p.all_reduce_(t, self.timeout_ms)
        self.comm.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPE[t.dtype], _OPS[op], self._stream())
        return t

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        self._check(t)
        self.comm.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPE[t.dtype], src, self._stream())
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] gathered in rank order."""
        self._check(t)
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        self.comm.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), _DTYPE[t.dtype], self._stream())
        return out

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """t: [world * n] -> this rank's reduced slice [n]."""
        self._check(t)
        n = t.numel() // self.world
        out = torch.empty(n, dtype=t.dtype, device=t.device)
        self.comm.reduce_scatter(t.data_ptr(), out.data_ptr(), n, _DTYPE[t.dtype], _OPS[op], self._stream())
        return out

    def barrier(self) -> None:
        if not self.comm.barrier(self._stream(), self.timeout_ms):
            raise RuntimeError(f"rank {self.rank}: RCCL barrier timed out or failed; communicator aborted")
        self.check_p2p()

    def wait(self, timeout_ms: Optional[int] = None) -> None:
        if not self.comm.wait(self._stream(), self.timeout_ms if timeout_ms is None else timeout_ms):
            raise RuntimeError(f"rank {self.rank}: RCCL collective timed out or failed; communicator aborted")
        self.check_p2p()

    def check_p2p(self) -> None:
        """A P2P all-reduce whose peer never arrived leaves only the local gradient in the buffer
        (the kernel records a sticky timeout and exits): surface it like an RCCL timeout, and abort
        the communicator so no later collective runs on diverged replicas."""
        if self.p2p is not None and self.p2p.status() != 0:
            self.abort()
            raise RuntimeError(f"rank {self.rank}: P2P all-reduce timed out waiting for a peer; communicator aborted")

    def abort(self) -> None:
        self.comm.abort()

    @property
    def aborted(self) -> bool:
        return self.comm.aborted


class FakeComm:
    """CPU stand-in with NativeComm's semantics (gloo process group), for multi-rank tests."""

    kind = "fake-gloo"

    def __init__(self, rank: int, world: int, group=None):
        import torch.distributed as dist

        self.rank, self.world, self.device = rank, world, torch.device("cpu")
        self._dist = dist
        self.group = group
        self.aborted = False

    _RED = {"sum": "SUM", "prod": "PRODUCT", "max": "MAX", "min": "MIN"}

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world > 1:
            if op == "avg":
                self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM, group=self.group)
                t.div_(self.world)
            else:
                self._dist.all_reduce(t, op=getattr(self._dist.ReduceOp, self._RED[op]), group=self.group)
        return t

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world > 1:
            self._dist.broadcast(t, src, group=self.group)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t.unsqueeze(0).clone()
        outs: List[torch.Tensor] = [torch.empty_like(t) for _ in range(self.world)]
        self._dist.all_gather(outs, t.contiguous(), group=self.group)
        return torch.stack(outs)

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        n = t.numel() // self.world
        full = self.all_reduce_(t.clone(), op)
        return full[self.rank * n:(self.rank + 1) * n].clone()

    def barrier(self) -> None:
        if self.world > 1:
            self._dist.barrier(group=self.group)

    def wait(self, timeout_ms: Optional[int] = None) -> None:
        return None

    def nranks(self) -> int:
        return self.world if self.group is None else self._dist.get_world_size(self.group)

    def abort(self) -> None:
        self.aborted = True


class TorchRcclComm(FakeComm):
    """torch.distributed's RCCL (the ``nccl`` backend) on a subgroup of all ranks, with NativeComm's
    API. Auto mode's second choice when the native communicator cannot initialise: the data plane
    stays on RCCL over xGMI (device tensors) instead of dropping to the host gloo group."""

    kind = "torch-rccl"

    def __init__(self, rank: int, world: int, device: torch.device):
        import torch.distributed as dist

        super().__init__(rank, world, group=dist.new_group(ranks=list(range(world)), backend="nccl"))
        self.device = device
        if world > 1:  # fail here, not in the first real collective
            self.all_reduce_(torch.zeros(1, device=device))
            torch.cuda.synchronize(device)

    def barrier(self) -> None:
        if self.world > 1:
            self.all_reduce_(torch.zeros(1, device=self.device))
            torch.cuda.synchronize(self.device)

    def wait(self, timeout_ms: Optional[int] = None) -> None:
        torch.cuda.current_stream(self.device).synchronize()


def measure_all_reduce(comm, nbytes: int, iters: int = 20) -> float:
    """Latency (seconds) of an in-place f32 sum all-reduce of ``nbytes`` (bus-bandwidth probes)."""
    t = torch.ones(max(1, nbytes // 4), dtype=torch.float32, device=comm.device)
    for _ in range(3):
        comm.all_reduce_(t)
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
    t0 = time.perf_counter()
    for _ in range(iters):
        comm.all_reduce_(t)
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
    return (time.perf_counter() - t0) / iters
