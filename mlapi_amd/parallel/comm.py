"""Process-group setup and the framework's collectives (RCCL over xGMI via torch.distributed).

One process per GPU. On ROCm the ``"nccl"`` backend of torch.distributed IS RCCL; CPU tests use
``"gloo"`` with the same code. Collectives used by the framework:

* C1 ``broadcast_model`` - rank 0's checkpoint to every replica at startup and on reload: the
  (kind, K, F, n_classes) header and the label JSON go first (tiny), then W|b packed into ONE
  flat float64 buffer so the weights cross xGMI in a single broadcast;
* C2 ``all_reduce_sum`` of the fused gradient buffer [gW | gb | loss | n_correct] per training
  step (C3 - the loss/accuracy scalars - piggyback on the same buffer);
* C4 ``barrier``.

All messages are <= ~1 MiB, i.e. latency-bound on xGMI: one fused buffer per step, never one
collective per tensor.

Data plane selection (``MLAPI_COMM``): ``auto`` (default) = ``native`` when the rank has a GPU,
``torch`` otherwise. ``native`` is the framework's own C++ RCCL communicator
(:class:`mlapi_amd.parallel.rccl.NativeComm`, csrc/dist/comm.cpp: RCCL called directly, on the
stream PyTorch hands over, with deadline/abort) with a gloo process group kept only as the host
control plane (rendezvous, unique-id exchange, reload control); ``torch`` uses torch.distributed
(``nccl`` = RCCL on GPUs, ``gloo`` on CPUs); ``fake`` runs the native code paths on CPU through
:class:`~mlapi_amd.parallel.rccl.FakeComm` (tests); ``p2p`` keeps float32/bfloat16 sum
all-reduces on the GPU through the one-shot P2P kernel (:class:`mlapi_amd.parallel.p2p.P2PComm`,
csrc/dist/p2p_allreduce.hip) and sends the rest through gloo - it also runs with several ranks on
one device, which RCCL refuses.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from mlapi_amd.models.linear import Kind, LinearModel


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: Optional[torch.device] = None  # None -> CPU
    backend: str = "none"
    comm: Optional[object] = None  # NativeComm / FakeComm when MLAPI_COMM selects one
    local_world: int = 1

    def comm_nranks(self) -> int:
        """Ranks of the data-plane communicator as the communicator itself reports them
        (ncclCommCount for the native RCCL comm; the process group size otherwise)."""
        if self.comm is not None and hasattr(self.comm, "nranks"):
            return int(self.comm.nranks())
        if self.world > 1 and dist.is_initialized():
            return dist.get_world_size()
        return self.world

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def gpu_shared_by_ranks() -> bool:
    """True when this node runs more ranks than it has visible GPUs (MLAPI_COMM=p2p rehearsals put
    several ranks on one device). Reads the launcher's env and torch.cuda.device_count(), which does
    not initialise the GPU on this image."""
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    n = torch.cuda.device_count()
    return n > 0 and local_world > n


def per_rank_cpus() -> int:
    """CPUs one rank of this host can keep busy: its share of its affinity mask (a core slice is the
    rank's own; a NUMA-node mask is shared by the ranks whose GPUs sit on that node; an unpinned
    mask by every rank), capped by its share of the cgroup quota (or of the machine)."""
    from mlapi_amd.utils.threads import cgroup_cpu_quota

    local_world = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    placement = os.environ.get("MLAPI_PLACEMENT", "none")
    if placement == "numa":
        from mlapi_amd.utils.affinity import gpu_numa_nodes, ranks_on_node

        share = ranks_on_node(local_rank, local_world, gpu_numa_nodes())
    else:
        share = 1 if placement == "cores" else local_world
    q = cgroup_cpu_quota()
    total = int(q) if q is not None else (os.cpu_count() or 1)
    return max(1, min(aff // share, total // local_world))


RESIDENT_MIN_CPUS = 8  # the smallest per-rank CPU budget measured with the resident path (no loss there)


def resident_auto_ok() -> bool:
    """resident=auto turns the resident SMALL-path kernel on for a rank with a GPU and at least
    RESIDENT_MIN_CPUS CPUs of its own. Measured on one MI355X (profiles/r6_resident_n/README.md):
    ranks sharing one card gain from it (2 ranks, io 4 : client 4 each: 2.69-2.77 M req/s on vs
    1.40-1.43 M off), a rank limited to 8 CPUs neither gains nor loses (1.14-1.15 vs 1.12-1.16 M),
    and 56 extra polling waves - the host-memory reads of 8 GPUs x 8 rings - cost nothing measurable
    (1.85 M median of 3 with and without). Round 5's 0.53 M two-rank collapse does not reproduce,
    neither with round 5's own tree (1.75-1.78 M) nor with this one."""
    return per_rank_cpus() >= RESIDENT_MIN_CPUS


def init_distributed(backend: Optional[str] = None, use_gpu: Optional[bool] = None,
                     comm: Optional[str] = None) -> DistInfo:
    """Initialise from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*); no-op for 1 process."""
    comm = (comm or os.environ.get("MLAPI_COMM", "auto")).lower()
    if comm not in ("auto", "torch", "native", "fake", "p2p"):
        raise ValueError(f"MLAPI_COMM must be auto, torch, native, fake or p2p (got {comm!r})")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if use_gpu is None:
        use_gpu = torch.cuda.is_available() and torch.cuda.device_count() > 0
    auto = comm == "auto"
    if comm == "auto":
        comm = "native" if use_gpu else "torch"
    device = None
    if use_gpu:
        ndev = torch.cuda.device_count()
        if local_world > ndev and comm in ("native", "torch"):
            # RCCL needs one GPU per rank; wrapping local_rank onto a shared device would only fail
            # later inside ncclCommInitRank (or, worse, run fewer GPUs than the job claims)
            raise RuntimeError(f"{local_world} ranks on this node but only {ndev} visible GPU(s): RCCL needs one GPU "
                               "per rank (MLAPI_COMM=p2p runs several ranks on one device)")
        device = torch.device("cuda", local_rank % ndev)
        torch.cuda.set_device(device)
    info = DistInfo(rank, world, local_rank, device, "none")
    info.local_world = local_world
    if comm in ("native", "p2p") and device is None:
        raise RuntimeError(f"MLAPI_COMM={comm} needs a GPU (use fake for CPU runs)")
    if world > 1:
        if not dist.is_initialized():
            if comm != "torch":
                backend = "gloo"  # host control plane only; the data plane is info.comm
            backend = backend or ("nccl" if use_gpu else "gloo")
            kw = {"device_id": device} if backend == "nccl" else {}
            dist.init_process_group(backend=backend, **kw)
        info.backend = dist.get_backend()
    if comm == "native":
        from mlapi_amd.parallel.rccl import FakeComm, NativeComm, TorchRcclComm

        try:
            info.comm = NativeComm(rank, world, device)
            info.backend = NativeComm.kind
        except Exception as e:  # noqa: BLE001
            if not auto or world == 1:
                raise
            # auto mode: a rank set whose native communicator cannot initialise first tries
            # torch.distributed's RCCL (still RCCL over xGMI), then the host gloo group; the backend
            # name says which in every bench line / log (bench.py refuses to report "gloo-fallback").
            import sys

            print(f"[mlapi] rank {rank}: native RCCL communicator init failed ({e}); trying torch's RCCL",
                  file=sys.stderr, flush=True)
            try:
                info.comm = TorchRcclComm(rank, world, device)
                info.backend = TorchRcclComm.kind
            except Exception as e2:  # noqa: BLE001
                print(f"[mlapi] rank {rank}: torch RCCL group failed too ({e2}); collectives fall back to gloo",
                      file=sys.stderr, flush=True)
                info.comm = FakeComm(rank, world)
                info.backend = "gloo-fallback"
    elif comm == "p2p":
        from mlapi_amd.parallel.p2p import P2PComm

        info.comm = P2PComm(rank, world, device)
        info.backend = P2PComm.kind
    elif comm == "fake":
        from mlapi_amd.parallel.rccl import FakeComm

        info.comm = FakeComm(rank, world)
        info.backend = FakeComm.kind
    return info


def _coll_device(info: DistInfo) -> torch.device:
    if info.comm is not None:
        return info.comm.device
    return info.device if (info.backend == "nccl" and info.device is not None) else torch.device("cpu")


def barrier(info: DistInfo) -> None:
    if info.comm is not None:
        info.comm.barrier()
        return
    if info.world > 1:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def all_reduce_max(value: float, info: DistInfo) -> float:
    if info.world == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(info))
    if info.comm is not None:
        info.comm.all_reduce_(t, "max")
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_floats(values, info: DistInfo) -> np.ndarray:
    t = torch.tensor(list(values), dtype=torch.float64, device=_coll_device(info))
    if info.world == 1:
        return t.cpu().numpy()[None, :]
    if info.comm is not None:
        return info.comm.all_gather(t).cpu().numpy()
    out = [torch.empty_like(t) for _ in range(info.world)]
    dist.all_gather(out, t)
    return torch.stack(out).cpu().numpy()


def all_reduce_sum_(t: torch.Tensor, info: DistInfo) -> torch.Tensor:
    """In-place sum over ranks (C2). ``t`` must live on the collective's device."""
    if info.world > 1:
        if info.comm is not None:
            info.comm.all_reduce_(t)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def _bcast(t: torch.Tensor, info: DistInfo, src: int) -> None:
    if info.comm is not None:
        info.comm.broadcast_(t, src)
    else:
        dist.broadcast(t, src)


def broadcast_(t: torch.Tensor, info: DistInfo, src: int = 0) -> torch.Tensor:
    """In-place broadcast of ``t`` from rank ``src`` (any device: staged through the collective's)."""
    if info.world == 1:
        return t
    dev = _coll_device(info)
    buf = t.detach().to(dev).contiguous()
    _bcast(buf, info, src)
    if buf is not t:
        t.copy_(buf)
    return t


def _broadcast_bytes(payload: Optional[bytes], info: DistInfo, src: int = 0) -> bytes:
    dev = _coll_device(info)
    n = torch.tensor([len(payload) if payload is not None else 0], dtype=torch.int64, device=dev)
    _bcast(n, info, src)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
    if info.rank == src:
        buf.copy_(torch.frombuffer(bytearray(payload), dtype=torch.uint8))
    _bcast(buf, info, src)
    return bytes(buf.cpu().numpy().tobytes())


def broadcast_model(model: Optional[LinearModel], info: DistInfo, src: int = 0) -> LinearModel:
    """C1: replicate ``model`` from ``src`` to every rank (RCCL broadcast over xGMI on GPUs)."""
    if info.world == 1:
        assert model is not None
        return model
    header = None
    if info.rank == src:
        header = json.dumps({
            "kind": int(model.kind), "K": model.n_outputs, "F": model.n_features,
            "classes": model.classes.tolist(),
            "classes_dtype": "object" if model.classes.dtype == object else model.classes.dtype.str,
        }).encode()
    h = json.loads(_broadcast_bytes(header, info, src))
    K, F = h["K"], h["F"]
    dev = _coll_device(info)
    flat = torch.empty(K * F + K, dtype=torch.float64, device=dev)
    if info.rank == src:
        flat.copy_(torch.from_numpy(np.concatenate([model.W.reshape(-1), model.b])))
    _bcast(flat, info, src)  # the one weight collective
    arr = flat.cpu().numpy()
    classes = np.array(h["classes"], dtype=object if h["classes_dtype"] == "object" else np.dtype(h["classes_dtype"]))
    return LinearModel(arr[:K * F].reshape(K, F), arr[K * F:], classes, Kind(h["kind"]))


def shutdown(info: DistInfo) -> None:
    info.comm = None  # drops the RCCL communicator (ncclCommDestroy) before the process group
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()
