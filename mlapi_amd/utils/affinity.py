"""CPU placement for one-process-per-GPU serving: physical cores, the GPU's NUMA node, the quota.

The serving path is CPU bound (HTTP parse, batching, JSON render run on host threads; the GPU leg
of a request is ~10 us), so where a rank's threads run decides whole-node req/s. Facts measured on
the MI355X hosts (``tools/probe_box.sh``, ``profiles/r1_session5/probe.txt``):

* 2 sockets x 64 cores x 2 SMT threads; logical CPUs N and N+128 are siblings; NUMA node 0 holds
  CPUs 0-63 and 128-191, node 1 holds 64-127 and 192-255; four GPUs hang off each node.
* The affinity mask shows all 256 CPUs, while the container's ``cpu.max`` allows 16 cores per GPU.

So a rank is placed on ``quota / ranks`` distinct physical cores of its own GPU's NUMA node (the
zero-copy request slots the kernel reads live in host memory of that node). Used by
``mlapi_amd.launch`` and by ``bench.py`` / ``mlapi_amd.serve`` under ``torchrun``.

Without core pinning, a rank can still be kept on its GPU's NUMA node (:func:`numa_rank_cpus`, the
launcher's default at N > 1): the node's whole CPU list as the mask, so the scheduler balances the
rank's threads over the node while its pinned host memory (first touched by those threads) and the
GPU's host link stay on one socket. The GPU -> node map comes from sysfs alone
(:func:`gpu_numa_nodes`: KFD topology order = HIP device order, PCI ``numa_node``), so a launcher
that must not initialise the GPU can compute it.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

SYS_CPU = "/sys/devices/system/cpu"
SYS_NODE = "/sys/devices/system/node"


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def parse_cpulist(s: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _core_key(cpu: int, sysfs: str) -> tuple:
    """(package, core) of a logical CPU; CPUs without topology info sort by their number."""
    pkg = _read(f"{sysfs}/cpu{cpu}/topology/physical_package_id")
    core = _read(f"{sysfs}/cpu{cpu}/topology/core_id")
    try:
        return (int(pkg), int(core))
    except (TypeError, ValueError):
        return (0, cpu)


def _cores(cpus: List[int], sysfs: str) -> List[List[int]]:
    """Physical cores (package-major) as lists of their logical CPUs among ``cpus``."""
    by_core: Dict[tuple, List[int]] = {}
    for c in sorted(cpus):
        by_core.setdefault(_core_key(c, sysfs), []).append(c)
    return [by_core[k] for k in sorted(by_core)]


def _threads_first(cores: List[List[int]]) -> List[int]:
    depth = max((len(c) for c in cores), default=0)
    return [core[t] for t in range(depth) for core in cores if t < len(core)]


def core_order(cpus: List[int], sysfs: str = SYS_CPU) -> List[int]:
    """Logical CPUs ordered one hardware thread per physical core first (package-major), then the
    SMT siblings in the same core order (numeric order would pair CPU N with its sibling N+128)."""
    return _threads_first(_cores(cpus, sysfs))


def _split_cores(cores: List[List[int]], nslices: int, per_slice: int) -> List[List[int]]:
    """``nslices`` disjoint slices of at most ``per_slice`` CPUs that never share a physical core:
    each slice owns whole cores, first threads first, and uses SMT siblings only of its own cores
    when its budget exceeds the cores it owns."""
    base, extra = divmod(len(cores), nslices)
    out, i = [], 0
    for j in range(nslices):
        n = base + (1 if j < extra else 0)
        out.append(_threads_first(cores[i:i + n])[:per_slice])
        i += n
    return out


def cpu_slices(nproc: int, cpus: Optional[List[int]] = None, budget: Optional[int] = None,
               sysfs: str = SYS_CPU) -> List[List[int]]:
    """Split the usable CPUs into ``nproc`` disjoint, near-equal slices of whole physical cores.

    ``budget`` caps the CPUs handed out (default when ``cpus`` is not given: the cgroup quota,
    :func:`mlapi_amd.utils.threads.effective_cpus`)."""
    from mlapi_amd.utils.threads import effective_cpus

    if cpus is None:
        cpus = sorted(os.sched_getaffinity(0))
        if budget is None:
            budget = effective_cpus()
    cpus = list(cpus)
    if nproc > len(cpus):  # oversubscribed: share round-robin
        order = core_order(cpus, sysfs)
        return [[order[i % len(order)]] for i in range(nproc)]
    budget = len(cpus) if budget is None else max(nproc, min(budget, len(cpus)))
    cores = _cores(cpus, sysfs)
    if len(cores) >= nproc:
        per, extra = divmod(budget, nproc)
        return [s[:per + (1 if r < extra else 0)] for r, s in enumerate(_split_cores(cores, nproc, budget))]
    order = core_order(cpus, sysfs)[:budget]  # fewer cores than ranks: slices share cores
    base, extra = divmod(len(order), nproc)
    out, i = [], 0
    for r in range(nproc):
        n = base + (1 if r < extra else 0)
        out.append(order[i:i + n])
        i += n
    return out


def node_cpus(node: int, sysnode: str = SYS_NODE) -> List[int]:
    s = _read(f"{sysnode}/node{node}/cpulist")
    return parse_cpulist(s) if s else []


def gpu_numa_node(device_index: int) -> Optional[int]:
    """NUMA node of a visible GPU (PCI location from the HIP device properties -> sysfs)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:
        return None
    s = _read(f"/sys/bus/pci/devices/{bdf}/numa_node")
    try:
        n = int(s)
    except (TypeError, ValueError):
        return None
    return n if n >= 0 else None


def rank_cpus(local_rank: int, local_world: int, gpu_nodes: Optional[List[Optional[int]]] = None,
              cpus: Optional[List[int]] = None, budget: Optional[int] = None, sysfs: str = SYS_CPU,
              sysnode: str = SYS_NODE) -> List[int]:
    """CPUs for ``local_rank``: its share of the budget, on its GPU's NUMA node when that node has
    room for every rank attached to it, else a plain physical-core slice."""
    from mlapi_amd.utils.threads import effective_cpus

    if cpus is None:
        cpus = sorted(os.sched_getaffinity(0))
        if budget is None:
            budget = effective_cpus()
    budget = len(cpus) if budget is None else min(budget, len(cpus))
    per_rank = max(1, budget // max(1, local_world))
    node = gpu_nodes[local_rank] if gpu_nodes and local_rank < len(gpu_nodes) else None
    if node is not None:
        peers = [r for r in range(local_world) if gpu_nodes[r] == node]
        allowed = set(cpus)
        cores = _cores([c for c in node_cpus(node, sysnode) if c in allowed], sysfs)
        if len(cores) >= len(peers) and sum(map(len, cores)) >= per_rank * len(peers):
            return _split_cores(cores, len(peers), per_rank)[peers.index(local_rank)]
    return cpu_slices(local_world, cpus, budget, sysfs)[local_rank]


def pin_this_rank(local_rank: int, local_world: int, device_index: Optional[int] = None) -> List[int]:
    """Pin the calling process (threads created afterwards inherit it) to :func:`rank_cpus`.

    GPU ``i`` of this node is assumed to be the device of local rank ``i`` (torchrun /
    ``mlapi_amd.launch`` convention). Returns the CPUs, or [] when pinning is not possible."""
    nodes: List[Optional[int]] = []
    try:
        import torch

        n = torch.cuda.device_count()
        nodes = [gpu_numa_node(i) if i < n else None for i in range(local_world)]
        if device_index is not None and local_rank < len(nodes):
            nodes[local_rank] = gpu_numa_node(device_index)
    except Exception:
        nodes = []
    try:
        cpus = rank_cpus(local_rank, local_world, nodes or None)
        os.sched_setaffinity(0, cpus)
        return cpus
    except (OSError, ValueError, IndexError):
        return []


SYS_KFD = "/sys/class/kfd/kfd/topology/nodes"
SYS_PCI = "/sys/bus/pci/devices"


def _kv(text: Optional[str]) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for line in (text or "").splitlines():
        parts = line.split()
        if len(parts) == 2:
            out[parts[0]] = parts[1]
    return out


def kfd_gpu_bdfs(sys_kfd: str = SYS_KFD) -> List[str]:
    """PCI addresses ("dddd:bb:dd.f") of the GPUs in KFD topology order - the order the ROCm runtime
    (and so HIP) enumerates them - read from sysfs without touching the GPU. CPU nodes (no SIMDs)
    are skipped."""
    try:
        nodes = sorted(int(d) for d in os.listdir(sys_kfd) if d.isdigit())
    except OSError:
        return []
    out = []
    for n in nodes:
        p = _kv(_read(f"{sys_kfd}/{n}/properties"))
        try:
            if int(p.get("simd_count", "0")) <= 0:
                continue
            loc, dom = int(p["location_id"]), int(p.get("domain", "0"))
        except (KeyError, ValueError):
            continue
        out.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}")
    return out


def _visible(n: int) -> List[int]:
    """Physical GPU indices behind HIP device ordinals 0.. (HIP/ROCR/CUDA_VISIBLE_DEVICES)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            try:
                idx = [int(x) for x in v.split(",") if x.strip() != ""]
                return [i for i in idx if 0 <= i < n]
            except ValueError:
                return list(range(n))
    return list(range(n))


def gpu_numa_nodes(sys_kfd: str = SYS_KFD, sys_pci: str = SYS_PCI) -> List[Optional[int]]:
    """NUMA node of each visible GPU, by HIP device ordinal (None where sysfs does not say)."""
    bdfs = kfd_gpu_bdfs(sys_kfd)
    out: List[Optional[int]] = []
    for i in _visible(len(bdfs)):
        s = _read(f"{sys_pci}/{bdfs[i]}/numa_node")
        try:
            node = int(s)
        except (TypeError, ValueError):
            node = -1
        out.append(node if node >= 0 else None)
    return out


def numa_rank_cpus(local_rank: int, nodes: List[Optional[int]], cpus: Optional[List[int]] = None,
                   sysnode: str = SYS_NODE) -> List[int]:
    """The CPU mask of a rank kept on its GPU's NUMA node (GPU ``local_rank``): the node's CPUs
    that the process may use - a node mask, not a core slice. [] when the node is unknown or has no
    usable CPU (the caller then leaves the rank unpinned)."""
    if local_rank >= len(nodes) or nodes[local_rank] is None:
        return []
    allowed = set(sorted(os.sched_getaffinity(0)) if cpus is None else cpus)
    return [c for c in node_cpus(nodes[local_rank], sysnode) if c in allowed]


def ranks_on_node(local_rank: int, local_world: int, nodes: List[Optional[int]]) -> int:
    """How many of this host's ranks (rank r uses GPU r % len(nodes)) sit on local_rank's GPU's NUMA
    node - the ranks that share its node mask under numa placement. local_world when the nodes are
    unknown (every rank then shares one mask)."""
    if not nodes or nodes[local_rank % len(nodes)] is None:
        return max(1, local_world)
    mine = nodes[local_rank % len(nodes)]
    return max(1, sum(1 for r in range(local_world) if nodes[r % len(nodes)] == mine))



def client_thread_cpus(local_rank: int, local_world: int, nthreads: int, mask: List[int],
                       nodes: Optional[List[Optional[int]]] = None, sysfs: str = SYS_CPU) -> List[int]:
    """One CPU per load-generator thread of this rank (bench.py pins its client threads, the loopback
    stand-in for NIC RX queues whose interrupts are pinned: every connection's segments then arrive
    from one stable CPU, which the server's SO_INCOMING_CPU steering relies on). Distinct physical
    cores of ``mask`` first, and ranks that share the mask (numa placement) take disjoint stretches
    of it, so no two ranks' client threads stack on one CPU. [] when the mask is empty."""
    if nthreads <= 0 or not mask:
        return []
    order = core_order(sorted(mask), sysfs)
    if nodes:
        mine = nodes[local_rank % len(nodes)]
        slot = sum(1 for r in range(local_rank) if nodes[r % len(nodes)] == mine)
        sharing = ranks_on_node(local_rank, max(local_world, local_rank + 1), nodes)
    else:
        slot, sharing = local_rank, max(1, local_world)
    stride = max(nthreads, len(order) // max(1, sharing))
    return [order[(slot * stride + i) % len(order)] for i in range(nthreads)]


def _siblings(cpu: int, sysfs: str) -> List[int]:
    s = _read(f"{sysfs}/cpu{cpu}/topology/thread_siblings_list")
    return parse_cpulist(s) if s else [cpu]


def _llc(cpu: int, sysfs: str) -> List[int]:
    s = _read(f"{sysfs}/cpu{cpu}/cache/index3/shared_cpu_list")
    return parse_cpulist(s) if s else []


def serve_thread_cpus(local_rank: int, local_world: int, n_client: int, n_io: int, mask: List[int],
                      nodes: Optional[List[Optional[int]]] = None, sysfs: str = SYS_CPU,
                      mode: str = "cores") -> tuple:
    """(client CPUs, IO-thread CPUs) of a serving rank, by ``mode``:

    * ``cores``: the load-generator threads' CPUs as :func:`client_thread_cpus` picks them, then the
      next ``n_io`` CPUs of the same stretch - physical cores of their own;
    * ``sibling``: the ranks sharing ``mask`` split its PHYSICAL cores into disjoint stretches; client
      thread i takes the first hardware thread of core i of this rank's stretch and IO thread i its
      SMT sibling (one core per pair, and no core shared between ranks);
    * ``llc``: client threads as ``sibling``; IO thread i on a free CPU of client thread i's
      last-level cache in the stretch (another core first, its sibling last).

    In the paired modes IO threads past the client threads get no CPU (the server leaves them
    unpinned: a core of their own was measured the worst placement), and client threads past the
    stretch's cores take the stretch's second hardware threads (their IO partners then stay
    unpinned). ([], []) for an empty mask."""
    if not mask or n_client + n_io <= 0:
        return [], []
    if mode == "cores":
        both = client_thread_cpus(local_rank, local_world, n_client + n_io, mask, nodes, sysfs)
        return both[:n_client], both[n_client:]
    if nodes:
        mine = nodes[local_rank % len(nodes)]
        slot = sum(1 for r in range(local_rank) if nodes[r % len(nodes)] == mine)
        sharing = ranks_on_node(local_rank, max(local_world, local_rank + 1), nodes)
    else:
        slot, sharing = local_rank, max(1, local_world)
    cores = _cores(sorted(mask), sysfs)
    stride = max(1, len(cores) // sharing)
    start = (slot * stride) % len(cores)
    mine_cores = [cores[(start + k) % len(cores)] for k in range(stride)]
    if n_client <= 0:
        return [], []
    cl = [mine_cores[i][0] if i < len(mine_cores) else mine_cores[i % len(mine_cores)][-1]
          for i in range(n_client)]
    stretch = [c for core in mine_cores for c in core]
    used, io = set(cl), []
    for i in range(min(n_io, n_client)):
        c = cl[i]
        core = next(k for k in mine_cores if c in k)
        sib = [x for x in core if x != c]
        if mode == "sibling":
            cands = sib
        else:  # llc
            llc = set(_llc(c, sysfs)) or set(stretch)
            others = [x for x in _threads_first([k for k in mine_cores if k is not core]) if x in llc]
            cands = others + sib
        pick = next((x for x in cands if x not in used), None)
        if pick is None:
            break  # no free partner: this and later IO threads stay unpinned
        used.add(pick)
        io.append(pick)
    return cl, io
