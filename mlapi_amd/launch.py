"""``python -m mlapi_amd.launch --nproc 8 [-m module | script.py] [args...]`` - one process per GPU.

The framework's own launcher ("spawns N rank processes, each pinned to a GPU"), an
alternative to ``torchrun`` with what a serving node needs:

* hosts the job's TCP key-value store (the host channel over which rank 0 publishes the RCCL
  unique id, :func:`mlapi_amd.parallel.rccl.exchange_unique_id`; torch.distributed's ``env://``
  init joins it as a client via ``TORCHELASTIC_USE_AGENT_STORE``);
* exports RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT, so every
  entry point (``bench.py``, ``mlapi_amd.serve``, ``mlapi_amd.train``) runs unchanged;
* places each rank (``--pin``): at N > 1 by default on its GPU's NUMA node (``numa``: the node's
  CPU list as the affinity mask, the scheduler balances the rank's threads over it and its pinned
  host memory is first touched there), at N = 1 on a disjoint slice of physical cores (``cores``,
  which also sizes OMP_NUM_THREADS); ``off`` / ``--no-pin`` leaves ranks unpinned. GPU
  ``local_rank`` is selected by the rank itself (all devices stay visible so RCCL can map peers);
* supervises: the first rank that exits non-zero brings the others down (SIGTERM, then SIGKILL
  after ``--grace``) and its exit code becomes the launcher's; with ``--restart N`` a failed rank
  is instead started again (at most N times per rank) while the others keep running, with
  ``MLAPI_REPLICA_RESTART=<n>`` in its environment (serving: it comes back as a standalone replica
  on the shared port, :func:`mlapi_amd.parallel.dp_serve.serve_replica`).

The launcher never touches the GPU itself, so starting the ranks with fork+exec is safe.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional

from mlapi_amd.utils.affinity import core_order, cpu_slices, gpu_numa_nodes, numa_rank_cpus  # noqa: F401


def _free_port(host: str) -> int:
    s = socket.socket()
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_placement(mode: str, nproc: int, **sysfs) -> List[List[int]]:
    """The CPU mask of every rank ([] = leave it unpinned) for --pin ``mode`` (numa / cores / off).
    numa: GPU r's NUMA-node CPUs for rank r (:func:`numa_rank_cpus`; unknown node -> unpinned);
    cores: disjoint physical-core slices of the CPU quota (:func:`cpu_slices`). ``sysfs`` overrides
    the sysfs roots (tests: sys_kfd, sys_pci, sysnode, cpus)."""
    if mode == "off":
        return [[] for _ in range(nproc)]
    if mode == "cores":
        return cpu_slices(nproc)
    cpus = sysfs.pop("cpus", None)
    nodes = gpu_numa_nodes(**{k: v for k, v in sysfs.items() if k in ("sys_kfd", "sys_pci")})
    kw = {"sysnode": sysfs["sysnode"]} if "sysnode" in sysfs else {}
    return [numa_rank_cpus(r, nodes, cpus, **kw) for r in range(nproc)]


def numa_omp_threads(placement: List[List[int]], r: int, quota: Optional[float] = -1.0) -> int:
    """OMP_NUM_THREADS for rank r under numa placement: its mask's CPUs split over the ranks that
    share that mask, capped by the rank's share of the cgroup CPU quota (``quota`` None = no quota,
    -1 = read it from the cgroup)."""
    from mlapi_amd.utils.threads import cgroup_cpu_quota

    mask = set(placement[r])
    sharing = max(1, sum(1 for c in placement if set(c) == mask))
    n = max(1, len(mask) // sharing)
    q = cgroup_cpu_quota() if quota == -1.0 else quota
    if q:
        n = min(n, max(1, int(q // max(1, len(placement)))))
    return n


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m mlapi_amd.launch", description=__doc__.split("\n\n")[0])
    ap.add_argument("--nproc", type=int, default=0, help="ranks (default: visible GPU count, at least 1)")
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0, help="0 = pick a free port")
    ap.add_argument("--pin", default="auto", choices=["auto", "numa", "cores", "off"],
                    help="rank placement: numa = its GPU's NUMA-node CPUs (mask), cores = a disjoint slice of "
                         "physical cores, off = unpinned; auto = numa at N > 1, cores at N = 1")
    ap.add_argument("--no-pin", action="store_true", help="same as --pin off")
    ap.add_argument("--grace", type=float, default=10.0, help="seconds between SIGTERM and SIGKILL on failure")
    ap.add_argument("--restart", type=int, default=0,
                    help="restart a rank that exits non-zero up to N times instead of stopping the job "
                         "(serving replicas; training jobs should keep 0)")
    ap.add_argument("-m", dest="module", default=None, help="run a module (like python -m)")
    ap.add_argument("target", nargs=argparse.REMAINDER, help="script.py args... (or module args with -m)")
    argv = list(sys.argv[1:] if argv is None else argv)
    module, mod_args = None, []
    if "-m" in argv:  # everything after `-m MODULE` belongs to the module, like `python -m`
        i = argv.index("-m")
        if i + 1 >= len(argv):
            ap.error("-m needs a module name")
        module, mod_args, argv = argv[i + 1], argv[i + 2:], argv[:i]
    args = ap.parse_args(argv)
    if module is not None:
        args.module, args.target = module, mod_args

    nproc = args.nproc
    if nproc <= 0:
        try:  # counting devices does not initialise the GPU on this image
            import torch

            nproc = max(1, torch.cuda.device_count())
        except Exception:  # pragma: no cover
            nproc = 1
    if args.module is None and not args.target:
        ap.error("nothing to run: give a script or -m module")
    cmd = [sys.executable] + (["-m", args.module] if args.module else []) + args.target

    import torch.distributed as dist

    port = args.master_port or _free_port(args.master_addr)
    store = dist.TCPStore(args.master_addr, port, nproc, is_master=True, wait_for_workers=False,
                          use_libuv=True)
    mode = "off" if args.no_pin else args.pin
    if mode == "auto":
        mode = "numa" if nproc > 1 else "cores"
    placement = rank_placement(mode, nproc)

    def _spawn(r: int, restart: int = 0) -> subprocess.Popen:
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc), "LOCAL_WORLD_SIZE": str(nproc),
                    "GROUP_RANK": "0", "MASTER_ADDR": args.master_addr, "MASTER_PORT": str(port),
                    "TORCHELASTIC_USE_AGENT_STORE": "True", "MLAPI_LAUNCHER": "1"})
        if restart:
            env["MLAPI_REPLICA_RESTART"] = str(restart)
        cpus = placement[r]
        if cpus and mode == "cores":
            env["OMP_NUM_THREADS"] = str(max(1, len(cpus)))
        elif cpus and mode == "numa" and "OMP_NUM_THREADS" not in os.environ:
            # a node mask is shared by the ranks whose GPUs sit on that node: each rank's OpenMP /
            # torch pool gets its share (and its share of the cgroup quota), not the whole mask
            env["OMP_NUM_THREADS"] = str(numa_omp_threads(placement, r))
        if cpus:
            env["MLAPI_PLACEMENT"] = mode
        pre = (lambda c=cpus: os.sched_setaffinity(0, c)) if cpus else None
        return subprocess.Popen(cmd, env=env, preexec_fn=pre)

    procs: List[subprocess.Popen] = [_spawn(r) for r in range(nproc)]
    restarts = [0] * nproc

    def _terminate(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:  # pragma: no cover
                    pass

    signal.signal(signal.SIGTERM, lambda *_: _terminate())
    code = 0
    try:
        while True:
            alive = 0
            for i, p in enumerate(procs):
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0 and code == 0 and restarts[i] < args.restart:
                    restarts[i] += 1
                    print(f"[mlapi_amd.launch] rank {i} exited with {rc}; restart {restarts[i]}/{args.restart}",
                          file=sys.stderr, flush=True)
                    procs[i] = _spawn(i, restarts[i])
                    alive += 1
                elif rc != 0 and code == 0:
                    code = rc if rc > 0 else 128 - rc
                    print(f"[mlapi_amd.launch] rank {i} exited with {rc}; stopping the job",
                          file=sys.stderr, flush=True)
                    _terminate()
                    deadline = time.monotonic() + args.grace
                    while time.monotonic() < deadline and any(q.poll() is None for q in procs):
                        time.sleep(0.05)
                    _terminate(signal.SIGKILL)
            if alive == 0:
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        _terminate(signal.SIGINT)
        for p in procs:
            p.wait()
        code = 130
    del store
    return code


if __name__ == "__main__":
    sys.exit(main())
