"""Per-thread CPU accounting from /proc (which native threads burn the CPU during a run).

The native runtime names its OS threads (``mlapi-io-N``, ``mlapi-batch``, ``mlapi-compl``,
``mlapi-loadgen``); :func:`cpu_by_group` sums utime+stime per name group so a benchmark can report
how many cores each stage of the serving pipeline used (the serving path is CPU-bound: the GPU
kernel per batch is a few microseconds).
"""
from __future__ import annotations

import os
import re
from typing import Dict

_TICK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100


def _group(name: str) -> str:
    name = name.strip()
    if name.startswith("mlapi-"):
        return re.sub(r"-\d+$", "", name)
    return "other"


def cpu_by_group(pid: int | None = None) -> Dict[str, float]:
    """{thread-name group: CPU seconds} for every thread of ``pid`` (default: this process)."""
    base = f"/proc/{pid or os.getpid()}/task"
    out: Dict[str, float] = {}
    try:  # whole process, including threads that already exited (e.g. load-generator workers)
        with open(f"/proc/{pid or os.getpid()}/stat") as f:
            s = f.read()
        fields = s[s.rfind(")") + 2:].split()
        out["process_total"] = (int(fields[11]) + int(fields[12])) / _TICK
    except OSError:
        pass
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"{base}/{tid}/stat") as f:
                s = f.read()
        except OSError:
            continue
        lp, rp = s.find("("), s.rfind(")")
        name = s[lp + 1:rp]
        fields = s[rp + 2:].split()
        ut, st = int(fields[11]), int(fields[12])  # utime, stime (fields 14, 15 of stat)
        g = _group(name)
        out[g] = out.get(g, 0.0) + (ut + st) / _TICK
    return out


def cgroup_cpu_quota(root: str = "/sys/fs/cgroup") -> float | None:
    """CPU bandwidth limit of this container in cores (cgroup v2 ``cpu.max`` or v1 CFS), or None.

    On the MI355X pool a 1-GPU box shows 256 CPUs in the affinity mask but ``cpu.max`` allows 16
    cores: sizing thread pools from the mask alone oversubscribes the quota and the kernel
    throttles the whole process for the rest of each 100 ms period.
    """
    try:
        with open(os.path.join(root, "cpu.max")) as f:
            quota, period = f.read().split()[:2]
        if quota != "max" and int(period) > 0:
            return int(quota) / int(period)
        return None
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(root, "cpu", "cpu.cfs_quota_us")) as f:
            quota_us = int(f.read().strip())
        with open(os.path.join(root, "cpu", "cpu.cfs_period_us")) as f:
            period_us = int(f.read().strip())
        if quota_us > 0 and period_us > 0:
            return quota_us / period_us
    except (OSError, ValueError):
        pass
    return None


def effective_cpus(root: str = "/sys/fs/cgroup") -> int:
    """CPUs this process can actually keep busy: min(affinity mask, cgroup quota)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    q = cgroup_cpu_quota(root)
    if q is not None:
        n = min(n, max(1, int(q)))
    return max(1, n)


def utilization(before: Dict[str, float], after: Dict[str, float], seconds: float) -> Dict[str, float]:
    """Cores busy per group over an interval."""
    keys = set(before) | set(after)
    return {k: round((after.get(k, 0.0) - before.get(k, 0.0)) / max(seconds, 1e-9), 2) for k in sorted(keys)}
