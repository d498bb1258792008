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


def utilization(before: Dict[str, float], after: Dict[str, float], seconds: float) -> Dict[str, float]:
    """Cores busy per group over an interval."""
    keys = set(before) | set(after)
    return {k: round((after.get(k, 0.0) - before.get(k, 0.0)) / max(seconds, 1e-9), 2) for k in sorted(keys)}
