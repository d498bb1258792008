"""Summarise serve bench logs with the paired and shuffled phases: one line per run.

    python tools/shuf_summary.py <dir> [prefix]
"""
import glob
import json
import os
import sys

d = sys.argv[1]
pre = sys.argv[2] if len(sys.argv) > 2 else ""
for f in sorted(glob.glob(os.path.join(d, pre + "*.log"))):
    lines = [x for x in open(f) if x.startswith("{")]
    if not lines:
        continue
    j = json.loads(lines[-1])
    if "cpu_breakdown_rank0" not in j:
        continue
    c = j["cpu_breakdown_rank0"]
    s = j.get("shuffled_rank0") or {}
    print("%-26s paired %5.3f M %4.2f us/req p99 %.3f | shuffled %5.3f M %4.2f us/req p99 %.3f | steered %s/%s "
          "pauses %s/%s | io %s lg %s | conns %s / %s"
          % (os.path.basename(f)[:-4], j["value"] / 1e6, c["server_cpu_us_per_req"], j["p99_latency_ms_c64"],
             (s.get("req_per_s") or 0) / 1e6, s.get("server_cpu_us_per_req", 0), s.get("p99_latency_ms_c64", 0),
             c.get("steered_conns"), s.get("steered_conns"), c.get("steer_pauses"), s.get("steer_pauses"),
             j["threads"]["io"], j["threads"]["loadgen"], c.get("io_conns_per_thread"), s.get("io_conns_per_thread")))
