"""Per-variant medians of interleaved serve-bench rounds (tools/variants.sh logs).

    python tools/variant_medians.py <dir> [<dir> ...]
"""
import collections
import glob
import json
import os
import re
import statistics
import sys

rows = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "*_r[0-9].log")):
        lines = [x for x in open(f) if x.startswith("{")]
        if not lines:
            continue
        j = json.loads(lines[-1])
        if "cpu_breakdown_rank0" not in j:
            continue
        name = re.sub(r"_r\d$", "", os.path.basename(f)[:-4])
        s = j.get("shuffled_rank0") or {}
        rows[(os.path.basename(d.rstrip("/")), name)].append(
            (j["value"] / 1e6, j["cpu_breakdown_rank0"]["server_cpu_us_per_req"],
             (s.get("req_per_s") or 0) / 1e6, s.get("server_cpu_us_per_req") or 0))
print("| session | variant | runs | paired M req/s (median; range) | µs/req | shuffled M req/s (median; range) | µs/req |")
print("|---|---|---|---|---|---|---|")
for (sess, name), v in sorted(rows.items()):
    p = [x[0] for x in v]
    sh = [x[2] for x in v]
    print("| %s | %s | %d | %.2f (%.2f-%.2f) | %.2f | %s | %s |" % (
        sess, name, len(v), statistics.median(p), min(p), max(p), statistics.median([x[1] for x in v]),
        "%.2f (%.2f-%.2f)" % (statistics.median(sh), min(sh), max(sh)) if any(sh) else "-",
        "%.2f" % statistics.median([x[3] for x in v]) if any(sh) else "-"))
