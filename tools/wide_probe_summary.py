"""Summarise tools/wide_probe.py's kernel trace: mean / median duration per phase (consecutive
runs of `iters` launches of the wide or split kernel, in the script's order)."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "wide" in r["Kernel_Name"] or "split" in r["Kernel_Name"]]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
labels = [f"{dt} B={B} probe={p}" for dt in ("f32", "f64") for B in (8, 24) for p in (1, 2, 0)]
labels += ["split f32 B=8", "split f32 B=24"]
for i, lab in enumerate(labels):
    chunk = rows[i * iters:(i + 1) * iters]
    if not chunk:
        break
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in chunk[10:]]
    print(f"{lab:24s} {chunk[0]['Kernel_Name'][:48]:48s} mean {statistics.mean(d):6.2f} us  median {statistics.median(d):6.2f} us")
