"""Summarise tools/pmc_profile.sh output: per bench and kernel, mean counter values per dispatch
plus derived rates (HBM bytes and GB/s, MFMA busy %, LDS bank-conflict cycles per LDS instruction)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
# (bench, kernel) -> counter -> [values per dispatch]; plus kernel durations
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for d in sorted(glob.glob(os.path.join(root, "*_*"))):
    if not os.path.isdir(d):
        continue
    bench = os.path.basename(d).rsplit("_", 1)[0]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)  # (dispatch, kernel, counter) summed over dimensions
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")
            per[(r.get("Dispatch_Id"), k, r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, k, c), v in per.items():
            vals[(bench, k)][c].append(v)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[(bench, r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def mean(x):
    return sum(x) / len(x) if x else float("nan")


print("| bench | kernel | µs | FETCH MB | WRITE MB | HBM GB/s* | bf16 TFLOP/s | LDS confl/instr | VALU instr/wave | "
      "wait % | wait-issue % | VALU-active % | LDS-active % | VMEM-active % | waves |")
print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
for (bench, k), cs in sorted(vals.items()):
    if not k.startswith("void mlapi") and "mlapi" not in k and not k.startswith("Cijk"):
        continue
    us = mean(dur.get((bench, k), []))
    fetch = mean(cs.get("FETCH_SIZE", [])) / 1024  # KB -> MB
    write = mean(cs.get("WRITE_SIZE", [])) / 1024
    lds_c = mean(cs.get("SQ_LDS_BANK_CONFLICT", []))
    lds_i = mean(cs.get("SQ_INSTS_LDS", []))
    name = k.replace("void mlapi::(anonymous namespace)::", "")[:60]
    gbs = (fetch + write) * 1e3 / us if us == us and us else float("nan")  # MB / us -> GB/s
    waves = mean(cs.get("SQ_WAVES", []))
    wcyc = mean(cs.get("SQ_WAVE_CYCLES", []))

    def pct(c):
        return 100 * mean(cs.get(c, [])) / wcyc if wcyc == wcyc and wcyc else float("nan")

    tflops = mean(cs.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", [])) * 512 / (us * 1e-6) / 1e12 if us == us and us else 0
    print(f"| {bench} | `{name}` | {us:.1f} | {fetch:.1f} | {write:.1f} | {gbs:.0f} | {tflops:.0f} | "
          f"{(lds_c / lds_i if lds_i else float('nan')):.3f} | {mean(cs.get('SQ_INSTS_VALU', [])) / waves:.0f} | "
          f"{pct('SQ_WAIT_ANY'):.0f} | {pct('SQ_WAIT_INST_ANY'):.0f} | {pct('SQ_ACTIVE_INST_VALU'):.0f} | "
          f"{pct('SQ_ACTIVE_INST_LDS'):.0f} | {pct('SQ_ACTIVE_INST_VMEM'):.0f} | {waves:.0f} |")
print()
# MFMA busy %: SQ_VALU_MFMA_BUSY_CYCLES is summed over all 1024 SIMDs, SQ_BUSY_CYCLES over the 32
# shader engines (8 XCDs x 4), so busy / (1024 x SQ_BUSY / 32) = busy / (32 x SQ_BUSY).
SE_COUNT = 32
print("| bench | kernel | L2 hit % | LDS-wait % | MFMA busy % | MISC-active % | SALU instr/wave |")
print("|---|---|---|---|---|---|---|")
for (bench, k), cs in sorted(vals.items()):
    if "mlapi" not in k and not k.startswith("Cijk"):
        continue
    name = k.replace("void mlapi::(anonymous namespace)::", "")[:60]
    hit, miss = mean(cs.get("TCC_HIT_sum", [])), mean(cs.get("TCC_MISS_sum", []))
    wcyc = mean(cs.get("SQ_WAVE_CYCLES", []))
    waves = mean(cs.get("SQ_WAVES", []))
    busy, sqb = mean(cs.get("SQ_VALU_MFMA_BUSY_CYCLES", [])), mean(cs.get("SQ_BUSY_CYCLES", []))

    def pc(c):
        return 100 * mean(cs.get(c, [])) / wcyc if wcyc == wcyc and wcyc else float("nan")

    print(f"| {bench} | `{name}` | {100 * hit / (hit + miss) if hit + miss else float('nan'):.1f} | "
          f"{pc('SQ_WAIT_INST_LDS'):.0f} | {100 * busy / sqb / SE_COUNT if sqb == sqb and sqb else float('nan'):.0f} | "
          f"{pc('SQ_ACTIVE_INST_MISC'):.0f} | {mean(cs.get('SQ_INSTS_SALU', [])) / waves if waves else float('nan'):.0f} |")
print()
print("*HBM GB/s = (FETCH_SIZE + WRITE_SIZE) / kernel time; on gfx950 FETCH_SIZE reads about half of")
print(" the streamed bytes (MI355X_MICROARCH.md), so the true read rate is up to 2x this column.")
print(" Kernel time here is measured under counter collection (serialised dispatches).")
print(" bf16 TFLOP/s = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 / kernel time (dense peak ~2500).")
print(" wait / active % = share of SQ_WAVE_CYCLES (summed over waves) spent waiting on anything /")
print(" on instruction issue, or with a VALU / LDS / VMEM instruction in flight.")

# L2 request rates (group l2req): vector-L1 -> L2 read requests and all L2 requests per µs, and the
# bytes they imply at 128 B per request (gfx950 L2 line) - the L2 bandwidth a kernel draws
rows = [(b, k, cs) for (b, k), cs in sorted(vals.items()) if "TCC_REQ_sum" in cs or "TCP_TCC_READ_REQ_sum" in cs]
if rows:
    print()
    print("| bench | kernel | µs | L1->L2 read req / µs | L2 req / µs | L2 read req / µs | L1->L2 read GB/s @128 B |")
    print("|---|---|---|---|---|---|---|")
    for b, k, cs in rows:
        us = mean(dur.get((b, k), []))
        r1 = mean(cs.get("TCP_TCC_READ_REQ_sum", [])) / us
        r2 = mean(cs.get("TCC_REQ_sum", [])) / us
        r3 = mean(cs.get("TCC_READ_sum", [])) / us
        print(f"| {b} | `{k[:60]}` | {us:.1f} | {r1:.0f} | {r2:.0f} | {r3:.0f} | {r1 * 128 / 1e3:.0f} |")

