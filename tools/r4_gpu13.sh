# Round 4 GPU session 13: kernel statistics of every bench mode on the round-4 tree (rocprofv3
# --kernel-trace --stats, one run each) + hardware counters of the kernel benches
set -o pipefail
O=gpurun_out/r4_final; mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
prof() {  # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  (cd /tmp && timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$n -o prof -- python3 $R/bench.py "$@" > $R/$O/prof_$n.log 2>&1) || { echo "prof $n failed"; tail -5 $R/$O/prof_$n.log; exit 1; }
  python3 - "$R/$O/prof_$n/prof_kernel_stats.csv" <<'PY' | tee $R/$O/prof_$n.top.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:6]:
    print(f"{r['Name'][:90]:90s} calls {r['Calls']:>7s} mean {float(r['AverageNs'])/1e3:9.2f} us  {float(r['Percentage']):6.2f} %")
PY
  echo "-- $n done"
}
prof serve 300 --steps 10 --warmup 2
prof serve_wide_f1024 300 --mode serve_wide --wide-features 1024 --steps 6 --warmup 2
prof serve_wide_f64 300 --mode serve_wide --wide-dtype f64 --steps 6 --warmup 2
prof gemv 200 --mode gemv --steps 20 --warmup 2
prof gemm_b1024 200 --mode gemm --steps 200 --warmup 10
prof gemm_b262144 200 --mode gemm --batch 262144 --steps 20 --warmup 2
prof train 200 --mode train --steps 20 --warmup 2
prof train_softmax 200 --mode train_softmax --steps 20 --warmup 2
prof train_softmax_f1024 300 --mode train_softmax --softmax-features 1024 --steps 10 --warmup 2
PMC_GROUPS="mfma valu active" timeout -k 10 900 bash tools/pmc_profile.sh > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
cp gpurun_out/pmc/summary.md $O/pmc_summary.md && cat $O/pmc_summary.md
