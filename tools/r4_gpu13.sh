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
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "softmax_grad_wide or wide_multiclass or gemm_softmax" > $O/pytest_rows.log 2>&1 || { echo "rows tests failed"; tail -30 $O/pytest_rows.log; exit 1; }
tail -1 $O/pytest_rows.log
for i in 1 2; do
  for v in 1 0; do
    MLAPI_ROWS_NT4=$v timeout -k 10 150 python bench.py --mode train_softmax --softmax-features 1024 --steps 20 --warmup 3 > $O/tsm_f1024_nt4_${v}_$i.json 2> $O/tsm_f1024_nt4_${v}_$i.err || { echo "tsm failed"; exit 1; }
    echo "nt4=$v $i $(python3 -c "import json; d=json.loads(open('$O/tsm_f1024_nt4_${v}_$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], round(d['tflops_incl_recompute'],1))")"
  done
done
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
