# Round 4 GPU session 14: 128 x 128 G^T X tiles for wide-F training (vs the 64 x 64 kernel)
set -o pipefail
O=gpurun_out/r4_s14; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "softmax_grad_wide or wide_multiclass_estimator" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for v in 128 64; do
    MLAPI_GDW_TILE=$v timeout -k 10 150 python bench.py --mode train_softmax --softmax-features 1024 --steps 20 --warmup 3 > $O/tsm_f1024_t${v}_$i.json 2> $O/tsm_f1024_t${v}_$i.err || { echo "tsm failed"; exit 1; }
    echo "tile=$v $i $(python3 -c "import json; d=json.loads(open('$O/tsm_f1024_t${v}_$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], round(d['tflops_incl_recompute'],1), d['final_loss'])")"
  done
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --mode train_softmax --softmax-features 1024 --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
cd $GRAFT_REPO_ROOT
rm -f $O/prof/prof_kernel_trace.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof/prof_kernel_stats.csv')))[:5]: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
PMC_GROUPS="mfma" PMC_BENCHES="tsm_f1024:--mode train_softmax --softmax-features 1024 --steps 3 --warmup 1" timeout -k 10 300 bash tools/pmc_profile.sh > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
cp gpurun_out/pmc/summary.md $O/pmc_summary.md && cat $O/pmc_summary.md | head -12
