# Round 4 GPU session 36: slab-reduce kernel with 16 loads in flight (vs 4, ab_old/)
set -o pipefail
O=gpurun_out/r4_s36; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "softmax or sgd or reduce or grad" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 150 python tools/ab_bench.py --mode train_softmax --steps 50 --warmup 5 > $O/old_$r.json 2> $O/old_$r.err || { echo "old failed"; tail $O/old_$r.err; exit 1; }
  timeout -k 10 150 python bench.py --mode train_softmax --steps 50 --warmup 5 > $O/new_$r.json 2> $O/new_$r.err || { echo "new failed"; tail $O/new_$r.err; exit 1; }
  for v in old new; do echo "$v r$r $(python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1000,2), 'us', d['final_loss'] if 'final_loss' in d else '')")"; done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o tsm -- python3 $GRAFT_REPO_ROOT/bench.py --mode train_softmax --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/tsm_kernel_stats.csv; find $O/prof -name "*kernel_trace.csv" -delete
python3 -c "
import csv
for r in csv.DictReader(open('$O/tsm_kernel_stats.csv')):
    if 'mlapi' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1000,2), r['Name'][:70])"
