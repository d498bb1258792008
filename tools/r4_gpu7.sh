# Round 4 GPU session 7: WIDE class merge rework (parallel exponentials, sc1 hand-off loads):
# numerics, phase timing sc1 vs acquire, serve_wide K=1000 f32/f64 and the split kernel
set -o pipefail
O=gpurun_out/r4_s7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $O/pytest_wide.log 2>&1 || { echo "wide tests failed"; tail -30 $O/pytest_wide.log; exit 1; }
tail -2 $O/pytest_wide.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/probe_sc1 -o prof -- python3 $GRAFT_REPO_ROOT/tools/wide_probe.py > $GRAFT_REPO_ROOT/$O/probe_sc1.log 2>&1 || { echo "probe failed"; exit 1; }
MLAPI_WIDE_ACQUIRE=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/probe_acq -o prof -- python3 $GRAFT_REPO_ROOT/tools/wide_probe.py > $GRAFT_REPO_ROOT/$O/probe_acq.log 2>&1 || { echo "probe2 failed"; exit 1; }
cd $GRAFT_REPO_ROOT
for d in probe_sc1 probe_acq; do f=$(ls $O/$d/*kernel_trace.csv | head -1); echo "== $d"; python3 tools/wide_probe_summary.py $f | tee $O/$d/summary.txt; done
for i in 1 2; do
  timeout -k 10 150 python bench.py --mode serve_wide --steps 10 --warmup 3 > $O/k1000_f32_$i.json 2> $O/k1000_f32_$i.err || { echo "default failed"; exit 1; }
  MLAPI_F32_SPLIT=1 timeout -k 10 150 python bench.py --mode serve_wide --steps 10 --warmup 3 > $O/k1000_split_$i.json 2> $O/k1000_split_$i.err || { echo "split failed"; exit 1; }
done
timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype f64 --steps 10 --warmup 3 > $O/k1000_f64.json 2> $O/k1000_f64.err || { echo "f64 failed"; exit 1; }
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d.get('p50_us'), {k:v for k,v in d.items() if 'leg' in k or 'gpu' in k})")"; done
