# Round 4 GPU session 11: WIDE merger = the row group's last class block; large-grid test; timing
set -o pipefail
O=gpurun_out/r4_s11; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $O/pytest_wide.log 2>&1 || { echo "wide tests failed"; tail -30 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/probe -o prof -- python3 $GRAFT_REPO_ROOT/tools/wide_probe.py > $GRAFT_REPO_ROOT/$O/probe.log 2>&1 || { echo "probe failed"; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(ls $O/probe/*kernel_trace.csv | head -1); python3 tools/wide_probe_summary.py $f | tee $O/probe/summary.txt
for dt in f32 f64; do
  timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype $dt --steps 10 --warmup 3 > $O/sw_$dt.json 2> $O/sw_$dt.err || { echo "sw failed"; exit 1; }
  echo "sw $dt $(python3 -c "import json; d=json.loads(open('$O/sw_$dt.json').read().strip().splitlines()[-1]); print(round(d['value']), round(d['gpu_leg_us_c64'],1))")"
done
