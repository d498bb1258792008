# Round 4 GPU session 6: WIDE serve latency - slot-private workspaces (unordered direct packets),
# direct dispatch for 1 MB models, the f32 split kernel for comparison, kernel traces
set -o pipefail
O=gpurun_out/r4_s6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $O/pytest_wide.log 2>&1 || { echo "wide tests failed"; tail -30 $O/pytest_wide.log; exit 1; }
for i in 1 2; do
  timeout -k 10 150 python bench.py --mode serve_wide --steps 10 --warmup 3 > $O/k1000_f32_default_$i.json 2> $O/k1000_f32_default_$i.err || echo "default failed"
  MLAPI_DIRECT_WIDE_MAX_WEIGHT_BYTES=1073741824 timeout -k 10 150 python bench.py --mode serve_wide --steps 10 --warmup 3 > $O/k1000_f32_direct_$i.json 2> $O/k1000_f32_direct_$i.err || echo "direct failed"
  MLAPI_F32_SPLIT=1 timeout -k 10 150 python bench.py --mode serve_wide --steps 10 --warmup 3 > $O/k1000_f32_split_$i.json 2> $O/k1000_f32_split_$i.err || echo "split failed"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o prof -- python3 bench.py --mode serve_wide --steps 4 --warmup 2 > $O/prof_default.log 2>&1 || echo "prof failed"
MLAPI_DIRECT_WIDE_MAX_WEIGHT_BYTES=1073741824 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_direct -o prof -- python3 bench.py --mode serve_wide --steps 4 --warmup 2 > $O/prof_direct.log 2>&1 || echo "prof2 failed"
