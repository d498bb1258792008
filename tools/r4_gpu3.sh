# Round 4 GPU session 3: wide kernel after the store-hazard fix, serve_wide on WIDE, lanes sweep
set -o pipefail
O=gpurun_out/r4_s3; mkdir -p $O
PYTHONPATH=. timeout -k 10 200 python tools/dbg/wide_partials.py > $O/dbg_partials.txt 2>&1 || { echo "dbg failed"; exit 1; }
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $O/pytest_wide.log 2>&1 || echo "wide tests failed"
timeout -k 10 150 python bench.py --mode serve_wide --steps 10 --warmup 3 > $O/serve_wide_k1000_f32.json 2> $O/serve_wide_k1000_f32.err || echo "serve_wide failed"
for i in 1 2; do
  for cfg in "MLAPI_LANES=0" "MLAPI_LANE_INFLIGHT=3" "MLAPI_LANE_INFLIGHT=6" "MLAPI_LANE_INFLIGHT=8"; do
    env $cfg timeout -k 10 150 python bench.py --steps 12 --warmup 4 > "$O/bench_${cfg}_$i.json" 2> "$O/bench_${cfg}_$i.err" || exit 1
  done
done
