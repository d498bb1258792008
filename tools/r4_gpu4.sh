# Round 4 GPU session 4: wide kernel after the workspace-layout fix; serve_wide on WIDE
set -o pipefail
O=gpurun_out/r4_s4; mkdir -p $O
PYTHONPATH=. timeout -k 10 200 python tools/dbg/wide_big.py > $O/dbg_big.txt 2>&1 || { echo "dbg failed"; exit 1; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $O/pytest_wide.log 2>&1 || { echo "wide tests failed"; tail -30 $O/pytest_wide.log; exit 1; }
for K in 1000 40 2; do
  for dt in f32 f64; do
    timeout -k 10 150 python bench.py --mode serve_wide --wide-classes $K --wide-dtype $dt --steps 10 --warmup 3 > $O/serve_wide_k${K}_${dt}.json 2> $O/serve_wide_k${K}_${dt}.err || echo "serve_wide $K $dt failed"
  done
done
