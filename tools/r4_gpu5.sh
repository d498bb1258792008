# Round 4 GPU session 5: serve_wide on the WIDE kernel with the in-kernel class merge
set -o pipefail
O=gpurun_out/r4_s5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $O/pytest_wide.log 2>&1 || { echo "wide tests failed"; tail -30 $O/pytest_wide.log; exit 1; }
for K in 1000 40; do
  for dt in f32 f64; do
    timeout -k 10 150 python bench.py --mode serve_wide --wide-classes $K --wide-dtype $dt --steps 10 --warmup 3 > $O/serve_wide_k${K}_${dt}.json 2> $O/serve_wide_k${K}_${dt}.err || echo "serve_wide $K $dt failed"
  done
done
MLAPI_F32_SPLIT=1 timeout -k 10 150 python bench.py --mode serve_wide --wide-classes 1000 --steps 10 --warmup 3 > $O/serve_wide_k1000_f32split.json 2> $O/serve_wide_k1000_f32split.err || echo "split failed"
mkdir -p $O/prof_k1000_f32 && cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_k1000_f32 -o prof -- python3 bench.py --mode serve_wide --wide-classes 1000 --steps 4 --warmup 2 > $O/prof_k1000_f32.log 2>&1 || echo "prof failed"
