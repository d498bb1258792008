# Round 4 GPU session 35: gemm tests + config-3 bench after restoring plain tag clears
set -o pipefail
O=gpurun_out/r4_s35; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_xcd_fallback_gpu.py tests/test_tensor_parallel_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for B in 1024 8192; do
  timeout -k 10 120 python bench.py --mode gemm --batch $B --steps 2000 --warmup 100 > $O/gemm_b$B.json 2> $O/gemm_b$B.err || { echo "gemm failed"; exit 1; }
  echo "gemm B=$B $(python3 -c "import json; d=json.loads(open('$O/gemm_b$B.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2), 'us')")"
done
