# G^T X kernel load depth: wide GPU tests, then the F = 1024 training step at MLAPI_GDW_DEPTH=1 / 2 interleaved x2
set -o pipefail
OUT=${OUT:-gpurun_out/gdw_depth}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "wide" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2; do
  for d in 1 2; do
    MLAPI_GDW_DEPTH=$d timeout -k 10 300 python -u bench.py --mode train_softmax --softmax-features 1024 --steps 50 --warmup 5 > $OUT/tsm_d${d}_r$r.log 2>&1 || exit 1
    grep '^{' $OUT/tsm_d${d}_r$r.log | cut -c1-200
  done
done
