set -u
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp
O=gpurun_out/r6xnt16; mkdir -p $O
for r in 1 2 3; do
  for g in 0 1; do
    MLAPI_GEMM_XNT16=$g timeout -k 10 120 python -u tools/probes/gemm16_xnt_ab.py >> $O/ab.log 2>&1 || { echo FAIL; tail -5 $O/ab.log; exit 1; }
  done
done
grep xnt16 $O/ab.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm or softmax" > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
