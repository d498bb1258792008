set -u
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp
O=gpurun_out/r6xnt; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm or softmax" > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/probes/gemm_xnt_ab.py > $O/ab.log 2>&1 || { echo AB FAILED; tail $O/ab.log; exit 1; }
tail -2 $O/ab.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --mode gemm --batch 262144 --steps 200 --warmup 20 > $O/gemm_big_r$r.log 2>&1 || { echo "BENCH FAILED"; exit 1; }
  timeout -k 10 200 python -u bench.py --mode gemm --steps 2000 --warmup 100 > $O/gemm_c3_r$r.log 2>&1 || { echo "BENCH FAILED"; exit 1; }
  timeout -k 10 300 python -u bench.py --mode train_softmax --steps 500 --warmup 200 > $O/tsm256_r$r.log 2>&1 || { echo "BENCH FAILED"; exit 1; }
  for f in gemm_big gemm_c3 tsm256; do python3 -c "
import json; d=json.loads([l for l in open('$O/${f}_r$r.log') if l.startswith('{')][-1])
print('$f r$r', '%.2f us/step' % (1000 * d['ms_per_step']), '%.4g' % d['value'], d['unit'])"; done
done
