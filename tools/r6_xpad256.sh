#!/bin/bash
# Round 6: X_aug rows padded to 128-byte lines on the F = 256 (1000-class) training step - GPU tests and
# an interleaved A/B of bench --mode train_softmax (steady state: --steps 500 --warmup 200), MLAPI_XAUG_PAD 1 / 0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6xpad256}; mkdir -p $O; O=$(cd $O && pwd)
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train.py tests/test_wide_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "softmax or sgd" > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for g in 1 0; do
    MLAPI_XAUG_PAD=$g timeout -k 10 300 python -u bench.py --mode train_softmax --steps 500 --warmup 200 \
      > $O/tsm256_g${g}_r$r.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/tsm256_g${g}_r$r.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/tsm256_g${g}_r$r.log') if l.startswith('{')][-1])
print('xpad=$g r$r', '%.2f us/step' % (1000 * d['ms_per_step']), 'loss %.6f' % d['final_loss'], '%.1f M samples/s' % (d['value']/1e6))"
  done
done
echo XPAD256 DONE
