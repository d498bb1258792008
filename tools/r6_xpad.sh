#!/bin/bash
# Round 6: wide X_aug rows padded to 128-byte lines - the GPU tests, an
# interleaved A/B of the F = 1024 training step (MLAPI_XAUG_PAD = 1 / 0) and a rocprofv3 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6xpad}; mkdir -p $O; O=$(cd $O && pwd)
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "softmax_grad_wide or sgd_wide or softmax_fused" > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for g in 1 0; do
    MLAPI_XAUG_PAD=$g timeout -k 10 300 python -u bench.py --mode train_softmax --softmax-features 1024 --steps 200 --warmup 50 \
      > $O/tsm1024_g${g}_r$r.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/tsm1024_g${g}_r$r.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/tsm1024_g${g}_r$r.log') if l.startswith('{')][-1])
print('xpad=$g r$r', '%.4f ms/step' % d['ms_per_step'], 'loss %.6f' % d['final_loss'], '%.1f M samples/s' % (d['value']/1e6))"
  done
done
for g in 1 0; do
  (cd /tmp && MLAPI_XAUG_PAD=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_g$g -o tsm1024 \
     -- python3 ${GRAFT_REPO_ROOT}/bench.py --mode train_softmax --softmax-features 1024 --steps 20 --warmup 5 > $O/prof_g$g.log 2>&1) \
     || { echo "PROF FAILED"; tail -20 $O/prof_g$g.log; exit 1; }
  find $O -name '*_trace.csv' -size +6M -delete
done
echo XPAD DONE
