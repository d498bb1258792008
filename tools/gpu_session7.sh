#!/bin/bash
# Session-7: fused softmax G+dW kernel correctness, sweep, train bench and kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s7
mkdir -p $O
cd $R
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -k "softmax_grad_dw or softmax_train_grad or softmax_sgd" -x -v --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1 || exit 11
timeout -k 10 180 python -u tools/softmax_train_sweep.py > $O/sweep.log 2>&1 || exit 12
cp gpurun_out/softmax_train_sweep.json $O/ || true
timeout -k 10 180 python -u bench.py --mode train_softmax --steps 50 --warmup 5 > $O/bench_train_softmax.log 2>&1 || exit 13
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_tsm -o tsm -- python3 $R/bench.py --mode train_softmax --steps 20 --warmup 3 > $O/prof_tsm.log 2>&1 || exit 14
echo done
