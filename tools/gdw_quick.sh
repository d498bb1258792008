#!/bin/bash
# Quick loop for the fused softmax G+dW kernel: its tests + the timing sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/gdw
mkdir -p $O
cd $R
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -k "softmax_grad_dw" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 11
timeout -k 10 180 python -u tools/softmax_train_sweep.py > $O/sweep.log 2>&1 || exit 12
echo done
