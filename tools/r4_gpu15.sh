# Round 4 GPU session 15: row-group kernel with 96-row blocks (KS = 2) vs 64-row blocks for wide F
set -o pipefail
O=gpurun_out/r4_s15; mkdir -p $O
export TMPDIR=/tmp
MLAPI_ROWS_NT=6 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "softmax_grad_wide or wide_multiclass" > $O/pytest_nt6.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest_nt6.log; exit 1; }
tail -1 $O/pytest_nt6.log
for i in 1 2; do
  for v in 6 4; do
    MLAPI_ROWS_NT=$v timeout -k 10 150 python bench.py --mode train_softmax --softmax-features 1024 --steps 20 --warmup 3 > $O/tsm_f1024_nt${v}_$i.json 2> $O/tsm_f1024_nt${v}_$i.err || { echo "tsm failed"; exit 1; }
    echo "nt=$v $i $(python3 -c "import json; d=json.loads(open('$O/tsm_f1024_nt${v}_$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], round(d['tflops_incl_recompute'],1), d['final_loss'])")"
  done
done
