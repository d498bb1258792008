# Round 4 GPU session 21: G^T X with 256 x 128 block tiles (8 waves) vs 128 x 128
set -o pipefail
O=gpurun_out/r4_s21; mkdir -p $O
export TMPDIR=/tmp
for t in 256 128; do
  MLAPI_GDW_TILE=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "softmax_grad_wide or wide_multiclass_estimator" > $O/pytest_t$t.log 2>&1 || { echo "tests $t failed"; tail -30 $O/pytest_t$t.log; exit 1; }
  tail -1 $O/pytest_t$t.log
done
for i in 1 2; do
  for t in 256 128; do
    MLAPI_GDW_TILE=$t timeout -k 10 150 python bench.py --mode train_softmax --softmax-features 1024 --steps 20 --warmup 3 > $O/tsm_f1024_t${t}_$i.json 2> $O/tsm_f1024_t${t}_$i.err || { echo "tsm failed"; exit 1; }
    echo "tile=$t $i $(python3 -c "import json; d=json.loads(open('$O/tsm_f1024_t${t}_$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], round(d['tflops_incl_recompute'],1), d['final_loss'])")"
  done
done
