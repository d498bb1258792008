set -u
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp
O=gpurun_out/r6gdwt; mkdir -p $O
for r in 1 2; do
  for t in 1024 512 1536; do
    MLAPI_GDW_TARGET=$t timeout -k 10 300 python -u bench.py --mode train_softmax --softmax-features 1024 --steps 200 --warmup 50 > $O/t${t}_r$r.log 2>&1 || { echo FAIL; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/t${t}_r$r.log') if l.startswith('{')][-1])
print('target=$t r$r', '%.4f ms/step' % d['ms_per_step'], 'loss %.6f' % d['final_loss'])"
  done
done
