# Two DP ranks sharing ONE GPU (MLAPI_COMM=p2p) through bench --mode train_softmax: the fused
# in-kernel exchange; each case under its own time limit, every case attempted.
set -u
cd "${GRAFT_REPO_ROOT}"; export TMPDIR=/tmp
O=gpurun_out/r6dp2; mkdir -p $O
one() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" MLAPI_COMM=p2p timeout -k 10 200 python -u bench.py --mode train_softmax --gpus 2 --steps 50 --warmup 10 $BARGS > $O/$n.log 2>&1
  local rc=$?
  python3 -c "
import json,sys
L=[l for l in open('$O/$n.log') if l.startswith('{')]
if not L: print('$n rc=$rc', [l.strip()[-160:] for l in open('$O/$n.log') if 'Error' in l][-1:]); sys.exit(0)
d=json.loads(L[-1]); print('$n', '%.4f ms/step' % d['ms_per_step'], 'loss %.6f' % d['final_loss'], d.get('dp_exchange'))"
}
BARGS="--softmax-features 1024" one f1024_nopack MLAPI_G2_PACKED=0
BARGS="--softmax-features 1024" one f1024_nopad MLAPI_XAUG_PAD=0
BARGS="--softmax-features 1024" one f1024_default X=1
