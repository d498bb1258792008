# Round 4 GPU session 9: wide-F training in 3 launches (row stats + G fused), DP two-shot / replica
# evidence at N=2 (two ranks on one GPU via the P2P kernel), N=1 fused vs local parity
set -o pipefail
O=gpurun_out/r4_s9; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_xcd_fallback_gpu.py -k "softmax_grad_wide or wide_multiclass_estimator or softmax_train or xcd or split" > $O/pytest_train.log 2>&1 || { echo "train tests failed"; tail -30 $O/pytest_train.log; exit 1; }
tail -1 $O/pytest_train.log
for i in 1 2; do
  timeout -k 10 150 python bench.py --mode train_softmax --softmax-features 1024 --steps 20 --warmup 3 > $O/tsm_f1024_3l_$i.json 2> $O/tsm_f1024_3l_$i.err || { echo "3l failed"; tail -5 $O/tsm_f1024_3l_$i.err; exit 1; }
  MLAPI_WIDE_TRAIN_5L=1 timeout -k 10 150 python bench.py --mode train_softmax --softmax-features 1024 --steps 20 --warmup 3 > $O/tsm_f1024_5l_$i.json 2> $O/tsm_f1024_5l_$i.err || { echo "5l failed"; exit 1; }
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_tsm_f1024 -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --mode train_softmax --softmax-features 1024 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof_tsm_f1024.log 2>&1 || { echo "prof failed"; exit 1; }
cd $GRAFT_REPO_ROOT
PMC_GROUPS="mfma valu" PMC_BENCHES="tsm_f1024:--mode train_softmax --softmax-features 1024 --steps 3 --warmup 1" timeout -k 10 300 bash tools/pmc_profile.sh > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
mkdir -p $O/pmc && cp gpurun_out/pmc/summary.md $O/pmc/ && cat $O/pmc/summary.md
# N=1: world 1 takes the local step (no exchange object): compare with round 3's local numbers
for m in train train_softmax; do
  timeout -k 10 150 python bench.py --mode $m --steps 50 --warmup 5 > $O/${m}_n1.json 2> $O/${m}_n1.err || { echo "$m n1 failed"; exit 1; }
done
# N=2 on one GPU (P2P kernel data plane), two-shot forced on for the multiclass exchange
for m in train train_softmax; do
  MLAPI_COMM=p2p MLAPI_DP_TWO_SHOT=1 timeout -k 10 200 python bench.py --gpus 2 --mode $m --steps 30 --warmup 5 > $O/${m}_n2.json 2> $O/${m}_n2.err || { echo "$m n2 failed"; tail -5 $O/${m}_n2.err; exit 1; }
done
for f in $O/*.json; do echo "$f $(python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print(round(d['value']), d.get('ms_per_step'), {k: d.get(k) for k in ('launches_per_step','tflops_incl_recompute','dp_exchange','replicas_bitwise_equal','p2p_selftest','two_shot')})")"; done
