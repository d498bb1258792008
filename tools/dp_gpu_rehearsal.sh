#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: N ranks share the GPU, MLAPI_COMM=p2p (RCCL refuses two
# ranks on one device; the P2P all-reduce + gloo control plane does not). Runs the headline serve
# bench and the DP training benches at N = 2 and 4 through torchrun, exactly as the driver launches
# bench.py on a multi-GPU node. Per-rank CPU and GPU shares shrink with N, so the numbers are a
# functional check of the DP path, not a scaling curve.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/dp_gpu}
mkdir -p "$O"
export MLAPI_COMM=p2p
port=29611
for n in ${NS:-2 4}; do
  for mode in ${MODES:-serve train train_softmax}; do
    port=$((port + 1))
    extra=""
    [ "$mode" = serve ] && extra="--reqs-per-conn 512 --pin ${PIN:-auto}"
    timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus "$n" --mode $mode --steps 20 --warmup 3 $extra > "$O/${mode}_n${n}${TAG:-}.log" 2>&1
    rc=$?
    tail -1 "$O/${mode}_n${n}${TAG:-}.log" | cut -c1-400
    [ $rc -eq 0 ] || { echo "STOP: $mode n=$n rc=$rc"; tail -20 "$O/${mode}_n${n}${TAG:-}.log"; exit $rc; }
  done
done
echo REHEARSAL DONE
