# Rehearse the multi-rank bench paths on a ONE-GPU box: N ranks share cuda:0, the data plane is
# FakeComm over gloo (RCCL refuses two ranks on one device), everything else - rank env, CPU
# pinning (--pin auto), per-rank engines/servers/load generators, max-over-ranks timing, the JSON
# line - is the code the driver runs at N=2/4/8 on a full node.
set -o pipefail
mkdir -p gpurun_out/dp_rehearsal
export MLAPI_COMM=fake
port=29611
for n in 2 4; do
  for mode in serve train; do
    port=$((port + 1))
    timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $n --mode $mode --steps 100 --warmup 10 \
      > gpurun_out/dp_rehearsal/${mode}_n$n.json 2> gpurun_out/dp_rehearsal/${mode}_n$n.err || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/dp_rehearsal/${mode}_n$n.json').read().strip().splitlines()[-1]);print('$mode n=$n', round(d['value']), d['unit'], d.get('threads'), d.get('cpu_cores_busy_rank0'))"
  done
done
