#!/bin/bash
# Sweep native-server / load-generator thread counts for the serving bench (1 GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "${@:-3 3}"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps ${STEPS:-150} --warmup 5 --io-threads $1 --client-threads $2 --c1-requests 1000 \
    > gpurun_out/sweep_io$1_cl$2${TAG:-}.log 2>&1 || { echo "sweep step failed rc=$?"; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_io$1_cl$2${TAG:-}.log').read().strip().splitlines()[-1]); print('io=$1 cl=$2', round(d['value']), 'req/s p50', d['p50_latency_ms_c64'], 'c1 p50', d['p50_latency_ms_batch1'], 'batch', round(d['mean_gpu_batch_rows'],2), d['cpu_cores_busy_rank0'])"
done
