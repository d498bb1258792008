#!/bin/bash
# A/B of serving engine modes, interleaved (box variance is large): bash tools/serve_ab.sh [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${1:-2}); do
  for mode in 0 1; do
    MLAPI_PERSISTENT=$mode timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/ab_p${mode}_r${r}.log 2>&1 \
      || { echo "STOP persistent=$mode"; tail -5 gpurun_out/ab_p${mode}_r${r}.log; exit 1; }
    tail -1 gpurun_out/ab_p${mode}_r${r}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('persistent=$mode', round(d['value']), 'p50', d['p50_latency_ms_c64'], 'c1', d['p50_latency_ms_batch1'], 'rows', round(d['mean_gpu_batch_rows'],1), 'gpu_leg', round(d['gpu_leg_us_c64'],1), round(d['gpu_leg_us_batch1'],1), d['cpu_cores_busy_rank0'])"
  done
done
