#!/bin/bash
# Serving engine knobs (batcher spin, slots in flight) at the default thread split; one bench per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${SWEEP:-"0:4" "30:4" "100:4" "30:8" "0:8"}; do
  spin=${cfg%%:*}; slots=${cfg##*:}
  MLAPI_SPIN_US=$spin MLAPI_SLOTS=$slots timeout -k 10 300 python bench.py --steps 200 --warmup 20 \
    > gpurun_out/sweep_spin${spin}_slots${slots}.log 2>&1 || { echo "STOP spin=$spin slots=$slots"; exit 1; }
  tail -1 gpurun_out/sweep_spin${spin}_slots${slots}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('spin=$spin slots=$slots', round(d['value']), 'p50', d['p50_latency_ms_c64'], 'c1', d['p50_latency_ms_batch1'], 'rows', round(d['mean_gpu_batch_rows'],1), 'gpu_leg', round(d['gpu_leg_us_c64'],1), round(d['gpu_leg_us_batch1'],1), d['cpu_cores_busy_rank0'])"
done
