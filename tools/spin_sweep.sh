cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/spinsweep
for r in a b; do
for cfg in "10 4 0" "6 4 50" "8 4 50" "4 4 50" "6 4 0"; do
  set -- $cfg
  MLAPI_IO_SPIN_US=$3 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --io-threads $1 --client-threads $2 --c1-requests 1000 \
    > gpurun_out/spinsweep/io$1_cl$2_spin$3_$r.log 2>&1 || { echo "failed rc=$?"; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/spinsweep/io$1_cl$2_spin$3_$r.log').read().strip().splitlines()[-1]); print('io=$1 cl=$2 spin=$3', round(d['value']), 'p50', d['p50_latency_ms_c64'], 'c1', d['p50_latency_ms_batch1'], d['cpu_cores_busy_rank0'])"
done
done
