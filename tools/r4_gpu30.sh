# Round 4 GPU session 30: headline serve A/B - kernarg ring in host memory (no HDP flush read-back)
set -o pipefail
O=gpurun_out/r4_s30; mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['cpu_breakdown_rank0']; print(round(d['value']), d['p50_latency_ms_c64'], d['p50_latency_ms_batch1'], round(d['gpu_leg_us_c64'],2), round(b['engine_queue_wait_us_per_req'],2), round(b['batcher_us_per_batch']['launch'],2), round(b['server_http_latency_us_mean'],2))"; }
for r in 1 2 3 4; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/def_$r.json 2> $O/def_$r.err || { echo "def failed"; tail $O/def_$r.err; exit 1; }
  echo "default r$r $(line $O/def_$r.json)"
  MLAPI_KERNARG_HOST=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/c16_$r.json 2> $O/c16_$r.err || { echo "c16 failed"; tail $O/c16_$r.err; exit 1; }
  echo "kernarg_host r$r $(line $O/c16_$r.json)"
done
