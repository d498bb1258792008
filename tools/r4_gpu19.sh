# Round 4 GPU session 19: default tree (wait-spin 3 us) - GPU serving tests, the driver's command x3
set -o pipefail
O=gpurun_out/r4_s19; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_serve_gpu.py tests/test_lanes_gpu.py tests/test_serve_wide_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_serve.log 2>&1 || { echo "serve tests failed"; tail -30 $O/pytest_serve.log; exit 1; }
tail -1 $O/pytest_serve.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || { echo "bench failed"; tail -5 $O/bench_$i.err; exit 1; }
  echo "bench $i $(python3 -c "import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); cb=d['cpu_breakdown_rank0']; print(round(d['value']), d['p50_latency_ms_c64'], d['p99_latency_ms_c64'], d['p50_latency_ms_batch1'], d['body_mismatches'], round(cb['server_http_latency_us_mean'],1), round(cb['engine_queue_wait_us_per_req'],1))")"
done
for dt in f32 f64; do
  timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype $dt --steps 10 --warmup 3 > $O/sw_$dt.json 2> $O/sw_$dt.err || { echo "sw failed"; exit 1; }
  echo "sw $dt $(python3 -c "import json; d=json.loads(open('$O/sw_$dt.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], round(d['gpu_leg_us_c64'],1))")"
done
