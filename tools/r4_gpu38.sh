# Round 4 GPU session 38: the driver's command x3 on the final tree (box-variance check)
set -o pipefail
O=gpurun_out/r4_s38; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$r.json 2> $O/bench_$r.err || { echo "bench failed"; tail $O/bench_$r.err; exit 1; }
  echo "r$r $(python3 -c "import json; d=json.loads(open('$O/bench_$r.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], d['p99_latency_ms_c64'], d['idle_path_batches']['c64'], round(d['mean_gpu_batch_rows'],2))")"
done
