# Interleaved A/B of the serve bench with and without CPU pinning (bench.py --pin off|on).
set -o pipefail
mkdir -p gpurun_out/pin_ab
for i in 1 2; do
  for p in off on; do
    timeout -k 10 120 python bench.py --steps 400 --warmup 40 --pin $p \
      > gpurun_out/pin_ab/serve_${p}_$i.json 2> gpurun_out/pin_ab/serve_${p}_$i.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/pin_ab/serve_${p}_$i.json'));print('$p',$i,round(d['value']),d['p50_latency_ms_c64'],d['p99_latency_ms_c64'],d['threads'],d['cpu_cores_busy_rank0'])"
  done
done
