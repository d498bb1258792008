# Round 4 GPU session 33: whole GPU tier + smoke on the final round-4 tree; headline, serve_wide, gemm lines
set -o pipefail
O=gpurun_out/r4_s33; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "gpu tier failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for K in 2 40; do
  for dt in f32 f64; do
    timeout -k 10 150 python bench.py --mode serve_wide --wide-classes $K --wide-dtype $dt --steps 10 --warmup 3 > $O/sw_k${K}_$dt.json 2> $O/sw_k${K}_$dt.err || { echo "sw failed"; exit 1; }
    echo "sw K=$K $dt $(python3 -c "import json; d=json.loads(open('$O/sw_k${K}_$dt.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], round(d['gpu_leg_us_c64'],1))")"
  done
done
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
echo "headline $(python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], d['p50_latency_ms_batch1'])")"
timeout -k 10 120 python bench.py --mode gemm --batch 1024 --steps 2000 --warmup 100 > $O/gemm_b1024.json 2> $O/gemm.err || { echo "gemm failed"; exit 1; }
echo "gemm B=1024 $(python3 -c "import json; d=json.loads(open('$O/gemm_b1024.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2), 'us')")"
