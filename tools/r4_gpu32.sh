# Round 4 GPU session 32: linear_split merge by tagged granules - tests + split probe timing
set -o pipefail
O=gpurun_out/r4_s32; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_xcd_fallback_gpu.py tests/test_serve_wide_gpu.py tests/test_serve_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 150 python tools/ab_bench.py --mode serve_wide --wide-dtype bf16 --steps 10 --warmup 3 > $O/old_bf16_$r.json 2> $O/old_bf16_$r.err || { echo "old failed"; tail $O/old_bf16_$r.err; exit 1; }
  timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype bf16 --steps 10 --warmup 3 > $O/new_bf16_$r.json 2> $O/new_bf16_$r.err || { echo "new failed"; tail $O/new_bf16_$r.err; exit 1; }
  for v in old new; do echo "$v r$r $(python3 -c "import json; d=json.loads(open('$O/${v}_bf16_$r.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], round(d['gpu_leg_us_c64'],1), d['kernel_batches'])")"; done
done
