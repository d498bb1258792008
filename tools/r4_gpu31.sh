# Round 4 GPU session 31: 32x32 kernel class splits at large B (granule merge makes splits cheap)
set -o pipefail
O=gpurun_out/r4_s31; mkdir -p $O
export TMPDIR=/tmp
SWEEP_PLANS="0,0,0 0,1,3 0,2,3 0,4,3" timeout -k 10 300 python tools/gemm_plan_sweep.py 65536 131072 262144 > $O/sweep_large.log 2>&1 || { echo "sweep failed"; tail $O/sweep_large.log; exit 1; }
grep "us graph" $O/sweep_large.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $O/pytest_wide.log 2>&1 || { echo "wide tests failed"; tail -30 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype f32 --steps 10 --warmup 3 > $O/sw_f32.json 2> $O/sw_f32.err || { echo "sw failed"; exit 1; }
echo "sw K=1000 f32 $(python3 -c "import json; d=json.loads(open('$O/sw_f32.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], round(d['gpu_leg_us_c64'],1))")"
