# Round 4 GPU session 22: f32-storage binary models on the WIDE kernel by default (f32_gemv = A/B)
set -o pipefail
O=gpurun_out/r4_s22; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_serve_wide_gpu.py tests/test_lanes_gpu.py tests/test_serve_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for g in 0 1; do
    MLAPI_F32_GEMV=$g timeout -k 10 150 python bench.py --mode serve_wide --wide-classes 2 --wide-dtype f32 --steps 10 --warmup 3 > $O/sw_k2_gemv${g}_$i.json 2> $O/sw_k2_gemv${g}_$i.err || { echo "sw failed"; exit 1; }
    echo "k2 f32_gemv=$g $i $(python3 -c "import json; d=json.loads(open('$O/sw_k2_gemv${g}_$i.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], round(d['gpu_leg_us_c64'],1))")"
  done
done
timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype f32 --steps 10 --warmup 3 > $O/sw_k1000.json 2> $O/sw_k1000.err || { echo "sw failed"; exit 1; }
echo "k1000 $(python3 -c "import json; d=json.loads(open('$O/sw_k1000.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], round(d['gpu_leg_us_c64'],1))")"
