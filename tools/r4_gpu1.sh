# Round 4 GPU session 1: dispatch-rate probe, lanes + wide-kernel tests, serving A/B (lanes on/off)
set -o pipefail
O=gpurun_out/r4_s1; mkdir -p $O
timeout -k 10 120 tools/bin/rate_probe tools/bin/probe.hsaco > $O/rate_probe.txt 2>&1 || echo "probe rc=$?" >> $O/rate_probe.txt
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_lanes_gpu.py > $O/pytest_new.log 2>&1 || { echo "new tests failed"; tail -30 $O/pytest_new.log; exit 1; }
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_serve_wide_gpu.py tests/test_serve_gpu.py > $O/pytest_serve.log 2>&1 || { echo "serve tests failed"; tail -30 $O/pytest_serve.log; exit 1; }
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench_lanes_$i.json 2> $O/bench_lanes_$i.err || exit 1
  MLAPI_LANES=0 timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench_nolanes_$i.json 2> $O/bench_nolanes_$i.err || exit 1
done
