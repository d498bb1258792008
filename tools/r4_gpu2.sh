# Round 4 GPU session 2: wide-kernel debug, new + touched GPU tests, serving A/B (lanes on/off)
set -o pipefail
O=gpurun_out/r4_s2; mkdir -p $O
PYTHONPATH=. timeout -k 10 200 python tools/dbg/wide_nfs.py > $O/dbg_wide.txt 2>&1 || { echo "dbg failed rc=$?"; tail -20 $O/dbg_wide.txt; exit 1; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_serve_gpu.py > $O/pytest_lanes.log 2>&1 || { echo "lanes tests failed"; tail -40 $O/pytest_lanes.log; exit 1; }
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench_lanes_$i.json 2> $O/bench_lanes_$i.err || exit 1
  MLAPI_LANES=0 timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench_nolanes_$i.json 2> $O/bench_nolanes_$i.err || exit 1
done
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_wide_gpu.py > $O/pytest_wide.log 2>&1 || echo "wide tests failed"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_comm_gpu.py > $O/pytest_comm.log 2>&1 || echo "comm tests failed"
