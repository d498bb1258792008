set -o pipefail
OUT=gpurun_out/r5_s16; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $OUT/pytest.log 2>&1 &&
OUT=$OUT bash tools/dbg/wide_trace_session.sh &&
timeout -k 10 300 python -u bench.py --mode serve_wide --wide-classes 1000 --wide-dtype f64 --steps 20 --warmup 5 > $OUT/sw1000.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; exit $rc
