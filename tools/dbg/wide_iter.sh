# one iteration of the small-batch WIDE kernel work: wide GPU tests, timeline, rocprofv3 phases
set -o pipefail
OUT=${OUT:-gpurun_out/wide_iter}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_wide_gpu.py tests/test_serve_wide_gpu.py > $OUT/pytest.log 2>&1 &&
OUT=$OUT bash tools/dbg/wide_trace_session.sh
rc=$?; tail -2 $OUT/pytest.log; exit $rc
