#!/bin/bash
# One GPU session: tests, smoke, benches, profiles. Stops at the first GPU fault / timeout.
# Usage (on the GPU box): bash tools/gpu_session.sh [steps...]   steps: test smoke serve kbench prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok_or_stop() {  # $1 = rc, $2 = allow test failures (1)
  local rc=$1
  if [ "$rc" -eq 0 ]; then return 0; fi
  if [ "${2:-0}" = "1" ] && [ "$rc" -eq 1 ]; then return 0; fi
  echo "STOP: step failed with rc=$rc"; exit "$rc"
}
steps="${*:-test smoke serve kbench prof}"
for s in $steps; do
  case $s in
    test)
      timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; tail -40 gpurun_out/pytest_gpu.log; ok_or_stop $rc 1 ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; tail -5 gpurun_out/smoke.log; ok_or_stop $rc ;;
    serve)
      timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_serve.log 2>&1
      rc=$?; tail -3 gpurun_out/bench_serve.log; ok_or_stop $rc ;;
    kbench)
      for m in gemv gemm train train_softmax; do
        timeout -k 10 300 python bench.py --mode $m --steps 100 --warmup 10 > gpurun_out/bench_$m.log 2>&1
        rc=$?; tail -2 gpurun_out/bench_$m.log; ok_or_stop $rc
      done ;;
    prof)
      for m in gemv gemm train train_softmax; do
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$m -o $m -- \
          python3 bench.py --mode $m --steps 20 --warmup 2 > gpurun_out/prof_$m.log 2>&1
        rc=$?; tail -2 gpurun_out/prof_$m.log; ok_or_stop $rc
      done
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_serve -o serve -- \
        python3 bench.py --steps 50 --warmup 5 > gpurun_out/prof_serve.log 2>&1
      rc=$?; tail -2 gpurun_out/prof_serve.log; ok_or_stop $rc ;;
  esac
done
echo "SESSION DONE"
