#!/bin/bash
# Round 6: rocprofv3 kernel statistics of the final tree's benches (serve headline, F = 1024
# training step, 1000-class predict at B = 262,144) -> gpurun_out/r6prof/<bench>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); export TMPDIR=/tmp
O=$R/gpurun_out/r6prof; mkdir -p $O
run() {  # name, bench args...
  local n=$1; shift
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o $n -- python3 $R/bench.py "$@" > $O/$n.log 2>&1) \
    || { echo "PROF $n FAILED"; tail -5 $O/$n.log; exit 1; }
  find $O -name '*_trace.csv' -size +4M -delete
  echo "done $n"
}
run serve --steps 20 --warmup 5
run tsm1024 --mode train_softmax --softmax-features 1024 --steps 20 --warmup 5
run gemm_big --mode gemm --batch 262144 --steps 50 --warmup 5
