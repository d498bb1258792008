#!/bin/bash
# Session-7 evidence: full GPU test tier, smoke, flagship serve bench, softmax-train bench + kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s7b
mkdir -p $O
cd $R
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 11
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
timeout -k 10 240 python -u bench.py > $O/bench_serve.log 2>&1 || exit 13
timeout -k 10 180 python -u bench.py --mode train_softmax --steps 50 --warmup 5 > $O/bench_train_softmax.log 2>&1 || exit 14
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tsm -o tsm -- python3 $R/bench.py --mode train_softmax --steps 20 --warmup 3 > $O/prof_tsm.log 2>&1 || exit 15
echo done
