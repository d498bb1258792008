#!/bin/bash
# Session-9 evidence: full GPU test tier, smoke, flagship serve bench, training benches + kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s9
mkdir -p $O
cd $R
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 11
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
timeout -k 10 240 python -u bench.py > $O/bench_serve.log 2>&1 || exit 13
timeout -k 10 180 python -u bench.py --mode train --steps 50 --warmup 5 > $O/bench_train.log 2>&1 || exit 14
timeout -k 10 180 python -u bench.py --mode train_softmax --steps 50 --warmup 5 > $O/bench_train_softmax.log 2>&1 || exit 15
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_train -o train -- python3 $R/bench.py --mode train --steps 20 --warmup 3 > $O/prof_train.log 2>&1 || exit 16
echo done
