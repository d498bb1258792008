# Round 4 GPU session 29: 1000-class training step kernel statistics (rocprofv3)
set -o pipefail
O=gpurun_out/r4_s29; mkdir -p $O
export TMPDIR=/tmp


cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o tsm -- python3 $GRAFT_REPO_ROOT/bench.py --mode train_softmax --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/tsm_kernel_stats.csv; cut -d, -f1-8 $O/tsm_kernel_stats.csv | head -12
find $O/prof -name "*kernel_trace.csv" -delete
