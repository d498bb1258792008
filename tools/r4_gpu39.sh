# Round 4 GPU session 39: WIDE kernel phase timing after the tag-clearing merge (B = 8 / 24)
set -o pipefail
O=gpurun_out/r4_s39; mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/probe -o prof -- python3 $GRAFT_REPO_ROOT/tools/wide_probe.py > $GRAFT_REPO_ROOT/$O/probe.log 2>&1 || { echo "probe failed"; tail $GRAFT_REPO_ROOT/$O/probe.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(ls $O/probe/*kernel_trace.csv | head -1); python3 tools/wide_probe_summary.py $f | tee $O/summary.txt
rm -f $O/probe/*kernel_trace.csv
