# wide kernel timeline (tools/wide_trace.py) + rocprofv3 phase durations (tools/wide_probe.py)
set -o pipefail
OUT=${OUT:-gpurun_out/wide_trace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 python3 -u tools/wide_trace.py 256 1000 200 > $OUT/trace.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 tools/wide_probe.py > $OUT/probe.log 2>&1 &&
python3 tools/wide_probe_summary.py "$(find $OUT/prof -name '*kernel_trace.csv' -print -quit)" > $OUT/probe_summary.txt 2>&1
rc=$?
cat $OUT/trace.log $OUT/probe_summary.txt
exit $rc
