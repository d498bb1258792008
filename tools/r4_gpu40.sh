# Round 4 GPU session 40: granule tag clears only in graph captures (WIDE, class-split): tests + phase timing
set -o pipefail
O=gpurun_out/r4_s40; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py tests/test_kernels_gpu.py tests/test_xcd_fallback_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/probe -o prof -- python3 $GRAFT_REPO_ROOT/tools/wide_probe.py > $GRAFT_REPO_ROOT/$O/probe.log 2>&1 || { echo "probe failed"; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(ls $O/probe/*kernel_trace.csv | head -1); python3 tools/wide_probe_summary.py $f | tee $O/summary.txt
rm -f $O/probe/*kernel_trace.csv
