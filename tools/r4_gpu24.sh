set -o pipefail
O=gpurun_out/r4_s24; mkdir -p $O; export PYTHONPATH=$PWD
for m in 0 1 2; do
MLAPI_XCD_POLL=$m timeout -k 10 120 python tools/dbg/gemm_merge_dbg.py 5000 256 1000 > $O/poll$m.log 2>&1; echo "poll=$m"; grep ^iter $O/poll$m.log
done
