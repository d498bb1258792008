# Round 4 GPU session 23: gemm_softmax split merge by tagged granules (no ticket) vs the ticket protocol
set -o pipefail
O=gpurun_out/r4_s23; mkdir -p $O
export TMPDIR=/tmp
PYTHONPATH=$PWD timeout -k 10 120 python tools/dbg/gemm_merge_dbg.py 5000 256 1000 > $O/dbg.log 2>&1 || { echo "dbg failed"; tail $O/dbg.log; exit 1; }
grep ^iter $O/dbg.log
for r in 1 2; do
  for B in 1024 100 8192 16384; do
    timeout -k 10 120 python tools/ab_bench.py --mode gemm --batch $B --steps 2000 --warmup 100 > $O/old_b${B}_$r.json 2> $O/old_b${B}_$r.err || { echo "old failed"; tail $O/old_b${B}_$r.err; exit 1; }
    timeout -k 10 120 python bench.py --mode gemm --batch $B --steps 2000 --warmup 100 > $O/new_b${B}_$r.json 2> $O/new_b${B}_$r.err || { echo "new failed"; tail $O/new_b${B}_$r.err; exit 1; }
    MLAPI_GEMM_XCD=0 timeout -k 10 120 python bench.py --mode gemm --batch $B --steps 2000 --warmup 100 > $O/agent_b${B}_$r.json 2> $O/agent_b${B}_$r.err || { echo "agent failed"; tail $O/agent_b${B}_$r.err; exit 1; }
    echo "B=$B r$r agent $(python3 -c "import json; d=json.loads(open('$O/agent_b${B}_$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2))")"
    echo "B=$B r$r old $(python3 -c "import json; d=json.loads(open('$O/old_b${B}_$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2))") new $(python3 -c "import json; d=json.loads(open('$O/new_b${B}_$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2))") us"
  done
done
