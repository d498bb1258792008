# Round 4 GPU session 34: gemm_softmax granule tag clear - plain stores (ab_old/) vs write-through
set -o pipefail
O=gpurun_out/r4_s34; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for B in 1024 8192; do
    timeout -k 10 120 python tools/ab_bench.py --mode gemm --batch $B --steps 2000 --warmup 100 > $O/plain_b${B}_$r.json 2> $O/plain_b${B}_$r.err || { echo "plain failed"; tail $O/plain_b${B}_$r.err; exit 1; }
    timeout -k 10 120 python bench.py --mode gemm --batch $B --steps 2000 --warmup 100 > $O/wt_b${B}_$r.json 2> $O/wt_b${B}_$r.err || { echo "wt failed"; tail $O/wt_b${B}_$r.err; exit 1; }
    echo "B=$B r$r plain $(python3 -c "import json; d=json.loads(open('$O/plain_b${B}_$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2))") write-through $(python3 -c "import json; d=json.loads(open('$O/wt_b${B}_$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2))") us"
  done
done
