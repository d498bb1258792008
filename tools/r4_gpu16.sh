# Round 4 GPU session 16: whole GPU tier + smoke + the driver's headline command on the final tree
set -o pipefail
O=gpurun_out/r4_s16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "gpu tier failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || { echo "bench failed"; tail -5 $O/bench_$i.err; exit 1; }
  echo "bench $i $(python3 -c "import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], d['p50_latency_ms_batch1'], d['body_mismatches'])")"
done
