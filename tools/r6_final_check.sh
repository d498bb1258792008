set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r6s8}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_r$r.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/bench_r$r.log; exit 1; }
done
python3 tools/shuf_summary.py $O bench
# serve_wide (the batcher path, io 10 : client 4) with the paired IO placement and without
for r in 1 2; do
  for p in sibling off; do
    timeout -k 10 300 python -u bench.py --mode serve_wide --steps 20 --warmup 5 --io-pin $p > $O/wide_${p}_r$r.log 2>&1 || { echo "WIDE BENCH FAILED"; tail -20 $O/wide_${p}_r$r.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$O/wide_${p}_r$r.log') if l.startswith('{')][-1])
print('wide $p r$r', '%.3f M req/s' % (d['value']/1e6), 'p99', d.get('p99_latency_ms_c64'), 'cpu', d['cpu_breakdown_rank0']['server_cpu_us_per_req'])"
  done
done
