# Round 4 GPU session 37: final tree - whole GPU tier, smoke, the driver command, config 3
set -o pipefail
O=gpurun_out/r4_s37; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "gpu tier failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
echo "headline $(python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(round(d['value']), d['p50_latency_ms_c64'], d['p50_latency_ms_batch1'])")"
timeout -k 10 120 python bench.py --mode gemm --batch 1024 --steps 2000 --warmup 100 > $O/gemm_b1024.json 2> $O/gemm.err || { echo "gemm failed"; exit 1; }
echo "gemm B=1024 $(python3 -c "import json; d=json.loads(open('$O/gemm_b1024.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2), 'us')")"
