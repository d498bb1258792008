# Round 4 GPU session 25: gemm_softmax split plans with the granule merge (auto = the new plan)
set -o pipefail
O=gpurun_out/r4_s25; mkdir -p $O
export TMPDIR=/tmp
SWEEP_PLANS="0,0,0 1,8,1 1,16,1 0,2,3 0,4,3 0,8,3" timeout -k 10 300 python tools/gemm_plan_sweep.py 1 100 1024 2048 4096 8192 16384 > $O/sweep_auto.log 2>&1 || { echo "sweep failed"; tail $O/sweep_auto.log; exit 1; }
grep "us graph" $O/sweep_auto.log
SWEEP_K=100 SWEEP_PLANS="0,0,0 1,1,1 1,2,1 0,0,1" timeout -k 10 300 python tools/gemm_plan_sweep.py 1024 8192 > $O/sweep_k100.log 2>&1 || { echo "sweep failed"; tail $O/sweep_k100.log; exit 1; }
grep "us graph" $O/sweep_k100.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_xcd_fallback_gpu.py tests/test_tensor_parallel_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for B in 1024 8192; do
    timeout -k 10 120 python tools/ab_bench.py --mode gemm --batch $B --steps 2000 --warmup 100 > $O/old_b${B}_$r.json 2> $O/old_b${B}_$r.err || { echo "old failed"; tail $O/old_b${B}_$r.err; exit 1; }
    timeout -k 10 120 python bench.py --mode gemm --batch $B --steps 2000 --warmup 100 > $O/new_b${B}_$r.json 2> $O/new_b${B}_$r.err || { echo "new failed"; tail $O/new_b${B}_$r.err; exit 1; }
    echo "B=$B r$r old $(python3 -c "import json; d=json.loads(open('$O/old_b${B}_$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2))") new $(python3 -c "import json; d=json.loads(open('$O/new_b${B}_$r.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1000,2))") us"
  done
done
