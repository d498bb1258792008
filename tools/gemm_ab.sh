# Interleaved A/B of bench.py --mode gemm (BASELINE config 3: B=1024, F=256, K=1000) between a
# stashed copy of the package (ab_old/mlapi_amd, previous extension build) and the working tree.
set -o pipefail
mkdir -p gpurun_out/gemm_ab
ARGS="--mode gemm --steps 2000 --warmup 100 ${EXTRA:-}"
for i in 1 2 3; do
  timeout -k 10 120 python -c "import sys; sys.path.insert(0, 'ab_old'); sys.argv = ['bench.py'] + sys.argv[1:]; import runpy; runpy.run_path('bench.py', run_name='__main__')" $ARGS \
    > gpurun_out/gemm_ab/old_$i.json 2>> gpurun_out/gemm_ab/err.log || exit 1
  timeout -k 10 120 python bench.py $ARGS > gpurun_out/gemm_ab/new_$i.json 2>> gpurun_out/gemm_ab/err.log || exit 1
  python -c "
import json
o = json.loads(open('gpurun_out/gemm_ab/old_$i.json').read().splitlines()[-1]); n = json.loads(open('gpurun_out/gemm_ab/new_$i.json').read().splitlines()[-1])
print('run $i old %.2f us  new %.2f us' % (o['ms_per_step'] * 1e3, n['ms_per_step'] * 1e3))"
done
