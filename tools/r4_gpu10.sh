# Round 4 GPU session 10: whole GPU tier + smoke, the headline bench, wide training after the
# gdw_gemm prefetch, serve_wide with direct dispatch for the 1 MB model (kernels overlap) vs default
set -o pipefail
O=gpurun_out/r4_s10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo "gpu tier failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
for i in 1 2; do
  timeout -k 10 150 python bench.py --mode train_softmax --softmax-features 1024 --steps 20 --warmup 3 > $O/tsm_f1024_$i.json 2> $O/tsm_f1024_$i.err || { echo "tsm failed"; exit 1; }
done
for i in 1 2; do
  for dt in f32 f64; do
    timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype $dt --steps 10 --warmup 3 > $O/sw_${dt}_$i.json 2> $O/sw_${dt}_$i.err || { echo "sw failed"; exit 1; }
    MLAPI_DIRECT_WIDE_MAX_WEIGHT_BYTES=1073741824 timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype $dt --steps 10 --warmup 3 > $O/sw_${dt}_direct_$i.json 2> $O/sw_${dt}_direct_$i.err || { echo "sw direct failed"; exit 1; }
  done
done
for f in $O/*.json; do echo "$f $(python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print(round(d['value']), d.get('ms_per_step'), {k: (round(v,1) if isinstance(v,float) else v) for k,v in d.items() if k in ('p50_latency_ms_c64','p50_latency_ms_batch1','gpu_leg_us_c64','launches_per_step','tflops_incl_recompute','direct_wide_batches')})")"; done
