#!/bin/bash
# Wide-model serving A/B on the box: the serving GPU tests, then serve_wide (K = 1000 f32 and K = 2
# bf16) with AB_VAR set to each of AB_VALS, interleaved x2; prints value and the engine's launch
# breakdown per batch. Usage: AB_VAR=MLAPI_PACK_STAGED AB_VALS="1 0" bash tools/wide_ab.sh
# (CFGS="1000 f32,1000 bf16": the "classes dtype" pairs, comma-separated; OUT: the output dir)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-wide_ab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_serve_wide_gpu.py tests/test_serve_gpu.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in $AB_VALS; do
    IFS=, read -ra cfgs <<< "${CFGS:-1000 f32,2 bf16}"
    for cfg in "${cfgs[@]}"; do
      set -- $cfg
      f=$O/k$1_$2_${AB_VAR}_${v}_r$r.log
      env "$AB_VAR=$v" timeout -k 10 300 python -u bench.py --mode serve_wide --wide-classes $1 --wide-dtype $2 \
        --steps 40 --warmup 5 > $f 2>&1 || { tail -5 $f; exit 1; }
      tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['cpu_breakdown_rank0']; print('$(basename $f)', round(d['value']), c['batcher_us_per_batch']['launch'], c['wide_launch_us_per_batch'])"
    done
  done
done
