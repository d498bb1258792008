#!/bin/bash
# GEMV completion by records vs the signal kernel (MLAPI_GEMV_RECORD_ROWS=2 / 0) on the wide binary
# serving bench, interleaved x2, after the serving GPU tests. One GPU session on the box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/gemv_rec; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_serve_wide_gpu.py tests/test_serve_gpu.py -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 2 0; do
    for dt in f32 bf16; do
      MLAPI_GEMV_RECORD_ROWS=$v timeout -k 10 300 python -u bench.py --mode serve_wide --wide-classes 2 --wide-dtype $dt \
        --steps 40 --warmup 5 > $O/k2_${dt}_rec${v}_r$r.log 2>&1 || { tail -5 $O/k2_${dt}_rec${v}_r$r.log; exit 1; }
      tail -1 $O/k2_${dt}_rec${v}_r$r.log | cut -c1-110
    done
  done
done
