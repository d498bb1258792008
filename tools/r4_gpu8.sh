# Round 4 GPU session 8: WIDE class merge by tagged granules (no ticket / fence); XCD-local
# misplacement fallback; f32 split row chunks; phase timing + serve_wide
set -o pipefail
O=gpurun_out/r4_s8; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_serve_wide_gpu.py tests/test_xcd_fallback_gpu.py > $O/pytest_wide.log 2>&1 || { echo "wide tests failed"; tail -30 $O/pytest_wide.log; exit 1; }
tail -2 $O/pytest_wide.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/probe -o prof -- python3 $GRAFT_REPO_ROOT/tools/wide_probe.py > $GRAFT_REPO_ROOT/$O/probe.log 2>&1 || { echo "probe failed"; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(ls $O/probe/*kernel_trace.csv | head -1); python3 tools/wide_probe_summary.py $f | tee $O/probe/summary.txt
for i in 1 2; do
  timeout -k 10 150 python bench.py --mode serve_wide --steps 10 --warmup 3 > $O/k1000_f32_$i.json 2> $O/k1000_f32_$i.err || { echo "default failed"; exit 1; }
  MLAPI_F32_SPLIT=1 timeout -k 10 150 python bench.py --mode serve_wide --steps 10 --warmup 3 > $O/k1000_split_$i.json 2> $O/k1000_split_$i.err || { echo "split failed"; exit 1; }
done
timeout -k 10 150 python bench.py --mode serve_wide --wide-dtype f64 --steps 10 --warmup 3 > $O/k1000_f64.json 2> $O/k1000_f64.err || { echo "f64 failed"; exit 1; }
for f in $O/*.json; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], {k:v for k,v in d.items() if 'leg' in k or 'p50' in k})")"; done
# packed-FP32 epilogue A/B: numerics, interleaved timing, PMC
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "t32pk" > $O/pytest_pk.log 2>&1 || { echo "pk tests failed"; tail -30 $O/pytest_pk.log; exit 1; }
tail -1 $O/pytest_pk.log
for i in 1 2; do
  for k in t32 t32pk; do
    timeout -k 10 120 python bench.py --mode gemm --batch 262144 --gemm-kernel $k --steps 50 --warmup 5 > $O/gemm_${k}_$i.json 2> $O/gemm_${k}_$i.err || { echo "gemm $k failed"; exit 1; }
    echo "gemm $k $i $(python3 -c "import json; d=json.loads(open('$O/gemm_${k}_$i.json').read().strip().splitlines()[-1]); print(d['tflops_per_gpu'], d['us_per_call'])")"
  done
done
PMC_GROUPS="mfma valu active" PMC_BENCHES="t32:--mode gemm --batch 262144 --gemm-kernel t32 --steps 5 --warmup 1|t32pk:--mode gemm --batch 262144 --gemm-kernel t32pk --steps 5 --warmup 1" timeout -k 10 600 bash tools/pmc_profile.sh > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
mkdir -p $O/pmc && cp gpurun_out/pmc/summary.md $O/pmc/ && cat $O/pmc/summary.md
