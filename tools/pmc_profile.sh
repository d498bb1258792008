#!/bin/bash
# Hardware counters for the hot kernels (one rocprofv3 run per counter group; counters are
# collected with --kernel-trace only, never with sys/runtime traces). Run on the GPU box:
#   bash tools/pmc_profile.sh      -> gpurun_out/pmc/<bench>_<group>/..._counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
# FETCH_SIZE / WRITE_SIZE are derived from many TCC channel counters: one per pass (together
# they exceed what one pass can collect and rocprofv3 aborts).
declare -A GROUPS_=(
  [fetch]="FETCH_SIZE"
  [write]="WRITE_SIZE"
  [mfma]="SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
  [lds]="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES"
  [valu]="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"
  [stall]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
  [active]="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
  [l2]="TCC_HIT_sum TCC_MISS_sum"
  [ldswait]="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
  [l2req]="TCP_TCC_READ_REQ_sum TCC_REQ_sum TCC_READ_sum"
)
GROUP_ORDER="${PMC_GROUPS:-fetch write mfma lds valu stall active l2 ldswait}"
BENCHES="${PMC_BENCHES:-gemv:--mode gemv --steps 5 --warmup 1|gemm:--mode gemm --steps 5 --warmup 1|gemm_big:--mode gemm --batch 262144 --steps 5 --warmup 1|train:--mode train --steps 5 --warmup 1|train_softmax:--mode train_softmax --steps 5 --warmup 1}"
IFS='|' read -ra BL <<< "$BENCHES"
for entry in "${BL[@]}"; do
  name="${entry%%:*}"; args="${entry#*:}"
  for g in $GROUP_ORDER; do
    out="gpurun_out/pmc/${name}_${g}"
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc ${GROUPS_[$g]} --output-format csv -d "$out" -o run -- \
      python3 bench.py $args > "$out.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP: $name/$g rc=$rc"; tail -5 "$out.log"; exit $rc; fi
    echo "done $name/$g"
  done
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.md && cat gpurun_out/pmc/summary.md
