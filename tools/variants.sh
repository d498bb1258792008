#!/bin/bash
# Interleaved A/B of serve-bench variants on one GPU box: each line of SPEC is
#   <name> <io threads> <load-generator threads> [ENV=value ...]
# and every round runs every line once (bench.py --gpus 1 --steps 20 --warmup 5, paired + shuffled
# phases). Output: <OUT>/<name>_r<round>.log; summary: python tools/shuf_summary.py <OUT>.
#   bash tools/variants.sh OUT=gpurun_out/sN SPEC=tools/variants/<file> [ROUNDS=2] [EXTRA="bench args"]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for a in "$@"; do export "$a"; done
mkdir -p "$OUT"
for r in $(seq 1 "${ROUNDS:-2}"); do
  while read -r name io lg envs; do
    [ -z "$name" ] && continue
    [[ "$name" == \#* ]] && continue
    echo "== $name r$r ($io:$lg $envs)"
    env $envs timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --io-threads "$io" \
      --client-threads "$lg" ${EXTRA:-} > "$OUT/${name}_r$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP: $name r$r rc=$rc"; tail -20 "$OUT/${name}_r$r.log"; exit $rc; fi
  done < "$SPEC"
done
python3 tools/shuf_summary.py "$OUT"
echo VARIANTS DONE
