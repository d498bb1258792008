#!/bin/bash
# Interleaved A/B of serve-bench variants on one GPU box: each line of SPEC is
#   <name> <io threads> <load-generator threads> [ENV=value ...]
# and every round runs every line once (bench.py --steps 20 --warmup 5, paired + shuffled phases).
# Pseudo-variables on a line: TASKSET=<cpulist> runs the bench under taskset; GPUS=<n> runs n ranks
# (MLAPI_COMM=p2p shares the one device); POLLLOAD=<waves> runs tools/bin/ring_probe's poll-only
# waves (the host-memory polling of that many busy resident rings) next to the bench; TREE=<dir>
# runs that directory's bench.py (a built checkout of another revision, e.g. ab_r5/); ARG=<token>
# appends one bench.py argument (e.g. ARG=--client-pin=off).
# Output: <OUT>/<name>_r<round>.log; summary: python tools/shuf_summary.py <OUT>.
#   bash tools/variants.sh OUT=gpurun_out/sN SPEC=tools/variants/<file> [ROUNDS=2] [EXTRA="bench args"]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for a in "$@"; do export "$a"; done
mkdir -p "$OUT"
# TASKSET=numa<k>: the first k CPUs of GPU 0's NUMA-node mask (the bench keeps a mask it is given
# when MLAPI_PLACEMENT=numa is set, so these variants set it)
numa_cpus() { python3 -c "
from mlapi_amd.utils.affinity import gpu_numa_nodes, numa_rank_cpus
m = numa_rank_cpus(0, gpu_numa_nodes()) or list(range(64))
print(','.join(str(c) for c in m[:$1]))"; }
for r in $(seq 1 "${ROUNDS:-2}"); do
  while read -r name io lg envs; do
    [ -z "$name" ] && continue
    [[ "$name" == \#* ]] && continue
    ts=""; gpus=1; poll=0; envv=""; tree="."; args=""
    for kv in $envs; do
      case $kv in
        ARG=*) args="$args ${kv#ARG=}" ;;
        TREE=*) tree=${kv#TREE=} ;;
        TASKSET=numa*) ts="taskset -c $(numa_cpus ${kv#TASKSET=numa})"; envv="$envv MLAPI_PLACEMENT=numa" ;;
        TASKSET=*) ts="taskset -c ${kv#TASKSET=}"; envv="$envv MLAPI_PLACEMENT=numa" ;;
        GPUS=*) gpus=${kv#GPUS=} ;;
        POLLLOAD=*) poll=${kv#POLLLOAD=} ;;
        *) envv="$envv $kv" ;;
      esac
    done
    echo "== $name r$r ($io:$lg gpus=$gpus poll=$poll ts='$ts' $envv)"
    ppid=""
    if [ "$poll" -gt 0 ]; then
      timeout -k 5 90 tools/bin/ring_probe v2 "$poll" 0 45 2 > "$OUT/${name}_r${r}_poll.log" 2>&1 &
      ppid=$!
      sleep 2
    fi
    (cd "$tree" && env $envv $ts timeout -k 10 300 python -u bench.py --gpus "$gpus" --steps 20 --warmup 5 \
      --io-threads "$io" --client-threads "$lg" $args ${EXTRA:-}) > "$OUT/${name}_r$r.log" 2>&1
    rc=$?
    if [ -n "$ppid" ]; then wait "$ppid"; prc=$?; [ $prc -eq 0 ] || { echo "STOP: poll load rc=$prc"; exit $prc; }; fi
    if [ $rc -ne 0 ]; then echo "STOP: $name r$r rc=$rc"; tail -20 "$OUT/${name}_r$r.log"; exit $rc; fi
  done < "$SPEC"
done
python3 tools/shuf_summary.py "$OUT"
echo VARIANTS DONE
