# round-5 resident-kernel probe (tools/ring_probe.hip): batch-1 ping-pong and loaded rings, host-memory rings only
set -e
mkdir -p gpurun_out/ring_probe
P=tools/bin/ring_probe
for a in "v1 1 1 2 1 64" "v2 1 1 2 1 16" "v2 1 1 2 2 16" "v2 1 1 2 4 16" "v2 10 6 2 2 16" "v2 10 6 2 4 16"; do
  timeout -k 5 30 $P $a | tee -a gpurun_out/ring_probe/results_v2.jsonl
done
