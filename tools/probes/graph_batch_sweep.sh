#!/bin/bash
# Same box, alternating processes: the default bench step (replayed graph) under
# the HIP runtime's graph packet-batch / packet-capture settings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
B="python bench.py --steps 30 --warmup 6 --no-cpu-baseline --no-heads --no-cfg5 --no-loader --no-parity-check --no-replay-census"
for round in 1 2; do
for cfg in "NONE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=4" "DEBUG_HIP_GRAPH_BATCH_SIZE=16" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  out=$(env $cfg timeout -k 10 150 $B 2>/dev/null | grep '^{"metric"')
  rc=$?
  [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; exit 1; }
  echo "$round $cfg $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
done
