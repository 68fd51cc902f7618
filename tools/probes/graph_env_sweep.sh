# Same box, alternating processes: GPU time per replayed step (host_enqueue.py
# 'total') under the HIP runtime's graph-queue settings.
set -u
cd "${GRAFT_REPO_ROOT}"
for round in 1 2; do
for cfg in "NONE=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=3"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/probes/host_enqueue.py 2>&1 | grep -E "enqueue" | head -3 || { echo "rc=$?"; break; }
done
done
