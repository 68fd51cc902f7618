#!/bin/bash
# A/B of an env knob on the large projection shapes (kbench --big) and the ZINC bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=$1; B=$2; ONLY=${3:-bwd_weight}
for v in "$A" "$B"; do
  env $v timeout -k 10 200 python -u tools/kbench.py --big --reps 10 --chain 5 --only "$ONLY" > gpurun_out/abbig.log 2>&1 || { tail -20 gpurun_out/abbig.log; exit 1; }
  echo "== $v"; grep '^{' gpurun_out/abbig.log | sed 's/"iso_us[^,]*, //'
done
bash tools/gpu_ab.sh "$A" "$B" "${4:-proj or linear or model}"
