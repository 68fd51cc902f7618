#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "HLHGAT_BN_PARTS=64 HLHGAT_BN_RED_THREADS=256" "HLHGAT_BN_PARTS=64 HLHGAT_BN_RED_THREADS=1024" "HLHGAT_BN_PARTS=128 HLHGAT_BN_RED_THREADS=256" "HLHGAT_BN_PARTS=256 HLHGAT_BN_RED_THREADS=256" "HLHGAT_BN_PARTS=16 HLHGAT_BN_RED_THREADS=1024"; do
  env $cfg timeout -k 10 120 python -u tools/kbench.py --only "bn_relu" --reps 20 --chain 20 > gpurun_out/bnsweep.log 2>&1 || { tail -10 gpurun_out/bnsweep.log; exit 1; }
  echo "== $cfg"; grep '^{' gpurun_out/bnsweep.log
done
