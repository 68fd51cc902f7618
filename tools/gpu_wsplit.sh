#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 0 4096 8192 16384; do
  echo "== WSPLIT_ROWS=$r"
  HLHGAT_WSPLIT_ROWS=$r timeout -k 10 200 python -u tools/kbench.py --big --reps 10 --chain 5 --only "bwd_weight" > gpurun_out/wsplit_$r.log 2>&1 || { tail -20 gpurun_out/wsplit_$r.log; exit 1; }
  grep '^{' gpurun_out/wsplit_$r.log
done
timeout -k 10 200 python -u tools/kbench.py --big --reps 10 --chain 5 --only "fwd|bwd_data" > gpurun_out/big_other.log 2>&1 || exit 1
grep '^{' gpurun_out/big_other.log
