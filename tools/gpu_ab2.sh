#!/bin/bash
# same-box bench A/B over several env settings (no tests): gpu_ab2.sh "A" "B" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cfg5 --no-heads --steps 30 > gpurun_out/ab2.log 2>&1 || { tail -20 gpurun_out/ab2.log; exit 1; }
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab2.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab2.log | head -1)"
  done
done
