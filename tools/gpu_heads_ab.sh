#!/bin/bash
# same-box A/B of the config 3-5 heads (bench.py heads leg) over env settings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$@"; do
    env $v timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --batches 2 --no-cpu-baseline --no-cfg5 > gpurun_out/hab.log 2>&1 || { tail -20 gpurun_out/hab.log; exit 1; }
    echo "$v $(grep '^\[heads\]' gpurun_out/hab.log | sed 's/(CPU oracle [0-9.]*)//' | tr '\n' ' ')"
  done
done
