#!/bin/bash
# rocprofv3 kernel stats of the config-3 (cifar) and config-5 (tsp) heads
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in cifar tsp; do
  rm -rf gpurun_out/prof_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- \
    python3 tools/heads_bench.py --configs $c --steps 5 --warmup 2 --batches 1 > gpurun_out/prof_$c.log 2>&1 \
    || { tail -30 gpurun_out/prof_$c.log; exit 1; }
  f=$(find gpurun_out/prof_$c -name "run_kernel_stats.csv" | head -1)
  python3 tools/prof_summary.py "$f" gpurun_out/prof_$c.md "config $c head (heads_bench, 7 steps)"
  head -28 gpurun_out/prof_$c.md
done
