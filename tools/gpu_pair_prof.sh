#!/bin/bash
# Kernel traces of the bench step with and without the paired convs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  HLHGAT_PAIR_CONV=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 4 --no-cpu-baseline --no-cfg5 --no-heads --batches 2 > gpurun_out/pp$v.log 2>&1 || { tail -20 gpurun_out/pp$v.log; exit 1; }
  python tools/step_kernels.py $(find gpurun_out/pp$v -name '*kernel_trace.csv' | head -1) > gpurun_out/step_kernels_pp$v.txt
done
