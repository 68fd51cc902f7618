#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_gaps
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_gaps -o run --output-format csv -- python3 bench.py --steps 10 --warmup 6 --no-cpu-baseline --no-cfg5 --prof-steps 0 > gpurun_out/prof_gaps.log 2>&1 || { tail -20 gpurun_out/prof_gaps.log; exit 1; }
f=$(find gpurun_out/prof_gaps -name "run_kernel_trace.csv" | head -1)
python3 tools/step_gaps.py "$f" --top 25
