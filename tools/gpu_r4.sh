#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python bench.py --no-cfg5 --no-cpu-baseline --no-loader > gpurun_out/r04_s_bench.json 2> gpurun_out/r04_s_bench.err
echo "=== bench noloader rc=$?"; grep -n "FAILED\|re-run\|heads\]" gpurun_out/r04_s_bench.err | head -5
exit 0
