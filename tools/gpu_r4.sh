#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python bench.py > gpurun_out/r04_q_bench.json 2> gpurun_out/r04_q_bench.err
echo "=== bench rc=$?"; grep -n "FAILED\|re-run\|Error\|heads\]" gpurun_out/r04_q_bench.err | head
exit 0
