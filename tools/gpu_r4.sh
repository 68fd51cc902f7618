#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export DEBUG_HIP_FORCE_GRAPH_QUEUES=2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipeline.py > gpurun_out/r04_g_pipe_tests.log 2>&1
rc=$?; echo "=== pipe tests rc=$rc"; tail -3 gpurun_out/r04_g_pipe_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/probes/cfg3_pipe.py > gpurun_out/r04_g_cfg3.log 2>&1
echo "=== cfg3 rc=$?"; tail -1 gpurun_out/r04_g_cfg3.log
timeout -k 10 300 python tools/probes/cfg3_pipe.py > gpurun_out/r04_g_cfg3b.log 2>&1
echo "=== cfg3 again rc=$?"; tail -1 gpurun_out/r04_g_cfg3b.log
exit 0
