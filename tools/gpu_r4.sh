#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export DEBUG_HIP_FORCE_GRAPH_QUEUES=2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_eig_pe.py tests/test_pipeline.py > gpurun_out/r04_t_tests.log 2>&1
rc=$?; echo "=== tests rc=$rc"; tail -1 gpurun_out/r04_t_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/probes/eig_probe.py > gpurun_out/r04_t_eig.log 2>&1
echo "=== eig rc=$?"; tail -1 gpurun_out/r04_t_eig.log
timeout -k 10 300 python tools/probes/cfg3_pipe.py > gpurun_out/r04_t_cfg3.log 2>&1
echo "=== cfg3 rc=$?"; tail -1 gpurun_out/r04_t_cfg3.log
exit 0
