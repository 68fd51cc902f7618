#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export DEBUG_HIP_FORCE_GRAPH_QUEUES=2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fold or nei_produced" > gpurun_out/r04_m_tests.log 2>&1
rc=$?; echo "=== tests rc=$rc"; tail -1 gpurun_out/r04_m_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 400 python tools/ab_step.py base prodbn base2 prodbn2 --rounds 4 > gpurun_out/r04_m_ab.log 2>&1
echo "=== ab rc=$?"; tail -1 gpurun_out/r04_m_ab.log
exit 0
