#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "spmm or basis or schedule or brain or conv or halo" > gpurun_out/pytest_spmm.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_spmm.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_spmm.log; exit $rc; }
timeout -k 10 300 python -u tools/brain_spmm.py > gpurun_out/brain_spmm.log 2>&1 || { tail -20 gpurun_out/brain_spmm.log; exit 1; }
grep '^{' gpurun_out/brain_spmm.log
timeout -k 10 300 python -u tools/cfg5_leg.py > gpurun_out/cfg5_leg.log 2>&1 || { tail -20 gpurun_out/cfg5_leg.log; exit 1; }
grep '^{' gpurun_out/cfg5_leg.log
