#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_train_step.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "brain or train or step or replay" > gpurun_out/pytest_brain.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_brain.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_brain.log; exit $rc; }
timeout -k 10 300 python -u tools/brain_spmm.py > gpurun_out/brain_spmm.log 2>&1 || { tail -20 gpurun_out/brain_spmm.log; exit 1; }
grep '^{' gpurun_out/brain_spmm.log
