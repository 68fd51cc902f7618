#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_step.py nolanes k2 nolanes2 --rounds 3 > gpurun_out/ab_k2.log 2>&1
rc=$?; echo "=== ab k2 rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_k2.log | tail -2 | cut -c1-600
timeout -k 10 300 python tools/kbench.py --big > gpurun_out/kbench_big.log 2>&1
rc=$?; echo "=== kbench big rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench_big.log | tail -30 | cut -c1-200
exit 0
