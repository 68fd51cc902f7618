#!/bin/bash
# Scratch GPU command: does the replayed step wait for the host's graph launch?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_step.py base noupload base2 noupload2 --rounds 6 > gpurun_out/ab.log 2>&1
rc=$?; echo "=== ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/probes/launch_lead.py --steps 20 --rounds 2 > gpurun_out/lead.log 2>&1
rc=$?; echo "=== lead rc=$rc"; grep -v amdgpu.ids gpurun_out/lead.log | tail -3
