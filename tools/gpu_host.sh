#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/host_profile.py > gpurun_out/host_profile.log 2>&1
rc=$?; echo "host rc=$rc"; head -c 9000 gpurun_out/host_profile.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o b --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
echo "prof rc=$?"
