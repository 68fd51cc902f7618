#!/bin/bash
# head throughput with and without the factored L1 (configs 3, 4, 5)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/heads_bench.py > gpurun_out/heads_fac.log 2>&1 || { tail -30 gpurun_out/heads_fac.log; exit 1; }
HLHGAT_FACTOR=0 timeout -k 10 400 python -u tools/heads_bench.py --configs cifar tsp > gpurun_out/heads_nofac.log 2>&1 || { tail -30 gpurun_out/heads_nofac.log; exit 1; }
grep '^{' gpurun_out/heads_fac.log gpurun_out/heads_nofac.log
