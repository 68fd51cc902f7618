#!/bin/bash
# Launch-group / weight-gradient-fork parity tests, then a same-box bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_launch_groups.py -m gpu > gpurun_out/pair_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pair_tests.log | tail -n 12
[ $rc -ne 0 ] && { tail -n 60 gpurun_out/pair_tests.log; exit $rc; }
for i in 1 2; do
  for v in "HLHGAT_PAIR_CONV=0" "HLHGAT_PAIR_CONV=1"; do
    env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cfg5 --no-heads --steps 30 > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_bench.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bench.log | head -1)"
  done
done
