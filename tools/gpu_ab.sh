#!/bin/bash
# A/B of an env knob on one box: tests with B, then bench A, B, A, B
# usage: gpu_ab.sh "VAR=a" "VAR=b" [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=$1; B=$2; K=${3:-norm or bn or model or train}
env $B timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_train_step.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" > gpurun_out/ab_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/ab_pytest.log; exit $rc; }
for i in 1 2; do
  for v in "$A" "$B"; do
    env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cfg5 --steps 30 > gpurun_out/ab_bench.log 2>&1 || { tail -20 gpurun_out/ab_bench.log; exit 1; }
    echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_bench.log | head -1)"
  done
done
