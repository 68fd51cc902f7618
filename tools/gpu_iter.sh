#!/bin/bash
# quick iteration: focused parity tests, head throughput, headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; grep '^{' "gpurun_out/$name.log" | cut -c1-400; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
step pytest_iter 300 python -u -m pytest tests/test_gpu_parity.py tests/test_train_step.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "${PYTEST_K:-norm or linear or proj or model or factor}"
step heads 400 python -u tools/heads_bench.py --configs ${HEADS:-cifar tsp}
step bench 300 python -u bench.py --no-cpu-baseline --no-cfg5
