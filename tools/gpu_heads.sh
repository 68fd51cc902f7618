#!/bin/bash
# attpool-head parity tests + config 3/4 throughput (stops at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
step pytest_heads 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "attpool or cluster_mean or tsp_model or zinc_model_vs"
step heads_bench 400 python -u tools/heads_bench.py ${HEADS_ARGS:-}
