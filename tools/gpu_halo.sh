#!/bin/bash
# GPU parity tests + cfg5 (TSP) SpMM variants.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 60 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_K:-}
step tsp_spmm 400 python tools/tsp_spmm.py ${TSP_ARGS:-} --out gpurun_out/tsp_spmm.json
cat gpurun_out/tsp_spmm.log | grep -v amdgpu.ids
