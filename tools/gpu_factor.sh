#!/bin/bash
# factored-L1 parity tests + config-5 SpMM comparison (stops at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 60 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
step pytest_factor 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "factor ${PYTEST_K:-}"
step tsp_spmm 400 python -u tools/tsp_spmm.py --tiles 24:160:768
grep '^{' gpurun_out/tsp_spmm.log
