#!/bin/bash
# Round-3 check: the new parity tests first (eval mode, frozen-mask gradients,
# segment-mean zero rows), then the whole GPU suite, then the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 80 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
step new_tests 400 python -u -m pytest tests/test_eval_mode.py tests/test_frozen_mask_grads.py tests/test_gpu_parity.py -k "eval or frozen or segment_mean or readout_grad" -m gpu -v -s -p no:cacheprovider --timeout 200 --timeout-method thread
[ "${NEW_ONLY:-0}" = 1 ] && exit 0
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
step bench 400 python bench.py
echo "=== done"
