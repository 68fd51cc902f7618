#!/bin/bash
# Round-3 check: the new parity tests first, then the whole GPU suite, then
# the default bench.  A failing test does not stop the later steps; a crash,
# abort or timeout does (no further GPU work after a fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  case $rc in
    0|1) ;;  # pass / test failures
    *) tail -n 60 "gpurun_out/$name.log"; exit $rc ;;
  esac
  return 0
}
NEW=${NEW:-"tests/test_frozen_mask_grads.py tests/test_multirank_trainstep.py tests/test_train_step.py tests/test_pipeline.py"}
KSEL=${KSEL:-"frozen or two_ranks or padded_levels or pipeline or mlgc"}
step new_tests 500 python -u -m pytest $NEW -k "$KSEL" -m gpu -v -s -p no:cacheprovider --timeout 200 --timeout-method thread
[ "${NEW_ONLY:-0}" = 1 ] && exit 0
[ "${SKIP_SUITE:-0}" = 1 ] || step pytest_gpu 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
step bench 600 python bench.py
echo "=== done"
