#!/bin/bash
# Scratch GPU command: the newest tests, a same-process A/B, kernel microbench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-2000
  case $rc in
    0|1) ;;
    *) tail -n 60 "gpurun_out/$name.log"; exit $rc ;;
  esac
  return 0
}
step t_new 300 python -u -m pytest tests/test_gpu_parity.py -k "batch_hook or spmm or basis or laguerre or cheb" -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
step ab 300 python tools/ab_step.py base nobatch base2 nobatch2 --rounds 6
step kb 200 python tools/kbench.py --only "laguerre|basis"
echo "=== done"
