#!/bin/bash
# Scratch GPU command: tests of the chain / replay paths, same-process A/B, timeline.
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
step t_new 500 python -u -m pytest tests/test_train_step.py tests/test_multirank_trainstep.py tests/test_gpu_parity.py -k "fork or replay or graph or zinc or chain or train or rank or padded" -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
step ab 400 python tools/ab_step.py base join nodefirst base2 join2 nodefirst2 --rounds 6
CAPS='{"rows_t": 23552, "rows_s": 25600, "nnz_t": 75776, "nnz_s": 112640}'
rm -rf gpurun_out/tl
step trace 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python3 bench.py --replay-probe "$CAPS" --steps 12 --warmup 4
T=$(find gpurun_out/tl -name '*kernel_trace.csv' | head -1)
python tools/replay_timeline.py "$T" --steps 3 --out gpurun_out/timeline4.csv && rm -rf gpurun_out/tl
echo "=== done"
