#!/bin/bash
# GPU tests + bench + kernel-trace profile of the bench (stops at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step bench 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-}
rm -rf gpurun_out/prof
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 6 --no-cpu-baseline ${BENCH_ARGS:-}
python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv --window-ms 60
python tools/step_kernels.py gpurun_out/prof/run_kernel_trace.csv | head -40
