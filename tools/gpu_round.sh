#!/bin/bash
# Round check on one MI355X: GPU parity tests, smoke, the default bench line,
# rocprofv3 kernel stats of the bench and of the config-5 SpMM tool.
# Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 60 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
rm -rf gpurun_out/prof gpurun_out/prof_tsp
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 6 --no-cpu-baseline --no-cfg5
step prof_tsp 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tsp -o run --output-format csv -- python3 tools/tsp_spmm.py --d 64 128
python tools/step_kernels.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) > gpurun_out/step_kernels.txt || true
echo "=== done"
