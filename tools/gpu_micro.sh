#!/bin/bash
# GPU tests + microbench (+ its rocprof kernel stats) + bench (stops on a fault)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -n 30 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -m pytest tests -m gpu -q -p no:cacheprovider
tail -n 5 gpurun_out/pytest_gpu.log
step microbench 600 python tools/microbench.py
step micro_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof -o m --output-format csv -- python tools/microbench.py --reps 20 --out gpurun_out/microbench_prof.json
step bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
tail -n 1 gpurun_out/bench.log
