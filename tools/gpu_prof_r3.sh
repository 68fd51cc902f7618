#!/bin/bash
# Step anatomy of the replayed cfg2 step: kernel + memory-copy trace (kept),
# census and gaps of a replayed step, per-launch shapes of the Linear
# backward, then SQ counters of the largest kernels (their own pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03_b}
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 30 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
B="python3 bench.py --steps 20 --warmup 6 --no-cpu-baseline --no-cfg5 --no-heads --no-loader --no-parity-check --no-replay-census --batches 3"
rm -rf gpurun_out/prof_$TAG
step trace 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- $B
T=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
python tools/step_kernels.py "$T" --step -3 > gpurun_out/${TAG}_step_kernels.txt
python tools/step_gaps.py "$T" --step -3 --top 40 > gpurun_out/${TAG}_step_gaps.txt
python tools/launch_shapes.py "$T" --step -3 > gpurun_out/${TAG}_launch_shapes.txt
head -5 gpurun_out/${TAG}_step_kernels.txt
step pmc_sq 200 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc_$TAG -o sq --output-format csv -- python3 bench.py --eager --steps 2 --warmup 1 --prof-steps 1 --no-cpu-baseline --no-cfg5 --no-heads --no-loader --no-parity-check --no-replay-census --batches 1
echo "=== done"
