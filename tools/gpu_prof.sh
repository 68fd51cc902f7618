#!/bin/bash
# Kernel stats (graph replay bench), eager bench, PMC FETCH/WRITE passes on the
# eager step (counters need per-dispatch serialisation; same kernels).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then tail -n 30 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
TAG=${1:-r01}
step bench_eager 300 python bench.py --eager --steps 10 --warmup 3 --no-cpu-baseline --no-heads --batches 2
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 6 --no-cpu-baseline --no-heads --no-cfg5 --batches 3
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o f --output-format csv -- python3 bench.py --eager --steps 2 --warmup 1 --prof-steps 1 --no-cpu-baseline --no-cfg5 --no-heads --batches 1
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o w --output-format csv -- python3 bench.py --eager --steps 2 --warmup 1 --prof-steps 1 --no-cpu-baseline --no-cfg5 --no-heads --batches 1
find gpurun_out/prof gpurun_out/pmcf gpurun_out/pmcw -name '*.csv' | head -20
python tools/pmc_traffic.py $(find gpurun_out/pmcf -name '*counter_collection.csv' | head -1) $(find gpurun_out/pmcw -name '*counter_collection.csv' | head -1) --kernel k_poly_step --kernel k_proj_fwd --kernel k_edge_gather2 --kernel k_bn_fwd_grid --kernel k_bn_bwd_reduce --kernel k_proj_bwd_fused --out gpurun_out/pmc_traffic.json --label "$TAG bench.py --eager cfg2 step" > /dev/null
python tools/timeline.py $(find gpurun_out/prof -name '*kernel_trace.csv' | head -1) --window-ms 60
python tools/step_kernels.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) --step 15 > gpurun_out/step_kernels.txt
