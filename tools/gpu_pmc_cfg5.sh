#!/bin/bash
# PMC passes over bench.py's config-5 leg (tools/cfg5_leg.py): L2 hit rate,
# HBM fetch and write bytes per dispatch of the factored-L1 and CSR kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for ctr in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc5_$i
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc5_$i -o run --output-format csv -- python3 tools/cfg5_leg.py > gpurun_out/pmc5_$i.log 2>&1 || { tail -5 gpurun_out/pmc5_$i.log; exit 1; }
done
python3 tools/pmc_kernel.py $(find gpurun_out/pmc5_1 gpurun_out/pmc5_2 gpurun_out/pmc5_3 -name "run_counter_collection.csv") > gpurun_out/pmc5_summary.txt
cat gpurun_out/pmc5_summary.txt
