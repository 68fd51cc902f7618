#!/bin/bash
# k_poly_step in the replayed step (kernel trace kept for the overlap
# analysis), L2 hit rates in the step vs isolated (PMC, dispatch-serialised),
# and the per-node cost of the replay (tools/probes/packet_cost.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pc_0
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pc_0 -o run --output-format csv -- python3 tools/probes/poly_context.py > gpurun_out/pc_0.log 2>&1
rc=$?; echo "=== trace rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pc_0.log; exit 1; }
T=$(find gpurun_out/pc_0 -name '*kernel_trace.csv' | head -1)
cp "$T" gpurun_out/r04_a_trace.csv
rm -rf gpurun_out/pmc_step gpurun_out/pmc_iso
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_step -o p --output-format csv -- python3 tools/probes/poly_context.py --steps 3 > gpurun_out/pmc_step.log 2>&1
echo "=== pmc step rc=$?"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_iso -o p --output-format csv -- python3 tools/kbench.py --only poly --reps 5 --chain 5 > gpurun_out/pmc_iso.log 2>&1
echo "=== pmc iso rc=$?"
for d in step iso; do
  C=$(find gpurun_out/pmc_$d -name '*counter_collection.csv' | head -1)
  python3 tools/pmc_kernel.py "$C" --match k_poly_step > gpurun_out/r04_a_pmc_poly_$d.txt 2>&1
  echo "--- $d"; head -12 gpurun_out/r04_a_pmc_poly_$d.txt
done
rm -rf gpurun_out/pmc_step gpurun_out/pmc_iso gpurun_out/pc_0
timeout -k 10 300 python3 tools/probes/packet_cost.py > gpurun_out/r04_a_packet_cost.log 2>&1
echo "=== packet cost rc=$?"; grep -v amdgpu.ids gpurun_out/r04_a_packet_cost.log | tail -1
exit 0
