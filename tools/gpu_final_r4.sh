#!/bin/bash
# Round-4 rehearsal on one MI355X: GPU suite, smoke, the default bench line,
# rocprofv3 kernel stats + step census/gaps of the replayed bench, and the
# PMC FETCH/WRITE passes for the roofline traffic.  Stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04_final}
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-600
  case $rc in
    0|1) ;;
    *) tail -n 40 "gpurun_out/$name.log"; exit $rc ;;
  esac
  return 0
}
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python bench.py
rm -rf gpurun_out/prof_$TAG gpurun_out/pmcf gpurun_out/pmcw
B="python3 bench.py --steps 20 --warmup 6 --no-cpu-baseline --no-cfg5 --no-heads --no-loader --no-parity-check --no-replay-census --batches 3"
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- $B
T=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
python tools/step_kernels.py "$T" --step -3 > gpurun_out/${TAG}_step_kernels.txt || true
python tools/step_gaps.py "$T" --step -3 --top 40 > gpurun_out/${TAG}_step_gaps.txt || true
S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
cp "$S" gpurun_out/${TAG}_bench_kernel_stats.csv || true
rm -f "$T"
E="python3 bench.py --eager --steps 2 --warmup 1 --prof-steps 1 --no-cpu-baseline --no-cfg5 --no-heads --no-loader --no-parity-check --no-replay-census --batches 1"
step pmc_fetch 200 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o f --output-format csv -- $E
step pmc_write 200 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o w --output-format csv -- $E
python tools/pmc_traffic.py $(find gpurun_out/pmcf -name '*counter_collection.csv' | head -1) $(find gpurun_out/pmcw -name '*counter_collection.csv' | head -1) --kernel k_poly_step --kernel k_proj_fwd --kernel k_edge_gather2 --kernel k_bn_fwd_grid --kernel k_bn_fwd_produced --kernel k_bn_bwd_reduce --kernel k_proj_bwd_fused --kernel k_proj_bn_fwd --out gpurun_out/${TAG}_pmc_traffic.json --label "$TAG bench.py --eager cfg2 step" > /dev/null || true
rm -rf gpurun_out/pmcf gpurun_out/pmcw
# k_poly_step's L2 behaviour in isolation (the replayed-step pass is in
# ${TAG}_pmc_poly_step via tools/probes/poly_context.py)
rm -rf gpurun_out/pmc_iso gpurun_out/pmc_step
step pmc_iso 150 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum -d gpurun_out/pmc_iso -o p --output-format csv -- python3 tools/kbench.py --only laguerre_step --reps 5 --chain 5
python3 tools/pmc_kernel.py $(find gpurun_out/pmc_iso -name '*counter_collection.csv' | head -1) --match k_poly_step > gpurun_out/${TAG}_pmc_poly_iso.txt 2>&1 || true
step pmc_step 150 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum -d gpurun_out/pmc_step -o p --output-format csv -- python3 tools/probes/poly_context.py --steps 3
python3 tools/pmc_kernel.py $(find gpurun_out/pmc_step -name '*counter_collection.csv' | head -1) --match k_poly_step > gpurun_out/${TAG}_pmc_poly_step.txt 2>&1 || true
rm -rf gpurun_out/pmc_iso gpurun_out/pmc_step
echo "=== done"
