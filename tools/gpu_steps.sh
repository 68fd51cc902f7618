#!/bin/bash
# GPU steps on one MI355X (every round's measurements go through this one script).
# Usage: tools/gpu_steps.sh TAG step [step ...]
#   sel     the GPU tests matching $SEL (pytest -k)
#   quick   the config-2 bench line alone (no heads, loader, census, CPU leg)
#   bn      the BatchNorm barrier tests (hand-over, CU hog, bitwise)
#   tests   the whole GPU suite
#   smoke   __graft_entry__.smoke()
#   bench   the default bench line (driver command)
#   pmcstep the config-2 step under rocprofv3 --pmc (serialised dispatch)
#   prof    rocprofv3 kernel stats + step census of the replayed bench
#   pmc     FETCH / WRITE passes for the roofline traffic
#   census  bench line with heads: k_poly_step per call site (tools/poly_census.py)
# Stops at the first crash / time-out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/${TAG}_$name.log" | cut -c1-800
  case $rc in
    0|1) ;;
    *) tail -n 40 "gpurun_out/${TAG}_$name.log"; exit $rc ;;
  esac
  return 0
}
PT="python -u -m pytest -p no:cacheprovider --timeout 200 --timeout-method thread"
for s in "$@"; do
  case $s in
    sel) step sel 600 $PT tests -m gpu -v -k "$SEL" ;;  # SEL="expr" tools/gpu_steps.sh TAG sel
    cfg3pipe) step cfg3pipe 600 python tools/probes/cfg3_pipe.py --cus "${CUS-0,32,64,128}" --prio "${PRIO-}" --rounds 2 ;;
    ab5env) for r in 1 2; do for v in ${AB5:-0 1}; do  # AB5ENV=NAME: cfg5 step with NAME=v
           env $AB5ENV=$v timeout -k 10 400 python3 bench.py --workload ${WL:-cfg5} --steps 10 --warmup 3 --batches 2 --no-cpu-baseline > gpurun_out/${TAG}_ab5env_${v}_$r.log 2>&1
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_ab5env_${v}_$r.log | head -1 | sed "s/^/${WL:-cfg5} $AB5ENV=$v run $r /" >> gpurun_out/${TAG}_ab5env.txt || true
         done; done; cat gpurun_out/${TAG}_ab5env.txt ;;
    glue) step glue3 300 python3 tools/probes/glue_ops.py --head cfg3_cifar_attpool &&
          step glue4 300 python3 tools/probes/glue_ops.py --head cfg4_pepfunc_attpool &&
          step glue5 300 python3 tools/probes/glue_ops.py --head cfg5_tsp_pyr ;;
    abstep) step abstep 900 python3 tools/ab_step.py ${AB:-base1 base2} --rounds 5 ;;
    quick) step quick 300 python bench.py --no-cfg5 --no-heads --no-cpu-baseline --no-replay-census --no-loader --steps 30 ;;
    bn) step bn 600 $PT tests/test_gpu_parity.py -m gpu -v -s -k "bn_ or proj_bn or handover or hog" ;;
    tests) step tests 1100 $PT tests -m gpu -q ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py ;;
    pmcstep) rm -rf gpurun_out/${TAG}_pmcstep_d
             step pmcstep 200 timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG}_pmcstep_d -o p --output-format csv -- python3 tools/probes/poly_context.py --steps 3
             rm -rf gpurun_out/${TAG}_pmcstep_d ;;
    prof) rm -rf gpurun_out/prof_$TAG
          B="python3 bench.py --steps 20 --warmup 6 --no-cpu-baseline --no-cfg5 --no-heads --no-loader --no-parity-check --no-replay-census --batches 3"
          step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- $B
          T=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
          python tools/step_kernels.py "$T" --step -3 --dump gpurun_out/${TAG}_step_dispatches.csv > gpurun_out/${TAG}_step_kernels.txt || true
          python tools/step_gaps.py "$T" --step -3 --top 40 > gpurun_out/${TAG}_step_gaps.txt || true
          S=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
          cp "$S" gpurun_out/${TAG}_bench_kernel_stats.csv || true
          rm -f "$T" ;;
    prof5) rm -rf gpurun_out/prof5_$TAG  # the config-5 head step (TSP 4x2500), replayed
          step prof5 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5_$TAG -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
          S=$(find gpurun_out/prof5_$TAG -name '*kernel_stats.csv' | head -1)
          cp "$S" gpurun_out/${TAG}_cfg5_kernel_stats.csv || true
          T=$(find gpurun_out/prof5_$TAG -name '*kernel_trace.csv' | head -1)
          python tools/step_kernels.py "$T" --step -3 --dump gpurun_out/${TAG}_cfg5_step_dispatches.csv > gpurun_out/${TAG}_cfg5_step_kernels.txt || true
          rm -rf gpurun_out/prof5_$TAG ;;
    prof3) rm -rf gpurun_out/prof3_$TAG  # the config-3 head step (CIFAR attpool), replayed
          step prof3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3_$TAG -o run --output-format csv -- python3 bench.py --workload cfg3 --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
          T=$(find gpurun_out/prof3_$TAG -name '*kernel_trace.csv' | head -1)
          python tools/step_kernels.py "$T" --step -3 --dump gpurun_out/${TAG}_cfg3_step_dispatches.csv > gpurun_out/${TAG}_cfg3_step_kernels.txt || true
          rm -rf gpurun_out/prof3_$TAG ;;
    prof4) rm -rf gpurun_out/prof4_$TAG  # the config-4 head step (peptides attpool), replayed
          step prof4 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4_$TAG -o run --output-format csv -- python3 bench.py --workload cfg4 --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
          T=$(find gpurun_out/prof4_$TAG -name '*kernel_trace.csv' | head -1)
          python tools/step_kernels.py "$T" --step -3 --dump gpurun_out/${TAG}_cfg4_step_dispatches.csv > gpurun_out/${TAG}_cfg4_step_kernels.txt || true
          rm -rf gpurun_out/prof4_$TAG ;;
    prof5s) rm -rf gpurun_out/prof5s_$TAG  # the same on ONE stream (HLHGAT_STREAM_FORK=0)
          HLHGAT_STREAM_FORK=0 step prof5s 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5s_$TAG -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
          T=$(find gpurun_out/prof5s_$TAG -name '*kernel_trace.csv' | head -1)
          python tools/step_kernels.py "$T" --step -3 --dump gpurun_out/${TAG}_cfg5s_step_dispatches.csv > gpurun_out/${TAG}_cfg5s_step_kernels.txt || true
          rm -rf gpurun_out/prof5s_$TAG ;;
    pmc) rm -rf gpurun_out/pmcf gpurun_out/pmcw
         E="python3 bench.py --eager --steps 2 --warmup 1 --prof-steps 1 --no-cpu-baseline --no-cfg5 --no-heads --no-loader --no-parity-check --no-replay-census --batches 1"
         step pmc_fetch 200 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o f --output-format csv -- $E
         step pmc_write 200 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o w --output-format csv -- $E
         python tools/pmc_traffic.py $(find gpurun_out/pmcf -name '*counter_collection.csv' | head -1) $(find gpurun_out/pmcw -name '*counter_collection.csv' | head -1) --kernel k_poly_step --kernel k_proj_fwd --kernel k_edge_gather2 --kernel k_bn_fwd_grid --kernel k_bn_bwd_reduce --kernel k_proj_bwd_fused --kernel k_proj_bn_fwd --out gpurun_out/${TAG}_pmc_traffic.json --label "$TAG bench.py --eager cfg2 step" > /dev/null || true
         rm -rf gpurun_out/pmcf gpurun_out/pmcw
         # the bench reads the newest profiles/*_pmc_traffic.json: this round's
         cp gpurun_out/${TAG}_pmc_traffic.json profiles/r06_pmc_traffic.json || true ;;
    census) step census 900 python3 bench.py --no-cpu-baseline --no-loader --no-parity-check --steps 20
          python3 tools/poly_census.py gpurun_out/${TAG}_census.log > gpurun_out/${TAG}_poly_census.txt || true ;;
    census1) HLHGAT_STREAM_FORK=0 step census1 900 python3 bench.py --no-cpu-baseline --no-loader --no-parity-check --no-replay-census --steps 10
          python3 tools/poly_census.py gpurun_out/${TAG}_census1.log > gpurun_out/${TAG}_poly_census_1stream.txt || true ;;
    fcalib) rm -rf gpurun_out/${TAG}_fc
          step fcalib 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_fc -o f --output-format csv -- python3 tools/probes/fetch_calib.py run --meta gpurun_out/${TAG}_fc_meta.json
          python3 tools/probes/fetch_calib.py parse $(find gpurun_out/${TAG}_fc -name '*counter_collection.csv' | head -1) --meta gpurun_out/${TAG}_fc_meta.json > gpurun_out/${TAG}_fetch_calib.json || true
          rm -rf gpurun_out/${TAG}_fc ;;
    pbphase) step pbphase 300 python3 tools/probes/proj_bn_phases.py --reps 20 ;;
    bnshapes) step bnshapes 300 python3 tools/probes/bn_shapes.py ;;
    fwdxcd) for v in 1 0; do HLHGAT_FWD_XCD=$v timeout -k 10 300 python3 tools/kbench.py --big --modes 0 --only "proj_fwd" --reps 10 --chain 5 > gpurun_out/${TAG}_fwdxcd_$v.log 2>&1 || exit 3; done
          grep -h '^{' gpurun_out/${TAG}_fwdxcd_1.log gpurun_out/${TAG}_fwdxcd_0.log ;;
    listctr) timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1; echo "=== listctr rc=$?" ;;
    heads) step heads 600 $PT tests -m gpu -v -k "reference_golden or state_dict" ;;
    pmcgemm) # SQ counters of k_proj_bwd_fused: isolated (kbench) and in the replayed step
         L=gpurun_out/${TAG}_counters.txt
         [ -s $L ] || timeout -k 10 120 rocprofv3 -L > $L 2>&1
         C=$(python3 tools/pick_counters.py $L SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT)
         echo "counters: $C"
         rm -rf gpurun_out/${TAG}_pg_iso gpurun_out/${TAG}_pg_step
         step pmcgemm_iso 200 timeout -s KILL 180 rocprofv3 --pmc $C -d gpurun_out/${TAG}_pg_iso -o p --output-format csv -- python3 tools/kbench.py --only "proj_bwd_fused" --reps 5 --chain 5
         python3 tools/pmc_kernel.py $(find gpurun_out/${TAG}_pg_iso -name '*counter_collection.csv' | head -1) --match k_proj_bwd_fused > gpurun_out/${TAG}_pmc_gemm_iso.txt 2>&1 || true
         step pmcgemm_step 200 timeout -s KILL 180 rocprofv3 --pmc $C -d gpurun_out/${TAG}_pg_step -o p --output-format csv -- python3 tools/probes/poly_context.py --steps 3
         python3 tools/pmc_kernel.py $(find gpurun_out/${TAG}_pg_step -name '*counter_collection.csv' | head -1) --match k_proj > gpurun_out/${TAG}_pmc_gemm_step.txt 2>&1 || true
         rm -rf gpurun_out/${TAG}_pg_iso gpurun_out/${TAG}_pg_step ;;
    census5) HLHGAT_LOG_PROJ=1 step census5 300 python3 bench.py --workload cfg5 --eager --steps 1 --warmup 0 --batches 1 --no-cpu-baseline
          grep "hlhgat proj" gpurun_out/${TAG}_census5.log | sort | uniq -c | sort -rn > gpurun_out/${TAG}_census5.txt || true ;;
    census2) HLHGAT_LOG_PROJ=1 step census2 300 python3 bench.py --eager --steps 1 --warmup 0 --prof-steps 1 --no-cpu-baseline --no-cfg5 --no-heads --no-loader --no-parity-check --no-replay-census --batches 1
          grep "hlhgat proj" gpurun_out/${TAG}_census2.log | sort | uniq -c | sort -rn > gpurun_out/${TAG}_census2.txt || true ;;
    kcensus) step kcensus 900 python3 tools/kbench_census.py profiles/r05_cfg5_proj_census.txt ;;
    kcensus2) step kcensus2 600 python3 tools/kbench_census.py profiles/r05_cfg2_proj_census.txt --modes 0 --min-gflop 0.1 --reps 10 --chain 10 ;;
    ab5) for r in 1 2; do for m in 0 -1; do
           HLHGAT_GEMM_BIG=$m step ab5_${m}_$r 400 python3 bench.py --workload cfg5 --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_ab5_${m}_$r.log | sed "s/^/big=$m run $r /" >> gpurun_out/${TAG}_ab5.txt || true
         done; done ;;
    ab5f) for f in 0 1; do for m in 0 -1; do
           HLHGAT_STREAM_FORK=$f HLHGAT_GEMM_BIG=$m step ab5f_${f}_${m} 400 python3 bench.py --workload cfg5 --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_ab5f_${f}_${m}.log | sed "s/^/fork=$f big=$m /" >> gpurun_out/${TAG}_ab5f.txt || true
         done; done ;;
    ab34) for w in cfg3 cfg4; do for m in 0 -1 0 -1; do
           HLHGAT_GEMM_BIG=$m step ab34_${w}_${m} 400 python3 bench.py --workload $w --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_ab34_${w}_${m}.log | sed "s/^/$w big=$m /" >> gpurun_out/${TAG}_ab34.txt || true
         done; done ;;
    abops) for w in cfg5 cfg3; do for o in x w fw dw; do
           HLHGAT_GEMM_BIG_OPS=$o step abops_${w}_${o} 400 python3 bench.py --workload $w --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_abops_${w}_${o}.log | sed "s/^/$w ops=$o /" >> gpurun_out/${TAG}_abops.txt || true
         done; done ;;
    abw) for w in cfg5 cfg3; do for v in x:1 dw:1 dw:4 dw:8 fdw:8; do o=${v%%:*}; r=${v##*:}
           HLHGAT_GEMM_BIG_OPS=$o HLHGAT_BIG_W_ROUNDS=$r step abw_${w}_${o}_$r 400 python3 bench.py --workload $w --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_abw_${w}_${o}_$r.log | sed "s/^/$w ops=$o rounds=$r /" >> gpurun_out/${TAG}_abw.txt || true
         done; done ;;
    abload) for d in 2 3 4 2 3 4; do
           step abload_$d 400 python3 bench.py --no-cfg5 --no-heads --no-cpu-baseline --no-parity-check --no-replay-census --loader-depth $d
           python3 -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{\"metric')][-1]; L=r['loader']; print('depth', sys.argv[2], r['ms_per_step'], L['loader_fed']['ms_per_step'], round(r['ms_per_step']/L['loader_fed']['ms_per_step'],3), L['loader_fed']['host_ms_per_step'])" gpurun_out/${TAG}_abload_$d.log $d >> gpurun_out/${TAG}_abload.txt || true
         done ;;
    abbn) for r in 1 2; do for v in 128 64 256 512; do
           HLHGAT_BN_BWD_PARTS=$v step abbn_${v}_$r 300 python3 bench.py --no-cfg5 --no-heads --no-cpu-baseline --no-parity-check --no-replay-census --no-loader --steps 30
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_abbn_${v}_$r.log | sed "s/^/bwd_parts=$v run $r /" >> gpurun_out/${TAG}_abbn.txt || true
         done; done ;;
    abws) for r in 1 2; do for v in 360 180 240 540; do
           HLHGAT_WSPLIT_TARGET=$v step abws_${v}_$r 300 python3 bench.py --no-cfg5 --no-heads --no-cpu-baseline --no-parity-check --no-replay-census --no-loader --steps 30
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_abws_${v}_$r.log | sed "s/^/wsplit_target=$v run $r /" >> gpurun_out/${TAG}_abws.txt || true
         done; done ;;
    abbn2) for r in 1 2; do for v in 128:256 128:16 512:256 256:16 512:16; do pp=${v%%:*}; fm=${v##*:}
           HLHGAT_BN_BWD_PARTS=$pp HLHGAT_BN_BWD_FLAT_MAX=$fm step abbn2_${pp}_${fm}_$r 300 python3 bench.py --no-cfg5 --no-heads --no-cpu-baseline --no-parity-check --no-replay-census --no-loader --steps 30
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_abbn2_${pp}_${fm}_$r.log | sed "s/^/parts=$pp flat_max=$fm run $r /" >> gpurun_out/${TAG}_abbn2.txt || true
         done; done ;;
    abnew) for r in 1 2 3; do for v in 360:256 240:16; do t=${v%%:*}; fm=${v##*:}
           HLHGAT_WSPLIT_TARGET=$t HLHGAT_BN_BWD_FLAT_MAX=$fm step abnew_${t}_${fm}_$r 300 python3 bench.py --no-cfg5 --no-heads --no-cpu-baseline --no-parity-check --no-replay-census --no-loader --steps 30
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_abnew_${t}_${fm}_$r.log | sed "s/^/wsplit=$t flat_max=$fm run $r /" >> gpurun_out/${TAG}_abnew.txt || true
         done; done ;;
    abload9) for r in 1 2; do for v in base host hostsl4 devsl4; do
           case $v in base) E=""; A="";; host) E="HLHGAT_STAGE_WAIT=host"; A="";; hostsl4) E="HLHGAT_STAGE_WAIT=host"; A="--loader-slots 4";; devsl4) E=""; A="--loader-slots 4";; esac
           step abload9_${v}_$r 400 env $E python3 bench.py --no-heads --no-cpu-baseline --no-replay-census $A
           python3 -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{\"metric')][-1]; L=r['loader']['loader_fed']; print(sys.argv[2], r['ms_per_step'], L['ms_per_step'], round(r['ms_per_step']/L['ms_per_step'],3), L['host_ms_per_step'], L.get('feeder_ms_per_batch'), L.get('stage_ms_per_batch'))" gpurun_out/${TAG}_abload9_${v}_$r.log $v >> gpurun_out/${TAG}_abload9.txt || true
         done; done ;;
    abopsf) for r in 1 2; do for w in cfg5 cfg3; do for o in x f; do
           HLHGAT_GEMM_BIG=-1 HLHGAT_GEMM_BIG_OPS=$o step abopsf_${w}_${o}_$r 400 python3 bench.py --workload $w --steps 10 --warmup 3 --batches 2 --no-cpu-baseline
           grep -o '"ms_per_step": [0-9.]*' gpurun_out/${TAG}_abopsf_${w}_${o}_$r.log | head -1 | sed "s/^/$w ops=$o run $r /" >> gpurun_out/${TAG}_abopsf.txt || true
         done; done; done ;;
    syncprobe) step syncprobe 900 python3 tools/probes/syncbn_capture_probe.py ${PROBE:-} ;;
    hog) step hog 300 python3 tools/probes/hog_probe.py ;;
    rccl) step rccl 600 $PT tests/test_rccl_capture.py tests/test_sync_bn.py tests/test_train_step.py -m gpu -v -k "rccl or sync or staged" ;;
    grad) step grad 900 $PT tests/test_frozen_mask_grads.py -m gpu -v -s ;;
    split) step split 300 $PT tests/test_gpu_parity.py -m gpu -q -k "proj_bn" ;;
    ab) step ab 900 python3 tools/ab_step.py base1 splitbn twolaunchbn nobarrier base2 --rounds 5 ;;
    big) step bigtests 400 $PT tests/test_proj_big.py -m gpu -v -s
         step bigbench 400 python3 tools/kbench.py --big --reps 10 --chain 5 ;;
    kbench) step kbench 300 python3 tools/kbench.py --only "proj" --reps 20 --chain 20 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
