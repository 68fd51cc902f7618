#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export DEBUG_HIP_FORCE_GRAPH_QUEUES=2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fold or nei_produced or fused_backward_zinc or bn_one" > gpurun_out/r04_k_tests.log 2>&1
rc=$?; echo "=== tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/r04_k_tests.log | head -12; [ $rc = 0 ] || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_train_step.py tests/test_rccl_capture.py tests/test_multirank_trainstep.py tests/test_eval_mode.py > gpurun_out/r04_k_tests2.log 2>&1
rc=$?; echo "=== tests2 rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/r04_k_tests2.log | head -12; [ $rc = 0 ] || exit 1
timeout -k 10 400 python tools/ab_step.py base noprodbn nobnfold base2 noprodbn2 nobnfold2 --rounds 4 > gpurun_out/r04_k_ab.log 2>&1
echo "=== ab rc=$?"; tail -8 gpurun_out/r04_k_ab.log
timeout -k 10 400 python bench.py --no-heads --no-cfg5 --no-cpu-baseline > gpurun_out/r04_k_bench.json 2> gpurun_out/r04_k_bench.err
echo "=== bench rc=$?"; tail -c 200 gpurun_out/r04_k_bench.err
timeout -k 10 300 python tools/kbench.py --only "proj_bwd_fused" > gpurun_out/r04_k_kbench.log 2>&1
echo "=== kbench rc=$?"; grep "^{" gpurun_out/r04_k_kbench.log | head -20
exit 0
