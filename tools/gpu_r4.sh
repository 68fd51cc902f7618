#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v -p no:cacheprovider --timeout 250 --timeout-method thread \
  tests/test_train_step.py tests/test_eval_mode.py tests/test_rccl_capture.py -m gpu -k "lane_replay or graph_replay_equals or head_graph_replay or chains_bitwise or stream_fork or rccl or infer_step" > gpurun_out/t4.log 2>&1
rc=$?; echo "=== tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|^E  " gpurun_out/t4.log | cut -c1-300 | tail -n 30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/ab_step.py base nolanes base2 nolanes2 --rounds 6 > gpurun_out/ab.log 2>&1
rc=$?; echo "=== ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | tail -8
exit $rc
