#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HLHGAT_TEST_VERBOSE=1 timeout -k 10 300 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_train_step.py -m gpu -k "lane_replay or graph_replay_equals_eager" > gpurun_out/t4.log 2>&1
rc=$?; echo "=== tests rc=$rc"; grep -E "host call|_run|PASSED|FAILED|passed|failed|^E  " gpurun_out/t4.log | cut -c1-250 | grep -v "err 0" | tail -n 40
exit 0
