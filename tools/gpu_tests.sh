#!/bin/bash
# Focused GPU parity run: the given pytest selection (default: the whole GPU
# suite), one process, stops at the first failure.  usage: gpu_tests.sh [pytest args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread "${args[@]}" > gpurun_out/tests.log 2>&1
rc=$?
echo "=== tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests.log | tail -n 40
[ $rc -ne 0 ] && tail -n 80 gpurun_out/tests.log
exit $rc
