#!/bin/bash
# round-end rehearsal: full GPU suite, smoke, the default bench (as the driver runs it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-3000
  if [ $rc -ne 0 ]; then tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python bench.py
