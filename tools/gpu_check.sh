#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEP_TIMEOUT=${STEP_TIMEOUT:-600}
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return $rc
}
MODE=${1:-all}
if [[ $MODE == all || $MODE == test ]]; then
  run pytest_gpu "$STEP_TIMEOUT" python -m pytest tests -m gpu -q -x -p no:cacheprovider
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $MODE == all || $MODE == bench ]]; then
  run bench 600 python bench.py --steps 20 --warmup 6
fi
if [[ $MODE == all || $MODE == prof ]]; then
  export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 6 --no-cpu-baseline
fi
echo "=== done"
