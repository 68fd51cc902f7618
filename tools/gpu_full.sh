#!/bin/bash
# full GPU test suite + smoke + 2-rank (gloo, shared GPU) bench rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "=== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
HLHGAT_DIST_BACKEND=gloo HLHGAT_SHARE_GPU=1 step bench2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 4
