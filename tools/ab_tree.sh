#!/bin/bash
# Same-box A/B of the config-2 bench line (or, with WL=cfg3|cfg4|cfg5, that
# head's replayed step) between this tree and another checkout (e.g. a git
# worktree of an earlier commit, built in place):
#   [WL=cfg4] tools/ab_tree.sh TAG OTHER_DIR [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=$1; OTHER=$2; R=${3:-2}
mkdir -p gpurun_out
for r in $(seq 1 "$R"); do
  for d in "$ROOT" "$ROOT/$OTHER"; do
    n=$([ "$d" = "$ROOT" ] && echo this || echo other)
    if [ -n "${WL:-}" ]; then
      B="bench.py --workload $WL --steps 10 --warmup 3 --batches 2 --no-cpu-baseline"
    else
      B="bench.py --no-cfg5 --no-heads --no-cpu-baseline --no-replay-census --no-loader --no-parity-check --steps 30"
    fi
    (cd "$d" && timeout -k 10 300 python3 $B) \
        > "gpurun_out/${TAG}_${n}_$r.log" 2>&1 || { echo "run $n $r failed"; exit 3; }
    grep -o '"ms_per_step": [0-9.]*' "gpurun_out/${TAG}_${n}_$r.log" | sed "s/^/$n run $r /" \
        | sed "s/^/${WL:-cfg2} /" | tee -a "gpurun_out/${TAG}_ab.txt"
  done
done
