#!/bin/bash
# run-to-run determinism of a small attpool head (eager) under each A/B knob
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export REPS=6 GRAPHS=0
for v in NONE NOFORK=1 HLHGAT_DEFER_REDUCE=0 HLHGAT_DEFER_NEI=0 HLHGAT_BN_ONE_LAUNCH=0 HLHGAT_GRAD_SINK=0 HLHGAT_PREPACK=0 HLHGAT_DENSE_SLAB=0; do
  timeout -k 10 120 env "X=$v" "${v/NONE/X=1}" python -u tools/head_graph_diag.py "${KIND:-peptides}" > "gpurun_out/hgd_$v.log" 2>&1 || exit $?
  echo "$v $(grep -o '"eager_distinct": [0-9]*' gpurun_out/hgd_$v.log | tr '\n' ' ')"
done
