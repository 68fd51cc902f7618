#!/bin/bash
# same-box A/B of the ZINC bench: current train.py vs the previous commit's
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-cfg5 --no-heads > "gpurun_out/ab_$1.log" 2>&1 || exit $?;
        echo "$1 $(grep -o '"value": [0-9.]*, "unit": "graphs/s", "n_gpus": 1, "steps": 20, "warmup": 6, "ms_per_step": [0-9.]*' gpurun_out/ab_$1.log)"; }
run cur1; cp tools/ab/train_prev.py hl-hgat_amd/hlhgat/train.py; run prev1
run prev2
