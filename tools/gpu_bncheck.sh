#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_train_step.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "norm or bn or model or train or step" > gpurun_out/bnc_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/bnc_pytest.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/bnc_pytest.log; exit $rc; }
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-cfg5 --steps 30 > gpurun_out/bnc_bench.log 2>&1 || { tail -20 gpurun_out/bnc_bench.log; exit 1; }; grep -o '"value": [0-9.]*' gpurun_out/bnc_bench.log | head -1; done
rm -rf gpurun_out/prof_bnc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bnc -o run --output-format csv -- python3 bench.py --steps 20 --warmup 6 --no-cpu-baseline --no-cfg5 > gpurun_out/prof_bnc.log 2>&1 || { tail -20 gpurun_out/prof_bnc.log; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/prof_bnc -name "run_kernel_stats.csv") gpurun_out/prof_bnc.md "bench kernel stats"
head -16 gpurun_out/prof_bnc.md
