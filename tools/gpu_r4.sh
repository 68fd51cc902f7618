#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_c_pipe2
export TMPDIR=/tmp
export DEBUG_HIP_FORCE_GRAPH_QUEUES=2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipeline.py tests/test_gpu_parity.py -k "pipeline or lanczos or hodge_builder or mlgc" > gpurun_out/r04_c_pipe_tests.log 2>&1
rc=$?; echo "=== tests rc=$rc"; tail -3 gpurun_out/r04_c_pipe_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/probes/pipeline_stages.py --batches 4 > gpurun_out/r04_c_pipe.log 2>&1
echo "=== stages rc=$?"; tail -1 gpurun_out/r04_c_pipe.log
timeout -k 10 300 python tools/probes/cfg3_pipe.py > gpurun_out/r04_c_cfg3.log 2>&1
echo "=== cfg3 rc=$?"; tail -1 gpurun_out/r04_c_cfg3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_c_pipe2 -o run -- python tools/probes/pipeline_stages.py --batches 4 > gpurun_out/r04_c_pipe_prof.log 2>&1
echo "=== prof rc=$?"
exit 0
