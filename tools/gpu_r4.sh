#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04_u_pytest.log 2>&1
echo "=== pytest rc=$?"; tail -2 gpurun_out/r04_u_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_u_smoke.log 2>&1
echo "=== smoke rc=$?"; tail -1 gpurun_out/r04_u_smoke.log
exit 0
