#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "
import sys, ctypes; sys.path[:0]=['.','hl-hgat_amd']
import torch; torch.zeros(1, device='cuda')
from hlhgat import _lib
c = ctypes.c_int64(0); _lib.LIB.hlhgat_proj_bn_fused_capacity(ctypes.byref(c)); print('proj_bn cap (share 2):', c.value)
" 2>&1 | grep cap
HLHGAT_BN_COLOCATE=3 timeout -k 10 700 python bench.py --no-cfg5 --no-cpu-baseline > gpurun_out/r04_r_bench.json 2> gpurun_out/r04_r_bench.err
echo "=== bench colocate3 rc=$?"; grep -n "FAILED\|re-run\|heads\]" gpurun_out/r04_r_bench.err | head
python - <<'PY'
import json
r=json.loads(open('gpurun_out/r04_r_bench.json').read().strip().splitlines()[-1])
print(r['value'], r['ms_per_step'], r['step_census']['dispatches_per_step'], r['heads'].get('bn_one_launch'))
PY
exit 0
