#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/probes/infer_probe.py > gpurun_out/ip.log 2>&1
rc=$?; echo "=== infer probe rc=$rc"; grep -v amdgpu.ids gpurun_out/ip.log | tail -4 | cut -c1-300
run_rc() {
  env MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 1000)) RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 "$@" > gpurun_out/rc_$i.log 2>&1
  rc=$?; echo "=== rccl $i [$*] rc=$rc"; grep -v "amdgpu.ids\|socket.cpp\|\[child\]" gpurun_out/rc_$i.log | grep "^{\|rror" | head -3 | cut -c1-600
}
i=1; run_rc timeout -k 10 200 python tests/test_rccl_capture.py cifar_global_max
i=2; run_rc TORCH_NCCL_CUDA_EVENT_CACHE=0 timeout -k 10 200 python tests/test_rccl_capture.py zinc_sync_bn
timeout -k 10 400 python tools/ab_step.py base nolanes base2 nolanes2 --rounds 6 > gpurun_out/ab.log 2>&1
rc=$?; echo "=== ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | tail -8
exit 0
