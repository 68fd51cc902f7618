set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "bn_fold" -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t23.log 2>&1
timeout -k 10 300 python tools/ab_step.py base nofold base2 nofold2 --rounds 8 > gpurun_out/ab23.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/suite23.log 2>&1
