#!/bin/bash
# igemm_big with the weight fragments loaded straight to registers (F3_BIG_BDIRECT=1): conv
# kernel parity, the layer-6 tcn forward time both ways, then the eager step A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F3_BIG_BDIRECT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "conv_kernel or conv_backward" > gpurun_out/bd_tests.log 2>&1 \
    || { echo "bd tests failed"; tail -30 gpurun_out/bd_tests.log; exit 1; }
tail -2 gpurun_out/bd_tests.log
for bd in 0 1 0 1; do
  F3_BIG_BDIRECT=$bd timeout -k 10 120 python -c "
import torch, bench
r = bench.roofline_kernels(torch.device('cuda'), 256, 18, 'bf16')
print('BDIRECT=$bd tcn_fwd', r['tcn_fwd']['ms_per_launch'], r['tcn_fwd']['frac'])" 2>/dev/null || exit 1
done
ROUNDS=2 bash tools/ab.sh env - F3_BIG_BDIRECT=1 || exit 1
