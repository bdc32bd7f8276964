#!/bin/bash
# Round-4 A/B: the first block's gcn on layer0.hip's fp32 kernels in the bf16x3 mode (F3_GCN0_X3):
# the bf16x3 / step parity tests with it on (the default), then the interleaved step A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instep.py tests/test_gpu_bnbwd_fr8.py -m gpu -x -q \
  -k "bf16x3 or benchmarked or fused_train or rmsprop or instep or fr8 or golden" \
  --timeout 240 --timeout-method thread > gpurun_out/gcn0_tests.log 2>&1 || { tail -40 gpurun_out/gcn0_tests.log; exit 1; }
tail -2 gpurun_out/gcn0_tests.log
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_GCN0_X3=0 2>&1 | tee gpurun_out/gcn0_ab.txt
