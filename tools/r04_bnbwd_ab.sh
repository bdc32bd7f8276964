#!/bin/bash
# Round-4 A/B: bn_bwd_apply with its first batch of loads issued before the coefficient prologue
# (F3_BNBWD_HOIST, default 1): parity tests, then the interleaved step A/B (bf16x3, bf16).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bnbwd_fr8.py tests/test_gpu_instep.py -m gpu -x -q \
  -k "golden or benchmarked or fused_train or fr8 or instep or bf16x3" \
  --timeout 240 --timeout-method thread > gpurun_out/bnbwd_tests.log 2>&1 || { tail -40 gpurun_out/bnbwd_tests.log; exit 1; }
tail -2 gpurun_out/bnbwd_tests.log
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_BNBWD_HOIST=0 2>&1 | tee gpurun_out/bnbwd_ab.txt
ROUNDS=2 tools/step_ab.sh bf16 - F3_BNBWD_HOIST=0 2>&1 | tee -a gpurun_out/bnbwd_ab.txt
