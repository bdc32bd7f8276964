#!/bin/bash
# Round-4 A/B: channel-attention backward pass 3 with one clip per workgroup (F3_CA_B3=1), parity
# tests with it on, then the interleaved step A/B (bf16x3 and bf16).
set -o pipefail
mkdir -p gpurun_out
F3_CA_B3=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "golden or benchmarked or fused_train" \
  --timeout 240 --timeout-method thread > gpurun_out/ca_tests.log 2>&1 || { tail -40 gpurun_out/ca_tests.log; exit 1; }
tail -2 gpurun_out/ca_tests.log
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_CA_B3=1 2>&1 | tee gpurun_out/ca_ab.txt
ROUNDS=2 tools/step_ab.sh bf16 - F3_CA_B3=1 2>&1 | tee -a gpurun_out/ca_ab.txt
