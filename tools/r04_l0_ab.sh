#!/bin/bash
# Round-4 tail A/B: bf16x3 parity tests with the layer-0 fp32 / 128-channel window options on,
# then interleaved step A/B (tools/step_ab.sh) of the options and the side-queue ordering knobs.
set -o pipefail
mkdir -p gpurun_out
F3_X3_L0_FP32=1 F3_WIN128_FWD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k bf16x3 \
  -x -q --timeout 240 --timeout-method thread > gpurun_out/l0_tests.log 2>&1 || { tail -30 gpurun_out/l0_tests.log; exit 1; }
tail -2 gpurun_out/l0_tests.log
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_X3_L0_FP32=1 F3_WIN128_FWD=1 F3_X3_L0_FP32=1,F3_WIN128_FWD=1 \
  F3_SIDE_EARLY=2 F3_SIDE_PRIO=1 2>&1 | tee gpurun_out/l0_ab.txt
