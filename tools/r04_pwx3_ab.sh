#!/bin/bash
# Round-4 A/B: the bf16x3 mode's K-concatenated 1x1 GEMMs (gcn input gradients, residual forwards)
# on the weight-stationary pw_gemm (F3_PW_X3=1): parity tests with it on, then the step A/B.
set -o pipefail
mkdir -p gpurun_out
F3_PW_X3=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instep.py -m gpu -x -q \
  -k "x3cat or bf16x3 or benchmarked or instep" \
  --timeout 240 --timeout-method thread > gpurun_out/pwx3_tests.log 2>&1 || { tail -40 gpurun_out/pwx3_tests.log; exit 1; }
tail -2 gpurun_out/pwx3_tests.log
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_PW_X3=1 2>&1 | tee gpurun_out/pwx3_ab.txt
