#!/bin/bash
# Round-4 A/B: 4-stage rings for wgrad_big (F3_WG_NST4): parity under them, the layer-5 roofline
# launch per setting, then the interleaved step A/B.
set -o pipefail
mkdir -p gpurun_out
F3_WG_NST4=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "conv_backward or x3cat or benchmarked" \
  --timeout 240 --timeout-method thread > gpurun_out/nst_tests.log 2>&1 || { tail -40 gpurun_out/nst_tests.log; exit 1; }
tail -2 gpurun_out/nst_tests.log
for v in 0 1 0 1; do
  F3_WG_NST4=$v timeout -k 10 120 python tools/roofline_pmc.py run wgrad_l5 2>&1 | tail -1 | sed "s/^/NST4=$v /" | tee -a gpurun_out/nst_roof.txt
done
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_WG_NST4=1 F3_WG_NST4=2 F3_WG_NST4=3 2>&1 | tee gpurun_out/nst_ab.txt
