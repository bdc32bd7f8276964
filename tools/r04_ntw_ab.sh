#!/bin/bash
# Round-4 wgrad tap-group A/B (F3_WG_NTW): parity under the tap groups and the side-queue split
# share (F3_SIDE_FRAC), the layer-5 roofline launch per setting, then the interleaved step A/B
# (+ side-queue priority).
set -o pipefail
mkdir -p gpurun_out
F3_WG_NTW=7 F3_SIDE_FRAC=50 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_instep.py -m gpu -x -q \
  -k "conv_backward or x3cat or benchmarked or train_step_matches or fused_train or bf16_step or instep" \
  --timeout 240 --timeout-method thread > gpurun_out/ntw_tests.log 2>&1 || { tail -40 gpurun_out/ntw_tests.log; exit 1; }
tail -2 gpurun_out/ntw_tests.log
for v in 0 1; do
  F3_WG_NTW=$v timeout -k 10 120 python tools/roofline_pmc.py run wgrad_l5 2>&1 | tail -1 | sed "s/^/NTW=$v /" | tee -a gpurun_out/ntw_roof.txt
done
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_WG_NTW=1 F3_WG_NTW=2 F3_WG_NTW=4 F3_WG_NTW=7 F3_SIDE_FRAC=50 F3_SIDE_FRAC=75 \
  F3_WG_NTW=7,F3_SIDE_FRAC=50 F3_SIDE_PRIO=2 2>&1 | tee gpurun_out/ntw_ab.txt
