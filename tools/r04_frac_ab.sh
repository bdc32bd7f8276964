#!/bin/bash
# Round-4 A/B: share of the chip the side-queue weight gradients are split for (F3_WGRAD_FRAC),
# with and without the tap groups (F3_WG_NTW)
set -o pipefail
mkdir -p gpurun_out
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_WGRAD_FRAC=50 F3_WGRAD_FRAC=75 "${NTW_BEST:-F3_WG_NTW=7}" \
  "${NTW_BEST:-F3_WG_NTW=7},F3_WGRAD_FRAC=50" "${NTW_BEST:-F3_WG_NTW=7},F3_WGRAD_FRAC=75" 2>&1 | tee gpurun_out/frac_ab.txt
