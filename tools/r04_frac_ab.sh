#!/bin/bash
# Round-4 A/B: which layers' side-queue weight gradients get split for part of the chip, and how
# large a part (F3_SIDE_FRAC / F3_SIDE_FRAC_FROM; default 75 from layer 2), + side priority
set -o pipefail
mkdir -p gpurun_out
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_SIDE_FRAC_FROM=1 F3_SIDE_FRAC_FROM=0 F3_SIDE_FRAC=60 F3_SIDE_FRAC=90 \
  F3_SIDE_PRIO=1 F3_SIDE_FRAC=0 2>&1 | tee gpurun_out/frac_ab.txt
