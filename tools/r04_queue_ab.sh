#!/bin/bash
# Round-4 tail A/B: hardware-queue count and side-queue submission order (tools/step_ab.sh)
set -o pipefail
mkdir -p gpurun_out
ROUNDS=3 tools/step_ab.sh bf16x3 - F3_WIN128_FWD=1 GPU_MAX_HW_QUEUES=8 F3_SIDE_LAG=0 \
  GPU_MAX_HW_QUEUES=8,F3_SIDE_LAG=0 2>&1 | tee gpurun_out/queue_ab.txt
