#!/bin/bash
# Round-4 last knob A/B at the final defaults (bf16x3 step, 4 interleaved rounds)
set -o pipefail
mkdir -p gpurun_out
ROUNDS=4 tools/step_ab.sh bf16x3 - F3_WG_NTW=3 F3_WG_NTW=7 F3_SIDE_FRAC=60 F3_CA_B3=1 2>&1 | tee gpurun_out/last_ab.txt
