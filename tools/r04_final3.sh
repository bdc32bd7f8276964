#!/bin/bash
# Round-4 final confirmation with the last default (128-channel tap groups): conv / step parity
# tests, bench, smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
PYTEST_K="conv or x3cat or bf16x3 or benchmarked or instep or golden or fused_train" F3_STEP_PREC=bf16x3 \
  bash tools/gpu_session.sh tests bench smoke
