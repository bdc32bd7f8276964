#!/bin/bash
# Round-4 last check with the final defaults: the whole -m gpu suite, bench, smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
F3_STEP_PREC=bf16x3 bash tools/gpu_session.sh tests bench smoke
