#!/bin/bash
# Round-4 closing session: the whole -m gpu suite at HEAD, bench, the headline roofline trace, smoke;
# then the pw_gemm bf16x3 A/B (tools/r04_pwx3_ab.sh). Every GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
F3_STEP_PREC=bf16x3 ROOF_KEYS="wgrad_l5" bash tools/gpu_session.sh tests bench roof_prof step_prof smoke || exit $?
bash tools/r04_pwx3_ab.sh
