#!/bin/bash
# Round-4 closing session on one MI355X (through gpurun; every GPU step under its own time limit,
# the session stops at a fault / abort / time limit): the whole -m gpu suite, bench, the headline
# roofline kernel trace + PMC passes, the step's kernel trace / timeline and PMC bytes, smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
F3_STEP_PREC=bf16x3 ROOF_KEYS="wgrad_l5 wgrad tcn_fwd" bash tools/gpu_session.sh tests bench roof_prof roof_pmc step_prof step_pmc smoke
