#!/bin/bash
# Kernel trace of the step alone + its timeline (per-queue busy time, gaps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/step_only.py 10 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/step -o run -- python tools/step_only.py 8 \
    > gpurun_out/step_prof.log 2>&1 || { tail -20 gpurun_out/step_prof.log; exit 1; }
python tools/timeline.py gpurun_out/step/run_results.db --list > gpurun_out/step_timeline.txt
head -6 gpurun_out/step_timeline.txt
