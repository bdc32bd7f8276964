#!/bin/bash
# Kernel durations without cross-stream contention: the step with every branch on one stream
# (F3_SERIAL=1) under rocprofv3 --kernel-trace; per-kernel summary into gpurun_out/serial.txt.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F3_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/ser -o run -- \
    python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/serial.log 2>&1 \
    || { echo "serial profile failed"; tail -20 gpurun_out/serial.log; exit 1; }
grep -h '^{' gpurun_out/serial.log | python -c "import json,sys; print('serial ms/step', json.loads(sys.stdin.readline())['ms_per_step'])"
python tools/timeline.py /tmp/ser/run_results.db | head -3
python tools/prof_summary.py /tmp/ser/run_results.db --top ${TOP:-40} --per-step 7 > gpurun_out/serial.txt
cat gpurun_out/serial.txt
