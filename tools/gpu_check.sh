#!/bin/bash
# One GPU-box pass: parity tests, the bench line, a rocprofv3 kernel-trace summary of the
# same bench command, and one of the roofline kernels launched alone (tools/roofline_pmc.py run). Every GPU step has its own time limit; the chain stops at the first
# failure. Outputs land in gpurun_out/ (merged back by gpurun).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MARK="gpu"
[ "$1" = "--fast" ] && MARK="gpu and not slow"
timeout -k 10 600 python -u -m pytest tests -m "$MARK" -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1 \
    || { echo "rocprof failed"; tail -30 gpurun_out/prof.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_roof -o run -- \
    python tools/roofline_pmc.py run > gpurun_out/prof_roof.log 2>&1 \
    || { echo "rocprof (roofline kernels) failed"; tail -30 gpurun_out/prof_roof.log; exit 1; }
echo "all done"
