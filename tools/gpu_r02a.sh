#!/bin/bash
# Round-2 GPU pass: full parity suite, bench line (with the config-2 TARGCN object), rocprofv3
# kernel summary of the TARGCN step. Each GPU step has its own time limit; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread -s \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tg -o run -- \
    python bench.py --model targcn --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tg.log 2>&1 \
    || { echo "rocprof targcn failed"; tail -30 gpurun_out/prof_tg.log; exit 1; }
echo "all done"
