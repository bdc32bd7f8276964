#!/bin/bash
# TARGCN: parity tests, then the config-2 bench line and a rocprofv3 kernel summary of it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_targcn_gpu.py -x -v -s --timeout 240 --timeout-method thread \
    > gpurun_out/tg_tests.log 2>&1 || { echo "tg tests failed"; tail -40 gpurun_out/tg_tests.log; exit 1; }
grep -E "TARGCN|v1[47]:" gpurun_out/tg_tests.log; tail -1 gpurun_out/tg_tests.log
timeout -k 10 200 python bench.py --model targcn --steps 10 --warmup 3 > gpurun_out/tg_bench.json 2> gpurun_out/tg_bench.err \
    || { echo "bench failed"; tail -30 gpurun_out/tg_bench.err; exit 1; }
cat gpurun_out/tg_bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tg -o run -- \
    python bench.py --model targcn --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_tg.log 2>&1 \
    || { echo "rocprof targcn failed"; tail -30 gpurun_out/prof_tg.log; exit 1; }
echo "all done"
