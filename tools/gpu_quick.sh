#!/bin/bash
# Full GPU test suite, then the bench line (no CPU baseline). Each step time-limited.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench_q.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['main_py_autograd_path'])"
