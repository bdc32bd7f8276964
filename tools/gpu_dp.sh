#!/bin/bash
# DP path on one GPU: two-rank gloo check (first step == RMSprop on mean shard gradient,
# replicas identical), then the bench line (phased-backward cost at N=1). Run under gpurun.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_parity.py -x -v -s --timeout 300 \
  --timeout-method thread -k "dp or replicas or benchmarked or golden" > gpurun_out/dp_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-targcn --no-cpu-baseline \
  > gpurun_out/bench_dp.json 2> gpurun_out/bench_dp.err
