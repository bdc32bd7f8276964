#!/bin/bash
# SkeletonTransformer GPU loop: parity tests, bench line, rocprof kernel trace (run under gpurun).
set -o pipefail
mkdir -p gpurun_out/prof_sktr
timeout -k 10 600 python -u -m pytest tests/test_sktr_gpu.py -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/sktr_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --model sktr --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/sktr_bench.json 2> gpurun_out/sktr_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_sktr/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sktr -o run -- \
  python -u bench.py --model sktr --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_sktr/log.txt 2>&1
