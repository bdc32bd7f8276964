#!/bin/bash
# musa_model GPU loop: bench line (+ depthwise conv roofline) and a rocprof kernel trace (run under gpurun).
set -o pipefail
mkdir -p gpurun_out/prof_musa
timeout -k 10 300 python -u bench.py --model musa --steps 10 --warmup 3 > gpurun_out/musa_bench.json \
  2> gpurun_out/musa_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_musa/*
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_musa -o run -- \
  python -u bench.py --model musa --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_musa/log.txt 2>&1
