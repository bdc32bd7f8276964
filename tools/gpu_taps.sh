#!/bin/bash
# wgrad_taps A/B pass: numerics + timing of the layer-6 weight gradient (and the measurement
# knobs), then the step-level parity tests that run it, then the bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/taps_ab.txt
for d in 0 1 2; do
  F3_TAPS_DBG=$d timeout -k 10 120 python tools/wgrad_ab.py >> gpurun_out/taps_ab.txt 2>&1 || { echo "wgrad_ab $d failed"; cat gpurun_out/taps_ab.txt; exit 1; }
done
cat gpurun_out/taps_ab.txt
grep -q "dW rel err [0-9.]*e-0[5-9]" <(head -2 gpurun_out/taps_ab.txt) || { echo "numerics off"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "conv_backward or benchmarked or top1 or train_step_matches" > gpurun_out/taps_tests.log 2>&1 \
    || { echo "tests failed"; tail -40 gpurun_out/taps_tests.log; exit 1; }
tail -3 gpurun_out/taps_tests.log
grep "held-out" gpurun_out/taps_tests.log || true
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_taps.json 2> gpurun_out/bench_taps.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench_taps.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_taps.json')); print(d['value'], d['ms_per_step'], d['roofline'], d['roofline_wgrad_kernel']['ms_per_launch'])"
bash tools/wgrad_pmc.sh > /dev/null || exit 1
cat gpurun_out/wpmc.txt
echo "all done"
