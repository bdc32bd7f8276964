#!/bin/bash
# wgrad kernel A/B on the box: the conv-backward parity tests, the isolated layer-6 wgrad
# launch under each setting of F3_WGRAD_BIG, then the whole step interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "conv_backward" -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/wgrad_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/wgrad_tests.log; exit 1; }
tail -2 gpurun_out/wgrad_tests.log
for v in ${VALS:-0 1}; do
  F3_WGRAD_BIG=$v timeout -k 10 120 python tools/roofline_pmc.py run || { echo "roofline run failed"; exit 1; }
done
bash tools/ab_env.sh F3_WGRAD_BIG "${VALS:-0 1}" ${ROUNDS:-2}
