#!/bin/bash
# A/B of two library builds on the step and the tcn-forward roofline launch (F3_LIB), after the
# window-form parity tests of the build under test.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread \
    -k "conv or benchmarked_config or cfg3 or bf16_step or fused_train_step or poison" \
    > gpurun_out/nst_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/nst_tests.log; exit 1; }
tail -2 gpurun_out/nst_tests.log
for r in 1 2; do
  for lib in "$1" fall_multimodal_amd/libfall3.so; do
    tag=$(basename $lib .so)
    F3_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-targcn > gpurun_out/nst_$tag.json \
        2> gpurun_out/nst_$tag.err || { echo "bench $lib failed"; tail -20 gpurun_out/nst_$tag.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print('$tag', d['ms_per_step'], 'ms/step', d['value'], 'clips/s', 'tcn_fwd', d['roofline_tcn_fwd']['ms_per_launch'], d['roofline_tcn_fwd']['frac'])" gpurun_out/nst_$tag.json
  done
done
echo "all done"
