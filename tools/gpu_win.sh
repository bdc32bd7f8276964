#!/bin/bash
# Clip-window igemm_big (F3_BIG_WIN): kernel parity (conv fwd / input-gradient shapes incl. the
# 256-channel T=8 ones), the benchmarked-config and top-1 parity tests, then the eager bench line
# with the window form off and on (the tcn forward roofline launch and the step time).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
F3_BIG_WIN=1 F3_BIG_ASM=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread \
    -k "conv or benchmarked_config or cfg3 or bf16_step or fused_train_step or poison" \
    > gpurun_out/win_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/win_tests.log; exit 1; }
tail -3 gpurun_out/win_tests.log
for r in $(seq ${ROUNDS:-2}); do
  for cfg in "F3_BIG_WIN=0 F3_BIG_ASM=0" "F3_BIG_WIN=1 F3_BIG_ASM=0" "F3_BIG_WIN=1 F3_BIG_ASM=1"; do
    tag=$(echo $cfg | tr -dc '0-9')
    env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --no-targcn > gpurun_out/win_bench_$tag.json \
        2> gpurun_out/win_bench_$tag.err || { echo "bench $cfg failed"; tail -20 gpurun_out/win_bench_$tag.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print('$cfg', d['ms_per_step'], 'ms/step', d['value'], 'clips/s', 'tcn_fwd', d['roofline_tcn_fwd']['ms_per_launch'], d['roofline_tcn_fwd']['frac'])" gpurun_out/win_bench_$tag.json
  done
done
F3_BIG_WIN=1 F3_BIG_ASM=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_win -o run -- \
    python tools/roofline_pmc.py run > gpurun_out/prof_win.log 2>&1 \
    || { echo "rocprof (roofline kernels) failed"; tail -30 gpurun_out/prof_win.log; exit 1; }
echo "all done"
