#!/bin/bash
# The round's final measurement session on one MI355X (run through gpurun; every GPU step under
# its own time limit, the session stops at a fault / abort / time limit):
#   bench + the roofline kernel traces and PMC passes + the step's PMC bytes and concurrent
#   timeline + the RGB kernels' PMC bytes + smoke; then the musa depthwise-conv store A/B
#   (F3_DW_STORE=1 after its GPU tests pass)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
F3_STEP_PREC=bf16x3 bash tools/gpu_session.sh bench roof_prof roof_pmc step_pmc step_prof rgb_pmc smoke
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 env F3_DW_STORE=1 python -u -m pytest tests/test_musa_gpu.py -q -m gpu --timeout 240 \
  --timeout-method thread > gpurun_out/musa_dwstore_tests.log 2>&1
rc=$?
tail -3 gpurun_out/musa_dwstore_tests.log
[ $rc -le 1 ] || exit $rc
for e in F3_DW_STORE=0 F3_DW_STORE=1; do
  timeout -k 10 300 env $e python bench.py --model musa --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/musa_$e.json 2>> gpurun_out/musa_ab.err || exit $?
  cut -c1-300 gpurun_out/musa_$e.json
done
