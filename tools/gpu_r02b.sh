#!/bin/bash
# Round-2 re-entry pass: the full GPU check (tests, bench, rocprof), then the wgrad_taps
# measurement knobs (F3_TAPS_DBG 0/1/2) and two SQ counter passes over the roofline kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh || exit 1
for d in 0 1 2; do
  F3_TAPS_DBG=$d timeout -k 10 120 python tools/wgrad_ab.py >> gpurun_out/taps_dbg.txt 2>&1 || { echo "wgrad_ab $d failed"; exit 1; }
done
cat gpurun_out/taps_dbg.txt
bash tools/wgrad_pmc.sh || exit 1
COUNTERS="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
  bash tools/wgrad_pmc.sh || exit 1
echo "all done"
