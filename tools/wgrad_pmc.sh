#!/bin/bash
# SQ counters of the roofline kernels launched alone (tools/roofline_pmc.py run), one pass.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${COUNTERS:-"SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"}
timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d /tmp/wpmc -o run -- python tools/roofline_pmc.py run \
    > gpurun_out/wpmc.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/wpmc.log; exit 1; }
python tools/pmc_kernels.py /tmp/wpmc/run_results.db wgrad igemm_big | tee gpurun_out/wpmc.txt
