#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one each, own time limit) over bench.py's roofline kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/rpmc_$C -o run -- python tools/roofline_pmc.py run \
      > gpurun_out/rpmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -20 gpurun_out/rpmc_$C.log; exit 1; }
done
echo "roofline pmc done"
