#!/bin/bash
# HBM traffic per kernel: two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over a short
# bench run, each in its own run and time limit (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE do not fit one pass; on gfx950 FETCH_SIZE reads 1/2 of wide streaming reads).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${ARGS:-"--no-cpu-baseline --steps 3 --warmup 1"}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_$C -o run -- python bench.py $ARGS \
      > gpurun_out/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -20 gpurun_out/pmc_$C.log; exit 1; }
done
echo "pmc done"
