#!/bin/bash
# Round-2 PMC set (run under gpurun): the roofline kernels' HBM bytes per launch (two passes over
# tools/roofline_pmc.py run) and the whole step's per-kernel HBM traffic (tools/gpu_pmc.sh).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/rpmc_$C
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/rpmc_$C -o run -- python tools/roofline_pmc.py run \
      > gpurun_out/rpmc_$C.log 2>&1 || { echo "roofline pmc $C failed"; tail -20 gpurun_out/rpmc_$C.log; exit 1; }
  db=$(find gpurun_out/rpmc_$C -name "*.db" | head -1); [ "$db" != "gpurun_out/rpmc_$C/run_results.db" ] && mv "$db" gpurun_out/rpmc_$C/run_results.db
done
python tools/roofline_pmc.py summarize gpurun_out > gpurun_out/r02_roofline_pmc.json || exit 1
ARGS="--no-cpu-baseline --no-targcn --steps 3 --warmup 1" bash tools/gpu_pmc.sh || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  db=$(find gpurun_out/pmc_$C -name "*.db" | head -1); [ "$db" != "gpurun_out/pmc_$C/run_results.db" ] && mv "$db" gpurun_out/pmc_$C/run_results.db
done
python tools/pmc_summary.py gpurun_out > gpurun_out/r02_step_hbm_traffic.txt || exit 1
echo done
