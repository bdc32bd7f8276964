#!/bin/bash
# Window-GEMM probe timings (tools/probe_build.sh N...): tools/kbench.py per probe library, the
# default library first. PROBES: the probe numbers to time (default "8 1 2 4 16").
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/win1_probe.txt
for L in default ${PROBES:-8 1 2 4 16}; do
  if [ "$L" = default ]; then lib=""; else lib="F3_LIB=$PWD/fall_multimodal_amd/libfall3_probe$L.so"; fi
  echo "== probe $L" >> gpurun_out/win1_probe.txt
  env $lib timeout -k 10 120 python tools/kbench.py l8d l8f l5d l7d l1d >> gpurun_out/win1_probe.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/win1_probe.txt
