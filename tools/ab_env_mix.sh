#!/bin/bash
# A/B of an env knob: serial kernel profile + eager bench per setting
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for G in ${GRIDS:-1024 2048 4096}; do
  F3_MIX_GRID=$G F3_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/abe_$G -o run -- \
      python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/abe_$G.log 2>&1 || { echo fail $G; exit 1; }
  python tools/prof_summary.py /tmp/abe_$G/run_results.db --top 200 --per-step 7 > gpurun_out/abe_$G.txt
  echo "== $G"; grep -E "mix_fwd|total" gpurun_out/abe_$G.txt
  F3_MIX_GRID=$G timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/abe_bench_$G.json 2>/dev/null || { echo bench fail; exit 1; }
  python -c "import json;print('$G', json.load(open('gpurun_out/abe_bench_$G.json'))['ms_per_step'], 'ms/step')"
done
