#!/bin/bash
# A/B of two library builds (F3_LIB): serial-step kernel durations (F3_SERIAL=1, no cross-stream
# contention) and the eager bench line for each. Usage: tools/ab_serial.sh A.so B.so [kernel-regex]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PAT=${3:-.}
for L in "$1" "$2"; do
  tag=$(basename "$L" .so)
  F3_LIB=$PWD/$L F3_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/ab_$tag -o run -- \
      python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/ab_$tag.log 2>&1 \
      || { echo "serial profile $tag failed"; tail -20 gpurun_out/ab_$tag.log; exit 1; }
  python tools/prof_summary.py /tmp/ab_$tag/run_results.db --top 200 --per-step 7 > gpurun_out/ab_$tag.txt
  echo "== $tag"; grep -E "$PAT" gpurun_out/ab_$tag.txt || true
  F3_LIB=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_bench_$tag.json 2>/dev/null \
      || { echo "bench $tag failed"; exit 1; }
  python -c "import json;print('$tag', json.load(open('gpurun_out/ab_bench_$tag.json'))['ms_per_step'], 'ms/step')"
done
