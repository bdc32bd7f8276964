#!/bin/bash
# A/B an environment toggle on the full bench step, interleaved rounds in one box call:
#   bash tools/ab_env.sh VAR "0 1" [rounds]
# prints ms_per_step per (round, value); with PMC=1 also one FETCH/WRITE pass per value
# into gpurun_out/ab_<value>/.
set -o pipefail
VAR=$1; VALS=$2; R=${3:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for v in $VALS; do
    out=$(env $VAR=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 --warmup 5) || { echo "bench failed"; exit 1; }
    echo "round $r $VAR=$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", d["value"], "clips/s")')"
  done
done
if [ "$PMC" = "1" ]; then
  for v in $VALS; do
    for C in FETCH_SIZE WRITE_SIZE; do
      env $VAR=$v timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/ab_$v/pmc_$C -o run -- \
          python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_$v.$C.log 2>&1 \
          || { echo "pmc failed"; exit 1; }
    done
  done
fi
echo done
