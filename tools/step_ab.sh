#!/bin/bash
# A/B of tools/step_only.py (10 steps) over environment settings, interleaved over ROUNDS rounds:
#   tools/step_ab.sh PREC "CFG1" "CFG2" ...   (CFG: comma-separated VAR=VALUE list, "-" = defaults)
# Each run is its own process under its own time limit; output lines "cfg ms/step" to stdout.
prec=$1
shift
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in "$@"; do
    envs=()
    [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
    out=$(env "${envs[@]}" F3_STEP_PREC=$prec timeout -k 10 120 python tools/step_only.py 10 2>/dev/null)
    rc=$?
    echo "round $r [$cfg] $(echo "$out" | grep ms/step)"
    if [ $rc -ne 0 ]; then echo "stopping: rc=$rc"; exit $rc; fi
  done
done
