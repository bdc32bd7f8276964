#!/bin/bash
# Eager-step A/B of env knobs: each config ("-" = defaults, else VAR=VAL[,VAR=VAL]) benched
# ROUNDS times, interleaved, so box drift hits every config alike.
#   tools/ab_env_bench.sh - F3_IGEMM_STAGES=3 F3_IGEMM_WIN=0
set -o pipefail
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
for r in $(seq "$ROUNDS"); do
  for cfg in "$@"; do
    envs=()
    [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 \
        > gpurun_out/abenv.json 2> gpurun_out/abenv.err || { echo "bench failed: $cfg"; tail -5 gpurun_out/abenv.err; exit 1; }
    python -c "import json,sys;print(sys.argv[1], json.load(open('gpurun_out/abenv.json'))['ms_per_step'], 'ms/step')" "$cfg"
  done
done
