#!/bin/bash
# Interleaved A/B of the bf16x3 training step alone (tools/step_only.py, B=256, V=18, S=6) over env
# configs: tools/ab_step.sh CFG... with CFG "-" (defaults) or VAR=VAL[,VAR=VAL...]; ROUNDS (default 3)
# rounds, STEPS (default 20) timed steps each. Each run under its own time limit; stops on a failure.
set -o pipefail
ROUNDS=${ROUNDS:-3}
STEPS=${STEPS:-20}
for r in $(seq "$ROUNDS"); do
  for cfg in "$@"; do
    envs=()
    [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
    out=$(env "${envs[@]}" timeout -k 10 180 python tools/step_only.py "$STEPS" 2>&1) || { echo "failed: $cfg"; echo "$out" | tail -5; exit 1; }
    echo "round $r [$cfg] $(echo "$out" | tail -1)"
  done
done
