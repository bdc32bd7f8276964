#!/bin/bash
# A/B harness for the 3-stream step on the GPU box (run under gpurun). One script, three modes:
#
#   tools/ab.sh env CFG...    eager bench per config, ROUNDS (default 2) interleaved rounds so box
#                             drift hits every config alike; CFG is "-" (defaults) or
#                             VAR=VAL[,VAR=VAL...]. SERIAL_PROF=1 adds a serial-step (F3_SERIAL=1)
#                             kernel profile per config filtered by PAT; PMC=1 adds one FETCH_SIZE and
#                             one WRITE_SIZE pass per config under gpurun_out/ab_<n>/.
#   tools/ab.sh libs A.so B.so [PAT]
#                             two library builds (F3_LIB): serial-step kernel durations matching PAT,
#                             then the eager bench line of each.
#   tools/ab.sh host CFG...   host enqueue cost per runtime env config (tools/host_enqueue.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
mode=$1; shift
ROUNDS=${ROUNDS:-2}
PAT=${PAT:-.}

bench_ms() {  # $1 = output json
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'], 'ms/step', d['value'], 'clips/s')" "$1"
}

serial_prof() {  # $1 tag; rest: env assignments
  local tag=$1; shift
  env "$@" F3_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/ab_$tag -o run -- \
      python bench.py --no-cpu-baseline --no-targcn --steps 5 --warmup 2 > gpurun_out/ab_$tag.log 2>&1 \
      || { echo "serial profile $tag failed"; tail -20 gpurun_out/ab_$tag.log; exit 1; }
  python tools/prof_summary.py /tmp/ab_$tag/run_results.db --top 200 --per-step 7 > gpurun_out/ab_$tag.txt
  echo "== $tag"; grep -E "$PAT" gpurun_out/ab_$tag.txt || true
}

case "$mode" in
  env)
    for r in $(seq "$ROUNDS"); do
      n=0
      for cfg in "$@"; do
        n=$((n + 1)); envs=()
        [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
        env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --no-targcn --steps 30 --warmup 5 \
            > gpurun_out/ab_env.json 2> gpurun_out/ab_env.err || { echo "bench failed: $cfg"; tail -5 gpurun_out/ab_env.err; exit 1; }
        echo "round $r [$cfg] $(bench_ms gpurun_out/ab_env.json)"
        if [ "$r" = 1 ] && [ "$SERIAL_PROF" = 1 ]; then serial_prof "cfg$n" "${envs[@]}"; fi
        if [ "$r" = 1 ] && [ "$PMC" = 1 ]; then
          for C in FETCH_SIZE WRITE_SIZE; do
            env "${envs[@]}" timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/ab_$n/pmc_$C -o run -- \
                python bench.py --no-cpu-baseline --no-targcn --steps 3 --warmup 1 > gpurun_out/ab_$n.$C.log 2>&1 \
                || { echo "pmc failed"; exit 1; }
          done
        fi
      done
    done ;;
  libs)
    [ -n "$3" ] && PAT=$3
    for L in "$1" "$2"; do
      tag=$(basename "$L" .so)
      serial_prof "$tag" F3_LIB=$PWD/$L
      F3_LIB=$PWD/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-targcn > gpurun_out/ab_bench_$tag.json \
          2>/dev/null || { echo "bench $tag failed"; exit 1; }
      echo "$tag $(bench_ms gpurun_out/ab_bench_$tag.json)"
    done ;;
  host)
    for e in "$@"; do
      out=$(env $e timeout -k 10 120 python tools/host_enqueue.py --steps 40) || { echo "$e failed"; exit 1; }
      echo "$e $out"
    done ;;
  *) echo "usage: tools/ab.sh env|libs|host ..."; exit 2 ;;
esac
