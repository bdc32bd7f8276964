#!/bin/bash
# One GPU-box session: runs the named steps in order, each under its own time limit, output under
# gpurun_out/. A step that FAILS (exit 1: a test or check failed) does not stop the session; a
# step that faults, aborts or hits its limit (exit >= 124, 134, 139) ends it at once.
#   tools/gpu_session.sh tests step_prof bench [pytest args for "tests" via PYTEST_ARGS]
# Steps:
#   tests       pytest -m gpu over ${TESTS:-tests} (+ PYTEST_ARGS; PYTEST_K: a -k expression) -> gpurun_out/gpu_tests.log
#   step_time   tools/step_only.py 10 for each precision in ${PRECS:-bf16}   -> gpurun_out/step_time.log
#   step_prof   rocprofv3 kernel trace + stats of the bench step alone  -> gpurun_out/step_kernels.txt
#   step_prof_ag  the same for the reference loop body through the custom ops -> gpurun_out/step_ag_*.txt
#   step_prof_serial  the bench step with every queue joined (F3_SERIAL=1): per-kernel alone times
#                     -> gpurun_out/step_serial_kernels.txt
#   kbench      tools/kbench.py over ${KB_KEYS} (tcn GEMMs alone)       -> gpurun_out/kbench.txt
#   kpmc        SQ / LDS / MFMA counter passes of the same               -> gpurun_out/kpmc.txt
#   step_pmc    FETCH_SIZE / WRITE_SIZE passes of the step alone        -> gpurun_out/step_hbm_traffic.txt
#   roof_prof   rocprofv3 kernel trace of bench.py's roofline launches, one process per key in
#               ${ROOF_KEYS:-wgrad_l1 dgrad_l8 wgrad_l5 wgrad wgrad_kernel tcn_fwd gcn_l5 gcn_l6}          -> gpurun_out/roof_kernels_KEY.txt
#   roof_pmc    FETCH_SIZE / WRITE_SIZE passes of the same, per key     -> gpurun_out/roofline_pmc.json
#   rgb_pmc     FETCH_SIZE / WRITE_SIZE passes of the RGB branch kernels -> gpurun_out/rgb_pmc.json
#   bench       bench.py (default run, 20 steps)                        -> gpurun_out/bench.json
#   bench_fp32  bench.py --precision fp32 --no-targcn                   -> gpurun_out/bench_fp32.json
#   ab          tools/ab.sh env $AB_CFGS (eager bench A/B, optional serial profiles) -> gpurun_out/ab.log
#   bench_tg    bench.py --model targcn per TG_CFGS config                -> gpurun_out/bench_tg_*.json
#   smoke       __graft_entry__.smoke()
#   exit_prof   tools/exit_check.py under rocprofv3 --kernel-trace (exit status after finalisation) -> gpurun_out/exit_prof.log
#   py:<file>   python <file> (a tool script)                           -> gpurun_out/<name>.log
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# raw rocprofv3 databases stay on the box (gpurun copies back at most 64 MiB of gpurun_out/); only the
# summaries made from them go to gpurun_out/
export PROF_DIR=${PROF_DIR:-/tmp/f3prof}
P=$PROF_DIR
mkdir -p "$P"
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
rc_all=0
run() {  # name limit cmd...
  local name=$1 lim=$2
  shift 2
  echo "== $name ($(date +%T))" >&2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "== $name rc=$rc ($(date +%T))" >&2
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "== stopping: $name ended with $rc"
    exit $rc
  fi
  [ $rc -ne 0 ] && rc_all=1
  return 0
}
for step in "$@"; do
  case $step in
    tests)
      if [ -n "${PYTEST_K:-}" ]; then
        run tests 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -s --timeout 300 --timeout-method thread \
          -k "$PYTEST_K" ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
      else
        run tests 900 python -u -m pytest ${TESTS:-tests} -m gpu -q --timeout 300 --timeout-method thread \
          ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
      fi
      tail -5 gpurun_out/gpu_tests.log ;;
    step_prof)
      run step_prof 300 rocprofv3 --kernel-trace --stats -d $P/step -o run -- \
        python tools/step_only.py 8 > gpurun_out/step_prof.log 2>&1
      python tools/prof_summary.py $P/step/run_results.db --per-step 11 --top 60 \
        > gpurun_out/step_kernels.txt 2>&1
      python tools/timeline.py $P/step/run_results.db --list > gpurun_out/step_timeline.txt 2>&1
      head -25 gpurun_out/step_kernels.txt ;;
    step_time)
      for pr in ${PRECS:-bf16}; do
        echo "precision $pr" >> gpurun_out/step_time.log
        run "step_time[$pr]" 300 env F3_STEP_PREC=$pr python tools/step_only.py 10 >> gpurun_out/step_time.log 2>&1
      done
      cat gpurun_out/step_time.log ;;
    step_prof_ag)
      run step_prof_ag 300 rocprofv3 --kernel-trace --stats -d $P/step_ag -o run -- \
        python tools/step_only.py 8 autograd > gpurun_out/step_prof_ag.log 2>&1
      python tools/prof_summary.py $P/step_ag/run_results.db --per-step 11 --top 60 \
        > gpurun_out/step_ag_kernels.txt 2>&1
      python tools/timeline.py $P/step_ag/run_results.db --list > gpurun_out/step_ag_timeline.txt 2>&1
      head -25 gpurun_out/step_ag_kernels.txt ;;
    step_prof_serial)
      export F3_SERIAL=1
      run step_prof_serial 300 rocprofv3 --kernel-trace --stats -d $P/step_serial -o run -- \
        python tools/step_only.py 8 > gpurun_out/step_prof_serial.log 2>&1
      unset F3_SERIAL
      python tools/prof_summary.py $P/step_serial/run_results.db --per-step 11 --top 80 \
        > gpurun_out/step_serial_kernels.txt 2>&1
      head -25 gpurun_out/step_serial_kernels.txt ;;
    kbench)
      run kbench 120 python tools/kbench.py ${KB_KEYS:-l1f l1d l4f l4d l5f l5d l7f l7d l8f l8d} > gpurun_out/kbench.txt 2>&1
      cat gpurun_out/kbench.txt ;;
    kpmc)
      # SQ stall / LDS / MFMA counters of tools/kbench.py's kernels, one pass per set
      i=0
      for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVES SQ_INST_CYCLES_VMEM" \
                 "FETCH_SIZE"; do
        i=$((i + 1))
        rm -rf $P/kpmc_$i
        run kpmc_$i 90 rocprofv3 --pmc $SET -d $P/kpmc_$i -o run -- python tools/kbench.py \
          ${KB_KEYS:-l1f l1d l4f l4d l5f l5d l7f l7d l8f l8d} > gpurun_out/kpmc_$i.log 2>&1
        db=$(find $P/kpmc_$i -name "*.db" | head -1)
        python tools/pmc_kernels.py "$db" >> gpurun_out/kpmc.txt 2>&1
      done
      tail -40 gpurun_out/kpmc.txt ;;
    step_pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        rm -rf $P/pmc_$C
        run pmc_$C 120 rocprofv3 --pmc $C -d $P/pmc_$C -o run -- python tools/step_only.py 2 \
          > gpurun_out/step_pmc_$C.log 2>&1
        db=$(find $P/pmc_$C -name "*.db" | head -1)
        [ -n "$db" ] && [ "$db" != "$P/pmc_$C/run_results.db" ] && mv "$db" $P/pmc_$C/run_results.db
      done
      python tools/pmc_summary.py $P --top 60 > gpurun_out/step_hbm_traffic.txt 2>&1
      head -30 gpurun_out/step_hbm_traffic.txt ;;
    roof_prof)
      for K in ${ROOF_KEYS:-wgrad_l1 dgrad_l8 wgrad_l5 wgrad wgrad_kernel tcn_fwd gcn_l5 gcn_l6}; do
        run roof_prof_$K 300 rocprofv3 --kernel-trace --stats -d $P/roof_$K -o run -- \
          python tools/roofline_pmc.py run $K > gpurun_out/roof_prof_$K.log 2>&1
        python tools/prof_summary.py $P/roof_$K/run_results.db --top 30 > gpurun_out/roof_kernels_$K.txt 2>&1
        head -8 gpurun_out/roof_kernels_$K.txt
      done ;;
    roof_pmc)
      for K in ${ROOF_KEYS:-wgrad_l1 dgrad_l8 wgrad_l5 wgrad wgrad_kernel tcn_fwd gcn_l5 gcn_l6}; do
        for C in FETCH_SIZE WRITE_SIZE; do
          rm -rf $P/rpmc_${K}_$C
          run rpmc_${K}_$C 120 rocprofv3 --pmc $C --kernel-trace -d $P/rpmc_${K}_$C -o run -- \
            python tools/roofline_pmc.py run $K > gpurun_out/roof_pmc_${K}_$C.log 2>&1
          db=$(find $P/rpmc_${K}_$C -name "*.db" | head -1)
          [ -n "$db" ] && [ "$db" != "$P/rpmc_${K}_$C/run_results.db" ] && mv "$db" $P/rpmc_${K}_$C/run_results.db
        done
      done
      python tools/roofline_pmc.py summarize $P > gpurun_out/roofline_pmc.json 2>&1
      cat gpurun_out/roofline_pmc.json | head -40 ;;
    rgb_pmc)   # HBM traffic of the RGB branch kernels (bench.py rgb_branch) -> gpurun_out/rgb_pmc.json
      for C in FETCH_SIZE WRITE_SIZE; do
        rm -rf $P/pmc_$C
        run rgbpmc_$C 180 rocprofv3 --pmc $C -d $P/pmc_$C -o run -- python tools/rgb_bench.py \
          > gpurun_out/rgb_pmc_$C.log 2>&1
        db=$(find $P/pmc_$C -name "*.db" | head -1)
        [ -n "$db" ] && [ "$db" != "$P/pmc_$C/run_results.db" ] && mv "$db" $P/pmc_$C/run_results.db
      done
      python tools/rgb_pmc.py gpurun_out > gpurun_out/rgb_pmc.json 2>&1
      cat gpurun_out/rgb_pmc.json ;;
    bench)
      run bench 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
      cut -c1-600 gpurun_out/bench.json ;;
    bench_fp32)
      run bench_fp32 300 python bench.py --steps 20 --warmup 5 --precision fp32 --no-targcn --no-cpu-baseline \
        > gpurun_out/bench_fp32.json 2> gpurun_out/bench_fp32.err
      cut -c1-400 gpurun_out/bench_fp32.json ;;
    ab)   # eager bench A/B over AB_CFGS (tools/ab.sh env; SERIAL_PROF / PAT / ROUNDS pass through)
      run ab 900 bash tools/ab.sh env ${AB_CFGS:--} > gpurun_out/ab.log 2>&1
      grep -E "ms/step|==" gpurun_out/ab.log | head -40 ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    exit_prof)  # tools/exit_check.py under a rocprofv3 kernel trace: the exit status after finalisation
      run exit_prof 240 rocprofv3 --kernel-trace --stats -d $P/exitprof -o run -- \
        python tools/exit_check.py > gpurun_out/exit_prof.log 2>&1
      grep -E "exit_check|Abort|SIGSEGV" gpurun_out/exit_prof.log ;;
    bench_tg)  # the TARGCN (cfg 2) line alone, A/B over TG_CFGS (env assignments, "-" = defaults)
      for cfg in ${TG_CFGS:--}; do
        envs=(); [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
        run "bench_tg[$cfg]" 300 env "${envs[@]}" python bench.py --model targcn --steps 10 --warmup 3 \
          --no-cpu-baseline > "gpurun_out/bench_tg_${cfg//[^A-Za-z0-9]/_}.json" 2>> gpurun_out/bench_tg.err
        cut -c1-300 "gpurun_out/bench_tg_${cfg//[^A-Za-z0-9]/_}.json"
      done ;;
    py:*)
      f=${step#py:}
      n=$(basename "$f" .py)
      run "$n" 600 python -u $f > "gpurun_out/$n.log" 2>&1
      tail -15 "gpurun_out/$n.log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit $rc_all
