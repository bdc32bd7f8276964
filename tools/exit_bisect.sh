set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${EXIT_MODES:-torch lib cnn targcn both}; do
  echo "== $w"
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/exitb_$w -o run -- python tools/exit_check.py $w > gpurun_out/exitb_$w.log 2>&1
  rc=$?
  echo "== $w rc=$rc"
  grep -E "exit_check|SIGSEGV" gpurun_out/exitb_$w.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
