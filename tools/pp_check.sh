set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "win1_matches" --timeout 120 --timeout-method thread > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -2 gpurun_out/pp_tests.log
: > gpurun_out/pp_kbench.txt
for pp in 0 1 0 1; do
  echo "== F3_WIN1_PP=$pp" >> gpurun_out/pp_kbench.txt
  F3_WIN1_PP=$pp timeout -k 10 120 python tools/kbench.py l8d l8f l5d l5f l7d l7f l4d l4f l1d >> gpurun_out/pp_kbench.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/pp_kbench.txt
