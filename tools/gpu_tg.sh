set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_targcn_gpu.py -x -v -s --timeout 240 --timeout-method thread > gpurun_out/tg_tests.log 2>&1; rc=$?
tail -40 gpurun_out/tg_tests.log
exit $rc
