#!/bin/bash
# Graph-mix backward on bf16 MFMA: kernel parity (both kernels), the step parity tests in bf16,
# then an eager-step A/B against the fp32-MFMA kernel (F3_MIX_BWD_BF16=0).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "graph_mix or benchmarked or cfg3 or bf16_step" > gpurun_out/mix_tests.log 2>&1 \
    || { echo "tests failed"; tail -40 gpurun_out/mix_tests.log; exit 1; }
tail -3 gpurun_out/mix_tests.log
ROUNDS=2 bash tools/ab.sh env - ${AB_CFG:-F3_MIX_BWD_BF16=0} || exit 1
timeout -k 10 120 python -c "
import json, torch, bench
r = bench.mix_roofline(torch.device('cuda'), 256, 18, 'bf16')
print(json.dumps(r))" > gpurun_out/mix_roof.json 2>gpurun_out/mix_roof.err || { tail gpurun_out/mix_roof.err; exit 1; }
cat gpurun_out/mix_roof.json
env ${AB_CFG:-F3_MIX_BWD_BF16=0} timeout -k 10 120 python -c "
import json, torch, bench
r = bench.mix_roofline(torch.device('cuda'), 256, 18, 'bf16')
print(json.dumps(r))" > gpurun_out/mix_roof0.json 2>>gpurun_out/mix_roof.err || { tail gpurun_out/mix_roof.err; exit 1; }
cat gpurun_out/mix_roof0.json
