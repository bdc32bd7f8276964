#!/bin/bash
# Kernel + HIP API trace of the step alone: when was each kernel submitted vs when did it run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/step_api -o run -- python tools/step_only.py 8 \
    > gpurun_out/step_api.log 2>&1 || { tail -20 gpurun_out/step_api.log; exit 1; }
python - <<'PY'
import sqlite3
c = sqlite3.connect("gpurun_out/step_api/run_results.db")
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print(tabs)
for t in ("kernels", "regions", "rocpd_region", "rocpd_kernel_dispatch"):
    if t in tabs:
        print(t, [r[1] for r in c.execute(f"pragma table_info({t})")])
PY
