#!/bin/bash
# Depthwise-conv BN-sum variants (env knobs of f3_mu_dwconv_fwd) under a rocprofv3 kernel trace;
# prints per-variant median kernel times with / without the sums. Run under gpurun.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dws
IFS="|" read -ra CFGS <<< "${DW_CFGS:-0 1024|0 512|0 2048}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  d=gpurun_out/dws/f$1_g$2
  rm -rf "$d"
  F3_FIN_NOZERO_SET=$1; if [ "$1" = "9" ]; then export F3_FIN_NOZERO=1; else unset F3_FIN_NOZERO; fi
  F3_DW_BLOCK=${3:-512} F3_DW_GRID=$2 timeout -k 10 90 rocprofv3 --kernel-trace -d "$d" -o run -- python -u tools/dwconv_prof.py \
    > "$d.log" 2>&1 || exit 1
  python - "$d" "$cfg" <<'PY'
import sqlite3, statistics, sys, glob
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, start, end from kernels order by start").fetchall()
out = []
for key in ("<3, 1>", "<5, 2>"):
    d = [(e - s) / 1000 for n, s, e in rows if key in n]
    out.append(f"{key} sums {statistics.median(d[:50]):.2f} nosum {statistics.median(d[50:]):.2f}")
fin = [(e - s) / 1000 for n, s, e in rows if "finalize" in n]
print("flush/grid", sys.argv[2], "|", " | ".join(out), "| fin", f"{statistics.median(fin):.2f}" if fin else "-")
PY
done
