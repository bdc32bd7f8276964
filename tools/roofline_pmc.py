#!/usr/bin/env python3
"""HBM traffic per launch of bench.py's roofline kernels, from rocprofv3 PMC counters.

    run:        python tools/roofline_pmc.py run          (the kernels bench.py times, 20 launches each)
    on the box: timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/rpmc_FETCH_SIZE -o run -- python tools/roofline_pmc.py run
                timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/rpmc_WRITE_SIZE -o run -- python tools/roofline_pmc.py run
    summarize:  python tools/roofline_pmc.py summarize gpurun_out > profiles/r01_roofline_pmc.json

FETCH_SIZE on gfx950 counts 1/2 of the bytes of wide streaming reads (MI355X_MICROARCH.md,
HBM section; calibrated here on rmsprop_kernel: 51.6 MB read = 2 x FETCH_SIZE), so fetch is
doubled; WRITE_SIZE is exact for 16-B stores and for float atomics. Separate passes: the
two counters do not fit one TCC pass.
"""
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

_TAPS = os.environ.get("F3_WGRAD_TAPS", "1") != "0"
_WG = "wgrad_taps<5>" if _TAPS else "wgrad_big<4, 2, 4, 4, 64>"
_RED = "wgrad_taps_reduce_kernel" if _TAPS else "wgrad_slab_reduce_kernel"
# bench.py roofline key -> kernel name patterns whose per-launch means add up to one launch of it
KERNELS = {"wgrad": [_WG, _RED], "wgrad_kernel": [_WG],
           "wgrad_l5": ["wgrad_big<4, 2, 4, 4, 64>", "wgrad_slab_reduce_kernel"],
           "tcn_fwd": ["igemm_big<1, 2, 4, false, true," if os.environ.get("F3_BIG_WIN", "1") != "0" else "igemm_big<1, 1, 8,"]}
_SHAPE = "C=256, T=8, N=256, V=18"
_KN = _WG.replace(", ", ",")
NAMES = {"wgrad": f"{_KN} + slab reduce (tcn 9x1 weight gradient incl. the split-K reduce, {_SHAPE})",
         "wgrad_kernel": f"{_KN} alone (partials left in the slab, {_SHAPE})",
         "wgrad_l5": "wgrad_big<4,2,4,4,64> + slab reduce (tcn 9x1 weight gradient incl. the split-K reduce, "
                     "stride 2, C=256, T=15->8, N=256, V=18)",
         "tcn_fwd": ("igemm_big<1,2,4,false,true> (clip window)" if os.environ.get("F3_BIG_WIN", "1") != "0"
                     else "igemm_big<1,1,8>") + f" bf16-out (tcn 9x1 fwd, {_SHAPE})"}


def run():
    import torch
    import bench
    r = bench.roofline_kernels(torch.device("cuda"), 256, 18, "bf16")
    print(json.dumps({k: [v["kernel"], v["ms_per_launch"], v["frac"]] for k, v in r.items()}))


def per_launch(db, counter, pattern):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, value from counters_collection where counter_name = ?", (counter,)).fetchall()
    vals = [v * 1024.0 for name, v in rows if pattern in name]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def summarize(d):
    out = {}
    for key, pats in KERNELS.items():
        fetch = write = 0.0
        launches = []
        for pat in pats:
            f, nf = per_launch(os.path.join(d, "rpmc_FETCH_SIZE", "run_results.db"), "FETCH_SIZE", pat)
            w, nw = per_launch(os.path.join(d, "rpmc_WRITE_SIZE", "run_results.db"), "WRITE_SIZE", pat)
            if f is None or w is None:
                break
            fetch += 2.0 * f
            write += w
            launches.append([pat, nf, nw])
        else:
            out[key] = {"kernel": NAMES[key], "fetch_bytes": fetch, "write_bytes": write,
                        "bytes_per_launch": round(fetch + write), "launches": launches,
                        "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, mean over launches, "
                                "summed over the kernels of one launch"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2])
