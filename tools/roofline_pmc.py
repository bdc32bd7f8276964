#!/usr/bin/env python3
"""HBM traffic per launch of bench.py's roofline kernels (the bf16x3 headline mode), from rocprofv3
PMC counters. One profiled process per roofline key, so launches of the same kernel name in
different keys (layer 6 / layer 5 / the GEMM alone) never mix.

    run:        python tools/roofline_pmc.py run KEY   (bench.roofline_kernels(..., "bf16x3", only=KEY):
                                                       3 warm-up + 20 timed launches; writes the record
                                                       to gpurun_out/roof_names/KEY.json)
    on the box: per KEY and counter C: timeout -s KILL 60 rocprofv3 --pmc C --kernel-trace
                    -d gpurun_out/rpmc_KEY_C -o run -- python tools/roofline_pmc.py run KEY
                (tools/gpu_session.sh roof_pmc)
    summarize:  python tools/roofline_pmc.py summarize gpurun_out > profiles/r05_roofline_pmc_final.json

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

# bench.py roofline key -> kernel name patterns whose per-launch means add up to one launch of it
_RED = "wgrad_slab_reduce_kernel"
KERNELS = {"wgrad_l1": ["wgrad_big<2, 4, 2, 1, 32, 1, 3, true", _RED],
           "dgrad_l8": ["igemm_win1<16, 2, 4, 144"],
           "gcn_l5": ["igemm_big<6, 1, 8, 0"],
           "gcn_l6": ["igemm_big<6, 1, 8, 0"],
           "wgrad_l5": ["wgrad_big<4, 2, 4, 4, 32, 1, 3, true", _RED],
           "wgrad": ["wgrad_taps<5", "wgrad_taps_reduce_kernel"],
           "wgrad_kernel": ["wgrad_taps<5"],
           "tcn_fwd": ["igemm_win1<1, 2, 4, 144"]}


def run(key):
    import torch
    import bench
    r = bench.roofline_kernels(torch.device("cuda"), 256, 18, "bf16x3", only=key)
    out = os.environ.get("PROF_DIR", os.path.join(ROOT, "gpurun_out"))  # (tools/gpu_session.sh sets it)
    os.makedirs(os.path.join(out, "roof_names"), exist_ok=True)
    with open(os.path.join(out, "roof_names", key + ".json"), "w") as f:
        json.dump(r[key], f)
    print(json.dumps({k: [v["kernel"], v["ms_per_launch"], v["frac"]] for k, v in r.items()}))


def per_launch(db, counter, pattern):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, value from counters_collection where counter_name = ?", (counter,)).fetchall()
    vals = [v * 1024.0 for name, v in rows if pattern in name]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def summarize(d):
    out = {}
    for key, pats in KERNELS.items():
        names = os.path.join(d, "roof_names", key + ".json")
        if not os.path.exists(names):
            continue
        with open(names) as f:
            rec = json.load(f)
        fetch = write = 0.0
        launches = []
        for pat in pats:
            f, nf = per_launch(os.path.join(d, f"rpmc_{key}_FETCH_SIZE", "run_results.db"), "FETCH_SIZE", pat)
            w, nw = per_launch(os.path.join(d, f"rpmc_{key}_WRITE_SIZE", "run_results.db"), "WRITE_SIZE", pat)
            if f is None or w is None:
                break
            fetch += 2.0 * f
            write += w
            launches.append([pat, nf, nw])
        else:
            out[key] = {"kernel": rec["kernel"], "fetch_bytes": fetch, "write_bytes": write,
                        "bytes_per_launch": round(fetch + write), "launches": launches,
                        "ms_per_launch_in_profiled_run": rec["ms_per_launch"],
                        "note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, mean over launches, "
                                "summed over the kernels of one launch; one profiled process per key"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        summarize(sys.argv[2])
