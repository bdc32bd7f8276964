#!/usr/bin/env python3
"""Time the tcn weight-gradient kernel alone (f3_conv_wgrad_packed) over batch sizes:
separates per-row cost from fixed cost.   python tools/wgrad_sweep.py [C] [T]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import fall_multimodal_amd._lib as L
    lib = L.lib()
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    V, KT = 18, 9
    st = L.stream_handle()
    cap = 512 * 128 * 128 * max(1, int(os.environ.get("F3_SLAB_X", "1")))
    slab = torch.empty(cap, device="cuda")
    res = {}
    for N in (32, 64, 128, 256, 512):
        x = torch.randn(N, T, V, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, T, V, C, device="cuda").to(torch.bfloat16)
        f = lambda: lib.f3_conv_wgrad_packed(L.ptr(dy), L.ptr(x), L.ptr(slab), cap, N, T, V, C, C, KT, 1, 4, st)
        L.check(f(), "wgrad")
        ms = bench._time_launch(f)
        res[N] = round(ms * 1e3, 1)
    print(json.dumps({"C": C, "T": T, "us": res, "dbg": os.environ.get("F3_WG_DBG", "0"),
                      "big": os.environ.get("F3_WGRAD_BIG", "1")}), flush=True)


if __name__ == "__main__":
    main()
