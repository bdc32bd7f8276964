#!/usr/bin/env python3
"""Time the implicit-GEMM conv kernels on the step's layer shapes (B=256, V=18):
fwd / dgrad / wgrad in fp32, bf16-from-fp32 (register-staged) and bf16 (LDS-DMA).
    python tools/bench_gemm.py [--reps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fall_multimodal_amd._lib as L  # noqa: E402

SHAPES = [  # (name, N, T_in, V, Cin, Cout, KT, stride, pad)
    ("plain4k", 1, 4096, 1, 4096, 4096, 1, 1, 0),   # a plain 4096^3 GEMM (structure ceiling)
    ("tcn l1", 256, 30, 18, 64, 64, 9, 1, 4),
    ("tcn l3", 256, 30, 18, 128, 128, 9, 2, 4),
    ("tcn l4", 256, 15, 18, 128, 128, 9, 1, 4),
    ("tcn l5", 256, 15, 18, 256, 256, 9, 2, 4),
    ("tcn l6", 256, 8, 18, 256, 256, 9, 1, 4),
    ("gcn l1", 256, 30, 18, 192, 64, 1, 1, 0),
    ("gcn l6", 256, 8, 18, 768, 256, 1, 1, 0),
]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    lib = L.lib()
    d = torch.device("cuda")
    st = L.stream_handle()
    print(f"{'shape':8s} {'prec':12s} {'fwd us':>8s} {'TF':>6s} {'dgrad us':>9s} {'TF':>6s} {'wgrad us':>9s} {'TF':>6s}")
    only = os.environ.get("BENCH_GEMM_ONLY")
    for name, N, T, V, Ci, Co, KT, s, p in SHAPES:
        if only and name not in only.split(","):
            continue
        To = (T + 2 * p - KT) // s + 1
        flop = 2.0 * N * To * V * Co * KT * Ci
        x32 = torch.randn(N, T, V, Ci, device=d)
        dy32 = torch.randn(N, To, V, Co, device=d)
        w = torch.randn(Co, Ci, KT, device=d) / (Ci * KT) ** 0.5
        b = torch.zeros(Co, device=d)
        out = torch.empty(N, To, V, Co, device=d)
        dx = torch.empty(N, T, V, Ci, device=d)
        dw = torch.empty(Co, Ci, KT, device=d)
        db = torch.empty(Co, device=d)
        wp = torch.empty(Co * KT * Ci, device=d)
        precs = ((1, "bf16"),) if os.environ.get("BENCH_GEMM_BF16_ONLY") else ((0, "fp32"), (2, "bf16_fp32in"), (1, "bf16"))
        for prec, pname in precs:
            x = x32.to(torch.bfloat16) if prec == 1 else x32
            dy = dy32.to(torch.bfloat16) if prec == 1 else dy32
            L.check(lib.f3_conv_forward(L.ptr(x), L.ptr(w), L.ptr(b), L.ptr(out), L.ptr(wp), N, T, V, Ci, Co, KT, s,
                                        p, prec, st), "fwd")
            tf = timeit(lambda: lib.f3_conv_forward(L.ptr(x), None, L.ptr(b), L.ptr(out), L.ptr(wp), N, T, V, Ci, Co,
                                                    KT, s, p, prec, st), a.reps)
            td = timeit(lambda: lib.f3_conv_backward_data(L.ptr(dy), L.ptr(w), L.ptr(dx), L.ptr(wp), N, T, V, Ci, Co,
                                                          KT, s, p, prec, st), a.reps)
            tw = timeit(lambda: lib.f3_conv_backward_weight(L.ptr(dy), L.ptr(x), L.ptr(dw), L.ptr(db), N, T, V, Ci,
                                                            Co, KT, s, p, prec, st), a.reps)
            print(f"{name:8s} {pname:12s} {tf:8.1f} {flop / tf / 1e6:6.0f} {td:9.1f} {flop / td / 1e6:6.0f} "
                  f"{tw:9.1f} {flop / tw / 1e6:6.0f}", flush=True)


if __name__ == "__main__":
    main()
