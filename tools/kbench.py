#!/usr/bin/env python3
"""Time the bf16x3 tcn implicit GEMMs of the step alone (B=256, V=18), one shape per key:

    python tools/kbench.py KEY [KEY ...]      keys: l1 l4 l5 l7 l8 (layer), suffix f (forward) / d (dgrad) / w (weight gradient)

    l1: 64 ch, T 30, stride 1
    l4: 128 ch, T 30 -> 15, stride 2    l5: 128 ch, T 15, stride 1
    l7: 256 ch, T 15 -> 8, stride 2     l8: 256 ch, T 8, stride 1

Operands as the step stores them ([hi | lo] rows, f3_split_x3cat); 3 warm-up + 20 timed launches per
key, HIP events on the library's stream; prints one line per key (us per launch, algorithmic TF/s).
Meant to run under rocprofv3 --pmc for per-kernel counters (tools/gpu_session.sh kpmc).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"l1": (30, 64, 1), "l4": (30, 128, 2), "l5": (15, 128, 1), "l7": (15, 256, 2), "l8": (8, 256, 1)}


def main():
    import fall_multimodal_amd._lib as L
    lib, st = L.lib(), L.stream_handle()
    dev = torch.device("cuda")
    N, V, KT, P = 256, 18, 9, 4

    def split(t):
        rows, c = t.numel() // t.shape[-1], t.shape[-1]
        out = torch.empty(rows, 2 * c, device=dev, dtype=torch.bfloat16)
        L.check(lib.f3_split_x3cat(L.ptr(t), L.ptr(out), rows, c, st), "split")
        return out

    for key in sys.argv[1:]:
        T, C, S = SHAPES[key[:2]]
        To = (T + 2 * P - KT) // S + 1
        w = torch.randn(C, C, KT, device=dev) / 48.0
        b = torch.zeros(C, device=dev)
        wp = torch.empty(3 * C * KT * C // 2 + 64, device=dev)
        if key[2] == "f":
            x3 = split(torch.randn(N, T, V, C, device=dev))
            y = torch.empty(N, To, V, C, device=dev)
            L.check(lib.f3_conv_forward_x3cat(L.ptr(x3), L.ptr(w), L.ptr(b), L.ptr(y), L.ptr(wp), N, T, V, C, C, KT, S, P,
                                              st), "fwd")
            run = lambda: lib.f3_conv_forward_x3cat(L.ptr(x3), None, L.ptr(b), L.ptr(y), L.ptr(wp), N, T, V, C, C, KT, S,
                                                    P, st)
        elif key[2] == "w":  # the weight gradient (three row segments + the slab reduce)
            x3 = split(torch.randn(N, T, V, C, device=dev))
            dy3 = split(torch.randn(N, To, V, C, device=dev))
            dw = torch.empty(C, C, KT, device=dev)
            db = torch.empty(C, device=dev)
            run = lambda: lib.f3_conv_backward_weight_x3cat(L.ptr(dy3), L.ptr(x3), L.ptr(dw), L.ptr(db), N, T, V, C, C,
                                                            KT, S, P, st)
        else:
            dy3 = split(torch.randn(N, To, V, C, device=dev))
            dx = torch.empty(N, T, V, C, device=dev)
            L.check(lib.f3_conv_backward_data_x3cat(L.ptr(dy3), L.ptr(w), L.ptr(dx), L.ptr(wp), N, T, V, C, C, KT, S, P,
                                                    st), "dgrad")
            run = lambda: lib.f3_conv_backward_data_x3cat(L.ptr(dy3), None, L.ptr(dx), L.ptr(wp), N, T, V, C, C, KT, S,
                                                          P, st)
        for _ in range(3):
            L.check(run(), key)
        s = torch.cuda.ExternalStream(st) if st else torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            L.check(run(), key)
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 20
        flop = 2.0 * N * (T if key[2] == "d" else To) * V * C * C * KT / (S if key[2] == "d" else 1)
        print(f"{key}: {us:8.1f} us/launch  {flop / us / 1e6:7.1f} TF/s algorithmic", flush=True)


if __name__ == "__main__":
    main()
