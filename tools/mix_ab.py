"""Graph-mix forward/backward timing at the step's three layer shapes (bf16 operands, B=256, V=18,
K=3): (Cin=64, T=30), (128, 15), (256, 8), live HIP-event timing, HBM fraction of x + z (+dx).
Run with F3_MIX_WAVE=0/1 to A/B the forward kernels. GPU only: python tools/mix_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timed(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    import fall_multimodal_amd._lib as L
    lib, st, dev = L.lib(), L.stream_handle(), torch.device("cuda")
    K, V, B = 3, 18, 256
    for Cin, T in ((64, 30), (128, 15), (256, 8)):
        frames = B * T
        A = torch.rand(K, V, V, device=dev) / V
        x = torch.randn(frames, V, Cin, device=dev).to(torch.bfloat16)
        z = torch.empty(frames, V, K, Cin, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(frames, V, Cin, device=dev)
        dA = torch.empty(K, V, V, device=dev)
        msf = timed(lambda: lib.f3_graph_mix_forward_ex(L.ptr(A), L.ptr(x), L.ptr(z), frames, K, V, Cin, 3, st))
        ref = torch.einsum("kvw,fvc->fwkc", A.double(), x.double().cpu().to(dev).double())
        err = float((z.double() - ref).abs().max() / ref.abs().max())
        msb = timed(lambda: lib.f3_graph_mix_backward_ex(L.ptr(A), L.ptr(x), L.ptr(z), L.ptr(dx), L.ptr(dA), frames, K,
                                                         V, Cin, 1, st))
        nx = frames * V * Cin
        bf, bb = nx * 2 + nx * K * 2, nx * 2 + nx * K * 2 + nx * 4
        print(f"Cin={Cin} T={T}: fwd {msf * 1e3:.1f} us = {bf / msf / 1e9 / 8000:.3f} of HBM (rel err {err:.1e}); "
              f"bwd {msb * 1e3:.1f} us = {bb / msb / 1e9 / 8000:.3f}", flush=True)


if __name__ == "__main__":
    main()
