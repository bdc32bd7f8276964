"""Layer-6 tcn weight gradient (C=256, T=8, V=18, 9 taps, bf16, B=256) timed live: the kernel +
slab reduce (f3_conv_backward_weight) and the kernel alone (f3_conv_wgrad_packed), plus a numerics
check of dW against torch on the bf16 operands. Run twice with F3_WGRAD_TAPS=0/1 to A/B.
GPU only: python tools/wgrad_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import fall_multimodal_amd._lib as L
    lib, st, dev = L.lib(), L.stream_handle(), torch.device("cuda")
    N, T, V, C, KT = 256, 8, 18, 256, 9
    torch.manual_seed(0)
    x = torch.randn(N, T, V, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, T, V, C, device=dev).to(torch.bfloat16)
    dw = torch.empty(C, C, KT, device=dev)
    db = torch.empty(C, device=dev)
    fn = lambda: lib.f3_conv_backward_weight(L.ptr(dy), L.ptr(x), L.ptr(dw), L.ptr(db), N, T, V, C, C, KT, 1, 4, 1, st)  # noqa
    L.check(fn(), "wgrad")
    torch.cuda.synchronize()
    # reference: dW[co][ci][dt] = sum_rows dY[row][co] * x[row shifted by (dt-4) frames][ci]
    xf, dyf = x.float().cpu().double(), dy.float().cpu().double()
    ref = torch.zeros(C, C, KT, dtype=torch.float64)
    for dt in range(KT):
        sh = dt - 4
        xs = torch.zeros_like(xf)
        if sh >= 0:
            xs[:, :T - sh] = xf[:, sh:]
        else:
            xs[:, -sh:] = xf[:, :T + sh]
        ref[:, :, dt] = dyf.reshape(-1, C).t() @ xs.reshape(-1, C)
    err = float((dw.cpu().double() - ref).abs().max() / ref.abs().max())
    dberr = float((db.cpu().double() - dyf.reshape(-1, C).sum(0)).abs().max() / dyf.reshape(-1, C).sum(0).abs().max())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        fn()
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    cap = 16 * 256 * 256 * 9
    slab = torch.empty(cap, device=dev)
    g = lambda: lib.f3_conv_wgrad_packed(L.ptr(dy), L.ptr(x), L.ptr(slab), cap, N, T, V, C, C, KT, 1, 4, st)  # noqa
    L.check(g(), "packed")
    for _ in range(5):
        g()
    e0.record()
    for _ in range(20):
        g()
    e1.record()
    torch.cuda.synchronize()
    msk = e0.elapsed_time(e1) / 20
    flop = 2.0 * N * T * V * C * KT * C
    print(f"F3_WGRAD_TAPS={os.environ.get('F3_WGRAD_TAPS', '1')}: with reduce {ms * 1e3:.1f} us "
          f"({flop / ms / 1e9:.0f} TF/s, {flop / ms / 1e9 / 2500:.3f} of peak), kernel alone {msk * 1e3:.1f} us "
          f"({flop / msk / 1e9:.0f} TF/s); dW rel err {err:.2e}, db rel err {dberr:.2e}", flush=True)


if __name__ == "__main__":
    main()
