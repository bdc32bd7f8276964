"""Layer-6 tcn weight gradient inside the bf16 TrainStep (B=256, V=18) vs torch on the step's own
dh / u tensors (f3_net_debug_tensor), per stream. GPU only: python tools/taps_debug.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import fall_multimodal_amd as f3
    import fall_multimodal_amd._lib as L
    from oracle.prng import synthetic_batch
    d = torch.device("cuda")
    B, V, S, C, T = 256, 18, 6, 256, 8
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, S, device=d,
                                      precision="bf16")
    step = f3.TrainStep(model, B, lr=0.0)
    batch = [torch.from_numpy(x).to(d) for x in synthetic_batch(B, V, 11, S, 257)]
    step(*batch)
    torch.cuda.synchronize()
    lib = L.lib()
    lib.f3_net_debug_tensor.restype = ctypes.c_void_p
    lib.f3_net_debug_tensor.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_char_p]
    h = model._native.h
    grads = {n: p.grad for n, p in model.named_parameters()}
    for si, pre in ((0, "stgcan_1"), (1, "stgcan_2")):
        n = B * T * V * C
        out = {what: lib.f3_net_debug_tensor(h, B, L.ptr(step.ws), si, 6, what.encode()) for what in ("dh", "u")}
        # copy via hipMemcpy
        hipMemcpy = ctypes.CDLL("libamdhip64.so").hipMemcpy
        hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        host = {}
        for what, ptr in out.items():
            a = np.empty(n, dtype=np.uint16)
            assert hipMemcpy(a.ctypes.data, ptr, n * 2, 2) == 0
            host[what] = torch.from_numpy(a.view(np.int16)).view(torch.bfloat16).float().double().reshape(B, T, V, C)
        dh, u = host["dh"], host["u"]
        ref = torch.zeros(C, C, 9, dtype=torch.float64)
        for dt in range(9):
            sh = dt - 4
            us = torch.zeros_like(u)
            if sh >= 0:
                us[:, :T - sh] = u[:, sh:]
            else:
                us[:, -sh:] = u[:, :T + sh]
            ref[:, :, dt] = dh.reshape(-1, C).t() @ us.reshape(-1, C)
        g = grads[f"{pre}.st_gcan_networks.6.tcn.2.weight"].detach().cpu().double().reshape(C, C, 9)
        # the same kernel standalone on the step's own tensors
        dhd = torch.from_numpy(np.ascontiguousarray(dh.float().numpy())).to(d).to(torch.bfloat16)
        ud = torch.from_numpy(np.ascontiguousarray(u.float().numpy())).to(d).to(torch.bfloat16)
        dws = torch.empty(C, C, 9, device=d)
        L.check(lib.f3_conv_backward_weight(L.ptr(dhd), L.ptr(ud), L.ptr(dws), None, B, T, V, C, C, 9, 1, 4, 1,
                                            L.stream_handle()), "wgrad")
        torch.cuda.synchronize()
        es = float((dws.cpu().double() - ref).abs().max() / ref.abs().max())
        print(f"{pre}: standalone on the step's dh/u: rel {es:.2e}; finite dh {bool(torch.isfinite(dh).all())} "
              f"u {bool(torch.isfinite(u).all())} max|dh| {float(dh.abs().max()):.3e} max|u| {float(u.abs().max()):.3e}",
              flush=True)
        err = (g - ref).abs()
        print(f"{pre} layer-6 tcn wgrad: max|ref| {float(ref.abs().max()):.3e} max err {float(err.max()):.3e} "
              f"rel {float(err.max() / ref.abs().max()):.2e}; bad entries {int((err > 1e-2 * ref.abs().max()).sum())}",
              flush=True)
        if float(err.max() / ref.abs().max()) > 1e-3:
            bad = (err > 1e-2 * ref.abs().max()).nonzero()
            print("  first bad (co, ci, dt):", bad[:10].tolist(), flush=True)
            co = bad[:, 0].unique(); ci = bad[:, 1].unique(); dts = bad[:, 2].unique()
            print("  co range", int(co.min()), int(co.max()), "n", co.numel(), "ci range", int(ci.min()), int(ci.max()),
                  "n", ci.numel(), "dts", dts.tolist(), flush=True)


if __name__ == "__main__":
    main()
