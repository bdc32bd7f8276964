"""Launch the depthwise temporal conv forward (musa_model's Conv1D) at the bench shapes, with and
without the fused BatchNorm sums, so that a rocprofv3 kernel trace separates the conv kernel from
the lane finalize. GPU only; usage:
    rocprofv3 --kernel-trace --stats -d gpurun_out/dw -- python tools/dwconv_prof.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import fall_multimodal_amd._lib as L  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    lib, st = L.lib(), L.stream_handle()
    B, C, T, V = 256, 128, 30, 14
    for K, S in ((3, 1), (5, 2)):
        xin = torch.randn(B, T, V, C, device=dev)
        To = (T - 1) // S + 1
        y = torch.empty(B, To, V, C, device=dev)
        w = torch.randn(C, K, device=dev)
        bb = torch.randn(C, device=dev)
        sums = torch.zeros(2 * C, dtype=torch.float64, device=dev)
        for use_sums in (True, False):
            for _ in range(50):
                L.check(lib.f3_dwconv_t_forward(L.ptr(xin), L.ptr(w), L.ptr(bb), L.ptr(y),
                                                L.ptr(sums) if use_sums else None, B, T, V, C, K, S,
                                                (K - 1) // 2, st), "dwconv")
        torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
