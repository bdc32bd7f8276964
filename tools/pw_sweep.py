"""Per-launch time of the 1x1 conv GEMM (f3_pointwise_conv: pw_gemm where eligible) against the
row count, to split a launch into fixed and per-tile cost. HIP events around 20 launches each.
    python tools/pw_sweep.py [F3_PW=0 for the igemm path]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import fall_multimodal_amd._lib as L
    d = torch.device("cuda")
    lib = L.lib()
    # (Cin, Cout, stride, transposed, epi, T_in, T_out)
    shapes = [(192, 64, 1, 0, 6, 30, 30), (64, 192, 1, 1, 0, 30, 30), (64, 128, 2, 0, 5, 30, 15),
              (192, 128, 1, 0, 6, 30, 30), (256, 768, 1, 1, 0, 8, 8)]
    for Cin, Cout, s, tr, epi, T_in, T_out in shapes:
        for N in (16, 64, 256, 512):
            V = 18
            x = torch.randn(N, T_in, V, Cin, device=d).to(torch.bfloat16)
            w = torch.randn(Cout, Cin, device=d).to(torch.bfloat16)
            bias = torch.randn(V * Cout, device=d)
            out = torch.empty(N, T_out, V, Cout, device=d, dtype=torch.bfloat16)
            st = torch.zeros(2, Cout, dtype=torch.float64, device=d)

            def run():
                L.check(lib.f3_pointwise_conv(L.ptr(x), L.ptr(w), L.ptr(bias), L.ptr(out), 1, L.ptr(st[0]),
                                              L.ptr(st[1]), N, T_in, T_out, V, Cin, Cout, s, tr, epi,
                                              L.stream_handle()), "pw")
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            mb = (x.numel() * (1 if s == 1 else 0.5) + out.numel()) * 2 / 1e6
            print(f"K={Cin:3d} N={Cout:3d} s={s} tr={tr} epi={epi:2d} clips={N:3d} rows={N * T_out * V:7d} "
                  f"{us:7.2f} us  {mb:6.1f} MB  {mb / us:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
