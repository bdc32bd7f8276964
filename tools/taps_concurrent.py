"""wgrad_taps numerics with other work on the GPU at the same time: the layer-6 weight gradient
(f3_conv_backward_weight, bf16, B=256) on torch's current stream while a second stream runs
matmuls and LDS-heavy convolutions; dW checked against torch each time. GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import fall_multimodal_amd._lib as L
    lib, dev = L.lib(), torch.device("cuda")
    N, T, V, C, KT = 256, 8, 18, 256, 9
    torch.manual_seed(0)
    x = torch.relu(torch.randn(N, T, V, C, device=dev)).to(torch.bfloat16)
    dy = torch.randn(N, T, V, C, device=dev).to(torch.bfloat16)
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
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    xc = torch.randn(64, 3, 30, 18, device=dev)
    wc = torch.randn(64, 3, 9, 1, device=dev)
    # a second library workload on the side stream: the graph-mix / GEMM kernels of the 3-stream step
    for it in range(6):
        dw = torch.empty(C, C, KT, device=dev)
        with torch.cuda.stream(side):
            for _ in range(20):
                a = (a @ a).clamp_(-1, 1)
                torch.nn.functional.conv2d(xc, wc, padding=(4, 0))
        st = L.stream_handle()
        L.check(lib.f3_conv_backward_weight(L.ptr(dy), L.ptr(x), L.ptr(dw), None, N, T, V, C, C, KT, 1, 4, 1, st),
                "wgrad")
        torch.cuda.synchronize()
        err = float((dw.cpu().double() - ref).abs().max() / ref.abs().max())
        print(f"iter {it}: dW rel err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
