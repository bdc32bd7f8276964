"""The 1x1 conv GEMM of the bf16 step (pw_gemm.hip, through f3_pointwise_conv and the step's own
dispatch) against torch fp64 on the same bf16 operands, for every epilogue the step uses:
  gcn forward        out = Z . W^T + bias_eff[v] (bf16) and BN sums     stgcan.py:50-56
  gcn input gradient dZ = dg . W (bf16)                                  (autograd of the above)
  residual forward   r = x[:, ::2] . W^T + b (bf16) and BN sums          stgcan.py:123-133
  residual dgrad     dx[:, ::2] += dr . W (fp32, odd frames untouched)   stgcan.py:143-144
plus a plain conv. Shapes are the step's (K, N) at a few clips with a ragged
last tile. Tolerance: the bf16 rounding of the output (2^-8 relative) plus 1e-5 of the max for the
fp32 accumulation; BN sums within 1e-5 relative (fp32 per-lane sums, fp64 across workgroups)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

EPI_BIAS, EPI_BIASV, EPI_STATS, EPI_ADD = 1, 2, 4, 32

# (N, T_in, T_out, V, Cin, Cout, stride, transposed, epi, out_bf16)
CASES = [
    (5, 30, 30, 18, 192, 64, 1, 0, EPI_BIASV | EPI_STATS, 1),    # gcn forward, 64-channel layers
    (5, 30, 30, 18, 192, 128, 1, 0, EPI_BIASV | EPI_STATS, 1),   # layer 3
    (3, 15, 15, 18, 384, 128, 1, 0, EPI_BIASV | EPI_STATS, 1),   # layer 4 (32-row tiles)
    (3, 15, 15, 18, 384, 256, 1, 0, EPI_BIASV | EPI_STATS, 1),   # layer 5
    (5, 8, 8, 18, 768, 256, 1, 0, EPI_BIASV | EPI_STATS, 1),     # layer 6 (half the waves store)
    (4, 8, 8, 14, 768, 256, 1, 0, EPI_BIASV | EPI_STATS, 1),     # V = 14
    (5, 30, 30, 18, 64, 192, 1, 1, 0, 1),                        # gcn input gradient, 64-channel layers
    (5, 30, 30, 18, 128, 192, 1, 1, 0, 1),                       # layer 3
    (3, 15, 15, 18, 128, 384, 1, 1, 0, 1),                       # layer 4
    (3, 15, 15, 18, 256, 384, 1, 1, 0, 1),                       # layer 5
    (3, 8, 8, 18, 256, 768, 1, 1, 0, 1),                         # layer 6
    (5, 30, 15, 18, 64, 128, 2, 0, EPI_BIAS | EPI_STATS, 1),     # residual forward, layer 3
    (4, 29, 15, 18, 64, 128, 2, 0, EPI_BIAS | EPI_STATS, 1),     # motion stream (T = 29)
    (3, 15, 8, 18, 128, 256, 2, 0, EPI_BIAS | EPI_STATS, 1),     # layer 5
    (5, 15, 30, 18, 128, 64, 2, 1, EPI_ADD, 0),                  # residual input gradient, layer 3
    (4, 15, 29, 18, 128, 64, 2, 1, EPI_ADD, 0),                  # ... motion stream: 15 -> 29 frames
    (3, 8, 15, 18, 256, 128, 2, 1, EPI_ADD, 0),                  # layer 5
    (5, 30, 30, 14, 64, 192, 1, 0, EPI_BIAS, 1),                 # plain conv (V = 14)
]


def _case_id(c):
    N, T, To, V, ci, co, s, tr, epi, ob = c
    return f"N{N}T{T}-{To}V{V}_{ci}to{co}_s{s}{'_tr' if tr else ''}_e{epi}{'_bf16' if ob else ''}"


@pytest.mark.parametrize("case", CASES, ids=[_case_id(c) for c in CASES])
def test_pointwise_conv_matches_torch(case):
    import fall_multimodal_amd._lib as L
    N, T_in, T_out, V, Cin, Cout, s, tr, epi, out_bf16 = case
    d = torch.device("cuda")
    g = torch.Generator().manual_seed(Cin * 7 + Cout + T_in)
    x = torch.randn(N, T_in, V, Cin, generator=g).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, generator=g) / np.sqrt(Cin)).to(torch.bfloat16)
    xd, wd = x.double(), w.double()
    if tr:
        ref = torch.zeros(N, T_out, V, Cout, dtype=torch.float64)
        ref[:, ::s] = torch.einsum("ntvc,jc->ntvj", xd, wd)
    else:
        ref = torch.einsum("ntvc,jc->ntvj", xd[:, ::s], wd)
    bias = None
    if epi & EPI_BIASV:
        bias = torch.randn(V, Cout, generator=g)
        ref = ref + bias.double()[None, None]
    elif epi & EPI_BIAS:
        bias = torch.randn(Cout, generator=g)
        ref = ref + bias.double()
    base = None
    if epi & EPI_ADD:
        base = torch.randn(N, T_out, V, Cout, generator=g)
        ref = ref + base.double()
    xg, wg = x.contiguous().to(d), w.contiguous().to(d)
    bg = bias.contiguous().to(d) if bias is not None else None
    if base is not None:
        out = base.clone().to(d)
    else:
        out = torch.full((N, T_out, V, Cout), float("nan"), device=d,
                         dtype=torch.bfloat16 if out_bf16 else torch.float32)
    st = torch.zeros(2, Cout, dtype=torch.float64, device=d)
    L.check(L.lib().f3_pointwise_conv(L.ptr(xg), L.ptr(wg), L.ptr(bg) if bg is not None else None, L.ptr(out),
                                      out_bf16, L.ptr(st[0]), L.ptr(st[1]), N, T_in, T_out, V, Cin, Cout, s, tr, epi,
                                      L.stream_handle()), "pointwise conv")
    got = out.double().cpu()
    tol = (ref.abs() * 2.0 ** -8 if out_bf16 else 0) + 1e-5 * float(ref.abs().max())
    err = (got - ref).abs() - tol
    assert bool((err <= 0).all()), f"max excess {float(err.max()):.3e} at {np.unravel_index(int(err.argmax()), err.shape)}"
    if epi & EPI_STATS:
        s1, s2 = ref.sum((0, 1, 2)), (ref * ref).sum((0, 1, 2))
        st = st.cpu()
        np.testing.assert_allclose(st[0].numpy(), s1.numpy(), rtol=0, atol=1e-5 * float(s1.abs().max()) + 1e-6)
        np.testing.assert_allclose(st[1].numpy(), s2.numpy(), rtol=1e-5, atol=1e-6)
