"""HIP path vs the oracle / the reference's golden vectors (needs an MI355X)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import model_cpu as oc
from oracle.prng import synthetic_batch
from tests.golden_util import check_grads_conditioned, check_packed, check_post, load

pytestmark = pytest.mark.gpu

TAGS = ["har", "ns", "two", "stgcn", "bilstm", "ur_nb", "ur_sensor"]


def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda")


def build_from_spec(spec, device, precision="fp32"):
    """The golden case's module in the given skeleton-stream precision (the sensor-only models have
    no skeleton GEMMs: precision does not apply to them)."""
    import fall_multimodal_amd as f3
    g = {"layout": spec.layout, "strategy": spec.strategy}
    if spec.model == "stgcn":
        return f3.STGCAN(spec.in_channels, g, spec.num_class, device=device, precision=precision)
    if spec.model == "bilstm" and spec.sensor == "cnn_bilstm":
        return f3.CNN_BiLSTM(hidden_size=16, num_layers=1, dropout_prob=0.3, num_classes=2, feature="mean",
                             device=device)
    if spec.model == "bilstm":
        return f3.BiLSTM(spec.sensor_dim, num_classes=spec.num_class, device=device)
    if spec.model == "two_stgcan":
        return f3.TwoStreamSTGCAN(3, g, spec.num_class, device=device, precision=precision)
    if spec.naming == "notebook":
        return f3.TwoStreamSpatialTemporalGraph(g, spec.num_class, sensor=spec.sensor, sensor_dim=spec.sensor_dim,
                                                sensor_classes=spec.sensor_classes, device=device,
                                                precision=precision)
    return f3.TwoStreamSTGCAN_BiLSTM(3, g, spec.num_class, spec.sensor_dim, device=device, precision=precision)


def call(model, spec, skel, sensor):
    if spec.naming == "notebook":
        return model((skel, skel[:, :2, 1:] - skel[:, :2, :-1], sensor))
    if spec.model == "bilstm" and spec.sensor == "cnn_bilstm":
        return model(sensor)
    if spec.model == "bilstm":
        return model(None, sensor)
    return model(skel, sensor)


PRECISIONS = [0, 1, 2, 4]
PREC_IDS = ["fp32", "bf16", "bf16_fp32in", "bf16x3"]
# bf16x3 (split-bf16, gemm_x3.hip): operands are NOT rounded (fp32 in); each product carries ~2^-16
# relative error, so its gate is against the fp64 result on the fp32 operands at 1e-4 of the max
# (the bf16 modes' 2e-5 is measured against fp64 on their bf16-ROUNDED operands)
X3_TOL = 1e-4


def _q(t, precision):
    """Operand rounding of a precision mode: the bf16 modes round GEMM operands to bf16 (RNE)
    and accumulate in fp32, so the fp64 reference on bf16-rounded operands is exact up to
    fp32 accumulation error."""
    return t.to(torch.bfloat16).to(t.dtype) if precision in (1, 2) else t


def _act(t_cl, precision, d):
    """Activation tensor as the kernel entry takes it: bf16 for precision 1, else fp32."""
    t = t_cl.to(d)
    return t.to(torch.bfloat16).contiguous() if precision == 1 else t.float().contiguous()


@pytest.mark.parametrize("precision", PRECISIONS, ids=PREC_IDS)
def test_conv_kernel_matches_torch(precision):
    d = dev()
    import fall_multimodal_amd._lib as L
    torch.manual_seed(0)
    for (N, T, V, Ci, Co, KT, s, p) in [(3, 30, 14, 64, 64, 9, 1, 4), (2, 30, 18, 64, 128, 9, 2, 4),
                                         (2, 15, 14, 128, 256, 1, 2, 0), (2, 30, 14, 9, 64, 1, 1, 0),
                                         (4, 8, 18, 256, 256, 9, 1, 4), (2, 15, 18, 256, 128, 9, 1, 4),
                                         (3, 8, 25, 64, 64, 9, 1, 4)]:
        x = torch.randn(N, Ci, T, V)
        w = torch.randn(Co, Ci, KT, 1) / np.sqrt(Ci * KT)
        b = torch.randn(Co)
        ref = torch.nn.functional.conv2d(_q(x.double(), precision), _q(w.double(), precision), b.double(),
                                         stride=(s, 1), padding=(p, 0)).float()  # [N,Co,To,V]
        xg = _act(x.permute(0, 2, 3, 1).contiguous(), precision, d)
        To = (T + 2 * p - KT) // s + 1
        out = torch.empty(N, To, V, Co, device=d)
        wp = torch.empty(Co * KT * Ci, device=d)
        wg, bg = w.contiguous().to(d), b.to(d)  # keep alive until the async launches have consumed them
        st = L.lib().f3_conv_forward(L.ptr(xg), L.ptr(wg), L.ptr(bg), L.ptr(out), L.ptr(wp),
                                     N, T, V, Ci, Co, KT, s, p, precision, L.stream_handle())
        L.check(st, "conv")
        got = out.cpu().permute(0, 3, 1, 2)
        np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
        if precision == 4:
            print(f"bf16x3 conv fwd {N, T, V, Ci, Co, KT, s, p}: max err / max "
                  f"{float((got - ref).abs().max() / ref.abs().max()):.2e}")


CONV_SHAPES = [(3, 30, 14, 64, 64, 9, 1, 4), (2, 30, 18, 64, 128, 9, 2, 4), (4, 15, 14, 256, 256, 9, 2, 4),
               (4, 29, 14, 128, 128, 9, 2, 4), (2, 15, 14, 128, 256, 1, 2, 0), (4, 8, 18, 256, 256, 9, 1, 4),
               (2, 30, 14, 9, 64, 1, 1, 0), (2, 30, 18, 64, 192, 1, 1, 0), (3, 30, 18, 192, 64, 1, 1, 0),
               (2, 15, 14, 256, 128, 9, 1, 4), (2, 15, 18, 128, 128, 9, 1, 4),
               # the tap-reuse weight gradient (wgrad_taps): T*V = 144 (5 k steps, 16 splits) and 112 (4)
               (40, 8, 18, 256, 256, 9, 1, 4), (5, 8, 14, 128, 64, 9, 1, 4),
               # its clip-segment / stride-2 form (wgrad_seg): the motion stream's T = 29 layers,
               # layer 5's 15 -> 8 stride 2 at V = 18, and enough clips for multi-unit splits
               (6, 29, 18, 64, 64, 9, 1, 4), (3, 15, 18, 256, 256, 9, 2, 4), (12, 30, 18, 64, 64, 9, 1, 4)]


@pytest.mark.parametrize("precision", PRECISIONS, ids=PREC_IDS)
@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_backward_kernels_match_torch(shape, precision):
    d = dev()
    import fall_multimodal_amd._lib as L
    N, T, V, Ci, Co, KT, s, p = shape
    torch.manual_seed(1)
    x = _q(torch.randn(N, Ci, T, V, dtype=torch.float64), precision).requires_grad_(True)
    w = _q(torch.randn(Co, Ci, KT, 1, dtype=torch.float64) / np.sqrt(Ci * KT), precision).requires_grad_(True)
    b = torch.zeros(Co, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.conv2d(x, w, b, stride=(s, 1), padding=(p, 0))
    dy = _q(torch.randn_like(y), precision)
    y.backward(dy)
    To = y.shape[2]
    dyg = _act(dy.permute(0, 2, 3, 1).contiguous(), precision, d)
    xg = _act(x.detach().permute(0, 2, 3, 1).contiguous(), precision, d)
    wg = w.detach().float().contiguous().to(d)
    dx = torch.empty(N, T, V, Ci, device=d)
    wp = torch.empty(Co * KT * Ci, device=d)
    dw = torch.empty(Co, Ci, KT, device=d)
    db = torch.empty(Co, device=d)
    L.check(L.lib().f3_conv_backward_data(L.ptr(dyg), L.ptr(wg), L.ptr(dx), L.ptr(wp), N, T, V, Ci, Co, KT, s, p,
                                          precision, L.stream_handle()), "dgrad")
    L.check(L.lib().f3_conv_backward_weight(L.ptr(dyg), L.ptr(xg), L.ptr(dw), L.ptr(db), N, T, V, Ci, Co, KT, s, p,
                                            precision, L.stream_handle()), "wgrad")
    ref_dx = x.grad.permute(0, 2, 3, 1).numpy()
    tol = X3_TOL if precision == 4 else 2e-5
    if precision == 4:
        print(f"bf16x3 {shape}: dx {np.abs(dx.cpu().numpy() - ref_dx).max() / np.abs(ref_dx).max():.2e}, dw "
              f"{np.abs(dw.cpu().numpy() - w.grad.reshape(Co, Ci, KT).numpy()).max() / np.abs(w.grad.numpy()).max():.2e}")
    np.testing.assert_allclose(dx.cpu().numpy(), ref_dx, rtol=0, atol=tol * np.abs(ref_dx).max() + 1e-6)
    ref_dw = w.grad.reshape(Co, Ci, KT).numpy()
    np.testing.assert_allclose(dw.cpu().numpy(), ref_dw, rtol=0, atol=tol * np.abs(ref_dw).max() + 1e-6)
    np.testing.assert_allclose(db.cpu().numpy(), b.grad.numpy(), rtol=0, atol=2e-5 * np.abs(b.grad.numpy()).max())


X3CAT_SHAPES = [(3, 30, 14, 64, 64, 9, 1, 4), (2, 30, 18, 64, 128, 9, 2, 4), (4, 15, 14, 256, 256, 9, 2, 4),
                (2, 15, 14, 128, 256, 1, 2, 0), (4, 8, 18, 256, 256, 9, 1, 4), (2, 30, 18, 64, 192, 1, 1, 0),
                (3, 30, 18, 192, 64, 1, 1, 0), (3, 15, 18, 256, 256, 9, 2, 4), (2, 29, 18, 128, 128, 9, 1, 4),
                # the clip-window classes of igemm_big at the step's V = 18: 64 channels at T = 30 / 29
                # (540-row clips), 128 channels at T = 15 (270) and the stride-2 30 / 29 -> 15 layer
                # (forward by input-frame parity, input gradient by output-frame parity)
                (3, 30, 18, 64, 64, 9, 1, 4), (2, 29, 18, 64, 64, 9, 1, 4), (3, 15, 18, 128, 128, 9, 1, 4),
                (3, 30, 18, 128, 128, 9, 2, 4), (3, 29, 18, 128, 128, 9, 2, 4)]


@pytest.mark.parametrize("shape", X3CAT_SHAPES)
def test_conv_x3cat_kernels_match_torch(shape):
    """bf16x3 as the step runs it: fp32 operands split by f3_split_x3cat into [hi | lo] rows, the
    weights packed per tap in 32-channel blocks [W_hi 32 | W_lo 32] (prep code 4), and the bf16 LDS-DMA
    kernels issuing x_hi W_hi + x_lo W_hi + x_hi W_lo per k step (the native split form: forward, input
    gradient); the weight gradient from the same [hi | lo] rows (dY_hi X_hi + dY_lo X_hi + dY_hi X_lo).
    Each against fp64 on the fp32 operands within X3_TOL of the max (the split-bf16 product, ~2^-16 per
    term)."""
    d = dev()
    import fall_multimodal_amd._lib as L
    lib, st = L.lib(), L.stream_handle()
    N, T, V, Ci, Co, KT, s, p = shape
    torch.manual_seed(5)
    x = torch.randn(N, Ci, T, V, dtype=torch.float64, requires_grad=True)
    w = (torch.randn(Co, Ci, KT, 1, dtype=torch.float64) / np.sqrt(Ci * KT)).requires_grad_(True)
    b = torch.randn(Co, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.conv2d(x, w, b, stride=(s, 1), padding=(p, 0))
    dy = torch.randn_like(y)
    y.backward(dy)
    To = y.shape[2]

    def split(t_cl):
        t = t_cl.float().contiguous().to(d)
        rows, C = t.numel() // t.shape[-1], t.shape[-1]
        out = torch.empty(rows, 2 * C, device=d, dtype=torch.bfloat16)
        L.check(lib.f3_split_x3cat(L.ptr(t), L.ptr(out), rows, C, st), "split")
        torch.cuda.synchronize()
        hi = t.to(torch.bfloat16)
        lo = (t - hi.float()).to(torch.bfloat16)
        ref = torch.cat([hi.reshape(rows, C), lo.reshape(rows, C)], 1)
        assert torch.equal(out.view(torch.int16), ref.view(torch.int16))  # bit-exact RNE split
        return out

    x3 = split(x.detach().permute(0, 2, 3, 1))
    dy3 = split(dy.permute(0, 2, 3, 1))
    wg, bg = w.detach().float().contiguous().to(d), b.detach().float().to(d)
    wp = torch.empty(3 * Co * KT * Ci // 2 + 64, device=d)
    out = torch.empty(N, To, V, Co, device=d)
    L.check(lib.f3_conv_forward_x3cat(L.ptr(x3), L.ptr(wg), L.ptr(bg), L.ptr(out), L.ptr(wp), N, T, V, Ci, Co, KT, s, p,
                                      st), "fwd")
    dx = torch.empty(N, T, V, Ci, device=d)
    wpt = torch.empty(3 * Co * KT * Ci // 2 + 64, device=d)
    L.check(lib.f3_conv_backward_data_x3cat(L.ptr(dy3), L.ptr(wg), L.ptr(dx), L.ptr(wpt), N, T, V, Ci, Co, KT, s, p,
                                            st), "dgrad")
    dw = torch.empty(Co, Ci, KT, device=d)
    db = torch.empty(Co, device=d)
    L.check(lib.f3_conv_backward_weight_x3cat(L.ptr(dy3), L.ptr(x3), L.ptr(dw), L.ptr(db), N, T, V, Ci, Co, KT, s, p,
                                              st), "wgrad")
    torch.cuda.synchronize()
    errs = {}
    for name, got, ref in (("y", out.cpu().double(), y.detach().permute(0, 2, 3, 1)),
                           ("dx", dx.cpu().double(), x.grad.permute(0, 2, 3, 1)),
                           ("dw", dw.cpu().double(), w.grad.reshape(Co, Ci, KT)),
                           ("db", db.cpu().double(), b.grad)):
        errs[name] = float((got - ref).abs().max() / ref.abs().max())
    print(f"bf16x3 cat {shape}: " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    assert max(errs.values()) <= X3_TOL, errs


@pytest.mark.parametrize("shape", [(4, 8, 18, 256, 256, 1), (3, 15, 18, 128, 128, 1), (3, 30, 18, 64, 64, 1),
                                   (2, 29, 18, 64, 64, 1), (3, 8, 18, 256, 256, 1), (3, 15, 18, 256, 256, 2),
                                   (4, 15, 18, 256, 256, 2), (3, 30, 18, 128, 128, 2), (3, 29, 18, 128, 128, 2)])
def test_win1_matches_runtime_tap_schedule_bitwise(shape, monkeypatch):
    """igemm_win1 (the clip-window GEMM with its tap schedule unrolled at compile time: stride 1, and
    stride 2 by output-frame parity (input gradient, one launch per parity) or by even / odd input
    frames (forward)) against igemm_big's run-time schedule (F3_WIN1=0): the same staged bytes,
    fragment reads and MFMA order, so forward (bias epilogue), input gradient and, at stride 1, the
    step's RELUMASK input gradient (with its BN1-backward sums) must agree bit for bit, on ragged clip
    counts (odd N at two clips per workgroup) and T = 29. The ping-pong form (F3_WIN1_PP=1) too."""
    d = dev()
    import fall_multimodal_amd._lib as L
    lib, st = L.lib(), L.stream_handle()
    N, T, V, Ci, Co, S = shape
    To = (T + 8 - 9) // S + 1
    torch.manual_seed(21)

    def split(t):
        t = t.float().contiguous().to(d)
        out = torch.empty(t.numel() // t.shape[-1], 2 * t.shape[-1], device=d, dtype=torch.bfloat16)
        L.check(lib.f3_split_x3cat(L.ptr(t), L.ptr(out), t.numel() // t.shape[-1], t.shape[-1], st), "split")
        return out

    x3 = split(torch.randn(N, T, V, Ci))
    dy3 = split(torch.randn(N, To, V, Co))
    w = (torch.randn(Co, Ci, 9) / np.sqrt(9 * Ci)).to(d)
    b = torch.randn(Co).to(d)
    g = torch.randn(N, T, V, Ci, device=d)
    gam, bet = torch.rand(Ci, device=d) + 0.5, torch.randn(Ci, device=d) * 0.3
    gd = g.reshape(-1, Ci).double()
    bsum, bsq = gd.sum(0), (gd * gd).sum(0)

    def run():
        y = torch.empty(N, To, V, Co, device=d)
        wp = torch.empty(Co * Ci * 9 + 64, device=d)
        L.check(lib.f3_conv_forward_x3cat(L.ptr(x3), L.ptr(w), L.ptr(b), L.ptr(y), L.ptr(wp), N, T, V, Ci, Co, 9, S, 4,
                                          st), "fwd")
        dx = torch.empty(N, T, V, Ci, device=d)
        wpt = torch.empty(Co * Ci * 9 + 64, device=d)
        L.check(lib.f3_conv_backward_data_x3cat(L.ptr(dy3), L.ptr(w), L.ptr(dx), L.ptr(wpt), N, T, V, Ci, Co, 9, S, 4,
                                                st), "dgrad")
        if S == 2:
            torch.cuda.synchronize()
            return y, dx
        dv = torch.empty(N, T, V, Ci, device=d)
        s1 = torch.zeros(Ci, dtype=torch.float64, device=d)
        s2 = torch.zeros_like(s1)
        L.check(lib.f3_conv_step_x3cat(1, L.ptr(dy3), L.ptr(w), L.ptr(wpt), L.ptr(dv), None, L.ptr(g), L.ptr(gam),
                                       L.ptr(bet), L.ptr(bsum), L.ptr(bsq), float(N * T * V), L.ptr(s1), L.ptr(s2), N, T,
                                       V, Ci, Co, st), "dgrad relumask")
        torch.cuda.synchronize()
        return y, dx, dv

    new = run()
    monkeypatch.setenv("F3_WIN1_PP", "1")  # the ping-pong form: the same MFMAs in the same order per wave
    pp = run()
    monkeypatch.delenv("F3_WIN1_PP")
    monkeypatch.setenv("F3_WIN1", "0")
    old = run()
    for name, p, q, r in zip(("y", "dx", "dv"), new, old, pp):
        assert torch.isfinite(p).all(), name
        assert torch.equal(p, q), (name, float((p - q).abs().max()))
        assert torch.equal(r, p), ("ping-pong " + name, float((r - p).abs().max()))


@pytest.mark.parametrize("shape", [(3, 15, 18, 384, 256, 1), (3, 8, 18, 768, 256, 1), (2, 15, 14, 128, 256, 2),
                                   (3, 30, 18, 128, 128, 1), (3, 29, 18, 128, 256, 2)])
def test_k1_staging_matches_generic_staging_bitwise(shape, monkeypatch):
    """igemm_big's 1x1 (K1) staging, fixed source pointers advanced per k step, against the generic
    per-step staging (F3_K1=0): the same bytes staged, so forward (bias), input gradient (stride-2: the
    parity tiles) and the step's gcn epilogue (graph-mixed bias + BN1 sums, f3_conv_step_x3cat kind 0)
    agree bit for bit. Shapes: the layer-5 / 6 gcn GEMMs, the stride-2 residual convs, a ragged T = 29."""
    d = dev()
    import fall_multimodal_amd._lib as L
    lib, st = L.lib(), L.stream_handle()
    N, T, V, Ci, Co, S = shape
    To = (T - 1) // S + 1
    torch.manual_seed(23)

    def split(t):
        t = t.float().contiguous().to(d)
        out = torch.empty(t.numel() // t.shape[-1], 2 * t.shape[-1], device=d, dtype=torch.bfloat16)
        L.check(lib.f3_split_x3cat(L.ptr(t), L.ptr(out), t.numel() // t.shape[-1], t.shape[-1], st), "split")
        return out

    x3 = split(torch.randn(N, T, V, Ci))
    dy3 = split(torch.randn(N, To, V, Co))
    w = (torch.randn(Co, Ci, 1) / np.sqrt(Ci)).to(d)
    b = torch.randn(Co).to(d)
    bv = (torch.randn(V, Co) * 0.1).to(d)

    def run():
        y = torch.empty(N, To, V, Co, device=d)
        wp = torch.empty(Co * Ci + 64, device=d)
        L.check(lib.f3_conv_forward_x3cat(L.ptr(x3), L.ptr(w), L.ptr(b), L.ptr(y), L.ptr(wp), N, T, V, Ci, Co, 1, S, 0,
                                          st), "fwd")
        dx = torch.empty(N, T, V, Ci, device=d)
        wpt = torch.empty(Co * Ci + 64, device=d)
        L.check(lib.f3_conv_backward_data_x3cat(L.ptr(dy3), L.ptr(w), L.ptr(dx), L.ptr(wpt), N, T, V, Ci, Co, 1, S, 0,
                                                st), "dgrad")
        outs = [y, dx]
        if S == 1:
            gq = torch.empty(N, T, V, Co, device=d)
            s1 = torch.zeros(Co, dtype=torch.float64, device=d)
            s2 = torch.zeros_like(s1)
            L.check(lib.f3_conv_step_x3cat(0, L.ptr(x3), None, L.ptr(wp), L.ptr(gq), L.ptr(bv), None, None, None, None,
                                           None, 0.0, L.ptr(s1), L.ptr(s2), N, T, V, Ci, Co, st), "gcn step")
            outs.append(gq)
        torch.cuda.synchronize()
        return outs

    new = run()
    monkeypatch.setenv("F3_K1", "0")
    old = run()
    for name, p, q in zip(("y", "dx", "gcn"), new, old):
        assert torch.isfinite(p).all(), name
        assert torch.equal(p, q), (name, float((p - q).abs().max()))


@pytest.mark.parametrize("kind,T,Cin,Cout", [(0, 15, 384, 256), (0, 8, 768, 256), (1, 8, 256, 256)])
def test_conv_step_x3cat_epilogues_match_torch(kind, T, Cin, Cout):
    """f3_conv_step_x3cat, the entry bench.py's roofline_gcn / roofline (dgrad_l8) keys time: the step's
    gcn 1x1 GEMM with the graph-mixed bias and BN1 sums (kind 0, skeleton layers 5 / 6 shapes), and the
    T=8 tcn input gradient with the RELUMASK epilogue (kind 1: dv masked where bn1(g) <= 0, the
    BN1-backward sums sum(dv), sum(dv g_hat)). Against fp64 on the fp32 operands within X3_TOL of the
    max; the sums within 1e-4 of their max."""
    d = dev()
    import fall_multimodal_amd._lib as L
    lib, st = L.lib(), L.stream_handle()
    N, V = 3, 18
    torch.manual_seed(11 + kind)
    M = N * T * V
    ind = Cin if kind == 0 else Cout  # channels of the GEMM's input rows

    def split(t):
        t = t.float().contiguous().to(d)
        out = torch.empty(t.numel() // t.shape[-1], 2 * t.shape[-1], device=d, dtype=torch.bfloat16)
        L.check(lib.f3_split_x3cat(L.ptr(t), L.ptr(out), t.numel() // t.shape[-1], t.shape[-1], st), "split")
        return out

    xin = torch.randn(N, T, V, ind, dtype=torch.float64)
    in3 = split(xin)
    ssum = torch.zeros(Cout if kind == 0 else Cin, dtype=torch.float64, device=d)
    ssq = torch.zeros_like(ssum)
    if kind == 0:
        w = torch.randn(Cout, Cin, dtype=torch.float64) / np.sqrt(Cin)
        bv = torch.randn(V, Cout, dtype=torch.float64) * 0.1
        out = torch.empty(N, T, V, Cout, device=d)
        wp = torch.empty(Cout * Cin + 64, device=d)
        # (device copies held in names: a temporary freed after ptr() would be reused by the next one)
        wd, bvd = w.float().to(d), bv.float().to(d)
        L.check(lib.f3_conv_step_x3cat(0, L.ptr(in3), L.ptr(wd), L.ptr(wp), L.ptr(out), L.ptr(bvd), None, None, None,
                                       None, None, 0.0, L.ptr(ssum), L.ptr(ssq), N, T, V, Cin, Cout, st), "gcn step")
        ref = xin @ w.T + bv.view(1, 1, V, Cout)
        rs, rq = ref.reshape(-1, Cout).sum(0), (ref.reshape(-1, Cout) ** 2).sum(0)
    else:
        w = torch.randn(Cout, Cin, 9, 1, dtype=torch.float64) / np.sqrt(9 * Cin)
        g = torch.randn(N, T, V, Cin, dtype=torch.float64)
        gam, bet = torch.rand(Cin, dtype=torch.float64) + 0.5, torch.randn(Cin, dtype=torch.float64) * 0.3
        for _ in range(8):  # no element within 1e-3 of the ReLU kink (fp32 vs fp64 would flip its mask)
            gs = g.reshape(-1, Cin)
            bsum, bsq = gs.sum(0), (gs * gs).sum(0)
            mean = bsum / M
            rstd = 1.0 / torch.sqrt(bsq / M - mean * mean + 1e-5)
            z = (g - mean) * rstd * gam + bet
            near = z.abs() < 1e-3
            if not bool(near.any()):
                break
            g = torch.where(near, g + 0.01, g)
        out = torch.empty(N, T, V, Cin, device=d)
        wp = torch.empty(Cout * Cin * 9 + 64, device=d)
        wd = w.float().reshape(Cout, Cin, 9).contiguous().to(d)
        gd, gamd, betd, bsd, bqd = g.float().to(d), gam.float().to(d), bet.float().to(d), bsum.to(d), bsq.to(d)
        L.check(lib.f3_conv_step_x3cat(1, L.ptr(in3), L.ptr(wd), L.ptr(wp), L.ptr(out), None, L.ptr(gd), L.ptr(gamd),
                                       L.ptr(betd), L.ptr(bsd), L.ptr(bqd), float(M), L.ptr(ssum), L.ptr(ssq), N, T, V,
                                       Cin, Cout, st), "dgrad step")
        # dv = relu'(bn1(g)) * conv_T(dh): the input gradient of conv2d(x, w, padding (4, 0))
        xx = torch.zeros(N, Cin, T, V, dtype=torch.float64, requires_grad=True)
        y = torch.nn.functional.conv2d(xx, w, padding=(4, 0))
        y.backward(xin.permute(0, 3, 1, 2))
        dv = xx.grad.permute(0, 2, 3, 1)
        ghat = (g - mean) * rstd
        ref = torch.where(ghat * gam + bet > 0, dv, torch.zeros_like(dv))
        rs, rq = ref.reshape(-1, Cin).sum(0), (ref * ghat).reshape(-1, Cin).sum(0)
    torch.cuda.synchronize()
    e = float((out.cpu().double() - ref).abs().max() / ref.abs().max())
    es = float((ssum.cpu() - rs).abs().max() / rs.abs().max())
    eq = float((ssq.cpu() - rq).abs().max() / rq.abs().max())
    print(f"step kind {kind} T={T} {Cin}->{Cout}: out {e:.2e}, sums {es:.2e} / {eq:.2e}")
    assert e <= X3_TOL and es <= 1e-4 and eq <= 1e-4, (e, es, eq)


@pytest.mark.parametrize("V,K,Cin,F", [(14, 3, 64, 40), (18, 3, 64, 37), (18, 3, 256, 20), (14, 3, 3, 30),
                                        (18, 3, 2, 29), (18, 1, 128, 9), (14, 2, 128, 11)])
def test_graph_mix_kernels_match_torch(V, K, Cin, F):
    """z = einsum('kvw,fvc->fwkc', A, x) and its gradients (stgcan.py:54 applied to the input)."""
    d = dev()
    import fall_multimodal_amd._lib as L
    torch.manual_seed(V * 100 + Cin)
    A = torch.rand(K, V, V, dtype=torch.float64, requires_grad=True)
    x = torch.randn(F, V, Cin, dtype=torch.float64, requires_grad=True)
    z = torch.einsum("kvw,fvc->fwkc", A, x)
    dz = torch.randn_like(z)
    z.backward(dz)
    Ag, xg, dzg = (t.detach().float().contiguous().to(d) for t in (A, x, dz))
    zo = torch.empty(F, V, K, Cin, device=d)
    dx = torch.empty(F, V, Cin, device=d)
    dA = torch.empty(K, V, V, device=d)
    L.check(L.lib().f3_graph_mix_forward(L.ptr(Ag), L.ptr(xg), L.ptr(zo), F, K, V, Cin, L.stream_handle()), "mix")
    L.check(L.lib().f3_graph_mix_backward(L.ptr(Ag), L.ptr(xg), L.ptr(dzg), L.ptr(dx), L.ptr(dA), F, K, V, Cin,
                                          L.stream_handle()), "mixbwd")
    for got, ref in ((zo, z.detach()), (dx, x.grad), (dA, A.grad)):
        r = ref.numpy()
        np.testing.assert_allclose(got.cpu().numpy(), r, rtol=0, atol=1e-5 * np.abs(r).max())


@pytest.mark.parametrize("V,K,Cin,F", [(18, 3, 64, 300), (14, 3, 128, 77), (18, 3, 256, 41), (18, 1, 64, 9)])
def test_graph_mix_x3_z3_rows(V, K, Cin, F):
    """The bf16x3 mix forward writing Z as the step stores it for the gcn GEMM (F3_MIX_Z3): per
    (frame, node) the bf16 row [z_hi | z_lo] of 2 K Cin. z_hi + z_lo against fp64 within X3_TOL of
    the max, and z_hi / z_lo bit-exactly the RNE split of the kernel's own fp32 z (F3_MIX_X3 alone)."""
    d = dev()
    import fall_multimodal_amd._lib as L
    torch.manual_seed(V + K + Cin)
    A = torch.rand(K, V, V, dtype=torch.float64) / V
    x = torch.randn(F, V, Cin, dtype=torch.float64)
    ref = torch.einsum("kvw,fvc->fwkc", A, x)  # [F][V][K][Cin]
    Ad, xd = A.float().contiguous().to(d), x.float().contiguous().to(d)
    zf = torch.empty(F, V, K, Cin, device=d)
    z3 = torch.empty(F, V, 2 * K * Cin, device=d, dtype=torch.bfloat16)
    st = L.stream_handle()
    L.check(L.lib().f3_graph_mix_forward_ex(L.ptr(Ad), L.ptr(xd), L.ptr(zf), F, K, V, Cin, 4, st), "mix x3")
    L.check(L.lib().f3_graph_mix_forward_ex(L.ptr(Ad), L.ptr(xd), L.ptr(z3), F, K, V, Cin, 4 | 8, st), "mix z3")
    torch.cuda.synchronize()
    hi, lo = z3[..., :K * Cin].reshape(F, V, K, Cin), z3[..., K * Cin:].reshape(F, V, K, Cin)
    assert torch.equal(hi, zf.to(torch.bfloat16))
    assert torch.equal(lo, (zf - zf.to(torch.bfloat16).float()).to(torch.bfloat16))
    got = (hi.double() + lo.double()).cpu()
    err = float((got - ref).abs().max() / ref.abs().max())
    print(f"mix z3 V={V} K={K} Cin={Cin} F={F}: {err:.2e}")
    assert err <= X3_TOL, err


@pytest.mark.parametrize("V,Cin,F", [(18, 64, 300), (14, 128, 77), (18, 256, 41), (17, 64, 5), (18, 64, 7680)])
@pytest.mark.parametrize("a_bf16", [True, False], ids=["A_bf16", "A_fp32"])
def test_graph_mix_bf16_forward(V, Cin, F, a_bf16):
    """The bf16-mode mix forward (x, Z bf16; bf16 MFMA with A_eff split into bf16 hi + lo, output
    rounded to bf16) against fp64 on the bf16-rounded x: every element within the bf16 rounding of
    the output (2^-8 relative) plus 1e-6 of the max, for a bf16-representable A_eff (the
    reference's autocast einsum rounds it) and a plain fp32 one (the hi + lo split, 2^-17)."""
    d = dev()
    import fall_multimodal_amd._lib as L
    torch.manual_seed(V + Cin)
    K = 3
    A = (torch.rand(K, V, V) / V)
    A = A.to(torch.bfloat16) if a_bf16 else A
    x = torch.randn(F, V, Cin).to(torch.bfloat16)
    ref = torch.einsum("kvw,fvc->fwkc", A.double(), x.double())
    Ad, xd = A.float().contiguous().to(d), x.contiguous().to(d)
    z = torch.empty(F, V, K, Cin, device=d, dtype=torch.bfloat16)
    L.check(L.lib().f3_graph_mix_forward_ex(L.ptr(Ad), L.ptr(xd), L.ptr(z), F, K, V, Cin, 3, L.stream_handle()), "mix")
    got = z.cpu().double()
    # bf16 rounding of the output (<= 2^-9 relative) + the split's |A - hi - lo| <= 2^-16 |A| summed
    # over the joints (it matters only where the sum cancels) + fp32 accumulation
    split = torch.einsum("kvw,fvc->fwkc", A.double().abs(), x.double().abs()) * 2.0 ** -15
    tol = ref.abs() * 2.0 ** -8 + split + 1e-7 * float(ref.abs().max())
    assert bool(((got - ref).abs() <= tol).all()), float(((got - ref).abs() - tol).max())


@pytest.mark.parametrize("V,K,Cin,F", [(18, 3, 64, 300), (14, 3, 128, 77), (18, 3, 256, 41), (17, 1, 64, 5),
                                        (18, 3, 64, 7680)])
@pytest.mark.parametrize("bf16_kernel", [True, False], ids=["bf16mfma", "fp32mfma"])
def test_graph_mix_bf16_backward(V, K, Cin, F, bf16_kernel, monkeypatch):
    """The bf16-mode mix backward (x, dZ bf16; dx fp32, dA fp32) against fp64 on the same bf16
    operands, for the bf16-MFMA kernel (A~ split into bf16 hi + lo: |A~ - hi - lo| <= 2^-17 |A~|)
    and the fp32 16x16x4 kernel (F3_MIX_BWD_BF16=0, a fresh process reads the knob): dx within
    2e-5 of its max, dA (exact bf16 products, fp32 sums over F*Cin terms) within 1e-5 of its max.
    F=7680 is the benchmarked 64-channel layer (B=256, T=30)."""
    d = dev()
    import subprocess
    import sys
    if not bf16_kernel:
        code = (f"import sys; sys.path.insert(0, {os.getcwd()!r}); import tests.test_gpu_parity as t; "
                f"t._mix_bwd_bf16_check({V}, {K}, {Cin}, {F})")
        env = dict(os.environ, F3_MIX_BWD_BF16="0")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        return
    _mix_bwd_bf16_check(V, K, Cin, F, d)


def _mix_bwd_bf16_check(V, K, Cin, F, d=None):
    import fall_multimodal_amd._lib as L
    d = d or torch.device("cuda")
    torch.manual_seed(V * 7 + Cin + F)
    A = torch.rand(K, V, V, dtype=torch.float64) / V            # fp32 A_eff (not bf16-representable)
    A = A.float().double().requires_grad_(True)
    x = torch.randn(F, V, Cin).to(torch.bfloat16).double().requires_grad_(True)
    z = torch.einsum("kvw,fvc->fwkc", A, x)
    dz = torch.randn_like(z).to(torch.bfloat16).double()
    z.backward(dz)
    Ag = A.detach().float().contiguous().to(d)
    xg = x.detach().to(torch.bfloat16).contiguous().to(d)
    dzg = dz.to(torch.bfloat16).contiguous().to(d)
    dx = torch.empty(F, V, Cin, device=d)
    dA = torch.empty(K, V, V, device=d)
    L.check(L.lib().f3_graph_mix_backward_ex(L.ptr(Ag), L.ptr(xg), L.ptr(dzg), L.ptr(dx), L.ptr(dA), F, K, V, Cin, 1,
                                             L.stream_handle()), "mixbwd")
    for got, ref, rel in ((dx, x.grad, 2e-5), (dA, A.grad, 1e-5)):
        r = ref.numpy()
        np.testing.assert_allclose(got.cpu().double().numpy(), r, rtol=0, atol=rel * np.abs(r).max())


@pytest.mark.parametrize("V,K,Cin,F", [(18, 3, 64, 300), (14, 3, 128, 77), (18, 3, 256, 41), (17, 1, 64, 5),
                                        (18, 3, 64, 7680)])
def test_graph_mix_bf16x3_kernels(V, K, Cin, F):
    """The bf16x3 mode's mix forward and backward (fp32 x / z / dz; both operands split into bf16 hi +
    lo, three MFMA products each) against fp64 on the fp32 operands: z, dx, dA within X3_TOL of
    their max (each product carries ~2^-16)."""
    d = dev()
    import fall_multimodal_amd._lib as L
    torch.manual_seed(V * 11 + Cin + F)
    A = (torch.rand(K, V, V, dtype=torch.float64) / V).float().double().requires_grad_(True)
    x = torch.randn(F, V, Cin, dtype=torch.float64).float().double().requires_grad_(True)
    z = torch.einsum("kvw,fvc->fwkc", A, x)
    dz = torch.randn_like(z).float().double()
    z.backward(dz)
    Ag, xg, dzg = (t.detach().float().contiguous().to(d) for t in (A, x, dz))
    zo = torch.empty(F, V, K, Cin, device=d)
    dx = torch.empty(F, V, Cin, device=d)
    dA = torch.empty(K, V, V, device=d)
    L.check(L.lib().f3_graph_mix_forward_ex(L.ptr(Ag), L.ptr(xg), L.ptr(zo), F, K, V, Cin, 4, L.stream_handle()), "mix")
    L.check(L.lib().f3_graph_mix_backward_ex(L.ptr(Ag), L.ptr(xg), L.ptr(dzg), L.ptr(dx), L.ptr(dA), F, K, V, Cin, 4,
                                             L.stream_handle()), "mixbwd")
    errs = {}
    for name, got, ref in (("z", zo, z.detach()), ("dx", dx, x.grad), ("dA", dA, A.grad)):
        r = ref.numpy()
        errs[name] = float(np.abs(got.cpu().double().numpy() - r).max() / np.abs(r).max())
        np.testing.assert_allclose(got.cpu().double().numpy(), r, rtol=0, atol=X3_TOL * np.abs(r).max())
    print(f"bf16x3 mix V={V} K={K} Cin={Cin} F={F}: " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))


# the skeleton cases run in both parity modes; the sensor-only ones (no skeleton GEMMs) in fp32
GOLDEN_CASES = [(t, "fp32") for t in TAGS] + [(t, "bf16x3") for t in ("har", "ns", "two", "stgcn", "ur_nb")]


@pytest.mark.parametrize("tag,precision", GOLDEN_CASES)
def test_train_step_matches_reference_golden(tag, precision):
    """fp32 and bf16x3 paths vs the reference's own outputs (golden, B=4):
    * forward: logits within 1e-3 (north-star gate; measured ~1e-6 fp32), identical argmax, loss;
    * BN running stats after the step;
    * gradients: conditioning-aware (see golden_util.check_grads_conditioned — at B=4 the
      reference's gradients move by up to ~1e-1 under 1e-6 perturbations of its BN outputs). bf16x3's
      products carry ~2^-16 relative error, so its envelope is the oracle's sensitivity to 2^-14
      perturbations (the same probe at a few split ulps, see below) and its running-stat bound 1e-3;
    * RMSprop: post-step parameters exactly as torch.optim.RMSprop would produce from our grads.
    The notebook cases (har / ns: softmax output, ur_nb: the UR CNN1D sensor branch) cover those
    variants in bf16x3 too."""
    d = dev()
    import fall_multimodal_amd as f3
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    g, spec = load(tag)
    st = oc.init_state(spec, int(g["seed"][0]))
    model = build_from_spec(spec, d, precision)
    model.load_state_dict(st, strict=True)
    model.train()
    skel = torch.from_numpy(g["skel"]).to(d)
    sensor = torch.from_numpy(g["sensor"]).to(d)
    label = torch.from_numpy(g["label"]).to(d)
    out = call(model, spec, skel, sensor)
    ref_out = g["out"]
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref_out, rtol=0, atol=1e-3)
    assert (out.detach().cpu().numpy().argmax(1) == ref_out.argmax(1)).all()
    loss = torch.nn.CrossEntropyLoss()(out, label)
    np.testing.assert_allclose(loss.item(), g["loss"][0], rtol=1e-4, atol=1e-5)
    opt = f3.RMSprop(model.parameters(), lr=1e-3)
    opt.zero_grad()
    loss.backward()
    pre = {n: p.detach().cpu().numpy().copy() for n, p in model.named_parameters()}
    grads = {n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters() if p.grad is not None}
    x3 = precision == "bf16x3"
    # bf16x3: the products carry ~2^-16 relative error and a K-term GEMM sum carries several of them;
    # at B=4 a ReLU kink next to the data flips under errors of that size (a flip moved layer-4's
    # channel-attention weight gradient by 0.135 of its max in one of two identical runs against a
    # 2^-16 envelope of 0.008), so the probe is 2^-14 (four split ulps)
    env = oc.gradient_sensitivity(st, spec, *(torch.from_numpy(g[k]) for k in ("skel", "sensor", "label")),
                                  eps=2.0 ** -14 if x3 else 1e-6, trials=5, per_param=True)
    dlogit = float(np.abs(out.detach().cpu().numpy() - ref_out).max())
    cosg = check_grads_conditioned(g, grads, env, what=f"{tag} {precision}")
    _record("golden_train_step", {"tag": tag, "precision": precision, "max_abs_dlogit": dlogit, "grad_cosine": cosg})
    opt.step()
    for name, p in model.named_parameters():
        if name not in grads:
            continue
        gg = grads[name].astype(np.float64)
        sq = 0.01 * gg * gg
        expect = pre[name] - 1e-3 * gg / (np.sqrt(sq) + 1e-8)
        np.testing.assert_allclose(p.detach().cpu().numpy(), expect, rtol=0, atol=2e-6, err_msg=name)
    sd = model.state_dict()
    for name, b in sd.items():
        if name.endswith(("running_mean", "running_var")):
            check_packed(g, "buf:" + name, b.cpu().numpy(), rtol=1e-3 if x3 else 1e-4, atol=1e-5, what=tag + " ")
        if name.endswith("num_batches_tracked"):
            assert int(b) == 1, name


def test_gradient_accumulation_keeps_flat_rmsprop():
    """model/main.py:115-132 accumulates loss.backward() over accum_iter batches before
    optimizer.step(). Two backwards through fall3::net_backward add into the same .grad views
    (autograd accumulates in place), the flat RMSprop path still applies (one launch over the flat
    range), and the update equals torch.optim.RMSprop on the summed gradient."""
    d = dev()
    import fall_multimodal_amd as f3
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    st = oc.init_state(spec, 9)
    b1 = [torch.from_numpy(x).to(d) for x in synthetic_batch(64, 18, 11, 6, 31)]
    b2 = [torch.from_numpy(x).to(d) for x in synthetic_batch(64, 18, 11, 6, 32)]
    loss_fn = torch.nn.CrossEntropyLoss()

    def grads_of(batch):
        m = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d)
        m.load_state_dict(st)
        loss_fn(m(batch[0], batch[1]), batch[2]).backward()
        return [p.grad.detach().clone() for p in m.parameters()]
    g1, g2 = grads_of(b1), grads_of(b2)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d)
    model.load_state_dict(st)
    params = list(model.parameters())
    opt = f3.RMSprop(params, lr=1e-3)
    opt.zero_grad()
    loss_fn(model(b1[0], b1[1]), b1[2]).backward()
    first = [p.grad for p in params]
    loss_fn(model(b2[0], b2[1]), b2[2]).backward()
    for p, f in zip(params, first):
        assert p.grad is f or p.grad.data_ptr() == f.data_ptr()   # accumulated in place
    # the separate runs differ only by float-atomic ordering noise (chaotic at this batch size per
    # tensor, tiny on the whole gradient)
    acc = torch.cat([p.grad.reshape(-1) for p in params]).double()
    ref_sum = torch.cat([(a + b).reshape(-1) for a, b in zip(g1, g2)]).double()
    cos = float(acc @ ref_sum / (acc.norm() * ref_sum.norm()))
    assert cos > 0.9999, cos
    assert abs(float(acc.norm() / ref_sum.norm()) - 1) < 1e-3
    assert opt._flat(opt.param_groups[0]) is not None
    twins = [p.detach().clone().requires_grad_(True) for p in params]
    for t, p in zip(twins, params):
        t.grad = p.grad.detach().clone()
    ref = torch.optim.RMSprop(twins, lr=1e-3)
    opt.step()
    ref.step()
    for p, t in zip(params, twins):
        torch.testing.assert_close(p.detach(), t.detach(), rtol=1e-6, atol=1e-7)


def test_rmsprop_flat_path_matches_torch():
    """f3.RMSprop's one-launch flat path (parameters, autograd gradients and square_avg states
    all views of one buffer each) gives torch.optim.RMSprop's parameters over 3 steps, and the
    per-tensor path (states not laid out flat) gives the same."""
    d = dev()
    import fall_multimodal_amd as f3
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    st = oc.init_state(spec, 5)
    batch = [torch.from_numpy(x).to(d) for x in synthetic_batch(8, 18, 11, 6, 17)]
    for mode in ("flat", "per_tensor"):
        model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d)
        model.load_state_dict(st)
        params = list(model.parameters())
        opt = f3.RMSprop(params, lr=1e-3)
        if mode == "per_tensor":  # pre-made states in their own storage: not flat
            for p in params:
                opt.state[p]["square_avg"] = torch.zeros_like(p)
                opt.state[p]["step"] = torch.zeros((), dtype=torch.float32)
        # torch.optim.RMSprop on copies, fed the same gradients each step
        twins = [p.detach().clone().requires_grad_(True) for p in params]
        ref_opt = torch.optim.RMSprop(twins, lr=1e-3)
        for _ in range(3):
            opt.zero_grad()
            torch.nn.CrossEntropyLoss()(model(batch[0], batch[1]), batch[2]).backward()
            assert (opt._flat(opt.param_groups[0]) is not None) == (mode == "flat"), mode
            for p, t in zip(params, twins):
                t.grad = p.grad.detach().clone()
            opt.step()
            ref_opt.step()
            for p, t in zip(params, twins):
                torch.testing.assert_close(p.detach(), t.detach(), rtol=1e-6, atol=1e-7)
                p.data.copy_(t.detach())  # keep both sides on identical values
        if mode == "flat":
            sq = [opt.state[p]["square_avg"] for p in params]
            assert len({s.untyped_storage().data_ptr() for s in sq}) == 1
            assert int(opt.state[params[0]]["step"]) == 3


@pytest.mark.parametrize("precision", ["bf16x3", "fp32", "bf16"])
def test_backward_rmsprop_per_layer_updates(precision):
    """TrainStep at world 1 runs f3_net_backward_rmsprop: each skeleton layer's RMSprop update is
    issued on the queue that finishes its gradients, the rest after the join. Over two steps the
    parameters and square_avg must equal torch's RMSprop arithmetic applied to the step's own
    gradients (step.grads) from the previous state - every parameter updated exactly once."""
    d = dev()
    import fall_multimodal_amd as f3
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    st = oc.init_state(spec, 9)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d,
                                      precision=precision)
    model.load_state_dict(st)
    B, lr, alpha, eps = 32, 1e-3, 0.99, 1e-8
    step = f3.TrainStep(model, B, lr=lr)
    assert step.fused_optimizer
    for k in range(2):
        sk, se, lb = (torch.from_numpy(x).to(d) for x in synthetic_batch(B, 18, 11, 6, 40 + k))
        p0 = model.flat_parameters().detach().clone()
        sq0 = step.square_avg.clone()
        step(sk, se, lb)
        torch.cuda.synchronize()
        g = step.grads
        sq = alpha * sq0 + (1 - alpha) * g * g
        p = p0 - lr * g / (sq.sqrt() + eps)
        # (a contracted multiply-add in the kernel: ~1 ulp from torch's separately rounded ops)
        torch.testing.assert_close(step.square_avg, sq, rtol=1e-5, atol=1e-12)
        torch.testing.assert_close(model.flat_parameters().detach(), p, rtol=1e-6, atol=1e-7)
        if k == 0:  # from square_avg = 0 every update is ~lr in size: nothing may be skipped
            moved = (model.flat_parameters().detach() != p0) | (g == 0)
            assert bool(moved.all()), int((~moved).sum())


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
@pytest.mark.parametrize("layout,S,B", [("coco_mmpose", 6, 32), ("coco_cut", 15, 24), ("coco_mmpose", 6, 13)])
def test_fused_train_step_vs_oracle(layout, S, B, precision):
    """TrainStep (native fwd + CE + bwd + RMSprop) vs the CPU oracle at a larger batch: the HAR
    layout (V=14, S=15; the motion stream's T=29 and the V=14 tilings of the native split-form kernels)
    and a ragged batch (B=13). Logits within 1e-3 with identical argmax, gradients conditioning-aware
    (bf16x3: envelope at the split's 2^-16)."""
    d = dev()
    import fall_multimodal_amd as f3
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    spec = oc.Spec(model="two_stgcan_bilstm", layout=layout, num_class=11, sensor_dim=S)
    st = oc.init_state(spec, 77)
    V = 18 if layout == "coco_mmpose" else 14
    skel, sensor, label = synthetic_batch(B, V, 11, S, 5)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": layout, "strategy": "spatial"}, 11, S, device=d,
                                      precision=precision)
    model.load_state_dict(st)
    step = f3.TrainStep(model, B, lr=1e-3)
    loss = step(torch.from_numpy(skel).to(d), torch.from_numpy(sensor).to(d), torch.from_numpy(label).to(d))
    out_ref, loss_ref, grads_ref = oc.train_step(st, spec, *(torch.from_numpy(x) for x in (skel, sensor, label)))
    np.testing.assert_allclose(step.out.cpu().numpy(), out_ref.numpy(), atol=1e-3, rtol=0)
    assert (step.out.cpu().numpy().argmax(1) == out_ref.numpy().argmax(1)).all()
    np.testing.assert_allclose(loss.item(), loss_ref.item(), rtol=1e-4)
    env = oc.gradient_sensitivity(oc.init_state(spec, 77), spec, *(torch.from_numpy(x) for x in (skel, sensor, label)),
                                  eps=2.0 ** -16 if precision == "bf16x3" else 1e-6, trials=3, per_param=True)
    fake = {"grad:" + k: v.numpy().reshape(-1) for k, v in grads_ref.items()}
    ours = {name: p.grad.detach().cpu().numpy() for (name, shape, off), p in zip(model.param_views(), model.parameters())}
    cosg = check_grads_conditioned(fake, ours, env, what=f"{layout} B={B} {precision}")
    _record("fused_train_step_vs_oracle", {"layout": layout, "S": S, "B": B, "precision": precision,
                                           "max_abs_dlogit": float(np.abs(step.out.cpu().numpy() - out_ref.numpy()).max()),
                                           "grad_cosine": cosg})


@pytest.mark.parametrize("tag,precision", [(t, "fp32") for t in ("har", "ur_nb", "stgcn", "bilstm", "ur_sensor")]
                         + [("har", "bf16x3"), ("stgcn", "bf16x3")])
def test_workspace_poison_no_uninitialized_reads(tag, precision):
    """Every workspace byte a step reads must have been written by that step: with the
    workspace pre-filled with NaN (0xFF) or huge (0x7F) bytes the outputs and gradients
    must stay finite, the forward identical to a zero-filled run, the gradients the same
    up to this model's fp32 conditioning (cosine)."""
    d = dev()
    g, spec = load(tag)
    st = oc.init_state(spec, int(g["seed"][0]))
    model = build_from_spec(spec, d, precision)
    skel = torch.from_numpy(g["skel"]).to(d)
    sensor = torch.from_numpy(g["sensor"]).to(d)
    N, C = skel.shape[0], spec.num_class
    dout = torch.randn(N, C, generator=torch.Generator().manual_seed(3)).to(d)
    res = []
    for fill in (0x00, 0xFF, 0x7F):
        model.load_state_dict(st)
        ws = torch.full((model._native.workspace_bytes(N),), fill, dtype=torch.uint8, device=d)
        out = torch.empty(N, C, device=d)
        sk = None if spec.model == "bilstm" else skel
        se = sensor if spec.model in ("bilstm", "two_stgcan_bilstm") else None
        model.native_forward(sk, se, out, ws, True)
        grads = torch.full((model._native.nparam,), float("nan"), device=d)
        model.native_backward(N, dout, grads, ws)
        torch.cuda.synchronize()
        assert torch.isfinite(out).all(), f"fill {fill:#x}: non-finite output"
        assert torch.isfinite(grads).all(), f"fill {fill:#x}: non-finite gradients"
        res.append((out.cpu().double(), grads.cpu().double()))
    for o, gr in res[1:]:
        torch.testing.assert_close(o, res[0][0], rtol=1e-5, atol=1e-5)
        cos = float(gr @ res[0][1] / (gr.norm() * res[0][1].norm()))
        assert cos > 0.999, cos


def _train_gpu(st, layout, S, precision, batches, d, steps, evaluate=None, checkpoints=()):
    """Train `steps` RMSprop steps through TrainStep; evaluate(model) at each checkpoint."""
    import fall_multimodal_amd as f3
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": layout, "strategy": "spatial"}, 11, S, device=d,
                                      precision=precision)
    model.load_state_dict(st)
    B = batches[0][0].shape[0]
    step = f3.TrainStep(model, B, lr=1e-3)
    evals = []
    for i in range(steps):
        step(*(torch.from_numpy(x).to(d) for x in batches[i % len(batches)]))
        if i + 1 in checkpoints:
            evals.append(evaluate(model))
    return model, evals


def test_bf16_step_tracks_oracle():
    """bf16 mode (activations stored bf16, GEMM operands bf16, fp32 accumulate): one step vs the
    fp32 oracle. This is the fast, lower-precision mode, not a parity mode (the parity modes, bf16x3 --
    the default and the headline -- and fp32, are held to logits within 1e-3 elsewhere in this file).
    Bounds, measured on MI355X with margin: logits within 3e-2 of the oracle's, same argmax on >= 95 %
    of clips, whole-model gradient cosine >= 0.99."""
    d = dev()
    import fall_multimodal_amd as f3
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    layout, S, B = "coco_mmpose", 6, 64
    spec = oc.Spec(model="two_stgcan_bilstm", layout=layout, num_class=11, sensor_dim=S)
    st = oc.init_state(spec, 91)
    batch = synthetic_batch(B, 18, 11, S, 9)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": layout, "strategy": "spatial"}, 11, S, device=d,
                                      precision="bf16")
    model.load_state_dict(st)
    step = f3.TrainStep(model, B, lr=1e-3)
    step(*(torch.from_numpy(x).to(d) for x in batch))
    out_ref, loss_ref, grads_ref = oc.train_step(st, spec, *(torch.from_numpy(x) for x in batch))
    out = step.out.cpu()
    err = (out - out_ref).abs().max().item()
    agree = (out.argmax(1) == out_ref.argmax(1)).double().mean().item()
    ours = torch.cat([p.grad.detach().cpu().reshape(-1) for p in model.parameters()]).double()
    names = [n for n, _ in model.named_parameters()]
    ref = torch.cat([grads_ref[n].reshape(-1) if n in grads_ref else torch.zeros_like(p.grad.cpu()).reshape(-1)
                     for n, p in zip(names, model.parameters())]).double()
    cos = float(ours @ ref / (ours.norm() * ref.norm()))
    print(f"bf16 vs oracle: logits max err {err:.3e}, argmax agreement {agree:.3f}, grad cosine {cos:.5f}, "
          f"loss {step.loss.item():.6f} vs {loss_ref.item():.6f}")
    assert err < 3e-2
    assert agree >= 0.95
    assert cos >= 0.99
    assert abs(step.loss.item() - loss_ref.item()) < 1e-2


@pytest.mark.slow
def test_top1_accuracy_parity():
    """BASELINE metric's 'top-1 acc parity': the oracle (reference algorithm, CPU fp32), the
    fp32 HIP path and the bf16 HIP path trained identically (same init, same 8 synthetic
    batches cycled for 48 RMSprop steps, B=32), held-out top-1 accuracy on 256 fresh clips
    averaged over the checkpoints after 24, 30, 36, 42 and 48 steps.

    Two read-outs per checkpoint:
    * batch-statistics accuracy (BN normalising over the 256 held-out clips): what the
      network has learned, independent of the running-statistics lag — gated within 6 points;
    * eval-mode accuracy (BN running statistics, the reference's test-loop protocol) —
      gated within 15 points. At this horizon it is dominated by the running statistics
      (momentum 0.1) trailing weights that still move ~lr per step: single checkpoints swing
      by ~10 points between neighbouring steps, with the CPU's thread count alone, and
      between two runs of the SAME fp32 GPU path (its float atomics reorder sums): measured
      on MI355X, fp32 [0.199, 0.273, 0.348] in one run and [0.434, 0.348, 0.309] in another
      against the oracle's [0.188, 0.277, 0.340] at steps 36/42/48.
    The batch-statistics read-out runs on copies of the BN buffers, so it does not perturb the
    running statistics the eval-mode read-out and the next steps see. Chance is 0.09."""
    d = dev()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    layout, S, B, steps, nb = "coco_mmpose", 6, 32, 48, 8
    checkpoints = (24, 30, 36, 42, 48)
    spec = oc.Spec(model="two_stgcan_bilstm", layout=layout, num_class=11, sensor_dim=S)
    batches = [synthetic_batch(B, 18, 11, S, 500 + i) for i in range(nb)]
    test_sk, test_se, test_lb = synthetic_batch(256, 18, 11, S, 999)
    truth = test_lb.argmax(1)
    st = oc.init_state(spec, 123)
    sq = {k: torch.zeros_like(v) for k, v in st.items() if not oc.is_buffer(k)}
    ref = {"eval": [], "batch": []}
    tsk, tse = torch.from_numpy(test_sk), torch.from_numpy(test_se)
    for i in range(steps):
        oc.train_step(st, spec, *(torch.from_numpy(x) for x in batches[i % nb]), sq=sq)
        if i + 1 in checkpoints:
            with torch.no_grad():
                out = oc.forward(st, spec, tsk, tse, training=False)
                ref["eval"].append(float((out.argmax(1).numpy() == truth).mean()))
                scratch = {k: (v.clone() if oc.is_buffer(k) else v) for k, v in st.items()}
                out = oc.forward(scratch, spec, tsk, tse, training=True)
                ref["batch"].append(float((out.argmax(1).numpy() == truth).mean()))
    sk_d, se_d = tsk.to(d), tse.to(d)

    def evaluate(model):
        res = {}
        with torch.no_grad():
            model.eval()
            res["eval"] = float((model(sk_d, se_d).argmax(1).cpu().numpy() == truth).mean())
            model.train()
            saved = (model._flat_buffers.clone(), model._flat_counters.clone())
            res["batch"] = float((model(sk_d, se_d).argmax(1).cpu().numpy() == truth).mean())
            model._flat_buffers.copy_(saved[0])
            model._flat_counters.copy_(saved[1])
        return res

    got, same_weights = {}, {}
    for prec in ("fp32", "bf16x3", "bf16"):
        model, ev = _train_gpu(oc.init_state(spec, 123), layout, S, prec, batches, d, steps, evaluate, checkpoints)
        got[prec] = {k: [e[k] for e in ev] for k in ("eval", "batch")}
        # SURVEY §8(d)'s +-0.5 % top-1 bar, on the weights the HIP path trained: the oracle's
        # eval-mode and batch-statistics forwards of the SAME state give the same held-out top-1
        # (the trajectories themselves diverge chaotically, as two runs of one path do, see above)
        trained = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
        with torch.no_grad():
            o_eval = oc.forward(trained, spec, tsk, tse, training=False)
            scratch = {k: (v.clone() if oc.is_buffer(k) else v) for k, v in trained.items()}
            o_batch = oc.forward(scratch, spec, tsk, tse, training=True)
        same_weights[prec] = {"eval": float((o_eval.argmax(1).numpy() == truth).mean()),
                              "batch": float((o_batch.argmax(1).numpy() == truth).mean())}
    print(f"held-out top-1 at steps {checkpoints}: oracle {ref}, fp32 {got['fp32']}, bf16x3 {got['bf16x3']}, "
          f"bf16 {got['bf16']}; "
          f"oracle forward of the HIP-trained weights at step {steps}: {same_weights}")
    _record("top1_accuracy_parity", {"checkpoints": list(checkpoints), "oracle": ref, "hip": got,
                                     "oracle_on_hip_weights_final": same_weights})
    # the HIP path's own forward vs the fp32 oracle's on the same weights: fp32 within SURVEY
    # §8(d)'s 0.5 % (measured identical); bf16 GEMM operands flip near-tie argmaxes of this
    # half-trained network (measured 2 of 256 clips in the batch-statistics read-out), gated at 3
    top1_gate = {"fp32": 0.005, "bf16x3": 0.005, "bf16": 3.0 / 256}
    for prec in got:
        for k in ("eval", "batch"):
            assert abs(got[prec][k][-1] - same_weights[prec][k]) <= top1_gate[prec], (
                prec, k, got[prec][k][-1], same_weights[prec][k])
    assert np.mean(ref["batch"]) > 2.0 / 11 and np.mean(ref["eval"]) > 1.5 / 11  # learnable in this budget
    bound = {"batch": 0.06, "eval": 0.15}
    for prec, r in got.items():
        for k, b in bound.items():
            assert abs(float(np.mean(r[k])) - float(np.mean(ref[k]))) <= b, (prec, k, r[k], ref[k])


def test_top1_at_convergence():
    """SURVEY §8(d)'s accuracy parity at convergence: the oracle (CPU restatement of the reference),
    the fp32, bf16x3 (the benchmarked mode) and bf16 HIP paths train the SAME recipe to a plateau — 400 RMSprop steps,
    B=32, fresh separable synthetic batches, cosine learning rate 1e-3 -> 0 (the reference's
    CosineLRScheduler), tools/gen_convergence.py — and their held-out top-1 (1024 clips) is compared
    at the end. The oracle's run is recorded in tests/golden/convergence.json (regenerated by that
    script; ~10 CPU minutes, so not repeated here).

    Two read-outs: batch statistics (BN over the 1024 held-out clips: what the network learned; the
    oracle reaches 99.8 %) and eval mode (BN running statistics, the reference's valid/test protocol;
    the oracle ends at 97.9 %: the running statistics of B=32 batch-norms, incl. the channel
    attention's BN over the 32 clips, trail the weights). The trajectories of any two
    implementations diverge chaotically step by step (float-atomic order alone does it: the fp32 HIP
    path is trained twice to show its own run-to-run spread), so the gates are on the plateau:
    batch-statistics top-1 within 0.5 % of the oracle's (fp32, bf16x3) / 1 % (bf16), eval-mode top-1 within
    2 % (both), recorded in profiles/r03_parity_record.jsonl."""
    import json
    d = dev()
    import fall_multimodal_amd as f3
    with open(os.path.join(os.path.dirname(__file__), "golden", "convergence.json")) as f:
        fx = json.load(f)
    r = fx["recipe"]
    kw = dict(separation=r["separation"], spread=r["spread"])
    spec = oc.Spec(model=r["model"], layout=r["layout"], num_class=r["classes"], sensor_dim=r["S"])
    tsk, tse, tlb = synthetic_batch(r["heldout"], r["V"], r["classes"], r["S"], r["heldout_seed"], **kw)
    truth = tlb.argmax(1)
    sk_d, se_d = torch.from_numpy(tsk).to(d), torch.from_numpy(tse).to(d)

    def train(prec):
        model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": r["layout"], "strategy": "spatial"}, r["classes"], r["S"],
                                          device=d, precision=prec)
        model.load_state_dict(oc.init_state(spec, r["init_seed"]))
        step = f3.TrainStep(model, r["batch"], lr=r["lr0"])
        res = {}
        for i in range(r["steps"]):
            step.lr = 0.5 * r["lr0"] * (1 + np.cos(np.pi * i / r["steps"]))
            step(*(torch.from_numpy(x).to(d) for x in synthetic_batch(r["batch"], r["V"], r["classes"], r["S"],
                                                                       r["batch_seed0"] + i, **kw)))
            if i + 1 in r["checkpoints"]:
                with torch.no_grad():
                    model.eval()
                    ev = float((model(sk_d, se_d).argmax(1).cpu().numpy() == truth).mean())
                    model.train()
                    saved = (model._flat_buffers.clone(), model._flat_counters.clone())
                    bt = float((model(sk_d, se_d).argmax(1).cpu().numpy() == truth).mean())
                    model._flat_buffers.copy_(saved[0])
                    model._flat_counters.copy_(saved[1])
                res[str(i + 1)] = {"eval": ev, "batch": bt}
        _progress(f"top1_at_convergence: {prec} done")
        return res
    got = {"fp32": train("fp32"), "fp32_rerun": train("fp32"), "bf16x3": train("bf16x3"), "bf16": train("bf16")}
    ref = fx["oracle"]
    last = str(r["steps"])
    _record("top1_at_convergence", {"oracle": ref, "hip": got, "heldout": r["heldout"], "recipe": r})
    print(f"held-out top-1 at {r['checkpoints']}: oracle {ref}, HIP {got}")
    assert ref[last]["batch"] > 0.95, ref          # the recipe converges
    gate = {"fp32": {"batch": 0.005, "eval": 0.02}, "fp32_rerun": {"batch": 0.005, "eval": 0.02},
            "bf16x3": {"batch": 0.005, "eval": 0.02}, "bf16": {"batch": 0.01, "eval": 0.02}}
    for run, g in gate.items():
        for k, b in g.items():
            assert abs(got[run][last][k] - ref[last][k]) <= b, (run, k, got[run][last][k], ref[last][k])


def test_eval_step_and_loader_match_oracle():
    """SURVEY §8f rows 1-2 on the device: the pinned, double-buffered WindowLoader feeds the
    eval step (fall_multimodal_amd.evaluate.test: eval-mode forward through the BN running
    statistics, top-k, macro P/R/F1) and the result equals the oracle's eval-mode forward on
    the same windows: logits within 1e-3 (fp32 mode), identical argmax and top-k."""
    d = dev()
    import fall_multimodal_amd as f3
    from fall_multimodal_amd import data as fd
    from fall_multimodal_amd import evaluate as fe
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    st = oc.init_state(spec, 31)
    # non-trivial running statistics (as after training): one oracle train-mode forward
    with torch.no_grad():
        oc.forward(st, spec, *(torch.from_numpy(x) for x in synthetic_batch(64, 18, 11, 6, 20)[:2]), training=True)
    skel, sensor, label = synthetic_batch(80, 18, 11, 6, 21)
    w = fd.Windows([f"v{i // 4}" for i in range(80)], np.ascontiguousarray(skel.transpose(0, 2, 3, 1)), sensor, label)
    loader = fd.WindowLoader(w, 32, shuffle=False, drop_last=False, device=d)
    got = [b for b in loader]
    assert [b[0].shape[0] for b in got] == [32, 32, 16]
    np.testing.assert_array_equal(torch.cat([b[0] for b in got]).cpu().numpy(), skel)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d)
    model.load_state_dict(st)
    out, _ = fe.predict(model, loader)
    with torch.no_grad():
        ref = oc.forward(st, spec, torch.from_numpy(skel), torch.from_numpy(sensor), training=False).numpy()
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=1e-3, rtol=0)
    assert (out.cpu().numpy().argmax(1) == ref.argmax(1)).all()
    res = fe.test(model, loader, torch.nn.CrossEntropyLoss(), top_k=(1, 5), num_classes=11)
    assert res["top_k"] == fe.cal_top_k_accuracy(torch.from_numpy(ref), torch.from_numpy(label), (1, 5))
    ref_m = fe.class_metrics(ref.argmax(1), label.argmax(1), 11)
    assert (res["precision"], res["recall"], res["f1"]) == (ref_m["precision"], ref_m["recall"], ref_m["f1"])


def _flat_grad_errors(model, grads_ref):
    """Per-tensor max |g - g_ref| / max |g_ref| and the whole-gradient cosine."""
    rel, a_all, r_all = {}, [], []
    for n, p in model.named_parameters():
        g = p.grad.detach().cpu().double().reshape(-1)
        r = grads_ref[n].double().reshape(-1) if n in grads_ref else torch.zeros_like(g)
        a_all.append(g)
        r_all.append(r)
        if n in grads_ref and float(r.abs().max()) > 0:
            rel[n] = float((g - r).abs().max() / r.abs().max())
    a, r = torch.cat(a_all), torch.cat(r_all)
    return rel, float(a @ r / (a.norm() * r.norm()))


def _record(name, values):
    """Append measured parity numbers to gpurun_out/parity_record.jsonl (copied to profiles/)."""
    import json
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "parity_record.jsonl"), "a") as f:
        f.write(json.dumps({"test": name, **values}) + "\n")


# tensors whose true gradient is ~0 (a bias feeding a train-mode BatchNorm): excluded from the
# per-tensor relative gate, covered by the cosine
_ZERO_GRAD = ("tcn.2.bias", "residual.0.bias", "atten.1.bias", "gcn.conv.bias")


_B256_ORACLE = {}


def _b256_oracle(seed, x3_env=False):
    """fp64 / fp32 oracle runs of the bench's configuration (B=256, V=18, S=6, 11 classes) for one seed
    pair (init seed, batch seed) = (seed, seed + 1), cached across tests (each fp64 step is ~10-20 s of
    host CPU). x3_env adds the per-tensor sensitivity envelope at 2^-16 (the bf16x3 gate)."""
    key = seed
    if key not in _B256_ORACLE:
        layout, S, B = "coco_mmpose", 6, 256
        spec = oc.Spec(model="two_stgcan_bilstm", layout=layout, num_class=11, sensor_dim=S)
        st = oc.init_state(spec, seed)
        batch = synthetic_batch(B, 18, 11, S, seed + 1)
        _progress(f"b256 oracle seed {seed}: fp64")
        st64 = {k: (v.double() if v.dtype == torch.float32 else v.clone()) for k, v in st.items()}
        out64, loss64, g64 = oc.train_step(st64, spec, *(torch.from_numpy(x).double() for x in batch))
        _progress(f"b256 oracle seed {seed}: fp32")
        _, _, g32 = oc.train_step({k: v.clone() for k, v in st.items()}, spec, *(torch.from_numpy(x) for x in batch))
        e32s = {}
        for n, r in g64.items():
            m = float(r.abs().max())
            if m > 0:
                e32s[n] = float((g32[n].double() - r).abs().max()) / m
        _B256_ORACLE[key] = {"spec": spec, "st": st, "batch": batch, "out64": out64, "loss64": float(loss64),
                             "g64": g64, "e32s": e32s, "env": None}
    o = _B256_ORACLE[key]
    if x3_env and o["env"] is None:
        # the split-bf16 products carry ~2^-16 relative error (fp32: 2^-24); the network's own
        # sensitivity to errors of that size - every BatchNorm / pooling output of the fp64 oracle
        # perturbed by 2^-16 relative noise, max over four draws - is the per-tensor envelope
        _progress(f"b256 oracle seed {seed}: 2^-16 envelope")
        o["env"] = oc.gradient_sensitivity(o["st"], o["spec"], *(torch.from_numpy(x) for x in o["batch"]),
                                           eps=2.0 ** -16, trials=4, per_param=True, base=o["g64"])
    return o


# the bf16x3 per-tensor gate: rel <= 8 env (the golden tests' conditioning factor, tests/golden_util.py)
# + 16 x the fp32 oracle's own error (the fp32 mode's gate); required margin: the worst tensor within
# X3_GATE_MARGIN of it on every seed (<= 0.7)
X3_GATE_MARGIN = 0.7
B256_SEEDS = (256, 1256, 2256)


def _x3_gate(rel_gated, o):
    x3ratio = {n: rel_gated[n] / (8.0 * o["env"].get(n, 0.0) + 16.0 * max(o["e32s"][n], 2.5e-4))
               for n in rel_gated if n in o["e32s"]}
    wx = max(x3ratio, key=x3ratio.get)
    return x3ratio, wx


@pytest.mark.parametrize("precision,seed", [("fp32", 256), ("bf16", 256)] + [("bf16x3", s) for s in B256_SEEDS])
def test_benchmarked_config_parity(precision, seed):
    """The bench's own configuration — TrainStep at B=256, V=18 (coco_mmpose), S=6, 11 classes —
    against the oracle run in fp64 (the reference's arithmetic without rounding) and in fp32.

    The gradient tolerance is per tensor and flat in the sense of needing no perturbation probe:
    the HIP error against fp64 must stay within 16x the oracle's OWN fp32-vs-fp64 error on that
    tensor, floored at 2.5e-4 of its max (so the gate is never tighter than 4e-3 relative: the
    HIP path's float-atomic reduction order varies run to run — two identical fp32 backward passes
    differ by ~1e-3 of max at small batch (tools/phase_check.py) — so the worst ratio is itself
    noisy: measured 6.1 and 8.7 on two runs, the latter on layer-2 tcn.2.weight, 8.1e-3 vs the
    oracle's 9.4e-4). The weights feeding a train-mode BatchNorm have gradients that
    are differences of nearly cancelling sums: measured on MI355X, the fp32 oracle itself is off by
    1.3e-2 of max|g| on stgcan_2 layer-5 residual.0.weight, and the HIP path by the same 1.3e-2
    (ratio 1.0; worst ratio over all tensors 6.2). Biases feeding a train-mode BN (true gradient
    ~1e-17) are covered by the cosine only. fp32 also: logits within 1e-3 (measured 7e-7),
    identical argmax, cosine >= 0.99999 (measured 0.9999998). bf16 gates ~2x the measured values
    (profiles/r02_parity_record.jsonl). bf16x3 (split-bf16 GEMMs on fp32 activations, the
    bench's parity mode), over three seeds: the north star's 1e-3 logits with identical argmax, cosine
    > 0.99999, and every gradient tensor within X3_GATE_MARGIN of 8x the network's own sensitivity to
    2^-16 relative errors (the split's precision) plus 16x the fp32 oracle's error."""
    d = dev()
    import fall_multimodal_amd as f3
    torch.set_num_threads(min(32, os.cpu_count() or 1))
    layout, S, B = "coco_mmpose", 6, 256
    o = _b256_oracle(seed, x3_env=precision == "bf16x3")
    st, batch, out64, loss64, g64 = o["st"], o["batch"], o["out64"], o["loss64"], o["g64"]
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": layout, "strategy": "spatial"}, 11, S, device=d,
                                      precision=precision)
    model.load_state_dict(st)
    step = f3.TrainStep(model, B, lr=1e-3)
    step(*(torch.from_numpy(x).to(d) for x in batch))
    out = step.out.cpu().double()
    err = float((out - out64).abs().max())
    agree = float((out.argmax(1) == out64.argmax(1)).double().mean())
    rel, cos = _flat_grad_errors(model, g64)
    gated = {k: v for k, v in rel.items() if not k.endswith(_ZERO_GRAD)}
    worst = max(gated, key=gated.get)
    rec = {"precision": precision, "seed": seed, "B": B, "max_abs_dlogit": err, "argmax_agreement": agree,
           "grad_cosine": cos, "worst_grad_rel": gated[worst], "worst_grad_tensor": worst,
           "loss": float(step.loss.item()), "loss_ref": loss64}
    if precision in ("fp32", "bf16x3"):
        ratio = {n: gated[n] / max(o["e32s"][n], 2.5e-4) for n in gated if n in o["e32s"]}
        wr = max(ratio, key=ratio.get)
        rec.update({"worst_ratio_to_oracle_fp32": ratio[wr], "worst_ratio_tensor": wr})
    if precision == "bf16x3":
        x3ratio, wx = _x3_gate(gated, o)
        rec.update({"worst_x3_gate_ratio": x3ratio[wx], "worst_x3_gate_tensor": wx,
                    "env_of_worst": o["env"].get(wx, 0.0), "rel_of_worst": gated[wx],
                    "top5_x3_gate": sorted(((round(v, 3), n) for n, v in x3ratio.items()), reverse=True)[:5]})
    _record("benchmarked_config_parity", rec)
    print(rec)
    if precision == "fp32":
        assert err < 1e-3 and agree == 1.0
        assert ratio[wr] <= 16.0, (wr, ratio[wr])
        assert cos > 0.99999
    elif precision == "bf16x3":
        assert err < 1e-3 and agree == 1.0
        assert x3ratio[wx] <= X3_GATE_MARGIN, (wx, x3ratio[wx])
        assert cos > 0.99999
    else:
        assert err < BF16_B256_LOGIT_GATE and agree >= BF16_B256_ARGMAX_GATE
        assert cos >= BF16_B256_COS_GATE
        assert abs(float(step.loss.item()) - float(loss64)) < 2e-3


def test_main_py_autograd_path_bf16x3_vs_oracle():
    """The reference's own loop body, unchanged (model/main.py:97-132): model = build_model(config) with
    ONE argument (so the default bf16x3 mode), pred = model(data, sensor) through the fall3 custom ops,
    loss = CrossEntropyLoss()(pred, label), loss.backward(), optimizer.step() with f3.RMSprop — at the
    bench's B=256 against the fp64 oracle with test_benchmarked_config_parity's bf16x3 gates, and the
    update equal to torch.optim.RMSprop's arithmetic on the autograd gradients."""
    d = dev()
    import fall_multimodal_amd as f3
    from fall_multimodal_amd.config import get_cfg_defaults
    torch.set_num_threads(min(32, os.cpu_count() or 1))
    seed = B256_SEEDS[0]
    o = _b256_oracle(seed, x3_env=True)
    cfg = get_cfg_defaults()
    cfg.merge_from_dict({"MODEL": {"NAME": "two_stgcan_bilstm"}, "GRAPH": {"LAYOUT": "coco_mmpose", "STRATEGY": "spatial"},
                         "DATA": {"NUM_CLASSES": 11, "SENSOR_DIM": 6}})
    if "F3_PRECISION" in os.environ:
        pytest.skip("F3_PRECISION overrides the default mode")
    model = f3.build_model(cfg, device=d)
    assert model.precision == "bf16x3" and model.spec.precision is None
    model.load_state_dict(o["st"])
    model.train()
    opt = f3.RMSprop(model.parameters(), lr=1e-3)
    skel, sensor, label = (torch.from_numpy(x).to(d) for x in o["batch"])
    opt.zero_grad()
    pred = model(skel, sensor)
    loss = torch.nn.CrossEntropyLoss()(pred, label)
    loss.backward()
    pre = model.flat_parameters().detach().clone()
    out = pred.detach().cpu().double()
    err = float((out - o["out64"]).abs().max())
    agree = float((out.argmax(1) == o["out64"].argmax(1)).double().mean())
    rel, cos = _flat_grad_errors(model, o["g64"])
    gated = {k: v for k, v in rel.items() if not k.endswith(_ZERO_GRAD)}
    x3ratio, wx = _x3_gate(gated, o)
    grads = [p.grad.detach().clone() for p in model.parameters()]
    opt.step()
    assert opt._flat(opt.param_groups[0]) is not None   # the one-launch flat path ran
    rec = {"precision": "bf16x3", "path": "autograd custom ops + f3.RMSprop", "seed": seed, "max_abs_dlogit": err,
           "argmax_agreement": agree, "grad_cosine": cos, "worst_x3_gate_ratio": x3ratio[wx],
           "worst_x3_gate_tensor": wx, "loss": float(loss.item()), "loss_ref": o["loss64"]}
    _record("main_py_autograd_path_parity", rec)
    print(rec)
    assert err < 1e-3 and agree == 1.0
    assert abs(float(loss.item()) - o["loss64"]) < 1e-4
    assert cos > 0.99999
    assert x3ratio[wx] <= X3_GATE_MARGIN, (wx, x3ratio[wx])
    for (name, shape, off), p, g in zip(model.param_views(), model.parameters(), grads):
        n = int(np.prod(shape))
        p0 = pre[off:off + n].view(shape)
        expect = p0 - 1e-3 * g / (torch.sqrt(0.01 * g * g) + 1e-8)
        torch.testing.assert_close(p.detach(), expect, rtol=1e-6, atol=1e-7, msg=name)


# bf16 gates at ~2x the values measured on MI355X (profiles/r02_parity_record.jsonl): B=256 3-stream
# max|dlogit| 3.3e-3, argmax agreement 1.0, gradient cosine 0.99725; config 3 (B=128, 2-stream)
# 4.1e-3, 1.0, 0.99658. (The round-1 gate was 3e-2 / 0.95 / 0.99.)
BF16_B256_LOGIT_GATE = 7e-3
BF16_B256_ARGMAX_GATE = 0.99
BF16_B256_COS_GATE = 0.994
BF16_CFG3_LOGIT_GATE = 9e-3
BF16_CFG3_COS_GATE = 0.993


def _progress(msg):
    """A line in gpurun_out/progress.log for long oracle runs (shows the box the run is alive)."""
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "progress.log"), "a") as f:
        f.write(msg + "\n")


def test_bf16_storage_parity():
    """The benchmarked bf16 step (TrainStep, B=256, V=18, S=6) gated PER GRADIENT TENSOR against
    the oracle's bf16-storage restatement (oracle/model_cpu.py st_gcan_block_bf16: the tensors the
    kernels store in bf16 rounded at the same points, arithmetic in fp64).

    What the restatement shows (profiles/r03_parity_record.jsonl): the bf16 step's per-tensor
    gradient errors against the plain fp64 oracle (worst ~0.4 of the tensor's max, e.g.
    edge_importance / data_bn.weight in round 2) are the storage rounding itself — the restatement
    moves as far from fp64 (median 0.11, worst 0.4 at B=256), almost all of it from rounding the
    forward activations (rounding only the stored gradients: <= 0.012 at B=64). And the bf16-mode
    gradient is CHAOTIC at the rounding boundaries: perturbing every value by 2^-24 (half an fp32
    ulp) before it is rounded — what any other valid fp32 summation order does — moves the
    restatement's own gradients by a median 0.1 of max and its logits by ~1.7e-3 (train-mode BNs
    amplify the 1-ulp bf16 flips). A per-tensor bound tighter than that envelope cannot hold for
    any fp32 implementation of this step, so the gate is the envelope, measured per tensor from
    two jittered restatement runs (env):
      |g_hip - g_storage| / max|g_storage| <= 2.5 env + 0.02     for every gradient tensor,
      logits within 2.5x the envelope's logit spread, identical argmax,
      gradient cosine >= 1 - 2.5 (1 - the envelope's worst cosine),
      |g_hip - g_fp64| <= |g_storage - g_fp64| + 2.5 env + 0.02 (the error vs fp64 IS the rounding).
    Biases feeding a train-mode BN (true gradient ~0) are on the cosine only."""
    d = dev()
    import fall_multimodal_amd as f3
    torch.set_num_threads(min(32, os.cpu_count() or 1))
    layout, S, B = "coco_mmpose", 6, 256
    spec = oc.Spec(model="two_stgcan_bilstm", layout=layout, num_class=11, sensor_dim=S)
    st = oc.init_state(spec, 256)
    batch = synthetic_batch(B, 18, 11, S, 257)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": layout, "strategy": "spatial"}, 11, S, device=d,
                                      precision="bf16")
    model.load_state_dict(st)
    step = f3.TrainStep(model, B, lr=1e-3)
    step(*(torch.from_numpy(x).to(d) for x in batch))
    out = step.out.cpu().double()

    def d64():
        return {k: (v.double() if v.dtype == torch.float32 else v.clone()) for k, v in st.items()}
    x64 = [torch.from_numpy(x).double() for x in batch]
    _progress("bf16_storage_parity: storage oracle")
    out_e, loss_e, g_e = oc.train_step(d64(), spec, *x64, storage="bf16")
    _progress("bf16_storage_parity: fp64 oracle")
    out_64, _, g_64 = oc.train_step(d64(), spec, *x64)
    names = [n for n in g_e if not n.endswith(_ZERO_GRAD) and float(g_e[n].abs().max()) > 0]

    def rel(a, b):
        return {n: float((a[n] - b[n]).abs().max() / b[n].abs().max()) for n in names}

    def cosine(a, b):
        x = torch.cat([a[n].reshape(-1) for n in g_e])
        y = torch.cat([b[n].reshape(-1) for n in g_e])
        return float(x @ y / (x.norm() * y.norm()))
    env, env_logit, env_cos = {n: 0.0 for n in names}, 0.0, 1.0
    for seed in (1, 2):
        _progress(f"bf16_storage_parity: jittered storage oracle {seed}")
        oc.storage_jitter(2.0 ** -24, seed)
        try:
            out_j, _, g_j = oc.train_step(d64(), spec, *x64, storage="bf16")
        finally:
            oc.storage_jitter(0.0, 0)
        r = rel(g_j, g_e)
        env = {n: max(env[n], r[n]) for n in names}
        env_logit = max(env_logit, float((out_j - out_e).abs().max()))
        env_cos = min(env_cos, cosine(g_j, g_e))
    ours = {n: p.grad.detach().cpu().double() for n, p in model.named_parameters()}
    rel_e, rel_64, e_emu64 = rel(ours, g_e), rel(ours, g_64), rel(g_e, g_64)
    cos = cosine(ours, g_e)
    dlog = float((out - out_e).abs().max())
    agree = float((out.argmax(1) == out_e.argmax(1)).double().mean())
    ratio = {n: rel_e[n] / (2.5 * env[n] + 0.02) for n in names}
    worst = max(names, key=ratio.get)
    rec = {"precision": "bf16", "B": B, "max_abs_dlogit_vs_storage_oracle": dlog,
           "envelope_dlogit": env_logit, "envelope_cosine": env_cos,
           "max_abs_dlogit_storage_oracle_vs_fp64": float((out_e - out_64).abs().max()),
           "max_abs_dlogit_vs_fp64": float((out - out_64).abs().max()), "argmax_agreement": agree,
           "grad_cosine_vs_storage_oracle": cos, "loss": float(step.loss.item()), "loss_storage_oracle": float(loss_e),
           "worst_ratio_to_gate": [worst, ratio[worst], rel_e[worst], env[worst]],
           "median_hip_vs_storage": float(np.median([rel_e[n] for n in names])),
           "median_envelope": float(np.median([env[n] for n in names])),
           "median_storage_vs_fp64": float(np.median([e_emu64[n] for n in names])),
           "median_hip_vs_fp64": float(np.median([rel_64[n] for n in names])),
           "per_tensor_hip_vs_storage_hip_vs_fp64_storage_vs_fp64_envelope": {
               n: [round(rel_e[n], 5), round(rel_64[n], 5), round(e_emu64[n], 5), round(env[n], 5)] for n in names}}
    _record("bf16_storage_parity", rec)
    print({k: v for k, v in rec.items() if not k.startswith("per_tensor")})
    assert dlog <= 2.5 * env_logit and agree == 1.0, (dlog, env_logit, agree)
    assert cos >= 1 - 2.5 * (1 - env_cos), (cos, env_cos)
    assert abs(float(step.loss.item()) - float(loss_e)) < 5e-4
    for n in names:
        assert rel_e[n] <= 2.5 * env[n] + 0.02, (n, rel_e[n], env[n])
        assert rel_64[n] <= e_emu64[n] + 2.5 * env[n] + 0.02, (n, rel_64[n], e_emu64[n], env[n])


def test_cfg3_two_stream_bf16_parity():
    """BASELINE config 3 — the Fall2 2-stream spatial+temporal model (build_model 'two_stgcan',
    combination.py:9-25 with its missing-argument bug fixed) in bf16 at B=128 — against the
    oracle; measured values recorded next to the 3-stream ones."""
    d = dev()
    import fall_multimodal_amd as f3
    torch.set_num_threads(min(32, os.cpu_count() or 1))
    B = 128
    spec = oc.Spec(model="two_stgcan", layout="coco_cut", num_class=11, sensor="none")
    st = oc.init_state(spec, 128)
    batch = synthetic_batch(B, 14, 11, 15, 129)
    model = f3.TwoStreamSTGCAN(3, {"layout": "coco_cut", "strategy": "spatial"}, 11, device=d, precision="bf16")
    model.load_state_dict(st)
    step = f3.TrainStep(model, B, lr=1e-3)
    step(torch.from_numpy(batch[0]).to(d), None, torch.from_numpy(batch[2]).to(d))
    st64 = {k: (v.double() if v.dtype == torch.float32 else v.clone()) for k, v in st.items()}
    out_ref, loss_ref, grads_ref = oc.train_step(st64, spec, torch.from_numpy(batch[0]).double(), None,
                                                 torch.from_numpy(batch[2]).double())
    out = step.out.cpu().double()
    err = float((out - out_ref).abs().max())
    agree = float((out.argmax(1) == out_ref.argmax(1)).double().mean())
    rel, cos = _flat_grad_errors(model, grads_ref)
    rec = {"precision": "bf16", "B": B, "model": "two_stgcan", "max_abs_dlogit": err, "argmax_agreement": agree,
           "grad_cosine": cos, "loss": float(step.loss.item()), "loss_ref": float(loss_ref)}
    _record("cfg3_two_stream_bf16_parity", rec)
    print(rec)
    assert err < BF16_CFG3_LOGIT_GATE and agree >= BF16_B256_ARGMAX_GATE
    assert cos >= BF16_CFG3_COS_GATE


def test_custom_ops_opcheck():
    """torch.library.opcheck on the native ops (schema, fake kernel vs real kernel, autograd
    registration) at a small batch."""
    d = dev()
    import fall_multimodal_amd as f3
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d)
    model.load_state_dict(oc.init_state(spec, 5))
    skel, sensor, _ = synthetic_batch(4, 18, 11, 6, 6)
    args = (model._op_id, list(model.parameters()), model._flat_buffers, model._flat_counters,
            torch.from_numpy(skel).to(d), torch.from_numpy(sensor).to(d), True)
    torch.library.opcheck(torch.ops.fall3.net_forward.default, args,
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))


@pytest.mark.parametrize("precision", ["bf16x3", "fp32"])
def test_ca_x_kernels_match_chain_kernels(precision, monkeypatch):
    """The channel-attention kernels with up-front loads (layers.hip ca_fwd1x / ca_fwd2x / ca_bwd1x /
    ca_bwd3x with ca_bwd2 folded in, F3_CA_X unset or 2, the default) against the load-chain kernels
    they replace (F3_CA_X=0), inside
    a B=256 training step of the 3-stream model (stgcan.py:59-74): logits within 1e-5 of max, the
    flattened gradients at cosine >= 0.999999, every gradient tensor within 5e-2 of its max, and the
    BN running statistics within 1e-5. The per-tensor bound is loose on purpose. The q1 / dhid / att
    sums run in another order, and the attention BN normalises over only the 256 clips, so the change
    reaches the attention weights through near-cancelling sums and ReLU kinks. Measured: 2.5e-2 on a
    layer-6 W1 gradient (bf16x3) and 6.4e-3 (fp32). The bf16x3 path itself is 4.5e-2 from fp64 on such
    tensors. test_benchmarked_config_parity holds the default (x) path to the oracle on three seeds."""
    d = dev()
    import fall_multimodal_amd as f3
    B, V, S = 256, 18, 6
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=S)
    st = oc.init_state(spec, 5)
    batch = [torch.from_numpy(x).to(d) for x in synthetic_batch(B, V, 11, S, 41)]
    res = {}
    for mode in ("0", "2"):  # 2 (= unset): the default, ca_bwd2 folded into ca_bwd3x
        monkeypatch.setenv("F3_CA_X", mode)
        model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, S, device=d,
                                          precision=precision)
        model.load_state_dict(st)
        step = f3.TrainStep(model, B, lr=0.0)
        step(*batch)
        torch.cuda.synchronize()
        res[mode] = (step.out.detach().cpu().double(),
                     {n: p.grad.detach().cpu().double() for n, p in model.named_parameters()},
                     {k: v.detach().cpu().double() for k, v in model.state_dict().items() if "running" in k})
    o0, g0, b0 = res["0"]
    o1, g1, b1 = res["2"]
    assert float((o1 - o0).abs().max()) <= 1e-5 * float(o0.abs().max())
    worst, gmax = 0.0, max(float(g.abs().max()) for g in g0.values())
    a0 = torch.cat([g.reshape(-1) for g in g0.values()])
    a1 = torch.cat([g1[n].reshape(-1) for n in g0])
    cos = float(a0 @ a1 / (a0.norm() * a1.norm()))
    assert cos >= 0.999999, cos
    for n in g0:
        scale = float(g0[n].abs().max())
        if scale < 1e-6 * gmax:  # rounding residue of an analytically zero gradient
            continue
        r = float((g1[n] - g0[n]).abs().max()) / scale
        if n.endswith(("tcn.2.bias", "residual.0.bias", "atten.1.bias")):  # BN-fed: analytically zero
            continue
        worst = max(worst, r)
        assert r <= 5e-2, (n, r)
    for k in b0:
        assert float((b1[k] - b0[k]).abs().max()) <= 1e-5 * max(float(b0[k].abs().max()), 1.0), k
    print(f"ca_x vs chain ({precision}): max |dlogit| {float((o1 - o0).abs().max()):.2e}, gradient cosine "
          f"{cos:.9f}, worst gradient rel {worst:.2e}")
