"""The asm-wait GEMM kernels checked INSIDE the 4-queue bf16 training step (needs an MI355X).

`wgrad_taps` (inline-asm transposed LDS reads with counted lgkmcnt waits) and the clip-window
`igemm_big` (batched inline-asm ds_read_b128 fragment reads, counted waits) rely on nothing touching
an asm read's destination before its wait. DESIGN.md §4.1b records one way that broke: under LDS
pressure inside the concurrent step, never in isolation, hipcc repacked asm destinations before the
wait and taps 2-3 of the weight gradient came out as garbage. The kernel unit tests run the kernels
alone, so this test checks their results on the step's own tensors after a full B=256 bf16
TrainStep (both skeleton streams, all four queues busy), at the shape they serve (layer 6:
C=256, T=8, V=18):
  * forward  h  = conv9x1(u, W) + b           (igemm_big clip window)      vs torch fp32
  * dgrad    dg = BN1-backward(relu-mask(conv9x1^T(dh, W)))  (clip window -- igemm_win1 in bf16x3 --
               transposed rows, RELUMASK epilogue; then bn_bwd_apply)   vs torch fp32 on the same dh, u, g
  * wgrad    dW = sum dh x shifted u           (wgrad_taps + its reduce)   vs torch fp32
A garbage tap or fragment shows up as O(max) errors; the bounds are bf16 output rounding."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle.prng import synthetic_batch

pytestmark = pytest.mark.gpu


def _view(ws, ptr, n, dtype):
    """The n-element workspace region at device pointer `ptr` as a torch tensor (no copy)."""
    es = torch.tensor([], dtype=dtype).element_size()
    off = int(ptr) - ws.data_ptr()
    assert 0 <= off and off + n * es <= ws.numel(), "debug tensor outside the workspace"
    return ws[off:off + n * es].view(dtype)


@pytest.mark.parametrize("precision", ["bf16", "bf16x3"])
@pytest.mark.parametrize("layer,C,T", [(6, 256, 8), (1, 64, 30)])  # T: the position stream's frames
def test_asm_wait_kernels_inside_the_step(layer, C, T, precision):
    """layer 6: igemm_big clip window + wgrad_taps; layer 1 (64 channels, T=30): the
    weight-stationary tcn64 forward / input gradient (tcn64.hip) and wgrad_big. bf16x3: the same
    path in the native split form (u, dh, dg stored as bf16 rows [x_hi | x_lo] of 2C, h / g fp32,
    weights fp32; the window GEMMs issue x_hi W_hi + x_lo W_hi + x_hi W_lo, the 64-channel T=30 layers
    through the WIN=540 clip windows, the tcn input gradients through igemm_win1), checked against
    torch fp64 on hi + lo at the split's 1e-4 of max."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import fall_multimodal_amd as f3
    import fall_multimodal_amd._lib as L
    d = torch.device("cuda")
    B, V, S = 256, 18, 6
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, S, device=d,
                                      precision=precision)
    x3 = precision == "bf16x3"
    step = f3.TrainStep(model, B, lr=0.0)
    batch = [torch.from_numpy(x).to(d) for x in synthetic_batch(B, V, 11, S, 257)]
    for _ in range(3):   # several steps: the check reads the last one's tensors
        step(*batch)
    torch.cuda.synchronize()
    lib, h = L.lib(), model._native.h
    params = dict(model.named_parameters())
    for si, pre in ((0, "stgcan_1"), (1, "stgcan_2")):
        if T == 30:
            T = 30 - si  # the motion stream (frame differences) has one frame less (combination.py:39)
        M = B * T * V
        def t(what, n=M * C, dtype=torch.bfloat16):
            p = lib.f3_net_debug_tensor(h, B, L.ptr(step.ws), si, layer, what.encode())
            assert p, what
            return _view(step.ws, p, n, dtype)

        def rows(what):   # NCHW view of a [B, T, V, C] row tensor as the precision stores it
            if x3 and what in ("u", "dh", "dg"):   # bf16 rows [hi | lo] of 2C: the value is hi + lo
                r = t(what, 2 * M * C).double().view(B, T, V, 2, C).sum(3)
            elif x3:
                r = t(what, M * C, torch.float32).double().view(B, T, V, C)
            else:
                r = t(what).float().view(B, T, V, C)
            return r.permute(0, 3, 1, 2)
        u, hh, dh, g, dg = rows("u"), rows("h"), rows("dh"), rows("g"), rows("dg")
        p = f"{pre}.st_gcan_networks.{layer}."
        W = params[p + "tcn.2.weight"].detach()
        W = W.double() if x3 else W.to(torch.bfloat16).float()
        bias = params[p + "tcn.2.bias"].detach().to(W.dtype)
        # forward (igemm_big clip window), bf16 output (bf16x3: fp32 output of the split products)
        ref = F.conv2d(u, W, bias, padding=(4, 0))
        err = float((hh - ref).abs().max() / ref.abs().max())
        assert err < (1e-4 if x3 else 2 ** -7), (pre, "forward", err)
        # weight gradient (wgrad_taps + reduce)
        dw_ref = torch.nn.grad.conv2d_weight(u, W.shape, dh, padding=(4, 0))
        dw = params[p + "tcn.2.weight"].grad.detach().to(W.dtype)
        err = float((dw - dw_ref).abs().max() / dw_ref.abs().max())
        assert err < 1e-4, (pre, "wgrad", err)
        for dt in range(9):   # per tap, so a garbage tap is named
            e = float((dw[..., dt, 0] - dw_ref[..., dt, 0]).abs().max() / dw_ref.abs().max())
            assert e < 1e-4, (pre, "wgrad tap", dt, e)
        # input gradient (igemm_big window, transposed rows, ReLU mask) through BN1's backward
        du = torch.nn.grad.conv2d_input(u.shape, W, dh, padding=(4, 0))
        dv = du * (u > 0)
        fs = t("bn1_fsum", C, torch.float64)
        fq = t("bn1_fsq", C, torch.float64)
        mean = fs / M
        var = (fq / M - mean * mean).clamp_min(0)
        rs = (1.0 / torch.sqrt(var + 1e-5)).to(W.dtype)
        gamma = params[p + "tcn.0.weight"].detach().to(W.dtype)
        xhat = (g - mean.to(W.dtype).view(1, C, 1, 1)) * rs.view(1, C, 1, 1)
        s1 = dv.sum((0, 2, 3))
        s2 = (dv * xhat).sum((0, 2, 3))
        bs = t("bn1_bsum", C, torch.float64).to(W.dtype)
        err = float((bs - s1).abs().max() / s1.abs().max())
        assert err < (1e-3 if x3 else 1e-2), (pre, "bn1 backward sums", err)
        dg_ref = (gamma * rs).view(1, C, 1, 1) * (dv - (s1 / M).view(1, C, 1, 1) - xhat * (s2 / M).view(1, C, 1, 1))
        err = float((dg - dg_ref).abs().max() / dg_ref.abs().max())
        assert err < (1e-3 if x3 else 2 ** -6), (pre, "dgrad", err)
        if not x3:
            frac = float(((dg - dg_ref).abs() > 2 ** -7 * dg_ref.abs().max()).double().mean())
            assert frac < 1e-4, (pre, "dgrad outliers", frac)
        print(f"{precision} layer {layer} {pre}: in-step forward / wgrad / dgrad ok")
