"""RGB spatial-conv branch (build-defined, PARITY UNPINNED: the reference has no RGB model arithmetic,
SURVEY.md section 8a row R-RGB). The HIP kernels (csrc/rgb.hip) are checked against the build's own
definition restated in oracle/rgb_cpu.py (fp64 on the bf16-rounded operands the kernels read)."""
import pytest
import torch

from oracle import rgb_cpu


def _case(B, T, seed):
    g = torch.Generator().manual_seed(seed)
    frames = torch.rand(B, T, 224, 224, 3, generator=g).to(torch.bfloat16)
    w = (torch.randn(64, 3, 8, 8, generator=g) * 0.1).to(torch.bfloat16).float()
    b = torch.randn(64, generator=g) * 0.1
    return frames, w, b


def test_pack_layout():
    w = torch.randn(64, 3, 8, 8)
    wp = rgb_cpu.pack_weight(w)
    for c, ch, dy, dx in [(0, 0, 0, 0), (5, 2, 7, 1), (63, 1, 3, 6)]:
        assert wp[c, (dy * 8 + dx) * 3 + ch] == w[c, ch, dy, dx]
    assert torch.equal(rgb_cpu.unpack_weight(wp), w)


def test_oracle_matches_patch_sum():
    """conv2d-based oracle == the kernels' formulation: 784 patches x packed [64, 192] weight."""
    frames, w, b = _case(1, 2, 0)
    feat = rgb_cpu.rgb_feat(frames, w, b)
    wp = rgb_cpu.pack_weight(w).double()
    acc = torch.zeros(64, dtype=torch.float64)
    for t in range(2):
        x = frames[0, t].double().reshape(28, 8, 28, 8, 3).permute(0, 2, 1, 3, 4).reshape(784, 192)
        acc += torch.relu(x @ wp.T + b.double()).sum(0)
    assert torch.allclose(feat[0], acc / (2 * 784), rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("B,T", [(2, 3), (5, 7), (1, 13)])
def test_rgb_kernels_vs_oracle(B, T):
    from fall_multimodal_amd import rgb  # noqa: F401 (registers the custom ops)
    frames, w, b = _case(B, T, 10 * B + T)
    dev = torch.device("cuda:0")
    fd, wd, bd = frames.to(dev), w.to(dev), b.to(dev)
    feat = torch.ops.fall3.rgb_forward(fd, wd, bd)
    torch.cuda.synchronize()
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    ref = rgb_cpu.rgb_feat(frames, wr, br)
    # fp32 accumulation of 192 bf16 products, then a mean over T*784 patches
    assert torch.allclose(feat.cpu().double(), ref.detach(), rtol=1e-4, atol=1e-5), \
        (feat.cpu().double() - ref.detach()).abs().max()
    dfeat = torch.randn(B, 64, generator=torch.Generator().manual_seed(7))
    dw, db = torch.ops.fall3.rgb_backward(fd, wd, bd, dfeat.to(dev))
    (ref * dfeat.double()).sum().backward()
    # dW: exact 0/1 relu mask x bf16 patches on MFMA, scaled by dfeat/(T*784) in fp32 (a mask bit
    # that flips between the fp32 and the fp64 pre-activation moves one patch term, ~1e-4 of max)
    tw = 5e-4 * wr.grad.abs().max().item()
    assert (dw.cpu().double() - wr.grad).abs().max().item() < tw
    assert (db.cpu().double() - br.grad).abs().max().item() < 1e-4 * max(1.0, br.grad.abs().max().item())


@pytest.mark.gpu
def test_rgb_branch_autograd_step():
    from fall_multimodal_amd.rgb import RGBBranch
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = RGBBranch(num_class=9, device=dev)
    frames = torch.rand(4, 5, 224, 224, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 9, (4,), device=dev)
    loss = torch.nn.functional.cross_entropy(m(frames), y)
    loss.backward()
    assert torch.isfinite(loss)
    assert m.conv.weight.grad is not None and m.conv.weight.grad.abs().sum() > 0
    assert m.conv.bias.grad is not None and torch.isfinite(m.conv.bias.grad).all()
    ref = rgb_cpu.rgb_feat(frames.cpu(), m.conv.weight.detach().cpu().to(torch.bfloat16).float(),
                           m.conv.bias.detach().cpu())
    got = m.conv(frames).detach().cpu().double()
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_fall3_with_rgb_step_vs_composed_oracle():
    """The north-star workload as one step (rgb.Fall3RGBStep: skeleton + IMU + RGB, late fusion by adding
    logits) against oracle/model_cpu (pinned to the reference) + oracle/rgb_cpu (the build's definition,
    parity unpinned) composed in fp64 with one soft-target CE: total logits within 1e-3 with identical
    argmax, loss, the gradients of the RGB parameters and of the fusion fc, and the RMSprop update of the
    RGB parameters."""
    import numpy as np

    import fall_multimodal_amd as f3
    from fall_multimodal_amd.rgb import Fall3RGBStep, Fall3WithRGB
    from oracle import model_cpu as oc
    from oracle.prng import synthetic_batch
    dev = torch.device("cuda:0")
    B, T, V, S, C = 4, 30, 18, 6, 11
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=C, sensor_dim=S)
    st = oc.init_state(spec, 5)
    skel, sensor, label = synthetic_batch(B, V, C, S, 9)
    base = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, C, S, device=dev)
    base.load_state_dict(st)
    torch.manual_seed(3)
    model = Fall3WithRGB(base, C, device=dev)
    with torch.no_grad():  # conv weights bf16-representable, as the kernels read them
        model.rgb.conv.weight.copy_(model.rgb.conv.weight.to(torch.bfloat16).float())
    rgb0 = [p.detach().cpu().clone() for p in (model.rgb.conv.weight, model.rgb.conv.bias, model.rgb.fc.weight,
                                               model.rgb.fc.bias)]
    frames = torch.rand(B, T, 224, 224, 3, generator=torch.Generator().manual_seed(4)).to(torch.bfloat16)
    step = Fall3RGBStep(model, B, lr=1e-3)
    step(*(torch.from_numpy(x).to(dev) for x in (skel, sensor)), frames.to(dev), torch.from_numpy(label).to(dev))
    torch.cuda.synchronize()
    # composed oracle (fp64)
    st64 = {k: (v.double() if v.dtype == torch.float32 else v.clone()) for k, v in st.items()}
    names = [k for k in st64 if not oc.is_buffer(k)]
    for k in names:
        st64[k] = st64[k].detach().clone().requires_grad_(True)
    rp = [t.double().requires_grad_(True) for t in rgb0]
    feat = rgb_cpu.rgb_feat(frames, rp[0], rp[1])
    total = oc.forward(st64, spec, torch.from_numpy(skel).double(), torch.from_numpy(sensor).double()) + \
        feat @ rp[2].t() + rp[3]
    loss = oc.soft_ce(total, torch.from_numpy(label).double())
    gl = torch.autograd.grad(loss, [st64["fc.weight"]] + rp)
    out = step.out.cpu().double()
    err = float((out - total.detach()).abs().max())
    assert err < 1e-3 and (out.argmax(1) == total.detach().argmax(1)).all(), err
    assert abs(step.loss.item() - loss.item()) < 1e-4
    fc_g = dict(base.named_parameters())["fc.weight"].grad.cpu().double()
    assert float((fc_g - gl[0]).abs().max()) < 1e-3 * float(gl[0].abs().max()) + 1e-7
    for p, ref, tol in zip((model.rgb.conv.weight, model.rgb.conv.bias, model.rgb.fc.weight, model.rgb.fc.bias),
                           gl[1:], (5e-4, 1e-4, 1e-5, 1e-5)):
        g = p.grad.detach().cpu().double()
        assert float((g - ref).abs().max()) <= tol * float(ref.abs().max()) + 1e-9, (p.shape, float((g - ref).abs().max()))
    # RMSprop (torch semantics) from the step's own gradients: p1 = p0 - lr g / (sqrt(0.01 g^2) + eps)
    for p, p0 in zip((model.rgb.conv.weight, model.rgb.conv.bias, model.rgb.fc.weight, model.rgb.fc.bias), rgb0):
        g = p.grad.detach().cpu()
        want = p0 - 1e-3 * g / (torch.sqrt(0.01 * g * g) + 1e-8)
        np.testing.assert_allclose(p.detach().cpu().numpy(), want.numpy(), rtol=0, atol=2e-6)
