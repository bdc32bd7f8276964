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
