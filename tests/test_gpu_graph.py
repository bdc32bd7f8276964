"""HIP-graph capture of TrainStep (needs an MI355X): the one-pass step and the two-phase (data
parallel) step captured with torch.cuda.graph and replayed give the eager step's logits, loss and
gradients. The phased capture is the DP path's (backward phase 1, all-reduce of the head bucket,
phase 2); at world 1 the collective is skipped and the capture/replay ordering is what is checked:
phase 1 must join its branch queues inside the capture (net.cpp Branches::mark_phase1)."""
import numpy as np
import pytest
import torch

from oracle import model_cpu as oc
from oracle.prng import synthetic_batch

pytestmark = pytest.mark.gpu

# biases feeding a train-mode BatchNorm (true gradient ~0): cosine-only
_ZERO_GRAD = ("tcn.2.bias", "residual.0.bias", "atten.1.bias", "gcn.conv.bias")


def _grads(model):
    return {n: p.grad.detach().double().cpu().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
@pytest.mark.parametrize("phased", [False, True], ids=["one_pass", "phased"])
def test_captured_step_matches_eager(phased, precision):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import fall_multimodal_amd as f3
    d = torch.device("cuda")
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    st = oc.init_state(spec, 61)
    B = 32
    sk, se, lb = (torch.from_numpy(x).to(d) for x in synthetic_batch(B, 18, 11, 6, 62))
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d,
                                      precision=precision)
    model.load_state_dict(st)
    step = f3.TrainStep(model, B, lr=1e-3, phased=phased)
    buf0 = model._flat_buffers.clone()
    # eager forward + backward (no optimizer step)
    lbl = step.prepare(sk, se, lb)
    step.forward_loss(sk, se, lbl)
    if phased:
        step.backward_phase(1)
        step.backward_phase(2)
    else:
        step.backward_phase(0)
    torch.cuda.synchronize()
    out_e, loss_e, g_e = step.out.clone(), float(step.loss.item()), _grads(model)
    # capture (its warm-up runs move the BN running statistics; restore them), then replay the
    # forward/backward graphs alone
    step.capture(sk, se, lbl)
    model._flat_buffers.copy_(buf0)
    step.grads.zero_()
    g_head, g_tail, _ = step.graph
    assert (g_tail is not None) == phased
    g_head.replay()
    if g_tail is not None:
        g_tail.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(step.out, out_e, rtol=0, atol=1e-5)
    assert abs(float(step.loss.item()) - loss_e) < 1e-5
    g_r = _grads(model)
    a = torch.cat([v.reshape(-1) for v in g_r.values()])
    b = torch.cat([v.reshape(-1) for v in g_e.values()])
    cos = float(a @ b / (a.norm() * b.norm()))
    assert cos > 0.99999, cos
    for n, v in g_e.items():
        if n.endswith(_ZERO_GRAD) or float(v.abs().max()) == 0:
            continue
        rel = float((g_r[n] - v).abs().max() / v.abs().max())
        assert rel < 5e-2, (n, rel)   # float-atomic ordering noise of this B=32 network (measured <= 0.021)
    # the whole captured step (incl. RMSprop) replays repeatedly; its loss trajectory is the eager one's
    model._flat_buffers.copy_(buf0)
    losses = [float(step(sk, se, lbl).item()) for _ in range(3)]
    twin = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d,
                                     precision=precision)
    twin.load_state_dict(st)
    tstep = f3.TrainStep(twin, B, lr=1e-3, phased=phased)
    ref = [float(tstep(sk, se, lbl).item()) for _ in range(3)]
    assert all(np.isfinite(losses)), losses
    # step 1 is the same forward; after it the two runs differ by float-atomic ordering noise, which
    # RMSprop's first steps amplify (lr*g/sqrt(v) ~ 10*lr*sign(g), also for gradients at rounding
    # level): measured 2e-4 after one update, 0.4-0.8 % after two. The bf16x3 step's reductions are
    # deterministic (tests/test_gpu_determinism.py): there the captured replay is bit-identical
    if precision == "bf16x3":
        assert losses == ref, (losses, ref)
    np.testing.assert_allclose(losses[:2], ref[:2], rtol=1e-3)
    np.testing.assert_allclose(losses[2], ref[2], rtol=2e-2)
