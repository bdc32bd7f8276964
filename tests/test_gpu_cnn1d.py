"""The sensor CNN1D's cooperative form (one launch per direction, sensor.hip cnn1d_coop_*) against
the per-layer launches it replaces in training (needs an MI355X). Parity against the oracle and the
reference's golden vectors is in test_gpu_parity.py (golden cases ur_sensor / ur_nb run the
cooperative form by default); here: the same step through both forms, ragged and multi-clip
workgroup batches, and run-to-run bit identity of the cooperative form (fixed-order reductions)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(model, x, dout, coop):
    os.environ["F3_CNN1D_COOP"] = "1" if coop else "0"
    try:
        N = x.shape[0]
        ws = torch.zeros(model._native.workspace_bytes(N), dtype=torch.uint8, device=x.device)
        out = torch.empty(N, dout.shape[1], device=x.device)
        model.native_forward(None, x, out, ws, True)
        grads = torch.zeros(model._native.nparam, device=x.device)
        model.native_backward(N, dout, grads, ws)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("F3_CNN1D_COOP", None)
    return out.cpu().double(), grads.cpu().double()


@pytest.mark.parametrize("N", [256, 5, 300, 600])
def test_cooperative_cnn1d_matches_per_layer_launches(N):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import fall_multimodal_amd as f3
    d = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = f3.CNN_BiLSTM(device=d)
    g = torch.Generator().manual_seed(N)
    x = torch.randn(N, 30, 4, generator=g).to(d)
    dout = torch.randn(N, model.spec.num_class, generator=g).to(d)
    o1, g1 = _step(model, x, dout, True)
    o0, g0 = _step(model, x, dout, False)
    assert torch.isfinite(o1).all() and torch.isfinite(g1).all()
    # the same arithmetic in another summation order (BN sums fp64 in both; weight-gradient sums
    # fp32 over clips): logits within 1e-5, each gradient tensor within 1e-4 of its own max
    torch.testing.assert_close(o1, o0, rtol=1e-5, atol=1e-5)
    worst, gmax = 0.0, float(g0.abs().max())
    for name, shape, off in model.param_views():
        n = 1
        for s in shape:
            n *= s
        a, b = g1[off:off + n], g0[off:off + n]
        if name.startswith("cnn.") and name.endswith(".0.bias"):
            # a conv bias feeding a batch-statistics BatchNorm has an exactly-zero gradient: both
            # forms leave rounding residue only
            assert float(a.abs().max()) <= 1e-5 * gmax and float(b.abs().max()) <= 1e-5 * gmax, name
            continue
        scale = max(float(b.abs().max()), 1e-12)
        r = float((a - b).abs().max()) / scale
        worst = max(worst, r)
        assert r <= 1e-4, (name, r)
    print(f"N={N}: max |dlogit| {float((o1 - o0).abs().max()):.2e}, worst gradient rel diff {worst:.2e}")


def test_cooperative_cnn1d_is_deterministic():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import fall_multimodal_amd as f3
    d = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = f3.CNN_BiLSTM(device=d)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(512, 30, 4, generator=g).to(d)
    dout = torch.randn(512, model.spec.num_class, generator=g).to(d)
    a = _step(model, x, dout, True)
    b = _step(model, x, dout, True)
    assert torch.equal(a[0], b[0])
    # the LSTM's own weight gradients use fixed-order partial rows too (f3_lstm_bwd)
    assert torch.equal(a[1], b[1]), int((a[1] != b[1]).sum())


def test_cooperative_cnn1d_barrier_timeout_is_reported(monkeypatch):
    """a group barrier of the cooperative CNN1D that times out writes NaN into its outputs,
    and the host must be told, as for TARGCN's GRU barriers. F3_CNN_SKIP_ARRIVE=1 makes workgroup 0
    skip its arrivals (every barrier of the launch then times out after 2^14 polls); the error word
    is copied to a pinned host ring after each launch (status_ring.h) and reported once as
    F3_EDEVICE by device_status() or the next forward / backward. A clean step before and after
    reports OK."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import fall_multimodal_amd as f3
    d = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = f3.CNN_BiLSTM(device=d)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, 30, 4, generator=g).to(d)
    dout = torch.randn(64, model.spec.num_class, generator=g).to(d)
    o, gr = _step(model, x, dout, True)
    model.device_status(wait=True)
    assert torch.isfinite(o).all() and torch.isfinite(gr).all()
    monkeypatch.setenv("F3_CNN_SKIP_ARRIVE", "1")
    with pytest.raises(RuntimeError, match="barrier"):
        _step(model, x, dout, True)
        model.device_status(wait=True)
    monkeypatch.delenv("F3_CNN_SKIP_ARRIVE")
    torch.cuda.synchronize()
    model.device_status(wait=True)  # reported once, then clear
    o, gr = _step(model, x, dout, True)
    model.device_status(wait=True)
    assert torch.isfinite(o).all() and torch.isfinite(gr).all()


def test_long_sensor_clips_take_the_per_layer_launches():
    """the cooperative form's per-clip tensors grow with the sensor frames; past its 64 KiB
    of LDS (T = 400 at Ci = 4 here) the step must take the per-layer launches instead of failing with
    F3_EINVAL. Checked against the per-layer form forced by F3_CNN1D_COOP=0: the same forward bit for bit,
    gradients within 1e-5 of their max (the per-layer backward's weight gradients use float atomics)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import fall_multimodal_amd as f3
    d = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = f3.CNN_BiLSTM(device=d, sensor_frames=400)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(16, 400, 4, generator=g).to(d)
    dout = torch.randn(16, model.spec.num_class, generator=g).to(d)
    o1, g1 = _step(model, x, dout, True)
    o0, g0 = _step(model, x, dout, False)
    assert torch.isfinite(o1).all() and torch.isfinite(g1).all()
    assert torch.equal(o1, o0)
    assert float((g1 - g0).abs().max()) <= 1e-5 * float(g0.abs().max())


@pytest.mark.parametrize("seed", [3, 17])
def test_cnn_bilstm_b256_step_vs_oracle(seed):
    """The sensor-only CNN_BiLSTM (UR notebook spec: S=4, 2 classes, hidden 16; GSTCAN_UR_conv.ipynb
    :493-514 CNN1D, :572-586 CNN_BiLSTM) at B=256 -- the batch the CNN1D runs as ONE cooperative
    launch per direction, group barriers over all its workgroups -- one TrainStep (native forward,
    soft CE, backward, RMSprop) against the CPU oracle: logits within 1e-3 with
    identical argmax, the loss, and the per-tensor conditioning-aware gradient gate of
    test_gpu_parity.py (tests/golden_util.check_grads_conditioned, fp32 envelope at 1e-6 probes).
    The conv biases that feed a batch-statistics BatchNorm have an exactly-zero true gradient and
    are checked as residue (<= 1e-5 of the largest gradient) instead."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import numpy as np
    import fall_multimodal_amd as f3
    from oracle import model_cpu as oc
    from oracle.prng import synthetic_batch
    from tests.golden_util import check_grads_conditioned, load
    d = torch.device("cuda", 0)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    _, spec = load("ur_sensor")
    B = 256
    _, sensor, label = synthetic_batch(B, 14, spec.num_class, spec.sensor_dim, seed)
    st = oc.init_state(spec, seed)
    model = f3.CNN_BiLSTM(hidden_size=16, num_layers=1, dropout_prob=0.3, num_classes=2, feature="mean", device=d)
    model.load_state_dict(st, strict=True)
    step = f3.TrainStep(model, B, lr=1e-3)
    loss = step(None, torch.from_numpy(sensor).to(d), torch.from_numpy(label).to(d))
    torch.cuda.synchronize()
    out_ref, loss_ref, grads_ref = oc.train_step(oc.init_state(spec, seed), spec, None, torch.from_numpy(sensor),
                                                 torch.from_numpy(label))
    out = step.out.cpu().numpy()
    np.testing.assert_allclose(out, out_ref.numpy(), atol=1e-3, rtol=0)
    assert (out.argmax(1) == out_ref.numpy().argmax(1)).all()
    np.testing.assert_allclose(loss.item(), loss_ref.item(), rtol=1e-4)
    ours = {name: p.grad.detach().cpu().numpy() for (name, shape, off), p in zip(model.param_views(), model.parameters())}
    gmax = max(float(np.abs(g).max()) for g in ours.values())
    fake = {"grad:" + k: v.numpy().reshape(-1) for k, v in grads_ref.items()}
    for name, g in ours.items():
        if "grad:" + name not in fake:  # CNN1D.fc: unused by the forward, no gradient in either
            fake["nograd:" + name] = np.zeros(1)
            assert not np.abs(g).any(), name
        elif name.startswith("cnn.") and name.endswith(".0.bias"):
            fake["nograd:" + name] = np.zeros(1)
            assert float(np.abs(g).max()) <= 1e-5 * gmax, name
    env = oc.gradient_sensitivity(oc.init_state(spec, seed), spec, None, torch.from_numpy(sensor),
                                  torch.from_numpy(label), eps=1e-6, trials=3, per_param=True)
    cosg = check_grads_conditioned(fake, ours, env, what=f"CNN_BiLSTM B=256 seed {seed}")
    # at B=256 the oracle's own envelope is ~1e-6 (no kink next to the data): hold every gated
    # tensor to 1e-4 of its max as well, the fp32-vs-fp32 summation-order bar
    worst = 0.0
    for k, v in grads_ref.items():
        if "nograd:" + k in fake:
            continue
        r = float(np.abs(ours[k].reshape(-1) - v.numpy().reshape(-1)).max() / max(float(v.abs().max()), 1e-30))
        assert r <= 1e-4, (k, r)
        worst = max(worst, r)
    print(f"CNN_BiLSTM B=256 seed {seed}: max |dlogit| {float(np.abs(out - out_ref.numpy()).max()):.2e}, "
          f"gradient cosine {cosg:.8f}, worst per-tensor rel {worst:.2e}")
