"""Run-to-run determinism of the native training step (needs an MI355X).

Every cross-workgroup reduction on the bf16x3 (headline) step's path sums partial rows in a fixed order
(f3_colsum: pooled means, per-clip block sums, channel-attention / data-BN / LSTM / bias weight
gradients, graph-mix dA, BN-backward column sums, split-K weight-gradient slabs), so two identical
steps give bit-identical outputs and gradients. The BN statistics accumulate float partials into fp64
atomics: exact, hence order-independent, while each channel's partials span at most
29 - ceil(log2 n) binades ("What the fp64 BN-statistic atomics guarantee"); a sum
that nearly cancels can fall outside that, so for those sums this test is a measurement, not a proof. This is what lets the parity gates elsewhere be fixed tolerances
instead of run-to-run floors. (The fp32 mode's own kernels — conv_wgrad_f32, the fp32 graph mix — keep
float atomics and are not covered.)

Shapes outside this guarantee (bf16x3), since nothing enforces it there:
- a tcn forward that does not fit a clip window (T*V > 540 at 64 channels, or > 270 at 128 / 256;
  e.g. V = 25 at T = 30) runs igemm_big's tiled form, which adds the channel-attention pool with
  float atomics (gemm_big.hip, EPI_GAP);
- a weight gradient whose split-K slab has no room for the bias rows falls back to float atomics
  on db (gemm_glds.hip). In bf16x3 the tcn and residual biases come from block_bwd_apply's rows and
  the gcn bias from gcn_bias_bwd, so only the other modes' weight gradients can take that fallback.
Every shape the bench and the parity tests run (V = 18 and V = 14, T <= 30) is inside it; this test
runs B = 32 at V = 18.
"""
import numpy as np
import pytest
import torch


def _run(precision, B, seed, steps):
    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=dev,
                                      precision=precision)
    step = f3.TrainStep(model, B, lr=1e-3)
    batch = [torch.from_numpy(x).to(dev) for x in synthetic_batch(B, 18, 11, 6, seed)]
    lab = step.prepare(*batch)
    step.forward_backward(batch[0], batch[1], lab)
    torch.cuda.synchronize()
    out = {"grads": step.grads.clone(), "logits": step.out.clone()}
    losses = []
    for i in range(steps):
        b = [torch.from_numpy(x).to(dev) for x in synthetic_batch(B, 18, 11, 6, seed + 1 + i)]
        losses.append(float(step(*b).item()))
    torch.cuda.synchronize()
    out["params"] = model.flat_parameters().clone()
    out["losses"] = losses
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16x3"])
def test_two_identical_steps_are_bit_identical(precision):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    a = _run(precision, 32, 7, 2)
    b = _run(precision, 32, 7, 2)
    assert torch.equal(a["logits"], b["logits"])
    diff = (a["grads"] - b["grads"]).abs()
    nz = int((diff != 0).sum())
    print(f"{precision}: gradient elements differing between two identical backward passes: {nz} of "
          f"{diff.numel()} (max {float(diff.max()):.3e}); losses {a['losses']} / {b['losses']}")
    assert nz == 0, (nz, float(diff.max()))
    # two RMSprop steps later (where rounding-level gradient noise used to reach ~1e-3 of the loss)
    assert a["losses"] == b["losses"]
    assert torch.equal(a["params"], b["params"])
