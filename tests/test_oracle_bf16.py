"""The oracle's bf16-storage restatement (oracle/model_cpu.py st_gcan_block_bf16), CPU.

It restates the skeleton block in the build's order (graph mix first, then the 1x1 GEMM with the
graph-mixed bias; BN statistics split from the values they normalise) and rounds the tensors the
bf16 kernels store. With the rounding switched off it must be the reference's own arithmetic
(pinned to the golden vectors through the fp32 path): this checks the reassociation and the split
BatchNorms exactly, in fp64. With the rounding on, only the stored tensors move: the logits stay
within bf16-storage distance and the running statistics are updated once per BatchNorm."""
import torch

from oracle import model_cpu as oc
from oracle.prng import synthetic_batch


def _case(B=8, seed=11):
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    st = oc.init_state(spec, seed)
    st64 = {k: (v.double() if v.dtype == torch.float32 else v.clone()) for k, v in st.items()}
    batch = [torch.from_numpy(x).double() for x in synthetic_batch(B, 18, 11, 6, seed + 1)]
    return spec, st64, batch


def test_storage_restatement_without_rounding_is_the_reference(monkeypatch):
    spec, st, batch = _case()
    a = {k: v.clone() for k, v in st.items()}
    b = {k: v.clone() for k, v in st.items()}
    o1, l1, g1 = oc.train_step(a, spec, *batch)
    monkeypatch.setattr(oc, "_to_bf16", lambda t: t)
    o2, l2, g2 = oc.train_step(b, spec, *batch, storage="bf16")
    assert float((o1 - o2).abs().max()) < 1e-12
    for k in g1:
        m = float(g1[k].abs().max())
        assert float((g1[k] - g2[k]).abs().max()) <= 1e-9 * max(m, 1e-3), k
    for k in a:   # running statistics, counters and the RMSprop update
        assert torch.allclose(a[k].double(), b[k].double(), rtol=0, atol=1e-10), k


def test_storage_rounding_moves_only_stored_tensors():
    spec, st, batch = _case()
    o1, _, g1 = oc.train_step({k: v.clone() for k, v in st.items()}, spec, *batch)
    s2 = {k: v.clone() for k, v in st.items()}
    o2, _, g2 = oc.train_step(s2, spec, *batch, storage="bf16")
    err = float((o1 - o2).abs().max())
    assert 1e-5 < err < 2e-2, err     # moved by the storage rounding, bounded
    assert all(int(s2[k]) == 1 for k in s2 if k.endswith("num_batches_tracked"))
    a = torch.cat([g1[k].reshape(-1) for k in g1])
    b = torch.cat([g2[k].reshape(-1) for k in g1])
    assert float(a @ b / (a.norm() * b.norm())) > 0.95
