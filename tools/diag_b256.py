"""Diagnostic: per-tensor gradient error of the fp32 HIP step at the benchmarked configuration
against the fp32 and fp64 oracle (the fp32-vs-fp64 oracle gap is the intrinsic fp32 noise)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fall_multimodal_amd as f3  # noqa: E402
from oracle import model_cpu as oc  # noqa: E402
from oracle.prng import synthetic_batch  # noqa: E402

torch.set_num_threads(32)
d = torch.device("cuda")
spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
st = oc.init_state(spec, 256)
batch = synthetic_batch(256, 18, 11, 6, 257)
model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d)
model.load_state_dict(st)
step = f3.TrainStep(model, 256, lr=1e-3)
step(*(torch.from_numpy(x).to(d) for x in batch))
_, _, g32 = oc.train_step({k: v.clone() for k, v in st.items()}, spec, *(torch.from_numpy(x) for x in batch))
st64 = {k: (v.double() if v.dtype == torch.float32 else v.clone()) for k, v in st.items()}
_, _, g64 = oc.train_step(st64, spec, *(torch.from_numpy(x).double() for x in batch))
rows = []
for n, p in model.named_parameters():
    if n not in g64:
        continue
    g = p.grad.detach().cpu().double()
    r = g64[n]
    m = float(r.abs().max())
    rows.append((float((g - r).abs().max()) / m, float((g32[n].double() - r).abs().max()) / m, m, n))
rows = [r for r in rows if r[2] > 1e-9]  # drop the biases feeding train-mode BN (true gradient ~0)
rows.sort(key=lambda r: -r[0])
for e, e32, m, n in rows[:12]:
    print(f"{e:.3e}  oracle32 {e32:.3e}  ratio {e / max(e32, 1e-30):8.2f}  max|g| {m:.3e}  {n}")
print("-- by ratio")
rows.sort(key=lambda r: -r[0] / max(r[1], 1e-30))
for e, e32, m, n in rows[:8]:
    print(f"{e:.3e}  oracle32 {e32:.3e}  ratio {e / max(e32, 1e-30):8.2f}  max|g| {m:.3e}  {n}")
print("worst ratio", max(r[0] / max(r[1], 1e-30) for r in rows))
