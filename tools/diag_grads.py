"""Diagnostic: per-parameter gradient error of the HIP path vs the fp64 oracle."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from oracle import model_cpu as oc
from tests.golden_util import load
from tests.test_gpu_parity import build_from_spec, call

tag = sys.argv[1] if len(sys.argv) > 1 else 'har'
d = torch.device('cuda')
g, spec = load(tag)
st = oc.init_state(spec, int(g['seed'][0]))
model = build_from_spec(spec, d)
model.load_state_dict(st)
model.train()
skel = torch.from_numpy(g['skel']).to(d); sensor = torch.from_numpy(g['sensor']).to(d)
label = torch.from_numpy(g['label']).to(d)
out = call(model, spec, skel, sensor)
loss = torch.nn.CrossEntropyLoss()(out, label)
loss.backward()
st64 = {k: (v.double() if v.dtype == torch.float32 else v) for k, v in st.items()}
o64, l64, g64 = oc.train_step(st64, spec, *(torch.from_numpy(g[k]).double() for k in ('skel', 'sensor', 'label')))
print('logit err', np.abs(out.detach().cpu().numpy() - o64.numpy()).max())
rows = []
for name, p in model.named_parameters():
    if name not in g64:
        continue
    a = g64[name].numpy().reshape(-1)
    b = p.grad.detach().cpu().double().numpy().reshape(-1)
    if np.abs(a).max() < 1e-7:
        continue
    rows.append((np.abs(a - b).max() / np.abs(a).max(), name))
for e, n in rows:
    print(f"{e:.2e} {n}")
