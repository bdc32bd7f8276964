"""Diagnostic: run the same train step R times and report which grads vary run to run."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from oracle import model_cpu as oc
from tests.golden_util import load
from tests.test_gpu_parity import build_from_spec, call

tag = sys.argv[1] if len(sys.argv) > 1 else 'har'
R = int(sys.argv[2]) if len(sys.argv) > 2 else 6
d = torch.device('cuda')
g, spec = load(tag)
st = oc.init_state(spec, int(g['seed'][0]))
model = build_from_spec(spec, d)
skel = torch.from_numpy(g['skel']).to(d); sensor = torch.from_numpy(g['sensor']).to(d)
label = torch.from_numpy(g['label']).to(d)
runs = []
outs = []
for r in range(R):
    model.load_state_dict(st)
    model.zero_grad(set_to_none=True)
    model.train()
    out = call(model, spec, skel, sensor)
    torch.nn.CrossEntropyLoss()(out, label).backward()
    outs.append(out.detach().cpu().numpy())
    runs.append({n: p.grad.detach().cpu().numpy().copy() for n, p in model.named_parameters() if p.grad is not None})
print("out variation", max(np.abs(o - outs[0]).max() for o in outs))
worst = {}
for r in range(1, R):
    for n, v in runs[r].items():
        ref = runs[0][n]
        den = np.abs(ref).max() + 1e-30
        if den < 1e-7:
            continue
        e = np.abs(v - ref).max() / den
        worst[n] = max(worst.get(n, 0), e)
for n, e in sorted(worst.items(), key=lambda x: -x[1])[:25]:
    print(f"{e:.2e} {n}")
