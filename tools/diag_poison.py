"""Diagnostic: same-fill reruns vs different workspace fills, per-parameter normrel diffs."""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from oracle import model_cpu as oc
from tests.golden_util import load
from tests.test_gpu_parity import build_from_spec

tag = sys.argv[1]
d = torch.device('cuda')
g, spec = load(tag)
st = oc.init_state(spec, int(g['seed'][0]))
model = build_from_spec(spec, d)
skel = torch.from_numpy(g['skel']).to(d); sensor = torch.from_numpy(g['sensor']).to(d)
N, C = skel.shape[0], spec.num_class
dout = torch.randn(N, C, generator=torch.Generator().manual_seed(3)).to(d)
def run(fill):
    model.load_state_dict(st)
    ws = torch.full((model._native.workspace_bytes(N),), fill, dtype=torch.uint8, device=d)
    out = torch.empty(N, C, device=d)
    sk = None if spec.model == "bilstm" else skel
    se = sensor if spec.model in ("bilstm", "two_stgcan_bilstm") else None
    model.native_forward(sk, se, out, ws, True)
    grads = torch.zeros(model._native.nparam, device=d)
    model.native_backward(N, dout, grads, ws)
    torch.cuda.synchronize()
    return out.cpu().double().numpy(), grads.cpu().double().numpy()
base = run(0)
for name, fill in (("zero-again", 0), ("zero-again2", 0), ("fill42", 0x42), ("fillC1", 0xC1)):
    o, gr = run(fill)
    rows = []
    for n, shape, off in model.param_views():
        n_el = int(np.prod(shape))
        a, b = base[1][off:off + n_el], gr[off:off + n_el]
        den = np.abs(a).max()
        if den < 1e-7 or n.endswith(("tcn.2.bias", "residual.0.bias", "atten.1.bias")):
            continue  # biases feeding a train-mode BatchNorm: true gradient is 0
        rows.append((np.abs(a - b).max() / den, n))
    rows.sort(reverse=True)
    print(name, "out diff", np.abs(o - base[0]).max(), "worst", [f"{e:.1e} {n}" for e, n in rows[:5]])
