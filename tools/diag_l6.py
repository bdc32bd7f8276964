"""Diagnostic: stream s layer l backward intermediates across repeated runs (early stop)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, '.')
from oracle import model_cpu as oc
from tests.golden_util import load
from tests.test_gpu_parity import build_from_spec
import fall_multimodal_amd._lib as L

class _Raw:
    def __init__(self, p, n, ts):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": ts, "data": (p, False), "version": 2}

s, l = [int(v) for v in os.environ['DIAG_SL'].split(',')]
STOPPED = 'F3_DEBUG_BWD_STOP' in os.environ
d = torch.device('cuda')
g, spec = load(sys.argv[1] if len(sys.argv) > 1 else 'two')
st = oc.init_state(spec, int(g['seed'][0]))
model = build_from_spec(spec, d)
skel = torch.from_numpy(g['skel']).to(d); sensor = torch.from_numpy(g['sensor']).to(d)
N, C, V = 4, spec.num_class, 14
Cl = [64, 64, 64, 128, 128, 256, 256][l]
To = {0: [30, 30, 30, 15, 15, 8, 8], 1: [29, 29, 29, 15, 15, 8, 8]}[s][l]
Ti = {0: [30, 30, 30, 30, 15, 15, 8], 1: [29, 29, 29, 29, 15, 15, 8]}[s][l]
lib = L.lib()
dout = torch.randn(N, C, generator=torch.Generator().manual_seed(3)).to(d)
items = [("dpool", N * 256, "<f4"), ("pool", N * 256, "<f4"), ("gap", N * Cl, "<f4"), ("q1", N * Cl // 4, "<f4"),
         ("hid", N * Cl // 4, "<f4"), ("att", N * Cl, "<f4"), ("P1", N * Cl, "<f4"), ("P2", N * Cl, "<f4"),
         ("dq2", N * Cl, "<f4"), ("dbn", N * Cl // 4, "<f4"), ("dq1", N * Cl // 4, "<f4"), ("e", N * Cl, "<f4"),
         ("bn2_bsum", Cl, "<f8"), ("bn2_bsq", Cl, "<f8"), ("ca_fsum", Cl // 4, "<f8"), ("ca_fsq", Cl // 4, "<f8"),
         ("dh", N * To * V * Cl, "<f4"), ("dv", N * Ti * V * Cl, "<f4")]
runs = []
for r in range(6):
    model.load_state_dict(st)
    ws = torch.zeros(model._native.workspace_bytes(N), dtype=torch.uint8, device=d)
    out = torch.empty(N, C, device=d)
    model.native_forward(skel, sensor if spec.model == "two_stgcan_bilstm" else None, out, ws, True)
    grads = torch.zeros(model._native.nparam, device=d)
    model.native_backward(N, dout, grads, ws)
    torch.cuda.synchronize()
    snap = {}
    for what, n, ts in items:
        p = lib.f3_net_debug_tensor(model._native.h, N, L.ptr(ws), s, l, what.encode())
        snap[what] = torch.as_tensor(_Raw(p, n, ts), device=d).clone().cpu().double().numpy()
    runs.append(snap)
for what, n, ts in items:
    base = runs[0][what]
    den = np.abs(base).max() + 1e-30
    diffs = [np.abs(r[what] - base).max() / den for r in runs[1:]]
    print(f"{what:9s} max {den:.3e} run-diffs " + " ".join(f"{x:.1e}" for x in diffs))
q = runs[0]["q1"].reshape(N, -1)
print("q1 per-unit var (min 5):", np.sort(q.var(0))[:5], " mean^2/var max", (q.mean(0)**2 / (q.var(0) + 1e-30)).max())

# ---- wgrad kernel on exactly these tensors, repeated, vs torch ----
ws_last = None
model.load_state_dict(st)
ws = torch.zeros(model._native.workspace_bytes(N), dtype=torch.uint8, device=d)
out = torch.empty(N, C, device=d)
model.native_forward(skel, sensor if spec.model == "two_stgcan_bilstm" else None, out, ws, True)
grads = torch.zeros(model._native.nparam, device=d)
model.native_backward(N, dout, grads, ws)
torch.cuda.synchronize()
def get(what, n, ts="<f4"):
    p = lib.f3_net_debug_tensor(model._native.h, N, L.ptr(ws), s, l, what.encode())
    return torch.as_tensor(_Raw(p, n, ts), device=d).clone()
dh = get("dh", N * To * V * Cl).view(N, To, V, Cl)
gg = get("g", N * Ti * V * Cl).view(N, Ti, V, Cl)
fs = get("bn1_fsum", Cl, "<f8"); fq = get("bn1_fsq", Cl, "<f8")
pre = 'stgcan_1.' if s == 0 else 'stgcan_2.'
sd = model.state_dict()
gam = sd[f'{pre}st_gcan_networks.{l}.tcn.0.weight'].double(); bet = sd[f'{pre}st_gcan_networks.{l}.tcn.0.bias'].double()
cnt = N * Ti * V
mu = fs / cnt; var = fq / cnt - mu * mu
u = torch.relu((gg.double() - mu) / torch.sqrt(var + 1e-5) * gam + bet).float().contiguous()
stride = [1, 1, 1, 2, 1, 2, 1][l]
ref = torch.nn.grad.conv2d_weight(u.permute(0, 3, 1, 2).double(), (Cl, Cl, 9, 1), dh.permute(0, 3, 1, 2).double(),
                                  stride=(stride, 1), padding=(4, 0)).reshape(Cl, Cl, 9)
if STOPPED:
    np.save('gpurun_out/l6_ref.npy', ref.cpu().numpy())
else:
    ref = torch.from_numpy(np.load('gpurun_out/l6_ref.npy')).to(d)
for rep in range(4 if STOPPED else 0):
    dw = torch.empty(Cl, Cl, 9, device=d); db = torch.empty(Cl, device=d)
    L.check(lib.f3_conv_backward_weight(L.ptr(dh), L.ptr(u), L.ptr(dw), L.ptr(db), N, Ti, V, Cl, Cl, 9, stride, 4, 0,
                                        L.stream_handle()), "wg")
    torch.cuda.synchronize()
    print("isolated wgrad vs torch", ((dw.double() - ref).abs().max() / ref.abs().max()).item())
# what the full backward produced for this weight
off = [o for n, sh, o in model.param_views() if n == f'{pre}st_gcan_networks.{l}.tcn.2.weight'][0]
full = grads[off:off + Cl * Cl * 9].view(Cl, Cl, 9).double()
print("full-backward tcn.2.weight vs torch(our dh,u)", ((full - ref).abs().max() / ref.abs().max()).item())
