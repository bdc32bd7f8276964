"""Diagnostic: check the layer-l tcn input-gradient (dv) of stream s against torch."""
import ctypes, sys
import numpy as np
import torch
import torch.nn.functional as F
sys.path.insert(0, '.')
from oracle import model_cpu as oc
from tests.golden_util import load
from tests.test_gpu_parity import build_from_spec, call
import fall_multimodal_amd._lib as L
import fall_multimodal_amd.model as M

d = torch.device('cuda')
g, spec = load('har')
st = oc.init_state(spec, int(g['seed'][0]))
model = build_from_spec(spec, d); model.load_state_dict(st); model.train()
skel = torch.from_numpy(g['skel']).to(d); sensor = torch.from_numpy(g['sensor']).to(d)
label = torch.from_numpy(g['label']).to(d)
saved = {}
orig = M._Fall3Fn.backward
def bw(ctx, dout):
    r = orig(ctx, dout); saved['ws'] = ctx.ws; return r
M._Fall3Fn.backward = staticmethod(bw)
out = call(model, spec, skel, sensor)
torch.nn.CrossEntropyLoss()(out, label).backward()
torch.cuda.synchronize()
ws = saved['ws']; N = 4; V = 14
lib = L.lib()
class _Raw:
    def __init__(self, p, n, ts):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": ts, "data": (p, False), "version": 2}
def T(s, l, what, shape):
    p = lib.f3_net_debug_tensor(model._native.h, N, L.ptr(ws), s, l, what.encode())
    return torch.as_tensor(_Raw(p, int(np.prod(shape)), "<f4"), device=d).clone().view(shape)
def Td(s, l, what, n):
    p = lib.f3_net_debug_tensor(model._native.h, N, L.ptr(ws), s, l, what.encode())
    return torch.as_tensor(_Raw(p, n, "<f8"), device=d).clone()
import os
STOP = [int(v) for v in os.environ['F3_DEBUG_BWD_STOP'].split(',')]
for s in (STOP[0],):
    pre = 'stgcan_1.' if s == 0 else 'stgcan_2.'
    for l in (STOP[1],):
        Lyr = model._native  # geometry
        Ti = {0: [30,30,30,30,15,15,8], 1: [29,29,29,29,15,15,8]}[s][l]
        To = {0: [30,30,30,15,15,8,8], 1: [29,29,29,15,15,8,8]}[s][l]
        C = [64,64,64,128,128,256,256][l]
        stride = [1,1,1,2,1,2,1][l]
        dh = T(s, l, 'dh', (N, To, V, C)).double()
        gg = T(s, l, 'g', (N, Ti, V, C)).double()
        dv = T(s, l, 'dv', (N, Ti, V, C)).double()
        fs = Td(s, l, 'bn1_fsum', C); fq = Td(s, l, 'bn1_fsq', C)
        cnt = N * Ti * V
        mu = fs / cnt; var = fq / cnt - mu * mu
        sd = model.state_dict()
        gam = sd[f'{pre}st_gcan_networks.{l}.tcn.0.weight'].double(); bet = sd[f'{pre}st_gcan_networks.{l}.tcn.0.bias'].double()
        W = sd[f'{pre}st_gcan_networks.{l}.tcn.2.weight'].double()
        # torch: dU = conv_transpose of dh
        dhn = dh.permute(0, 3, 1, 2)
        dU = F.conv_transpose2d(dhn, W, stride=(stride, 1), padding=(4, 0), output_padding=(Ti - ((To - 1) * stride - 8 + 9), 0))
        dU = dU.permute(0, 2, 3, 1)
        u = (gg - mu) / torch.sqrt(var + 1e-5) * gam + bet
        dv_ref = dU * (u > 0)
        err = (dv - dv_ref).abs().max().item() / dv_ref.abs().max().item()
        bad = ((dv - dv_ref).abs() > 1e-4 * dv_ref.abs().max()).nonzero()
        print(f"stream {s} layer {l}: dv normrel err {err:.2e} nbad {bad.shape[0]}", bad[:5].tolist())
        bs = Td(s, l, 'bn1_bsum', C); bq = Td(s, l, 'bn1_bsq', C)
        xh = (gg - mu) / torch.sqrt(var + 1e-5)
        rs = dv_ref.sum((0, 1, 2)); rq = (dv_ref * xh).sum((0, 1, 2))
        print("  bsum err", ((bs - rs).abs().max() / rs.abs().max()).item(), " bsq err", ((bq - rq).abs().max() / rq.abs().max()).item())
        print("  dh max", dh.abs().max().item(), "g var min", var.min().item(), "mean^2/var max", (mu*mu/var).max().item())

# ---- compare our dh with the fp64 oracle's gradient wrt the tcn conv output ----
import torch.nn.functional as F2
s, l = STOP
pre = 'stgcan_1.' if s == 0 else 'stgcan_2.'
st64 = {k: (v.double() if v.dtype == torch.float32 else v) for k, v in st.items()}
cap = {}
orig_conv = F2.conv2d
def hooked(x, w, b=None, stride=1, padding=0, *a, **k):
    y = orig_conv(x, w, b, stride, padding, *a, **k)
    if w.shape[2] == 9 and w is st64_ref[f'{pre}st_gcan_networks.{l}.tcn.2.weight']:
        y.retain_grad(); cap['h'] = y
    return y
st64_ref = {}
names = [k for k in st64 if not oc.is_buffer(k)]
for k in names:
    st64[k] = st64[k].detach().clone().requires_grad_(True)
st64_ref.update(st64)
oc.F.conv2d = hooked
out64 = oc.forward(st64, spec, *(torch.from_numpy(g[k]).double() for k in ('skel', 'sensor')), training=True)
loss64 = oc.soft_ce(out64, torch.from_numpy(g['label']).double())
loss64.backward()
oc.F.conv2d = orig_conv
dh_ref = cap['h'].grad.permute(0, 2, 3, 1).to(d)
To = dh_ref.shape[1]; C = dh_ref.shape[3]
dh = T(s, l, 'dh', (N, To, V, C)).double()
err = (dh - dh_ref).abs()
print("dh normrel err", (err.max() / dh_ref.abs().max()).item())
e_nc = (dh - dh_ref).mean((1, 2))
print("per-(n,c) mean err max", e_nc.abs().max().item(), " per-c mean err max", e_nc.mean(0).abs().max().item())
resid = (dh - dh_ref) - e_nc[:, None, None, :]
print("residual err after removing per-(n,c) mean", (resid.abs().max() / dh_ref.abs().max()).item())

# ---- dx handed down by layer l+1 (= grad of layer l's output) vs fp64 oracle ----
cap2 = {}
orig_block = oc.st_gcan_block
def blk(S_, p_, x, A_eff, cin, cout, stride, res_kind):
    if p_ == f"{pre}st_gcan_networks.{l + 1}.":
        x.retain_grad(); cap2['x'] = x
    return orig_block(S_, p_, x, A_eff, cin, cout, stride, res_kind)
oc.st_gcan_block = blk
st64b = {k: (v.double() if v.dtype == torch.float32 else v) for k, v in st.items()}
for k in names:
    st64b[k] = st64b[k].detach().clone().requires_grad_(True)
o = oc.forward(st64b, spec, *(torch.from_numpy(g[k]).double() for k in ('skel', 'sensor')), training=True)
oc.soft_ce(o, torch.from_numpy(g['label']).double()).backward()
oc.st_gcan_block = orig_block
dx_ref = cap2['x'].grad.permute(0, 2, 3, 1).to(d)
dxo = T(s, l, 'dx0', tuple(dx_ref.shape)).double()
print("dx(l+1 -> l) normrel err", ((dxo - dx_ref).abs().max() / dx_ref.abs().max()).item())
ee = (dxo - dx_ref).abs()
idx = (ee > 1e-3 * dx_ref.abs().max()).nonzero()
print(" nbad", idx.shape[0], "t values", sorted(set(idx[:, 1].tolist())), "v values", sorted(set(idx[:, 2].tolist()))[:20])
