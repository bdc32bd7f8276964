"""Diagnostic: forward twice, compare saved per-layer activations (debug accessor)."""
import sys
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

d = torch.device('cuda')
g, spec = load('har')
st = oc.init_state(spec, int(g['seed'][0]))
model = build_from_spec(spec, d)
model.load_state_dict(st)
skel = torch.from_numpy(g['skel']).to(d); sensor = torch.from_numpy(g['sensor']).to(d)
N = 4; V = 14
lib = L.lib()
snaps = []
for r in range(4):
    model.load_state_dict(st)
    ws = torch.zeros(model._native.workspace_bytes(N), dtype=torch.uint8, device=d)
    out = torch.empty(N, 11, device=d)
    model.native_forward(skel, sensor, out, ws, True)
    torch.cuda.synchronize()
    snap = {}
    for s in (0, 1):
        T = [30, 29][s]
        Ts = {0: [30,30,30,15,15,8,8], 1: [29,29,29,15,15,8,8]}[s]
        Ti = {0: [30,30,30,30,15,15,8], 1: [29,29,29,29,15,15,8]}[s]
        C = [64,64,64,128,128,256,256]
        for l in range(7):
            for what, rows, cols in (("g", N*Ti[l]*V, C[l]), ("h", N*Ts[l]*V, C[l]), ("out", N*Ts[l]*V, C[l]), ("att", N, C[l])):
                p = lib.f3_net_debug_tensor(model._native.h, N, L.ptr(ws), s, l, what.encode())
                snap[(s, l, what)] = torch.as_tensor(_Raw(p, rows*cols, "<f4"), device=d).clone().cpu().numpy()
    snaps.append(snap)
for k in snaps[0]:
    e = max(np.abs(sn[k] - snaps[0][k]).max() for sn in snaps[1:]) / (np.abs(snaps[0][k]).max() + 1e-30)
    if e > 1e-6:
        print(k, f"{e:.2e}")
print("done")
