"""ORACLE — test infrastructure only (never imported by the product path).

CPU fp32 restatement of the reference's skeleton-only TARGCN training step (BASELINE
config 2), written from scratch as functional PyTorch. It is the parity checker for the
HIP path (tests/, __graft_entry__.smoke) and is pinned to golden vectors produced by the
reference's own modules (tools/gen_golden.py -> tests/golden/targcn_*.npz,
tests/test_oracle_golden.py).

It follows, op for op (file:line relative to /root/reference):

* static adjacency sym_norm_Adj + 2x softmax  EmbGCN.py:14-26, 63-64, 78
* EmbGCN (adaptive supports, node weights)    EmbGCN.py:59-89
* graph GRU cell                              GRU.py:8-30
* AVWDCRNN (2 layers x T steps, then TA)      TRAGCN.py:134-175
* Transform / PositionalEncoding / TA layer   TA.py:22-108
* TARGCN head (end_conv -> pool -> Linear)    TRAGCN.py:177-224
* training: CE(out, soft labels), RMSprop     TARGCN_HAR_conv_10kfold.ipynb cell 3
  (model(pts.permute(0,2,3,1)); torch.nn.CrossEntropyLoss; RMSprop)

The reference only runs with adj=None (its default adj raises): the static
adjacency is then a V x V matrix of ones.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

T_STEPS, DIN, HID, EMB, HORIZON, OUT_DIM = 30, 3, 64, 64, 30, 64


def param_shapes(V: int, num_class: int = 11) -> "OrderedDict[str, tuple]":
    """state_dict order of TARGCN(adj=None, num_nodes=V) (TRAGCN.py:177-205)."""
    out = OrderedDict()
    out["node_embeddings"] = (V, EMB)
    for layer, din in enumerate((DIN, HID)):
        for part, o in (("gate", 2 * HID), ("update", HID)):
            p = f"encoder.dcrnn_cells.{layer}.{part}."
            i = din + HID
            out[p + "weights_pool"] = (EMB, i, o)
            out[p + "bias_pool"] = (EMB, o)
            out[p + "linear.weight"] = (o, i)
            out[p + "linear.bias"] = (o,)
    for l in range(2):
        p = f"encoder.trans_layer_T.trans_layers.{l}."
        out[p + "vff.weight"] = (OUT_DIM, OUT_DIM)
        out[p + "vff.bias"] = (OUT_DIM,)
        for c in ("conv1", "conv2"):
            out[p + c + ".weight"] = (T_STEPS, T_STEPS, 1, 3)
            out[p + c + ".bias"] = (T_STEPS,)
        for n in ("ln", "lnff"):
            out[p + n + ".weight"] = (OUT_DIM,)
            out[p + n + ".bias"] = (OUT_DIM,)
        out[p + "ff.0.weight"] = (OUT_DIM, OUT_DIM)
        out[p + "ff.0.bias"] = (OUT_DIM,)
        out[p + "ff.2.weight"] = (OUT_DIM, OUT_DIM)
        out[p + "ff.2.bias"] = (OUT_DIM,)
    out["encoder.trans_layer_T.PE.pe"] = (1, T_STEPS, 1, OUT_DIM)
    out["end_conv.weight"] = (HORIZON * OUT_DIM, 6, 1, HID)
    out["end_conv.bias"] = (HORIZON * OUT_DIM,)
    out["fc.2.weight"] = (num_class, OUT_DIM)
    out["fc.2.bias"] = (num_class,)
    return out


def is_buffer(name):
    return name.endswith(".pe")


def positional_encoding(T=T_STEPS, Fdim=OUT_DIM):
    """TA.py:75-86 (sin on even, cos on odd features), fp32 as the reference computes it."""
    pe = torch.zeros(T, Fdim)
    position = torch.arange(0, T).unsqueeze(1)
    div = torch.exp(torch.arange(0, Fdim, 2) * -(math.log(10000.0) / Fdim))
    pe[:, 0::2] = torch.sin(position * div)
    pe[:, 1::2] = torch.cos(position * div)
    return pe.unsqueeze(0).unsqueeze(2)


def static_colscale(V: int) -> torch.Tensor:
    """EmbGCN's static branch x_static = einsum('nm,bmc->bmc', softmax(M,-1), x) is a per-node
    scale of x by the column sums of M (EmbGCN.py:78), M = softmax(D^-1/2 (W + I/2) D^-1/2)
    (EmbGCN.py:14-26,63-64; implicit softmax dim = 1 for 2-D) with W = ones (adj=None,
    TRAGCN.py:191). Returns cs[m] = sum_n softmax(M, -1)[n, m] as fp32."""
    W = np.ones((V, V)) + 0.5 * np.identity(V)
    D = np.diag(1.0 / np.sum(W, axis=1))
    sym = np.dot(np.dot(np.sqrt(D), W), np.sqrt(D))
    M = F.softmax(torch.from_numpy(sym).to(torch.float32), dim=1)
    return torch.softmax(M, dim=-1).sum(0)


def init_state(V: int, seed: int, num_class: int = 11):
    from oracle.prng import param_value
    st = OrderedDict()
    for name, shape in param_shapes(V, num_class).items():
        if is_buffer(name):
            st[name] = positional_encoding()
        else:
            st[name] = torch.from_numpy(param_value(name, shape, seed))
    return st


def supports(E):
    """EmbGCN.py:74-75: softmax(relu(E E^T), dim=1) + I."""
    V = E.shape[0]
    return torch.eye(V) + F.softmax(F.relu(E @ E.t()), dim=1)


def embgcn(st, p, x, E, S, cs):
    """EmbGCN.forward (EmbGCN.py:69-89): node-specific weights + static gated branch."""
    xs = F.linear(x * cs.view(1, -1, 1), st[p + "linear.weight"], st[p + "linear.bias"])
    W = torch.einsum("nd,dio->nio", E, st[p + "weights_pool"])
    b = E @ st[p + "bias_pool"]
    xg = torch.einsum("nm,bmc->bnc", S, x)
    return torch.einsum("bni,nio->bno", xg, W) + b + torch.sigmoid(xs) * xs


def gru(st, p, x, h, E, S, cs):
    """GRU.forward (GRU.py:17-27)."""
    zr = torch.sigmoid(embgcn(st, p + "gate.", torch.cat([x, h], -1), E, S, cs))
    z, r = zr.split(HID, dim=-1)
    hc = torch.tanh(embgcn(st, p + "update.", torch.cat([x, r * h], -1), E, S, cs))
    return z * h + (1 - z) * hc


def transform(st, p, x):
    """Transform.forward (TA.py:40-69), x [B,T,N,C]."""
    c = x.shape[-1]
    q = F.conv2d(x, st[p + "conv1.weight"], st[p + "conv1.bias"]).permute(0, 2, 1, 3)
    k = F.conv2d(x, st[p + "conv2.weight"], st[p + "conv2.bias"]).permute(0, 2, 3, 1)
    v = F.linear(x, st[p + "vff.weight"], st[p + "vff.bias"]).permute(0, 2, 1, 3)
    A = torch.softmax((q @ k) / (c ** 0.5), -1)
    val = (A @ v).permute(0, 2, 1, 3) + x
    val = F.layer_norm(val, (c,), st[p + "ln.weight"], st[p + "ln.bias"])
    f = F.linear(F.relu(F.linear(val, st[p + "ff.0.weight"], st[p + "ff.0.bias"])),
                 st[p + "ff.2.weight"], st[p + "ff.2.bias"]) + val
    return F.layer_norm(f, (c,), st[p + "lnff.weight"], st[p + "lnff.bias"])


def forward(st, source):
    """TARGCN.forward (TRAGCN.py:207-224), source [B, T, N, 3] -> logits [B, C]."""
    B, T, V, _ = source.shape
    E = st["node_embeddings"]
    S = supports(E)
    cs = static_colscale(V)
    cur = source
    for layer in range(2):
        p = f"encoder.dcrnn_cells.{layer}."
        h = source.new_zeros(B, V, HID)
        outs = []
        for t in range(T):
            h = gru(st, p, cur[:, t], h, E, S, cs)
            outs.append(h)
        cur = torch.stack(outs, dim=1)
    x = cur + st["encoder.trans_layer_T.PE.pe"]
    for l in range(2):
        x = transform(st, f"encoder.trans_layer_T.trans_layers.{l}.", x)
    y = F.conv2d(x[:, -6:], st["end_conv.weight"], st["end_conv.bias"])
    y = y.squeeze(-1).reshape(-1, HORIZON, OUT_DIM, V).permute(0, 1, 3, 2)
    y = y.permute(0, 3, 1, 2).mean(dim=(2, 3))
    return F.linear(y, st["fc.2.weight"], st["fc.2.bias"])


def soft_ce(out, target):
    return -(target * F.log_softmax(out, dim=-1)).sum(dim=-1).mean()


def train_step(st, source, label, lr=1e-5, sq=None, alpha=0.99, eps=1e-8):
    """forward -> CE -> backward -> RMSprop (TARGCN notebook: RMSprop(lr=1e-5)).
    Mutates st; returns (logits, loss, grads) with grads taken before the update."""
    names = [k for k in st if not is_buffer(k)]
    for k in names:
        st[k] = st[k].detach().clone().requires_grad_(True)
    out = forward(st, source)
    loss = soft_ce(out, label)
    gl = torch.autograd.grad(loss, [st[k] for k in names])
    grads = OrderedDict((k, g.detach()) for k, g in zip(names, gl))
    with torch.no_grad():
        for k in names:
            st[k] = st[k].detach()
        if sq is None:
            sq = {k: torch.zeros_like(st[k]) for k in names}
        for k, g in grads.items():
            sq[k].mul_(alpha).addcmul_(g, g, value=1 - alpha)
            st[k].addcdiv_(g, sq[k].sqrt().add_(eps), value=-lr)
    return out.detach(), loss.detach(), grads


def synthetic_source(batch, V, num_class, seed, T=T_STEPS):
    """Skeleton windows in the notebook's TARGCN input layout pts.permute(0,2,3,1) = [B,T,V,3]
    (the same synthetic clips as oracle.prng.synthetic_batch) and soft labels."""
    from oracle.prng import synthetic_batch
    skel, _, label = synthetic_batch(batch, V, num_class, 1, seed, frames=T)
    return np.ascontiguousarray(skel.transpose(0, 2, 3, 1)), label
