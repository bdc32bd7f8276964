"""ORACLE — test infrastructure only (never imported by the product path).

CPU fp32 restatement of the reference's `musa_model.Model` training step (the model the root
Multimodal_Fall3/main.py trains: Model(num_class=11, num_point=14, max_frame=300,
graph=adjGraph('coco_cut', 'uniform'), bias=True, edge=True, block_size=41, embed_dim=64,
n_stage=1, act_type='tanh'), main.py:307-320), written from scratch as functional PyTorch and
pinned to golden vectors produced by the reference module (tools/gen_golden.py ->
tests/golden/musa_*.npz, tests/test_oracle_golden.py).

It follows (file:line relative to /root/reference/Multimodal_Fall3/model/musa_model.py):

* embed (cnn1x1 + ReLU, no norm)                       423-452, 528-529
* SpatialGraphConv (gcn 1x1 -> einsum with A*edge, BN; residual 1x1 + BN; DropBlocks; tanh)
                                                        101-146
* SepTemporal_Block (depthwise (k,1) conv + BN + tanh, pointwise 1x1 + BN; residual identity or
  strided 1x1 + BN; DropBlocks; tanh)                  148-199
* Sep_TCN (shortcut 1x1; DW3-BN-LeakyReLU-PW-BN, ReLU; DW1-BN-LeakyReLU-PW-BN, ReLU; + shortcut)
                                                        400-474
* Classification_Module (Linear-LeakyReLU-LayerNorm-LeakyReLU-Dropout-Linear)  476-490
* Model.forward: mot = x[:, :2, :-1] - x[:, :2, 1:]; two streams; mean over (T,V); concat with
  the mean of the raw positions; classifier                                   492-589

Randomness. DropBlock (Randomized_DropBlock_Ske / Randomized_DropBlockT_1d, 39-99; keep_prob 0.9
hard-coded at :509) draws torch.bernoulli masks and a torch.randperm of the frames; the head has
Dropout(0.2). Here every draw is a counter hash (`uniform24`) of (seed, call, index) that the HIP
kernels reproduce bit for bit, so train-mode steps with DropBlock agree between the two
implementations. The reference's golden vectors are produced with keep_prob = 1 (DropBlock off,
the modules return their input) and the head dropout p = 0.
"""
from __future__ import annotations

import warnings
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

EMBED = 64
KEEP_PROB = 0.9
BLOCK_SIZE = 41
LEAKY = 0.01


def adjacency_uniform_coco_cut():
    """adjGraph('coco_cut', 'uniform').A (musa_model.py:200-349): normalize_digraph of the
    1-hop adjacency (self links + 13 edges), shape [1, 14, 14]."""
    V = 14
    edges = [(i, i) for i in range(V)] + [(6, 4), (4, 2), (2, 13), (13, 1), (5, 3), (3, 1), (12, 10), (10, 8),
                                          (8, 2), (11, 9), (9, 7), (7, 1), (13, 0)]
    A = np.zeros((V, V))
    for i, j in edges:
        A[j, i] = 1
        A[i, j] = 1
    Dl = A.sum(0)
    Dn = np.diag([d ** -1 if d > 0 else 0 for d in Dl])
    return (A @ Dn)[None].astype(np.float32)


def _bn_entries(out, p, C):
    for leaf in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
        out[p + leaf] = () if leaf == "num_batches_tracked" else (C,)


def param_shapes(V=14, num_class=11):
    """state_dict order of the reference Model (printed from the module; 427,107 parameters, A included)."""
    out = OrderedDict()
    out["joint_embed_pos.cnn.0.cnn.weight"] = (EMBED, 3, 1, 1)
    out["joint_embed_pos.cnn.0.cnn.bias"] = (EMBED,)
    out["joint_embed_mos.cnn.0.cnn.weight"] = (EMBED, 2, 1, 1)
    out["joint_embed_mos.cnn.0.cnn.bias"] = (EMBED,)
    C = 2 * EMBED
    for s in ("stream_pos", "stream_mot"):
        p = s + ".0."
        out[p + "A"] = (1, V, V)
        out[p + "edge"] = (1, V, V)
        out[p + "gcn.weight"] = (C, EMBED, 1, 1)
        out[p + "gcn.bias"] = (C,)
        _bn_entries(out, p + "bn.", C)
        out[p + "residual.0.weight"] = (C, EMBED, 1, 1)
        out[p + "residual.0.bias"] = (C,)
        _bn_entries(out, p + "residual.1.", C)
        for b, k in ((1, 3), (2, 5)):
            p = f"{s}.{b}."
            out[p + "A"] = (1, V, V)
            out[p + "edge"] = (1, V, V)
            out[p + "depth_conv.0.weight"] = (C, 1, k, 1)
            out[p + "depth_conv.0.bias"] = (C,)
            _bn_entries(out, p + "depth_conv.1.", C)
            out[p + "point_conv.0.weight"] = (C, C, 1, 1)
            out[p + "point_conv.0.bias"] = (C,)
            _bn_entries(out, p + "point_conv.1.", C)
            if b == 2:
                out[p + "residual.0.weight"] = (C, C, 1, 1)
                out[p + "residual.0.bias"] = (C,)
                _bn_entries(out, p + "residual.1.", C)
        p = s + ".3."
        M = (2 * C - C) // 2 + C   # 192
        out[p + "sep31.seq.0.weight"] = (C, 1, 3, 1)
        out[p + "sep31.seq.0.bias"] = (C,)
        _bn_entries(out, p + "sep31.seq.1.", C)
        out[p + "sep31.seq.3.weight"] = (M, C, 1, 1)
        out[p + "sep31.seq.3.bias"] = (M,)
        _bn_entries(out, p + "sep31.seq.4.", M)
        out[p + "sep11.seq.0.weight"] = (M, 1, 1, 1)
        out[p + "sep11.seq.0.bias"] = (M,)
        _bn_entries(out, p + "sep11.seq.1.", M)
        out[p + "sep11.seq.3.weight"] = (2 * C, M, 1, 1)
        out[p + "sep11.seq.3.bias"] = (2 * C,)
        _bn_entries(out, p + "sep11.seq.4.", 2 * C)
        out[p + "shortcut.weight"] = (2 * C, C, 1, 1)
        out[p + "shortcut.bias"] = (2 * C,)
    F_IN = 4 * C + 3
    out["fc.seq.0.weight"] = (128, F_IN)
    out["fc.seq.0.bias"] = (128,)
    out["fc.seq.2.weight"] = (128,)
    out["fc.seq.2.bias"] = (128,)
    out["fc.seq.5.weight"] = (num_class, 128)
    out["fc.seq.5.bias"] = (num_class,)
    return out


def is_buffer(name):
    return name.endswith(("running_mean", "running_var", "num_batches_tracked"))


def is_frozen(name):
    """A is a Parameter with requires_grad=False (musa_model.py:112, 181)."""
    return name.endswith(".A")


def init_state(seed, V=14, num_class=11):
    from oracle.prng import param_value
    st = OrderedDict()
    A = torch.from_numpy(adjacency_uniform_coco_cut())
    for name, shape in param_shapes(V, num_class).items():
        if name.endswith("running_mean"):
            st[name] = torch.zeros(shape)
        elif name.endswith("running_var"):
            st[name] = torch.ones(shape)
        elif name.endswith("num_batches_tracked"):
            st[name] = torch.tensor(0, dtype=torch.int64)
        elif name.endswith(".A"):
            st[name] = A.clone()
        elif name.endswith(".edge"):
            st[name] = torch.from_numpy(param_value(name, shape, seed))  # ones in the reference; U(0.5,1.5) here
        else:
            st[name] = torch.from_numpy(param_value(name, shape, seed))
    return st


# ---------------------------------------------------------------------------------------------
# counter-hash draws (shared bit-for-bit with the HIP kernels, musa.hip)
# ---------------------------------------------------------------------------------------------
def _mix32(x):
    x = np.asarray(x, dtype=np.uint32).copy()
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def uniform24(seed, call, n):
    """u[e] in [0, 1): (mix32(mix32(seed ^ call*0x9E3779B9) + e) >> 8) / 2^24, e = 0..n-1."""
    with np.errstate(over="ignore"):
        base = _mix32(np.uint32((int(seed) ^ (int(call) * 0x9E3779B9)) & 0xFFFFFFFF))
        e = np.arange(n, dtype=np.uint64)
        h = _mix32(((e + np.uint64(base)) & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    return (h >> np.uint32(8)).astype(np.float64) / float(1 << 24)


def _bern(p, u):
    """torch.bernoulli(p) with the uniform draw u (float32 p; keep u < p)."""
    return (torch.from_numpy(u.astype(np.float32)).reshape(p.shape) < p).to(p.dtype)


def drop_masks(y, Ae, seed, call, keep_prob=KEEP_PROB, block_size=BLOCK_SIZE):
    """dropT(dropS(y)) as factors: returns fS [n, v] and fT [n, t] with
    dropT(dropS(y)) == y * fS[n, None, v] * fT[n, t, None] for y [N, T, V, C] (channels last).
    Randomized_DropBlock_Ske (:39-70) then Randomized_DropBlockT_1d (:73-99); A = A*edge [1,V,V]."""
    N, T, V, C = y.shape
    y = y.detach()
    # dropS
    a = y.abs().mean(dim=(1, 3))                                    # [n, v]: mean over c and t
    a = a / a.sum() * a.numel()
    gamma = (1.0 - keep_prob) / (1 + 1.92)                          # num_point 14: the "else" branch
    m_seed = _bern(torch.clamp(a * gamma, max=1.0), uniform24(seed, 2 * call, N * V))
    M = m_seed @ Ae.detach().reshape(V, V)
    M = (M > 0.001).to(y.dtype)                                     # M[M>0.001]=1; M[M<0.5]=0
    mS = 1 - M
    fS = mS * (mS.numel() / mS.sum())
    # dropT on dropS's output
    ys = y * fS[:, None, :, None]
    b = ys.abs().mean(dim=(2, 3))                                   # [n, t]: mean over v then c
    b = b / b.sum() * b.numel()
    gT = (1.0 - keep_prob) / block_size
    m = _bern(torch.clamp(b * gT, max=1.0), uniform24(seed, 2 * call + 1, N * T))
    msum = F.max_pool1d(m[:, None, :], kernel_size=block_size, stride=1, padding=block_size // 2)[:, 0]
    keys = uniform24(seed ^ 0x5BD1E995, call, T)
    idx = torch.from_numpy(np.argsort(keys, kind="stable"))
    rm = msum[:, idx]
    mT = 1 - rm
    fT = mT * (mT.numel() / mT.sum())
    return fS, fT


def _conv1x1(x, w, b, stride=1):
    """x [N, T, V, Cin] channels-last; w [Cout, Cin, 1, 1]; stride over T."""
    if stride > 1:
        x = x[:, ::stride]
    return F.linear(x, w.flatten(1), b)


def _bn(st, p, x, training, momentum=0.1, eps=1e-5):
    C = x.shape[-1]
    flat = x.reshape(-1, C)
    if training:
        mean, var = flat.mean(0), flat.var(0, unbiased=False)
        n = flat.shape[0]
        with torch.no_grad():
            st[p + "running_mean"].mul_(1 - momentum).add_(mean.detach(), alpha=momentum)
            st[p + "running_var"].mul_(1 - momentum).add_(var.detach() * n / max(n - 1, 1), alpha=momentum)
            st[p + "num_batches_tracked"] += 1
    else:
        mean, var = st[p + "running_mean"], st[p + "running_var"]
    return (x - mean) / torch.sqrt(var + eps) * st[p + "weight"] + st[p + "bias"]


def _dwconv_t(x, w, b, stride, pad):
    """depthwise (k,1) conv over T on channels-last x [N, T, V, C]; w [C, 1, k, 1]."""
    N, T, V, C = x.shape
    y = F.conv2d(x.permute(0, 3, 1, 2), w, b, stride=(stride, 1), padding=(pad, 0), groups=C)
    return y.permute(0, 2, 3, 1)


def _drop(y, Ae, draws, call, training):
    if not training or draws is None:
        return y
    fS, fT = drop_masks(y, Ae, draws, call)
    return y * fS[:, None, :, None] * fT[:, :, None, None]


def sgc(st, p, x, training, draws, call0):
    """SpatialGraphConv.forward (:127-146)."""
    Ae = st[p + "A"] * st[p + "edge"]
    res = _bn(st, p + "residual.1.", _conv1x1(x, st[p + "residual.0.weight"], st[p + "residual.0.bias"]), training)
    g = _conv1x1(x, st[p + "gcn.weight"], st[p + "gcn.bias"])
    h = torch.einsum("ntvc,vw->ntwc", g, Ae[0])                    # 'nctv,cvw->nctw' with the size-1 c broadcast
    z = _bn(st, p + "bn.", h, training)
    return torch.tanh(_drop(z, Ae, draws, call0, training) + _drop(res, Ae, draws, call0 + 1, training))


def sep_temporal(st, p, x, k, stride, training, draws, call0):
    """SepTemporal_Block.forward (:185-199), expand_ratio 0, act tanh."""
    Ae = st[p + "A"] * st[p + "edge"]
    if stride == 1:
        res = x
    else:
        res = _bn(st, p + "residual.1.", _conv1x1(x, st[p + "residual.0.weight"], st[p + "residual.0.bias"], stride),
                  training)
    d = torch.tanh(_bn(st, p + "depth_conv.1.", _dwconv_t(x, st[p + "depth_conv.0.weight"],
                                                          st[p + "depth_conv.0.bias"], stride, (k - 1) // 2),
                       training))
    q = _bn(st, p + "point_conv.1.", _conv1x1(d, st[p + "point_conv.0.weight"], st[p + "point_conv.0.bias"]),
            training)
    return torch.tanh(_drop(q, Ae, draws, call0, training) + _drop(res, Ae, draws, call0 + 1, training))


def sep_tcn(st, p, x, training):
    """Sep_TCN.forward (:469-474)."""
    res = _conv1x1(x, st[p + "shortcut.weight"], st[p + "shortcut.bias"])
    q = p + "sep31.seq."
    a = F.leaky_relu(_bn(st, q + "1.", _dwconv_t(x, st[q + "0.weight"], st[q + "0.bias"], 1, 1), training), LEAKY)
    a = torch.relu(_bn(st, q + "4.", _conv1x1(a, st[q + "3.weight"], st[q + "3.bias"]), training))
    q = p + "sep11.seq."
    b = F.leaky_relu(_bn(st, q + "1.", _dwconv_t(a, st[q + "0.weight"], st[q + "0.bias"], 1, 0), training), LEAKY)
    b = torch.relu(_bn(st, q + "4.", _conv1x1(b, st[q + "3.weight"], st[q + "3.bias"]), training))
    return b + res


def stream(st, s, x, training, draws, sidx):
    c = sidx * 3 * 2   # DropBlock call ids: (stream, block, branch)
    x = sgc(st, s + ".0.", x, training, draws, c)
    x = sep_temporal(st, s + ".1.", x, 3, 1, training, draws, c + 2)
    x = sep_temporal(st, s + ".2.", x, 5, 2, training, draws, c + 4)
    return sep_tcn(st, s + ".3.", x, training)


def forward(st, x, training=True, draws=None, head_dropout=0.2):
    """Model.forward (:561-589), x [N, 3, T, V] -> logits. draws: the step's hash seed (None: no
    DropBlock / dropout, i.e. keep_prob = 1 and Dropout p = 0)."""
    pts = x
    mot = x[:, :2, :-1] - x[:, :2, 1:]
    tp = pts.permute(0, 2, 3, 1)                                    # channels last [N, T, V, C]
    tm = mot.permute(0, 2, 3, 1)
    ep = torch.relu(_conv1x1(tp, st["joint_embed_pos.cnn.0.cnn.weight"], st["joint_embed_pos.cnn.0.cnn.bias"]))
    em = torch.relu(_conv1x1(tm, st["joint_embed_mos.cnn.0.cnn.weight"], st["joint_embed_mos.cnn.0.cnn.bias"]))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        o1 = stream(st, "stream_pos", ep, training, draws, 0).mean(dim=(1, 2))
        o2 = stream(st, "stream_mot", em, training, draws, 1).mean(dim=(1, 2))
    rp = pts.mean(dim=(2, 3))
    z = torch.cat([o1, o2, rp], dim=-1)
    z = F.leaky_relu(F.linear(z, st["fc.seq.0.weight"], st["fc.seq.0.bias"]), LEAKY)
    z = F.leaky_relu(F.layer_norm(z, (z.shape[-1],), st["fc.seq.2.weight"], st["fc.seq.2.bias"]), LEAKY)
    if training and draws is not None and head_dropout > 0:
        keep = torch.from_numpy((uniform24(draws ^ 0x1B873593, 0, z.numel()) >= head_dropout).astype(np.float32))
        z = z * keep.reshape(z.shape) / (1.0 - head_dropout)
    return F.linear(z, st["fc.seq.5.weight"], st["fc.seq.5.bias"])


def soft_ce(out, target):
    return -(target * F.log_softmax(out, dim=-1)).sum(dim=-1).mean()


def train_step(st, x, label, lr=1e-3, sq=None, alpha=0.99, eps=1e-8, draws=None):
    """forward -> CE -> backward -> RMSprop (root main.py: RMSprop lr 1e-3, CrossEntropyLoss).
    Mutates st; returns (logits, loss, grads) with grads taken before the update. Parameters
    without a gradient in the reference (A: requires_grad=False; the SepTemporal blocks' edge, used
    only inside DropBlock masks) get zero gradients here and are not updated."""
    names = [k for k in st if not is_buffer(k) and not is_frozen(k)]
    for k in names:
        st[k] = st[k].detach().clone().requires_grad_(True)
    out = forward(st, x, True, draws)
    loss = soft_ce(out, label)
    gl = torch.autograd.grad(loss, [st[k] for k in names], allow_unused=True)
    grads = OrderedDict((k, torch.zeros_like(st[k]) if g is None else g.detach()) for k, g in zip(names, gl))
    with torch.no_grad():
        for k in names:
            st[k] = st[k].detach()
        if sq is None:
            sq = {k: torch.zeros_like(st[k]) for k in names}
        for k, g in grads.items():
            sq[k].mul_(alpha).addcmul_(g, g, value=1 - alpha)
            st[k].addcdiv_(g, sq[k].sqrt().add_(eps), value=-lr)
    return out.detach(), loss.detach(), grads
