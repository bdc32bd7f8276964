"""ORACLE — test infrastructure only (never imported by the product path).

A CPU fp32 restatement of the reference's 3-stream fall-detection training step,
written from scratch as plain functional PyTorch on CPU, used (a) as the parity
checker for the HIP path in `tests/` and `__graft_entry__.smoke()`, and (b) as
the timed CPU baseline ("port") in `bench.py`.

It follows, op for op (file:line relative to /root/reference):

* skeleton graph A[K,V,V]               Multimodal_Fall3/model/graph.py:20-126
* STGCAN stream (data_bn, 7 st_gcan, pool) Multimodal_Fall3/model/stgcan.py:147-228
* st_gcan block (gcn, tcn, CA, residual)   Multimodal_Fall3/model/stgcan.py:79-144
* GraphConvolution (1x1 conv + einsum)     Multimodal_Fall3/model/stgcan.py:50-56
* Channel_Attention                        Multimodal_Fall3/model/stgcan.py:59-74
* BiLSTM sensor branch                     Multimodal_Fall3/model/bilstm.py:21-59
* CNN1D / CNN_BiLSTM (UR notebook)         GSTCAN_UR_conv.ipynb cell 2 (:493-586)
* sensor-only CNN_BiLSTM (BASELINE cfg 1)  GSTCAN_UR_sensor.ipynb cell 2 (:493-586)
* TwoStreamSTGCAN(_BiLSTM) fusion          Multimodal_Fall3/model/combination.py:9-46
* notebook 3-stream (+softmax)             GSTCAN_HAR_conv_10kfold.ipynb:390-444
* CE with soft targets                     Multimodal_Fall3/model/main.py:113,280
* RMSprop(lr) defaults                     Multimodal_Fall3/model/optimizer.py:20-21

Parity pin: tests/test_oracle_golden.py checks this restatement against golden
vectors produced by running the reference's own modules in the build container
(tools/gen_golden.py -> tests/golden/*.npz).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------
# graph (graph.py:20-126)
# --------------------------------------------------------------------------
_LAYOUTS = {
    # graph.py:26-32 — COCO with ears/eyes removed, centre node 13
    "coco_cut": (14, 13, [(6, 4), (4, 2), (2, 13), (13, 1), (5, 3), (3, 1), (12, 10),
                          (10, 8), (8, 2), (11, 9), (9, 7), (7, 1), (13, 0)]),
    # graph.py:34-49 — 17 COCO keypoints + centre node 17
    "coco_mmpose": (18, 17, [(0, 1), (1, 3), (0, 2), (2, 4), (17, 0), (17, 6), (6, 8),
                             (8, 10), (17, 5), (5, 7), (7, 9), (17, 12), (12, 14),
                             (14, 16), (17, 11), (11, 13), (13, 15)]),
}


def graph_adjacency(layout: str = "coco_cut", strategy: str = "spatial",
                    max_hop: int = 1, dilation: int = 1) -> np.ndarray:
    if layout not in _LAYOUTS:
        raise ValueError("This layout is not supported!")
    v, center, links = _LAYOUTS[layout]
    edges = [(i, i) for i in range(v)] + list(links)
    adj = np.zeros((v, v))
    for i, j in edges:
        adj[i, j] = adj[j, i] = 1
    hop = np.full((v, v), np.inf)
    reach = [np.linalg.matrix_power(adj, d) > 0 for d in range(max_hop + 1)]
    for d in range(max_hop, -1, -1):
        hop[reach[d]] = d
    hops = list(range(0, max_hop + 1, dilation))
    base = np.zeros((v, v))
    for h in hops:
        base[hop == h] = 1
    deg = base.sum(0)
    dinv = np.diag([1.0 / x if x > 0 else 0.0 for x in deg])
    norm = base @ dinv  # column-normalised (normalize_digraph, graph.py:118-126)
    if strategy == "uniform":
        return norm[None].copy()
    if strategy == "distance":
        out = np.zeros((len(hops), v, v))
        for i, h in enumerate(hops):
            out[i][hop == h] = norm[hop == h]
        return out
    if strategy == "spatial":
        parts = []
        for h in hops:
            root, close, far = (np.zeros((v, v)) for _ in range(3))
            for i in range(v):
                for j in range(v):
                    if hop[j, i] != h:
                        continue
                    if hop[j, center] == hop[i, center]:
                        root[j, i] = norm[j, i]
                    elif hop[j, center] > hop[i, center]:
                        close[j, i] = norm[j, i]
                    else:
                        far[j, i] = norm[j, i]
            if h == 0:
                parts.append(root)
            else:
                parts += [root + close, far]
        return np.stack(parts)
    raise ValueError("This strategy is not supported!")


# --------------------------------------------------------------------------
# model specification + parameter table (state_dict order of the reference)
# --------------------------------------------------------------------------
@dataclass
class Spec:
    model: str = "two_stgcan_bilstm"   # two_stgcan_bilstm | two_stgcan | stgcn | bilstm
    layout: str = "coco_cut"
    strategy: str = "spatial"
    num_class: int = 11
    in_channels: int = 3
    sensor: str = "bilstm"             # bilstm | cnn_bilstm | none
    sensor_dim: int = 15
    sensor_classes: int | None = None  # BiLSTM head width (defaults to num_class)
    softmax_output: bool = False       # notebook form returns softmax (nb :444)
    naming: str = "package"            # package | notebook

    @property
    def s_classes(self):
        return self.num_class if self.sensor_classes is None else self.sensor_classes


STREAM_CHANNELS = [(None, 64, 1, "none"), (64, 64, 1, "id"), (64, 64, 1, "id"),
                   (64, 128, 2, "conv"), (128, 128, 1, "id"), (128, 256, 2, "conv"),
                   (256, 256, 1, "id")]  # stgcan.py:182-194


def _bn(p, n, out):
    out[p + ".weight"] = (n,)
    out[p + ".bias"] = (n,)
    out[p + ".running_mean"] = (n,)
    out[p + ".running_var"] = (n,)
    out[p + ".num_batches_tracked"] = ()


def stream_shapes(prefix, cin, K, V, spec, num_class=None):
    out = OrderedDict()
    layers = "st_gcn_networks" if spec.naming == "notebook" else "st_gcan_networks"
    out[prefix + "A"] = (K, V, V)
    _bn(prefix + "data_bn", cin * V, out)
    for i, (ci, co, s, res) in enumerate(STREAM_CHANNELS):
        ci = cin if ci is None else ci
        p = f"{prefix}{layers}.{i}."
        out[p + "gcn.conv.weight"] = (K * co, ci, 1, 1)
        out[p + "gcn.conv.bias"] = (K * co,)
        _bn(p + "tcn.0", co, out)
        out[p + "tcn.2.weight"] = (co, co, 9, 1)
        out[p + "tcn.2.bias"] = (co,)
        _bn(p + "tcn.3", co, out)
        if res == "conv":
            out[p + "residual.0.weight"] = (co, ci, 1, 1)
            out[p + "residual.0.bias"] = (co,)
            _bn(p + "residual.1", co, out)
        q = p + "channel_attention_module.atten."
        out[q + "1.weight"] = (co // 4, co, 1, 1)
        out[q + "1.bias"] = (co // 4,)
        _bn(q + "2", co // 4, out)
        out[q + "4.weight"] = (co, co // 4, 1, 1)
        out[q + "4.bias"] = (co,)
    for i in range(len(STREAM_CHANNELS)):
        out[f"{prefix}edge_importance.{i}"] = (K, V, V)
    if num_class is not None:
        out[prefix + "cls.weight"] = (num_class, 256, 1, 1)
        out[prefix + "cls.bias"] = (num_class,)
    return out


def bilstm_shapes(prefix, S, H, C):
    out = OrderedDict()
    for sfx in ("", "_reverse"):
        out[f"{prefix}lstm1.weight_ih_l0{sfx}"] = (4 * H, S)
        out[f"{prefix}lstm1.weight_hh_l0{sfx}"] = (4 * H, H)
        out[f"{prefix}lstm1.bias_ih_l0{sfx}"] = (4 * H,)
        out[f"{prefix}lstm1.bias_hh_l0{sfx}"] = (4 * H,)
    _bn(prefix + "batchnorm", 2 * H, out)
    r = int(2 * H * (1 / 8))
    out[prefix + "channelattention.attention.0.weight"] = (r, 2 * H)
    out[prefix + "channelattention.attention.0.bias"] = (r,)
    out[prefix + "channelattention.attention.2.weight"] = (2 * H, r)
    out[prefix + "channelattention.attention.2.bias"] = (2 * H,)
    out[prefix + "fc.1.weight"] = (C, 2 * H)
    out[prefix + "fc.1.bias"] = (C,)
    return out


def cnn1d_shapes(prefix, S, T):
    out = OrderedDict()
    out[prefix + "layer1.0.weight"] = (16, S, 5)
    out[prefix + "layer1.0.bias"] = (16,)
    _bn(prefix + "layer1.1", 16, out)
    out[prefix + "layer2.0.weight"] = (32, 16, 5)
    out[prefix + "layer2.0.bias"] = (32,)
    _bn(prefix + "layer2.1", 32, out)
    out[prefix + "fc.weight"] = (32, 32 * ((T // 2) // 2))  # unused in forward (nb :507)
    out[prefix + "fc.bias"] = (32,)
    return out


def prefixes(spec):
    if spec.naming == "notebook":
        return "pts_stream.", "mot_stream.", "sensor.", "fcn."
    return "stgcan_1.", "stgcan_2.", "lstm.", "fc."


def param_shapes(spec: Spec, sensor_frames: int = 30) -> "OrderedDict[str, tuple]":
    A = graph_adjacency(spec.layout, spec.strategy)
    K, V = A.shape[0], A.shape[1]
    if spec.model == "stgcn":
        return stream_shapes("", spec.in_channels, K, V, spec, spec.num_class)
    if spec.model == "bilstm":
        if spec.sensor == "cnn_bilstm":  # sensor-only CNN_BiLSTM (GSTCAN_UR_sensor.ipynb:572-586)
            out = cnn1d_shapes("cnn.", spec.sensor_dim, sensor_frames)
            out.update(bilstm_shapes("bilstm.", 32, 64, spec.num_class))
            return out
        return bilstm_shapes("", spec.sensor_dim, 64, spec.num_class)
    p1, p2, ps, pf = prefixes(spec)
    out = OrderedDict()
    out.update(stream_shapes(p1, 3, K, V, spec))
    out.update(stream_shapes(p2, 2, K, V, spec))
    sens = OrderedDict()
    fc_in = 512
    if spec.model == "two_stgcan_bilstm":
        if spec.sensor == "cnn_bilstm":
            sens.update(cnn1d_shapes(ps + "cnn.", spec.sensor_dim, sensor_frames))
            sens.update(bilstm_shapes(ps + "bilstm.", 32, 64, spec.s_classes))
        else:
            sens.update(bilstm_shapes(ps, spec.sensor_dim, 64, spec.s_classes))
        fc_in += spec.s_classes
    fc = OrderedDict([(pf + "weight", (spec.num_class, fc_in)), (pf + "bias", (spec.num_class,))])
    # registration order: package lstm then fc (combination.py:31-34); notebook fcn then
    # sensor (GSTCAN_HAR_conv_10kfold.ipynb / GSTCAN_UR_conv.ipynb TwoStreamSpatialTemporalGraph)
    for part in ((fc, sens) if spec.naming == "notebook" else (sens, fc)):
        out.update(part)
    return out


def is_buffer(name):
    leaf = name.rsplit(".", 1)[-1]
    return leaf in ("running_mean", "running_var", "num_batches_tracked") or leaf == "A"


def init_state(spec: Spec, seed: int, sensor_frames: int = 30):
    """Full state dict (params from the portable PRNG, buffers at their defaults)."""
    from oracle.prng import param_value
    A = torch.tensor(graph_adjacency(spec.layout, spec.strategy), dtype=torch.float32)
    st = OrderedDict()
    for name, shape in param_shapes(spec, sensor_frames).items():
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "A":
            st[name] = A.clone()
        elif leaf == "running_mean":
            st[name] = torch.zeros(shape)
        elif leaf == "running_var":
            st[name] = torch.ones(shape)
        elif leaf == "num_batches_tracked":
            st[name] = torch.tensor(0, dtype=torch.long)
        else:
            st[name] = torch.from_numpy(param_value(name, shape, seed))
    return st


# --------------------------------------------------------------------------
# forward (functional; autograd supplies the backward)
# --------------------------------------------------------------------------
class _State:
    """Thin view over a state dict: params require grad, buffers are updated in place."""

    def __init__(self, st, training):
        self.st = st
        self.training = training

    def __getitem__(self, k):
        return self.st[k]

    def bn(self, x, p):
        out = F.batch_norm(x, self.st[p + ".running_mean"], self.st[p + ".running_var"],
                           self.st[p + ".weight"], self.st[p + ".bias"],
                           training=self.training, momentum=0.1, eps=1e-5)
        if self.training:
            self.st[p + ".num_batches_tracked"].add_(1)
        return out


def st_gcan_block(S, p, x, A_eff, cin, cout, stride, res_kind):
    # residual branch (stgcan.py:123-133)
    if res_kind == "none":
        res = 0
    elif res_kind == "id":
        res = x
    else:
        res = F.conv2d(x, S[p + "residual.0.weight"], S[p + "residual.0.bias"], stride=(stride, 1))
        res = S.bn(res, p + "residual.1")
    # gcn (stgcan.py:50-56): 1x1 conv to K*C then einsum over the K partitions
    y = F.conv2d(x, S[p + "gcn.conv.weight"], S[p + "gcn.conv.bias"])
    n, kc, t, v = y.shape
    K = A_eff.shape[0]
    y = y.view(n, K, kc // K, t, v)
    g = torch.einsum("nkctv,kvw->nctw", y, A_eff).contiguous()
    # tcn (stgcan.py:112-121): BN, ReLU, conv(9,1) stride (s,1) pad (4,0), BN, Dropout(0)
    h = F.relu(S.bn(g, p + "tcn.0"))
    h = F.conv2d(h, S[p + "tcn.2.weight"], S[p + "tcn.2.bias"], stride=(stride, 1), padding=(4, 0))
    h = S.bn(h, p + "tcn.3")
    # Channel_Attention (stgcan.py:59-74)
    q = p + "channel_attention_module.atten."
    a = F.adaptive_avg_pool2d(h, (1, 1))
    a = F.conv2d(a, S[q + "1.weight"], S[q + "1.bias"])
    a = F.relu(S.bn(a, q + "2"))
    a = torch.sigmoid(F.conv2d(a, S[q + "4.weight"], S[q + "4.bias"]))
    return F.relu(h * a + res)


# --------------------------------------------------------------------------
# bf16-storage restatement (test infrastructure for the HIP path's bf16 mode)
#
# The reference computes in fp32 throughout; the build's bf16 mode keeps its
# arithmetic in fp32 but STORES these tensors as bf16 (round-to-nearest-even of the fp32 value):
#   forward : data_bn output, Z = graph mix of the block input, g = gcn output, u = relu(bn1(g)),
#             h = tcn output, r = residual-conv output, the block output; the packed gcn / tcn /
#             residual weights are bf16 GEMM operands;
#   backward: dZ, dg (gcn output gradient), dv (gradient of bn1's output, after the ReLU mask),
#             dh (tcn output gradient), dres (residual-conv output gradient).
# BatchNorm statistics are taken from the fp32 values before rounding (GEMM epilogues), and the
# channel-attention pool from the fp32 h; the normalised values are computed from the stored
# (rounded) tensors. The gcn runs in the build's order (graph mix, then the 1x1 GEMM with the
# graph-mixed bias), which is the reference's arithmetic reassociated (stgcan.py:50-56).
# Run in fp64 this isolates the effect of the storage rounding; the HIP bf16 path is compared
# with it per gradient tensor (tests/test_gpu_parity.py::test_bf16_storage_parity).
# --------------------------------------------------------------------------
_JITTER = {"eps": 0.0, "gen": None}


def storage_jitter(eps, seed):
    """Relative noise `eps` applied to every value just before it is rounded to bf16 (eps=0: off).
    eps ~ 2^-23 stands in for another valid fp32 evaluation order: it moves a value across a bf16
    rounding boundary exactly where a different fp32 accumulation would. The spread of gradients
    over such runs is the restatement's own envelope for the bf16 mode (test_bf16_storage_parity)."""
    _JITTER["eps"] = float(eps)
    _JITTER["gen"] = torch.Generator().manual_seed(int(seed)) if eps else None


def _to_bf16(t):
    """Round through fp32 to bf16 (RNE), as a kernel rounds its fp32 result, back in t's dtype."""
    if _JITTER["eps"]:
        t = t * (1 + _JITTER["eps"] * torch.randn(t.shape, generator=_JITTER["gen"], dtype=t.dtype))
    return t.float().to(torch.bfloat16).to(t.dtype)


class _RoundValue(torch.autograd.Function):
    """Forward: the stored (rounded) value. Backward: the gradient passes unchanged."""

    @staticmethod
    def forward(ctx, t):
        return _to_bf16(t)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGrad(torch.autograd.Function):
    """Forward: identity. Backward: the gradient is stored as bf16."""

    @staticmethod
    def forward(ctx, t):
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        return _to_bf16(g)


_rv, _rg = _RoundValue.apply, _RoundGrad.apply


def _bn_split(S, stat_src, values, p):
    """BatchNorm whose batch statistics come from `stat_src` (the unrounded tensor) applied to
    `values` (the stored one); running statistics updated as nn.BatchNorm does."""
    rm, rv = S[p + ".running_mean"], S[p + ".running_var"]
    shape = [1, -1] + [1] * (values.dim() - 2)
    if S.training:
        dims = [0] + list(range(2, stat_src.dim()))
        mean = stat_src.mean(dims)
        var = stat_src.var(dims, unbiased=False)
        n = stat_src.numel() // stat_src.shape[1]
        with torch.no_grad():
            rm.mul_(0.9).add_(0.1 * mean.detach().to(rm.dtype))
            rv.mul_(0.9).add_(0.1 * (var.detach() * n / (n - 1)).to(rv.dtype))
            S[p + ".num_batches_tracked"].add_(1)
    else:
        mean, var = rm, rv
    inv = torch.rsqrt(var + 1e-5)
    return (values - mean.view(shape)) * (inv * S[p + ".weight"]).view(shape) + S[p + ".bias"].view(shape)


def st_gcan_block_bf16(S, p, x, A_eff, cin, cout, stride, res_kind):
    """st_gcan block (stgcan.py:79-144) with the bf16 mode's storage rounding. `x` is the stored
    (bf16-valued) block input. Returns (out fp32, out as stored)."""
    N, _, T, V = x.shape
    K = A_eff.shape[0]
    if res_kind == "none":
        res = 0
    elif res_kind == "id":
        res = x
    else:
        r = _rg(F.conv2d(x, _rv(S[p + "residual.0.weight"]), S[p + "residual.0.bias"], stride=(stride, 1)))
        res = _bn_split(S, r, _rv(r), p + "residual.1")
    # gcn: Z = graph mix of x (stored bf16, dZ bf16), g = W_bf16 . Z + graph-mixed bias
    Z = _rv(_rg(torch.einsum("nctv,kvw->nkctw", x, A_eff)))
    W = _rv(S[p + "gcn.conv.weight"]).view(K, cout, cin)
    b = S[p + "gcn.conv.bias"].view(K, cout)
    g = torch.einsum("nkitw,kci->nctw", Z, W) + torch.einsum("kc,kw->cw", b, A_eff.sum(1)).view(1, cout, 1, V)
    g = _rg(g)
    # tcn: u = relu(bn1(g_bf16)) stored bf16 (dv bf16), conv, h stored bf16 (dh bf16)
    u = _rv(F.relu(_rg(_bn_split(S, g, _rv(g), p + "tcn.0"))))
    h = _rg(F.conv2d(u, _rv(S[p + "tcn.2.weight"]), S[p + "tcn.2.bias"], stride=(stride, 1), padding=(4, 0)))
    hn_pool = _bn_split(S, h, h, p + "tcn.3")            # the pool reads the fp32 h
    hn = _bn_reuse(S, h, _rv(h), p + "tcn.3")
    q = p + "channel_attention_module.atten."
    a = F.adaptive_avg_pool2d(hn_pool, (1, 1))
    a = F.conv2d(a, S[q + "1.weight"], S[q + "1.bias"])
    a = F.relu(S.bn(a, q + "2"))
    a = torch.sigmoid(F.conv2d(a, S[q + "4.weight"], S[q + "4.bias"]))
    out = F.relu(hn * a + res)
    return out, _rv(out)


def _bn_reuse(S, stat_src, values, p):
    """The same BatchNorm applied a second time in one forward (no second running-stat update)."""
    shape = [1, -1] + [1] * (values.dim() - 2)
    if S.training:
        dims = [0] + list(range(2, stat_src.dim()))
        mean, var = stat_src.mean(dims), stat_src.var(dims, unbiased=False)
    else:
        mean, var = S[p + ".running_mean"], S[p + ".running_var"]
    inv = torch.rsqrt(var + 1e-5)
    return (values - mean.view(shape)) * (inv * S[p + ".weight"]).view(shape) + S[p + ".bias"].view(shape)


def stgcan_stream(S, prefix, x, spec, num_class=None, storage="fp32"):
    layers = "st_gcn_networks" if spec.naming == "notebook" else "st_gcan_networks"
    N, C, T, V = x.shape
    # data_bn over V*C channels, V-major (stgcan.py:213-218)
    z = x.permute(0, 3, 1, 2).contiguous().view(N, V * C, T)
    z = S.bn(z, prefix + "data_bn")
    x = z.view(N, V, C, T).permute(0, 2, 3, 1).contiguous()
    A = S[prefix + "A"]
    if storage == "bf16":
        x = _rv(x)
        for i, (ci, co, s, res) in enumerate(STREAM_CHANNELS):
            ci = C if ci is None else ci
            A_eff = A * S[f"{prefix}edge_importance.{i}"]
            out, x = st_gcan_block_bf16(S, f"{prefix}{layers}.{i}.", x, A_eff, ci, co, s, res)
        x = out  # the pool reads the fp32 block output
    else:
        for i, (ci, co, s, res) in enumerate(STREAM_CHANNELS):
            ci = C if ci is None else ci
            A_eff = A * S[f"{prefix}edge_importance.{i}"]
            x = st_gcan_block(S, f"{prefix}{layers}.{i}.", x, A_eff, ci, co, s, res)
    x = F.avg_pool2d(x, x.shape[2:])
    if num_class is not None:
        x = F.conv2d(x, S[prefix + "cls.weight"], S[prefix + "cls.bias"])
    return x.view(x.shape[0], -1)


def lstm_dir(x, w_ih, w_hh, b_ih, b_hh, reverse):
    """One LSTM direction, PyTorch gate order i,f,g,o (bilstm.py:29 / nn.LSTM)."""
    N, T, _ = x.shape
    H = w_hh.shape[1]
    h = x.new_zeros(N, H)
    c = x.new_zeros(N, H)
    outs = [None] * T
    steps = range(T - 1, -1, -1) if reverse else range(T)
    for t in steps:
        gates = x[:, t] @ w_ih.t() + b_ih + h @ w_hh.t() + b_hh
        i, f, g, o = gates.chunk(4, dim=1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
        h = torch.sigmoid(o) * torch.tanh(c)
        outs[t] = h
    return torch.stack(outs, dim=1)


def bilstm_head(S, p, x):
    """BiLSTM.forward with feature='mean' (bilstm.py:41-59)."""
    fw = lstm_dir(x, S[p + "lstm1.weight_ih_l0"], S[p + "lstm1.weight_hh_l0"],
                  S[p + "lstm1.bias_ih_l0"], S[p + "lstm1.bias_hh_l0"], False)
    bw = lstm_dir(x, S[p + "lstm1.weight_ih_l0_reverse"], S[p + "lstm1.weight_hh_l0_reverse"],
                  S[p + "lstm1.bias_ih_l0_reverse"], S[p + "lstm1.bias_hh_l0_reverse"], True)
    out = torch.cat([fw, bw], dim=2).mean(dim=1)
    out = S.bn(out, p + "batchnorm")
    q = p + "channelattention.attention."
    w = F.relu(F.linear(out, S[q + "0.weight"], S[q + "0.bias"]))
    w = torch.sigmoid(F.linear(w, S[q + "2.weight"], S[q + "2.bias"]))
    out = out * w
    return F.linear(out, S[p + "fc.1.weight"], S[p + "fc.1.bias"])


def cnn1d(S, p, x):
    """CNN1D front end (GSTCAN_UR_conv.ipynb cell 2): [N,T,S] -> [N,T/4,32]."""
    z = x.permute(0, 2, 1)
    for L in ("layer1", "layer2"):
        z = F.conv1d(z, S[f"{p}{L}.0.weight"], S[f"{p}{L}.0.bias"], padding=2)
        z = F.max_pool1d(F.relu(S.bn(z, f"{p}{L}.1")), 2)
    return z.permute(0, 2, 1)


def forward(st, spec: Spec, skel, sensor=None, training=True, storage="fp32"):
    """Returns the module output (logits, or softmax for the notebook form). storage="bf16":
    the skeleton streams with the build's bf16-mode storage rounding (st_gcan_block_bf16)."""
    S = _State(st, training)
    if spec.model == "stgcn":
        return stgcan_stream(S, "", skel, spec, spec.num_class, storage)
    if spec.model == "bilstm":
        if spec.sensor == "cnn_bilstm":
            return bilstm_head(S, "bilstm.", cnn1d(S, "cnn.", sensor))
        return bilstm_head(S, "", sensor)
    p1, p2, ps, pf = prefixes(spec)
    mot = skel[:, :2, 1:] - skel[:, :2, :-1]  # combination.py:39
    feats = [stgcan_stream(S, p1, skel, spec, storage=storage), stgcan_stream(S, p2, mot, spec, storage=storage)]
    if spec.model == "two_stgcan_bilstm":
        if spec.sensor == "cnn_bilstm":
            feats.append(bilstm_head(S, ps + "bilstm.", cnn1d(S, ps + "cnn.", sensor)))
        else:
            feats.append(bilstm_head(S, ps, sensor))
    out = F.linear(torch.cat(feats, dim=-1), st[pf + "weight"], st[pf + "bias"])
    if spec.softmax_output:
        out = F.softmax(out, dim=-1)
    return out


def soft_ce(out, target):
    """CrossEntropyLoss with probability targets, mean over batch, no renormalisation."""
    return -(target * F.log_softmax(out, dim=-1)).sum(dim=-1).mean()


def rmsprop_step(params, grads, sq, lr=1e-3, alpha=0.99, eps=1e-8):
    """torch.optim.RMSprop defaults (optimizer.py:21): v=a v+(1-a)g^2; p-=lr g/(sqrt(v)+eps)."""
    for k in grads:
        g = grads[k]
        sq[k].mul_(alpha).addcmul_(g, g, value=1 - alpha)
        params[k].addcdiv_(g, sq[k].sqrt().add_(eps), value=-lr)


def train_step(st, spec, skel, sensor, label, lr=1e-3, sq=None, storage="fp32"):
    """One reference training step: forward -> CE -> backward -> RMSprop.

    Mutates `st` (params updated, BN running stats updated). Returns
    (output, loss, grads) with grads computed before the update.
    """
    names = [k for k in st if not is_buffer(k)]
    for k in names:
        st[k] = st[k].detach().clone().requires_grad_(True)
    out = forward(st, spec, skel, sensor, training=True, storage=storage)
    loss = soft_ce(out, label)
    gl = torch.autograd.grad(loss, [st[k] for k in names], allow_unused=True)
    # unused parameters (CNN1D.fc, GSTCAN_UR_conv.ipynb cell 2) get no gradient: RMSprop skips them
    grads = OrderedDict((k, g.detach()) for k, g in zip(names, gl) if g is not None)
    with torch.no_grad():
        for k in names:
            st[k] = st[k].detach()
        if sq is None:
            sq = {k: torch.zeros_like(st[k]) for k in names}
        rmsprop_step({k: st[k] for k in names}, grads, sq, lr=lr)
    return out.detach(), loss.detach(), grads


def gradient_sensitivity(st, spec, skel, sensor, label, eps=1e-6, trials=3, per_param=False, base=None):
    """Conditioning probe (test infrastructure): max normalised change of any gradient
    when every BatchNorm / pooling output is perturbed by relative noise `eps` (fp64).

    Train-mode BatchNorm over a handful of samples (the channel-attention BN normalises
    over the batch only, stgcan.py:66) puts ReLU kinks right next to the data: a 1e-6
    perturbation can flip one and move whole gradients by 1e-2..1e-1. Gradient parity is
    only meaningful on cases where this probe is small; golden seeds are chosen so.
    Biases that feed a train-mode BN have a zero true gradient and are skipped.
    base: the unperturbed fp64 gradients if the caller already has them (saves one run).
    """
    st64 = {k: (v.double() if v.dtype == torch.float32 else v.clone()) for k, v in st.items()}
    args = [None if x is None else x.double() for x in (skel, sensor, label)]
    orig_bn, orig_pool = F.batch_norm, F.adaptive_avg_pool2d

    def run(seed):
        gen = torch.Generator().manual_seed(seed)

        def noisy(y):
            return y if seed < 0 else y * (1 + eps * torch.randn(y.shape, generator=gen, dtype=y.dtype))

        F.batch_norm = lambda *a, **k: noisy(orig_bn(*a, **k))
        F.adaptive_avg_pool2d = lambda *a, **k: noisy(orig_pool(*a, **k))
        try:
            s = {k: v.clone() for k, v in st64.items()}
            return train_step(s, spec, *args)[2]
        finally:
            F.batch_norm, F.adaptive_avg_pool2d = orig_bn, orig_pool

    base = run(-1) if base is None else base
    env = {}
    for t in range(trials):
        g = run(1000 + t)
        for k, a in base.items():
            m = a.abs().max().item()
            env[k] = max(env.get(k, 0.0), (g[k] - a).abs().max().item() / max(m, 1e-30))
    if per_param:
        return env
    return max((e for k, e in env.items() if not k.endswith(("tcn.2.bias", "residual.0.bias", "atten.1.bias"))
                and base[k].abs().max().item() >= 1e-9), default=0.0)
