"""ORACLE — test infrastructure only (never imported by the product path).

CPU fp32 restatement of the reference's SkeletonTransformer training step (BASELINE config 5,
`SkeletonTransformer(3, 14, 30, 11, 32, 6, 16, 8)`), written from scratch as functional PyTorch.
It is the parity checker for the HIP path and is pinned to golden vectors produced by the
reference's own module (tools/gen_golden.py -> tests/golden/sktr_*.npz, tests/test_oracle_golden.py).

It follows, op for op (file:line relative to /root/reference/skeleton_transformer.py):

* RelativePositionalMultiHeadSelfAttention   100-157  (w_qkv Linear, chunk q|k|v, per-head
  q.k^T * embed_dims^-0.5 + q.table[i-j+L-1], softmax over keys, P.v, merge Linear)
* B2TSpatialTenporalTransformerBlock         206-248  (x + SD(attn_s(x)) -> BN1;
  + SD(attn_t(.)) over frames -> BN2; + SD(FFN(.)); + x -> BN3; BatchNorm3d over (N,T,V,M))
* SkeletonTransformer                        360-435  (Linear-GELU-Linear-GELU embedding,
  6 blocks, mean over (T,V) then over M, 1x1 Conv2d classifier)

Randomness. The reference's train mode has two random parts:
* StochasticDepth(p, mode="batch") (torchvision; one Bernoulli(1-p) per call, scaled by
  1/(1-p)): here an explicit per-(block, branch) factor `sd[b][k]` in {0, 1/(1-p)} (1 for p=0),
  drawn by the caller; the reference's environment lacks torchvision, so its golden vectors are
  produced with SD = identity, i.e. sd = 1 everywhere.
* FFN Dropout(0.5): a counter-based hash mask `dropout_keep` that the HIP kernels compute
  identically (seeded per step and block), so a train step with dropout is reproducible across
  the two implementations. Golden vectors are produced with the dropout p set to 0.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

EMBED, HEADS, HEAD_DIM, NBLOCK = 32, 8, 16, 6
D = HEADS * HEAD_DIM          # 128: attention embed dims
FFN = 4 * EMBED               # 128
SD_RATES = np.linspace(0, 0.5, NBLOCK)   # skeleton_transformer.py:380


def param_shapes(V=14, T=30, num_class=11, in_channels=3):
    """state_dict order of SkeletonTransformer(in_channels, V, T, num_class, 32, 6, 16, 8)."""
    out = OrderedDict()
    out["embedding.0.weight"] = (EMBED // 2, in_channels)
    out["embedding.0.bias"] = (EMBED // 2,)
    out["embedding.2.weight"] = (EMBED, EMBED // 2)
    out["embedding.2.bias"] = (EMBED,)
    for b in range(NBLOCK):
        p = f"extractor.{b}."
        for att, L in (("multi_head_spatial_self_attention", V), ("multi_head_temporal_self_attention", T)):
            q = p + att + "."
            out[q + "relative_position_bias_table"] = (2 * L - 1, HEAD_DIM)
            out[q + "w_qkv.weight"] = (3 * D, EMBED)
            out[q + "w_qkv.bias"] = (3 * D,)
            out[q + "merge.weight"] = (EMBED, D)
            out[q + "merge.bias"] = (EMBED,)
            n = p + ("norm1." if att.startswith("multi_head_spatial") else "norm2.")
            for leaf in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
                out[n + leaf] = () if leaf == "num_batches_tracked" else (EMBED,)
        out[p + "feed_forward_network.0.weight"] = (FFN, EMBED)
        out[p + "feed_forward_network.0.bias"] = (FFN,)
        out[p + "feed_forward_network.2.weight"] = (EMBED, FFN)
        out[p + "feed_forward_network.2.bias"] = (EMBED,)
        for leaf in ("weight", "bias", "running_mean", "running_var", "num_batches_tracked"):
            out[p + "norm3." + leaf] = () if leaf == "num_batches_tracked" else (EMBED,)
    out["fcn.0.weight"] = (num_class, EMBED, 1, 1)
    out["fcn.0.bias"] = (num_class,)
    return out


def is_buffer(name):
    return name.endswith(("running_mean", "running_var", "num_batches_tracked"))


def init_state(seed, V=14, T=30, num_class=11):
    from oracle.prng import param_value
    st = OrderedDict()
    for name, shape in param_shapes(V, T, num_class).items():
        if name.endswith("running_mean"):
            st[name] = torch.zeros(shape)
        elif name.endswith("running_var"):
            st[name] = torch.ones(shape)
        elif name.endswith("num_batches_tracked"):
            st[name] = torch.tensor(0, dtype=torch.int64)
        else:
            st[name] = torch.from_numpy(param_value(name, shape, seed))
    return st


# ---------------------------------------------------------------------------------------------
# counter-based dropout mask (shared bit-for-bit with the HIP kernels, sktr.hip dropout_keep)
# ---------------------------------------------------------------------------------------------
def _mix32(x):
    x = np.asarray(x, dtype=np.uint32).copy()
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def dropout_keep(seed, block, n_elem, p):
    """keep[e] for element e = token*32 + channel of block `block`'s FFN output: the 24-bit
    uniform u = mix32(mix32(seed ^ (block * 0x9E3779B9)) + e) >> 8, kept when u >= p * 2^24."""
    with np.errstate(over="ignore"):
        base = _mix32(np.uint32((int(seed) ^ (int(block) * 0x9E3779B9)) & 0xFFFFFFFF))
        e = np.arange(n_elem, dtype=np.uint64)
        h = _mix32(((e + np.uint64(base)) & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    thr = np.uint32(min(int(round(p * (1 << 24))), 1 << 24))
    return (h >> np.uint32(8)) >= thr


# ---------------------------------------------------------------------------------------------
# model
# ---------------------------------------------------------------------------------------------
def rel_attention(st, p, x, L):
    """RelativePositionalMultiHeadSelfAttention.forward on sequences x [S, L, 32] -> [S, L, 32]."""
    S = x.shape[0]
    qkv = F.linear(x, st[p + "w_qkv.weight"], st[p + "w_qkv.bias"])
    q, k, v = qkv.chunk(3, dim=-1)
    q = q.reshape(S, L, HEADS, HEAD_DIM).permute(0, 2, 1, 3)
    k = k.reshape(S, L, HEADS, HEAD_DIM).permute(0, 2, 1, 3)
    v = v.reshape(S, L, HEADS, HEAD_DIM).permute(0, 2, 1, 3)
    dot = (q @ k.transpose(-1, -2)) * (D ** -0.5)
    idx = torch.arange(L)[:, None] - torch.arange(L)[None, :] + L - 1
    table = st[p + "relative_position_bias_table"][idx]          # [L, L, HD]
    rel = torch.einsum("shld,lrd->shlr", q, table)
    a = torch.softmax(dot + rel, dim=-1)
    o = (a @ v).permute(0, 2, 1, 3).reshape(S, L, D)
    return F.linear(o, st[p + "merge.weight"], st[p + "merge.bias"])


def batchnorm(st, p, x, training, momentum=0.1, eps=1e-5):
    """BatchNorm3d over every axis but the channel (last here); running stats updated in place."""
    C = x.shape[-1]
    flat = x.reshape(-1, C)
    if training:
        mean = flat.mean(0)
        var = flat.var(0, unbiased=False)
        n = flat.shape[0]
        with torch.no_grad():
            st[p + "running_mean"].mul_(1 - momentum).add_(mean.detach(), alpha=momentum)
            st[p + "running_var"].mul_(1 - momentum).add_(var.detach() * n / max(n - 1, 1), alpha=momentum)
            st[p + "num_batches_tracked"] += 1
    else:
        mean, var = st[p + "running_mean"], st[p + "running_var"]
    return (x - mean) / torch.sqrt(var + eps) * st[p + "weight"] + st[p + "bias"]


def block(st, b, x, training, sd, keep):
    """B2TSpatialTenporalTransformerBlock.forward (206-248) on tokens x [N, M, T, V, 32]."""
    p = f"extractor.{b}."
    N, M, T, V, C = x.shape
    a = rel_attention(st, p + "multi_head_spatial_self_attention.", x.reshape(-1, V, C), V).reshape(x.shape)
    out = batchnorm(st, p + "norm1.", x + sd[0] * a, training)
    xt = out.permute(0, 1, 3, 2, 4).reshape(-1, T, C)              # sequences over frames
    a = rel_attention(st, p + "multi_head_temporal_self_attention.", xt, T)
    a = a.reshape(N, M, V, T, C).permute(0, 1, 3, 2, 4)
    out = batchnorm(st, p + "norm2.", out + sd[1] * a, training)
    f = F.linear(F.gelu(F.linear(out, st[p + "feed_forward_network.0.weight"], st[p + "feed_forward_network.0.bias"])),
                 st[p + "feed_forward_network.2.weight"], st[p + "feed_forward_network.2.bias"])
    if keep is not None:
        f = f * keep.reshape(f.shape) * 2.0     # Dropout(0.5): kept elements scaled by 1/(1-p)
    out = out + sd[2] * f
    return batchnorm(st, p + "norm3.", x + out, training)


def forward(st, x, training=True, sd=None, dropout_seed=None, dropout_p=0.5):
    """SkeletonTransformer.forward (418-435), x [N, C, T, V, M] -> logits [N, num_class].
    sd: [6][3] stochastic-depth factors (None: identity); dropout_seed None: no dropout."""
    N, Cin, T, V, M = x.shape
    t = x.permute(0, 4, 2, 3, 1)                                  # [N, M, T, V, Cin]
    t = F.gelu(F.linear(t, st["embedding.0.weight"], st["embedding.0.bias"]))
    t = F.gelu(F.linear(t, st["embedding.2.weight"], st["embedding.2.bias"]))
    R = N * M * T * V
    for b in range(NBLOCK):
        keep = None
        if training and dropout_seed is not None and dropout_p > 0:
            keep = torch.from_numpy(dropout_keep(dropout_seed, b, R * EMBED, dropout_p).astype(np.float32))
        t = block(st, b, t, training, sd[b] if sd is not None else (1.0, 1.0, 1.0), keep)
    pooled = t.mean(dim=(2, 3)).mean(dim=1)                        # avg_pool2d over (T,V), mean over M
    return F.linear(pooled, st["fcn.0.weight"].flatten(1), st["fcn.0.bias"])


def soft_ce(out, target):
    return -(target * F.log_softmax(out, dim=-1)).sum(dim=-1).mean()


def train_step(st, x, label, lr=1e-3, sq=None, alpha=0.99, eps=1e-8, sd=None, dropout_seed=None):
    """forward -> CE -> backward -> RMSprop. Mutates st (params and BN running stats); returns
    (logits, loss, grads) with grads taken before the update."""
    names = [k for k in st if not is_buffer(k)]
    for k in names:
        st[k] = st[k].detach().clone().requires_grad_(True)
    out = forward(st, x, True, sd, dropout_seed)
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


def synthetic_clips(batch, V, num_class, seed, T=30, M=1):
    """Skeleton windows in the transformer's input layout [N, 3, T, V, M] (the same synthetic clips
    as oracle.prng.synthetic_batch, replicated over M persons with a small per-person offset)."""
    from oracle.prng import synthetic_batch
    skel, _, label = synthetic_batch(batch, V, num_class, 1, seed, frames=T)
    x = np.repeat(skel[..., None], M, axis=-1)
    if M > 1:
        x[:, :2] += (np.arange(M, dtype=np.float32) * 0.05)[None, None, None, None, :]
    return np.ascontiguousarray(x.astype(np.float32)), label
