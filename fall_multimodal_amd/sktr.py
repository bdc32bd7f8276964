"""SkeletonTransformer (BASELINE config 5) as a drop-in module backed by the gfx950 HIP library.

Reference interface mirrored here (file:line relative to /root/reference):
  SkeletonTransformer(in_channels, n_joints, seq_len, num_classes, embedding_dim=32, n_block=6,
                      head_dim=16, n_heads=8)                               skeleton_transformer.py:360-416
  SkeletonTransformer.forward(x[N, C, T, V, M]) -> logits[N, num_classes]   skeleton_transformer.py:418-435
  notebook loop (GSTCAN_HAR_conv_kfold_trans.ipynb): SkeletonTransformer(n_joints=14, seq_len=30);
  CrossEntropyLoss; one model per fold (10-fold CV: replicas, no collective)

The state_dict has the reference's exact keys, order and shapes (f3_sktr_entry): parameters are
views into one flat fp32 buffer, BatchNorm3d running statistics into a buffer array and
num_batches_tracked into an int64 counter array. Forward and backward are one native call each.

Train-mode randomness: torchvision StochasticDepth(p, mode="batch") draws one Bernoulli(1-p)
per call (three calls per block: spatial, temporal, FFN; p = linspace(0, 0.5, 6)[block]) — drawn
here on the host from the module's generator and passed to the kernels as scale factors; the FFN
Dropout(0.5) mask is a counter hash of (seed, block, element) computed in the kernels (the oracle
reproduces it bit for bit). `stochastic_depth=False` / `dropout_p=0` switch either off (the
reference's golden vectors were produced that way, its environment lacking torchvision).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib, ops
from ._lib import ENTRY_BUFFER, ENTRY_COUNTER, ENTRY_PARAM, check, lib, ptr, require_device, stream_handle

NBLOCK = 6
SD_RATES = np.linspace(0, 0.5, NBLOCK)  # skeleton_transformer.py:380


class _NativeSktr:
    def __init__(self, V, T, M, num_class, precision=0):
        L = lib()
        c = _lib.F3SktrConfig()
        c.num_joint, c.frames, c.persons, c.num_class, c.precision = V, T, M, num_class, precision
        h = ctypes.c_void_p()
        check(L.f3_sktr_create(ctypes.byref(c), ctypes.byref(h)), "f3_sktr_create")
        self.h = h
        self.entries = []
        name, kind, nd = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_int()
        shape, off = (ctypes.c_int64 * 8)(), ctypes.c_int64()
        for i in range(L.f3_sktr_num_entries(h)):
            check(L.f3_sktr_entry(h, i, ctypes.byref(name), ctypes.byref(kind), ctypes.byref(nd), shape,
                                  ctypes.byref(off)), "f3_sktr_entry")
            self.entries.append((name.value.decode(), kind.value, tuple(shape[d] for d in range(nd.value)),
                                 off.value))
        self.nparam = L.f3_sktr_param_count(h)
        self.nbuf = L.f3_sktr_buffer_count(h)
        self.ncnt = L.f3_sktr_counter_count(h)
        self._ws = {}

    def workspace_bytes(self, batch):
        if batch not in self._ws:
            self._ws[batch] = int(lib().f3_sktr_workspace_bytes(self.h, batch))
        return self._ws[batch]

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().f3_sktr_destroy(self.h)
        except Exception:
            pass


class SkeletonTransformer(nn.Module):
    """skeleton_transformer.py:360-435 on the MI355X path."""

    def __init__(self, in_channels: int = 3, n_joints: int = 14, seq_len: int = 30, num_classes: int = 11,
                 embedding_dim: int = 32, n_block: int = 6, head_dim: int = 16, n_heads: int = 8, persons: int = 1,
                 device=None, dropout_p: float = 0.5, stochastic_depth: bool = True, seed: int = 0,
                 precision: str = "fp32"):
        """precision: "fp32" (fp32 MFMA GEMMs; the parity mode) or "bf16" (BASELINE config 5: the six
        blocks' Linear layers - qkv, merge, FFN - on bf16 MFMA with fp32 accumulate; attention core,
        BatchNorm3d, embedding and head stay fp32)."""
        super().__init__()
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        object.__setattr__(self, "precision", precision)
        if (in_channels, embedding_dim, n_block, head_dim, n_heads) != (3, 32, 6, 16, 8):
            raise NotImplementedError("fall3 SkeletonTransformer implements the reference configuration "
                                      "(in_channels 3, embedding_dim 32, 6 blocks, head_dim 16, 8 heads)")
        object.__setattr__(self, "n_joints", n_joints)
        object.__setattr__(self, "seq_len", seq_len)
        object.__setattr__(self, "persons", persons)
        object.__setattr__(self, "num_classes", num_classes)
        object.__setattr__(self, "dropout_p", float(dropout_p))
        object.__setattr__(self, "stochastic_depth", bool(stochastic_depth))
        object.__setattr__(self, "_gen", torch.Generator().manual_seed(int(seed)))
        object.__setattr__(self, "_native", _NativeSktr(n_joints, seq_len, persons, num_classes,
                                                        1 if precision == "bf16" else 0))
        object.__setattr__(self, "_op_id", ops.register(self))
        if device is None:
            device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        self._alloc(torch.device(device))
        shapes = {n: s for n, k, s, o in self._native.entries}
        with torch.no_grad():
            for name, kind, shape, off in self._native.entries:
                t = self._view(kind, shape, off)
                t.copy_(self._default(name, shape, shapes))
                self._register(name, kind, t)

    def _alloc(self, dev):
        nat = self._native
        object.__setattr__(self, "_flat_params", torch.zeros(nat.nparam, dtype=torch.float32, device=dev))
        object.__setattr__(self, "_flat_buffers", torch.zeros(max(nat.nbuf, 1), dtype=torch.float32, device=dev))
        object.__setattr__(self, "_counters", torch.zeros(max(nat.ncnt, 1), dtype=torch.int64, device=dev))

    @staticmethod
    def _default(name, shape, shapes):
        """PyTorch default inits of the reference modules (trunc_normal(0.02) for the tables,
        skeleton_transformer.py:120)."""
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "relative_position_bias_table":
            return nn.init.trunc_normal_(torch.empty(shape), std=0.02)
        if leaf == "running_mean":
            return torch.zeros(shape)
        if leaf == "running_var":
            return torch.ones(shape)
        if leaf == "num_batches_tracked":
            return torch.zeros(shape, dtype=torch.int64)
        if ".norm" in name:  # BatchNorm3d affine
            return torch.ones(shape) if leaf == "weight" else torch.zeros(shape)
        if leaf == "bias":  # Linear / Conv bias: U(+-1/sqrt(fan_in of its weight))
            fan_in = int(np.prod(shapes[name[: -len("bias")] + "weight"][1:]))
        else:               # kaiming_uniform(a=sqrt 5) == U(+-1/sqrt(fan_in))
            fan_in = int(np.prod(shape[1:]))
        b = 1.0 / math.sqrt(fan_in)
        return torch.empty(shape).uniform_(-b, b)

    def _view(self, kind, shape, off):
        n = int(np.prod(shape)) if len(shape) else 1
        if kind == ENTRY_PARAM:
            return self._flat_params[off:off + n].view(shape)
        if kind == ENTRY_BUFFER:
            return self._flat_buffers[off:off + n].view(shape)
        return self._counters[off:off + 1].view(shape)

    def _owner(self, name):
        mod = self
        *path, leaf = name.split(".")
        for p in path:
            if p not in mod._modules:
                mod.add_module(p, nn.Module())
            mod = mod._modules[p]
        return mod, leaf

    def _register(self, name, kind, t):
        mod, leaf = self._owner(name)
        if kind == ENTRY_PARAM:
            mod.register_parameter(leaf, nn.Parameter(t))
        else:
            mod.register_buffer(leaf, t)

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        dev = next(iter(self.parameters())).device
        self._alloc(dev)
        with torch.no_grad():
            for name, kind, shape, off in self._native.entries:
                mod, leaf = self._owner(name)
                cur = mod._parameters[leaf] if leaf in mod._parameters else mod._buffers[leaf]
                view = self._view(kind, shape, off)
                view.copy_(cur.detach())
                if kind == ENTRY_PARAM:
                    cur.data = view
                else:
                    mod._buffers[leaf] = view
        return self

    def flat_parameters(self):
        return self._flat_params

    def param_views(self):
        return [(name, shape, off) for name, kind, shape, off in self._native.entries if kind == ENTRY_PARAM]

    def check_inputs(self, x):
        require_device(x, "x")
        want = (3, self.seq_len, self.n_joints, self.persons)
        if x.dim() != 5 or tuple(x.shape[1:]) != want:
            raise ValueError(f"x must be [N,{','.join(map(str, want))}], got {tuple(x.shape)}")

    def draw_randomness(self):
        """One training forward's draws: 18 stochastic-depth factors and the dropout seed."""
        sd = []
        for b in range(NBLOCK):
            p = float(SD_RATES[b])
            for _ in range(3):
                if p == 0 or not self.stochastic_depth:
                    sd.append(1.0)
                else:
                    keep = torch.rand((), generator=self._gen).item() < 1.0 - p
                    sd.append(1.0 / (1.0 - p) if keep else 0.0)
        seed = int(torch.randint(0, 2 ** 31 - 1, (), generator=self._gen).item())
        return sd, seed

    def native_forward(self, x, out, workspace, training, sd=None, seed=0, buffers=None, counters=None,
                       stream=None):
        st = stream if stream is not None else stream_handle()
        b = self._flat_buffers if buffers is None else buffers
        c = self._counters if counters is None else counters
        sd_arr = None if sd is None else (ctypes.c_float * 18)(*sd)
        check(lib().f3_sktr_forward(self._native.h, x.shape[0], int(training), ptr(self._flat_params), ptr(b), ptr(c),
                                    ptr(x), ptr(out), ptr(workspace), sd_arr, ctypes.c_uint(seed & 0xFFFFFFFF),
                                    ctypes.c_float(self.dropout_p if training else 0.0), st),
              "sktr forward")

    def native_backward(self, B, dout, grads, workspace, stream=None):
        st = stream if stream is not None else stream_handle()
        check(lib().f3_sktr_backward(self._native.h, B, ptr(self._flat_params), ptr(self._flat_buffers), ptr(dout),
                                     ptr(grads), ptr(workspace), st), "sktr backward")

    def forward(self, x):
        """One fall3::sktr_forward custom op (its autograd calls fall3::sktr_backward)."""
        x = x.detach().contiguous().float()
        self.check_inputs(x)
        if self.training:
            sd, seed = self.draw_randomness()
        else:
            sd, seed = [1.0] * 18, 0
        out, _, nb, nc = torch.ops.fall3.sktr_forward(self._op_id, list(self.parameters()), self._flat_buffers,
                                                      self._counters, x, self.training, sd, seed)
        if self.training:
            with torch.no_grad():
                self._flat_buffers.copy_(nb)
                self._counters.copy_(nc)
        return out


class SktrStep:
    """Fused SkeletonTransformer training step: forward -> soft-target CE -> backward -> RMSprop on
    one HIP stream, every buffer preallocated (the CV notebook's loop body for one fold)."""

    def __init__(self, model: SkeletonTransformer, batch, lr=1e-3, alpha=0.99, eps=1e-8):
        self.model, self.N = model, batch
        self.lr, self.alpha, self.eps = lr, alpha, eps
        dev = model.flat_parameters().device
        nat = model._native
        self.grads = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        self.square_avg = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        self.ws = torch.empty(nat.workspace_bytes(batch), dtype=torch.uint8, device=dev)
        self.out = torch.empty(batch, model.num_classes, dtype=torch.float32, device=dev)
        self.dout = torch.empty_like(self.out)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.last_draws = None
        for (name, shape, off), p in zip(model.param_views(), model.parameters()):
            p.grad = self.grads[off:off + int(np.prod(shape))].view(shape)

    def _check(self, x, label):
        self.model.check_inputs(x)
        if x.shape[0] != self.N or not x.is_contiguous() or x.dtype != torch.float32:
            raise ValueError(f"SktrStep: x must be contiguous fp32 with batch {self.N}")
        if tuple(label.shape) != (self.N, self.model.num_classes) or label.dtype != torch.float32 \
                or not label.is_contiguous() or label.device != x.device:
            raise ValueError(f"SktrStep: label must be contiguous fp32 [{self.N},{self.model.num_classes}] on the device")

    def forward_backward(self, x, label, sd=None, seed=None):
        self._check(x, label)
        m = self.model
        if sd is None or seed is None:
            dsd, dseed = m.draw_randomness()
            sd = dsd if sd is None else sd
            seed = dseed if seed is None else seed
        self.last_draws = (list(sd), int(seed))
        st = stream_handle()
        m.native_forward(x, self.out, self.ws, True, sd, seed, stream=st)
        check(lib().f3_soft_ce(ptr(self.out), ptr(label), self.N, m.num_classes, ptr(self.loss), ptr(self.dout), st),
              "soft ce")
        m.native_backward(self.N, self.dout, self.grads, self.ws, st)

    def __call__(self, x, label, sd=None, seed=None):
        self.forward_backward(x, label, sd, seed)
        check(lib().f3_rmsprop_step(ptr(self.model.flat_parameters()), ptr(self.square_avg), ptr(self.grads),
                                    self.grads.numel(), self.lr, self.alpha, self.eps, 1.0, stream_handle()),
              "rmsprop")
        return self.loss
