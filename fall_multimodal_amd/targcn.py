"""TARGCN (BASELINE config 2) as a drop-in module backed by the gfx950 HIP library.

Reference interface mirrored here (file:line relative to /root/reference):
  TARGCN(input_dim=3, num_classes=11, num_nodes=14, ..., adj=None)     TRAGCN.py:177-205
  TARGCN.forward(source[B, T, N, 3]) -> logits[B, num_classes]          TRAGCN.py:207-224
  notebook loop: out = model(pts.permute(0,2,3,1)); CrossEntropyLoss(out, lbs); RMSprop
                                                                        TARGCN_HAR_conv_10kfold.ipynb cell 3

The state_dict has the reference's exact keys, order and shapes (table from f3_targcn_entry):
parameters are views into one flat fp32 buffer (16-B aligned entries), the positional-encoding
table is a buffer. Forward and backward are one native call each (one autograd node); TargcnStep
is the fused forward -> CE -> backward -> RMSprop step with preallocated buffers.

The reference's default adj (Graph(...).A) raises inside its own __init__ and only adj=None works
(SURVEY §0.7); its weights_pool / bias_pool are uninitialised memory (EmbGCN.py:67-68), which is
why its logged run diverges to nan. Here they are initialised U(+-1/sqrt(fan_in)).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib, ops
from ._lib import ENTRY_PARAM, check, lib, ptr, require_device, stream_handle

PRECISION_IDS = {"fp32": 0, "bf16": 1}


def positional_encoding(T=30, F=64):
    """TA.py:75-86."""
    pe = torch.zeros(T, F)
    position = torch.arange(0, T).unsqueeze(1)
    div = torch.exp(torch.arange(0, F, 2) * -(math.log(10000.0) / F))
    pe[:, 0::2] = torch.sin(position * div)
    pe[:, 1::2] = torch.cos(position * div)
    return pe.view(1, T, 1, F)


class _NativeTargcn:
    def __init__(self, V, num_class, precision):
        if precision not in PRECISION_IDS:
            raise ValueError(f"precision must be one of {sorted(PRECISION_IDS)}, got {precision!r}")
        L = lib()
        c = _lib.F3TargcnConfig()
        c.num_node, c.num_class, c.precision = V, num_class, PRECISION_IDS[precision]
        h = ctypes.c_void_p()
        check(L.f3_targcn_create(ctypes.byref(c), ctypes.byref(h)), "f3_targcn_create")
        self.h = h
        self.entries = []
        name, kind, nd = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_int()
        shape, off = (ctypes.c_int64 * 8)(), ctypes.c_int64()
        for i in range(L.f3_targcn_num_entries(h)):
            check(L.f3_targcn_entry(h, i, ctypes.byref(name), ctypes.byref(kind), ctypes.byref(nd), shape,
                                    ctypes.byref(off)), "f3_targcn_entry")
            self.entries.append((name.value.decode(), kind.value, tuple(shape[d] for d in range(nd.value)),
                                 off.value))
        self.nparam = L.f3_targcn_param_count(h)
        self.nbuf = L.f3_targcn_buffer_count(h)
        self._ws = {}

    def workspace_bytes(self, batch):
        if batch not in self._ws:
            self._ws[batch] = int(lib().f3_targcn_workspace_bytes(self.h, batch))
        return self._ws[batch]

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().f3_targcn_destroy(self.h)
        except Exception:
            pass


class TARGCN(nn.Module):
    """TRAGCN.py:177-224 on the MI355X path (adj=None, the only form the reference runs)."""

    def __init__(self, input_dim=3, num_classes=11, num_nodes=14, rnn_units=64, output_dim=64, horizon=30,
                 num_layers=2, embed_dim=64, cheb_k=2, adj=None, device=None, precision="fp32"):
        super().__init__()
        if (input_dim, rnn_units, output_dim, horizon, num_layers, embed_dim) != (3, 64, 64, 30, 2, 64):
            raise NotImplementedError("fall3 TARGCN implements the reference configuration "
                                      "(input_dim 3, rnn_units 64, output_dim 64, horizon 30, 2 layers, embed_dim 64)")
        if adj is not None:
            raise ValueError("TARGCN: only adj=None is supported (the reference's default adj raises, TRAGCN.py:191)")
        object.__setattr__(self, "num_node", num_nodes)
        object.__setattr__(self, "num_class", num_classes)
        object.__setattr__(self, "precision", precision)
        object.__setattr__(self, "_native", _NativeTargcn(num_nodes, num_classes, precision))
        object.__setattr__(self, "_op_id", ops.register(self))
        if device is None:
            device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        nat = self._native
        dev = torch.device(device)
        object.__setattr__(self, "_flat_params", torch.zeros(nat.nparam, dtype=torch.float32, device=dev))
        object.__setattr__(self, "_flat_buffers", torch.zeros(max(nat.nbuf, 1), dtype=torch.float32, device=dev))
        shapes = {n: s for n, k, s, o in nat.entries}
        with torch.no_grad():
            for name, kind, shape, off in nat.entries:
                t = self._view(kind, shape, off)
                t.copy_(self._default(name, shape, shapes))
                self._register(name, kind, t)

    @staticmethod
    def _default(name, shape, shapes):
        """PyTorch default inits of the reference modules; the uninitialised pools get U(+-1/sqrt(fan_in))."""
        leaf = name.rsplit(".", 1)[-1]
        if name.endswith("PE.pe"):
            return positional_encoding()
        if name == "node_embeddings":
            return torch.randn(shape)  # TRAGCN.py:194
        if ".ln" in name:  # LayerNorm: ones / zeros
            return torch.ones(shape) if leaf == "weight" else torch.zeros(shape)
        if leaf == "bias":  # Linear / Conv bias: U(+-1/sqrt(fan_in of its weight))
            fan_in = int(np.prod(shapes[name[: -len("bias")] + "weight"][1:]))
        else:
            fan_in = int(np.prod(shape[1:]))
        b = 1.0 / math.sqrt(fan_in)
        return torch.empty(shape).uniform_(-b, b)

    def _view(self, kind, shape, off):
        n = int(np.prod(shape)) if len(shape) else 1
        flat = self._flat_params if kind == ENTRY_PARAM else self._flat_buffers
        return flat[off:off + n].view(shape)

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
        nat = self._native
        dev = next(iter(self.parameters())).device
        p = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        b = torch.zeros(max(nat.nbuf, 1), dtype=torch.float32, device=dev)
        object.__setattr__(self, "_flat_params", p)
        object.__setattr__(self, "_flat_buffers", b)
        with torch.no_grad():
            for name, kind, shape, off in nat.entries:
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

    def check_inputs(self, source):
        require_device(source, "source")
        if source.dim() != 4 or tuple(source.shape[1:]) != (30, self.num_node, 3):
            raise ValueError(f"source must be [B,30,{self.num_node},3], got {tuple(source.shape)}")

    def native_forward(self, source, out, workspace, stream=None):
        st = stream if stream is not None else stream_handle()
        check(lib().f3_targcn_forward(self._native.h, source.shape[0], ptr(self._flat_params),
                                      ptr(self._flat_buffers), ptr(source), ptr(out), ptr(workspace), st),
              "targcn forward")

    def native_backward(self, B, dout, grads, workspace, stream=None):
        st = stream if stream is not None else stream_handle()
        check(lib().f3_targcn_backward(self._native.h, B, ptr(self._flat_params), ptr(self._flat_buffers),
                                       ptr(dout), ptr(grads), ptr(workspace), st), "targcn backward")

    def device_status(self, wait=True):
        """Raise if a GRU group barrier of the last forward / backward timed out (F3_EDEVICE: the
        node-partitioned recurrences' outputs are then wrong); wait=False checks only a completed copy."""
        check(lib().f3_targcn_status(self._native.h, 1 if wait else 0), "targcn device status")

    def forward(self, source):
        """One fall3::targcn_forward custom op (its autograd calls fall3::targcn_backward)."""
        source = source.detach().contiguous().float()
        self.check_inputs(source)
        out, _ = torch.ops.fall3.targcn_forward(self._op_id, list(self.parameters()), self._flat_buffers, source)
        return out


class TargcnStep:
    """Fused TARGCN training step: forward -> soft-target CE -> backward -> RMSprop on one HIP
    stream, every buffer preallocated (the notebook's loop body, TARGCN_HAR_conv_10kfold.ipynb
    cell 3, with its RMSprop(lr=1e-5))."""

    def __init__(self, model: TARGCN, batch, lr=1e-5, alpha=0.99, eps=1e-8):
        self.model, self.N = model, batch
        self.lr, self.alpha, self.eps = lr, alpha, eps
        dev = model.flat_parameters().device
        nat = model._native
        self.grads = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        self.square_avg = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        self.ws = torch.empty(nat.workspace_bytes(batch), dtype=torch.uint8, device=dev)
        self.out = torch.empty(batch, model.num_class, dtype=torch.float32, device=dev)
        self.dout = torch.empty_like(self.out)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        for (name, shape, off), p in zip(model.param_views(), model.parameters()):
            p.grad = self.grads[off:off + int(np.prod(shape))].view(shape)

    def _check(self, source, label):
        self.model.check_inputs(source)
        if source.shape[0] != self.N or not source.is_contiguous() or source.dtype != torch.float32:
            raise ValueError(f"TargcnStep: source must be contiguous fp32 [{self.N},30,V,3]")
        if tuple(label.shape) != (self.N, self.model.num_class) or label.dtype != torch.float32 \
                or not label.is_contiguous() or label.device != source.device:
            raise ValueError(f"TargcnStep: label must be contiguous fp32 [{self.N},{self.model.num_class}] on the device")

    def forward_backward(self, source, label):
        self._check(source, label)
        m = self.model
        st = stream_handle()
        m.native_forward(source, self.out, self.ws, st)
        check(lib().f3_soft_ce(ptr(self.out), ptr(label), self.N, m.num_class, ptr(self.loss), ptr(self.dout), st),
              "soft ce")
        m.native_backward(self.N, self.dout, self.grads, self.ws, st)

    def __call__(self, source, label):
        # a flagged barrier of an earlier step surfaces here (or from the native calls themselves)
        self.model.device_status(wait=False)
        self.forward_backward(source, label)
        check(lib().f3_rmsprop_step(ptr(self.model.flat_parameters()), ptr(self.square_avg), ptr(self.grads),
                                    self.grads.numel(), self.lr, self.alpha, self.eps, 1.0, stream_handle()),
              "rmsprop")
        return self.loss
