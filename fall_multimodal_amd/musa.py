"""musa_model.Model (the model the root Multimodal_Fall3/main.py trains) as a drop-in module backed
by the gfx950 HIP library.

Reference interface mirrored here (file:line relative to /root/reference/Multimodal_Fall3):
  adjGraph(layout='coco_cut', strategy='uniform')                 model/musa_model.py:200-349
  Model(num_class, num_point, max_frame, graph, bias, edge, block_size, embed_dim=64, n_stage=1,
        act_type='tanh')                                          model/musa_model.py:492-559
  Model.forward(x[N, 3, T, V]) -> logits[N, num_class]            model/musa_model.py:561-589
  driver: Model(num_class=11, num_point=14, max_frame=300, graph=adjGraph('coco_cut','uniform'),
          bias=True, edge=True, block_size=41, embed_dim=64, n_stage=1, act_type='tanh')
                                                                  main.py:307-320

The state_dict has the reference's exact keys, order and shapes (f3_musa_entry), A included (a
Parameter with requires_grad=False, as the reference registers it). Train-mode randomness: the
DropBlocks (keep_prob 0.9 at musa_model.py:509) and the head's Dropout(0.2) are drawn in the kernels
from a counter hash of a per-step seed taken from the module's generator (the oracle reproduces the
draws); `dropblock=False` runs the reference with keep_prob 1 and p 0.
"""
from __future__ import annotations

import ctypes
import re
import math

import numpy as np
import torch
import torch.nn as nn

from . import _lib, ops
from ._lib import ENTRY_BUFFER, ENTRY_PARAM, check, lib, ptr, require_device, stream_handle


class adjGraph:  # noqa: N801  (reference name)
    """musa_model.py:200-349 for the layouts / strategies the driver uses: 'coco_cut' with 'uniform'
    (normalize_digraph of the 1-hop adjacency incl. self links), A of shape [1, V, V]."""

    def __init__(self, layout="coco_cut", strategy="uniform", max_hop=1, dilation=1):
        if layout != "coco_cut" or strategy != "uniform" or max_hop != 1 or dilation != 1:
            raise NotImplementedError("fall3 adjGraph: layout 'coco_cut', strategy 'uniform' (the driver's graph)")
        V = 14
        edges = [(i, i) for i in range(V)] + [(6, 4), (4, 2), (2, 13), (13, 1), (5, 3), (3, 1), (12, 10), (10, 8),
                                              (8, 2), (11, 9), (9, 7), (7, 1), (13, 0)]
        A = np.zeros((V, V))
        for i, j in edges:
            A[j, i] = A[i, j] = 1
        Dl = A.sum(0)
        Dn = np.diag([d ** -1 if d > 0 else 0 for d in Dl])
        self.num_node = V
        self.A = (A @ Dn)[None]


class _NativeMusa:
    def __init__(self, V, T, num_class, precision=0):
        L = lib()
        c = _lib.F3MusaConfig()
        c.num_point, c.frames, c.num_class, c.precision = V, T, num_class, precision
        h = ctypes.c_void_p()
        check(L.f3_musa_create(ctypes.byref(c), ctypes.byref(h)), "f3_musa_create")
        self.h = h
        self.entries = []
        name, kind, nd = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_int()
        shape, off = (ctypes.c_int64 * 8)(), ctypes.c_int64()
        for i in range(L.f3_musa_num_entries(h)):
            check(L.f3_musa_entry(h, i, ctypes.byref(name), ctypes.byref(kind), ctypes.byref(nd), shape,
                                  ctypes.byref(off)), "f3_musa_entry")
            self.entries.append((name.value.decode(), kind.value, tuple(shape[d] for d in range(nd.value)),
                                 off.value))
        self.nparam = L.f3_musa_param_count(h)
        self.nbuf = L.f3_musa_buffer_count(h)
        self.ncnt = L.f3_musa_counter_count(h)
        self._ws = {}

    def workspace_bytes(self, batch):
        if batch not in self._ws:
            self._ws[batch] = int(lib().f3_musa_workspace_bytes(self.h, batch))
        return self._ws[batch]

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().f3_musa_destroy(self.h)
        except Exception:
            pass


class Model(nn.Module):
    """musa_model.Model on the MI355X path (the driver's configuration)."""

    def __init__(self, num_class, num_point, max_frame, graph, bias, edge, block_size, embed_dim=64, n_stage=1,
                 act_type="tanh", device=None, dropblock=True, seed=0, frames=30, precision="fp32"):
        """precision: "fp32" (fp32 MFMA; the parity mode) or "bf16" (the root main.py trains under bf16
        autocast, Multimodal_Fall3/main.py:97: the streams' 1x1 convs on bf16 MFMA with fp32 accumulate;
        depthwise convs, graph mix, BatchNorms, DropBlock and the head stay fp32)."""
        super().__init__()
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        object.__setattr__(self, "precision", precision)
        if (embed_dim, n_stage, act_type, bool(bias), bool(edge), block_size) != (64, 1, "tanh", True, True, 41):
            raise NotImplementedError("fall3 musa Model implements the driver's configuration (embed_dim 64, "
                                      "n_stage 1, act 'tanh', bias, edge, block_size 41; main.py:307-320)")
        A = np.asarray(graph.A, dtype=np.float32)
        if A.shape != (1, num_point, num_point):
            raise ValueError(f"graph.A must be [1, {num_point}, {num_point}] (uniform strategy), got {A.shape}")
        object.__setattr__(self, "num_classes", num_class)
        object.__setattr__(self, "num_point", num_point)
        object.__setattr__(self, "frames", frames)
        object.__setattr__(self, "dropblock", bool(dropblock))
        object.__setattr__(self, "_gen", torch.Generator().manual_seed(int(seed)))
        object.__setattr__(self, "_native", _NativeMusa(num_point, frames, num_class, 1 if precision == "bf16" else 0))
        object.__setattr__(self, "_op_id", ops.register(self))
        if device is None:
            device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        self._alloc(torch.device(device))
        shapes = {n: s for n, k, s, o in self._native.entries}
        with torch.no_grad():
            for name, kind, shape, off in self._native.entries:
                t = self._view(kind, shape, off)
                t.copy_(torch.from_numpy(A) if name.endswith(".A") else self._default(name, shape, shapes))
                self._register(name, kind, t)

    def _alloc(self, dev):
        nat = self._native
        object.__setattr__(self, "_flat_params", torch.zeros(nat.nparam, dtype=torch.float32, device=dev))
        object.__setattr__(self, "_flat_buffers", torch.zeros(max(nat.nbuf, 1), dtype=torch.float32, device=dev))
        object.__setattr__(self, "_counters", torch.zeros(max(nat.ncnt, 1), dtype=torch.int64, device=dev))

    @staticmethod
    def _default(name, shape, shapes):
        """PyTorch default inits (init_param at musa_model.py:408-420 is never called)."""
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "edge":
            return torch.ones(shape)
        if leaf == "running_mean":
            return torch.zeros(shape)
        if leaf == "running_var":
            return torch.ones(shape)
        if leaf == "num_batches_tracked":
            return torch.zeros(shape, dtype=torch.int64)
        if len(shape) == 1 and leaf == "weight":   # BatchNorm / LayerNorm affine
            return torch.ones(shape)
        if len(shape) == 1 and leaf == "bias" and (name[: -len("bias")] + "weight") in shapes \
                and len(shapes[name[: -len("bias")] + "weight"]) == 1:
            return torch.zeros(shape)
        if leaf == "bias":
            fan_in = int(np.prod(shapes[name[: -len("bias")] + "weight"][1:]))
        else:
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
            mod.register_parameter(leaf, nn.Parameter(t, requires_grad=not name.endswith(".A")))
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
        want = (3, self.frames, self.num_point)
        if x.dim() != 4 or tuple(x.shape[1:]) != want:
            raise ValueError(f"x must be [N,{','.join(map(str, want))}], got {tuple(x.shape)}")

    def draw_seed(self):
        return int(torch.randint(0, 2 ** 31 - 1, (), generator=self._gen).item())

    def native_forward(self, x, out, workspace, training, seed=0, buffers=None, counters=None, stream=None):
        st = stream if stream is not None else stream_handle()
        b = self._flat_buffers if buffers is None else buffers
        c = self._counters if counters is None else counters
        check(lib().f3_musa_forward(self._native.h, x.shape[0], int(training), ptr(self._flat_params), ptr(b), ptr(c),
                                    ptr(x), ptr(out), ptr(workspace), ctypes.c_uint(seed & 0xFFFFFFFF),
                                    int(training and self.dropblock), st), "musa forward")

    def native_backward(self, B, dout, grads, workspace, stream=None):
        st = stream if stream is not None else stream_handle()
        check(lib().f3_musa_backward(self._native.h, B, ptr(self._flat_params), ptr(self._flat_buffers), ptr(dout),
                                     ptr(grads), ptr(workspace), st), "musa backward")

    def forward(self, x):
        """One fall3::musa_forward custom op (its autograd calls fall3::musa_backward)."""
        x = x.detach().contiguous().float()
        self.check_inputs(x)
        seed = self.draw_seed() if self.training else 0
        out, _, nb, nc = torch.ops.fall3.musa_forward(self._op_id, list(self.parameters()), self._flat_buffers,
                                                      self._counters, x, self.training, seed)
        if self.training:
            with torch.no_grad():
                self._flat_buffers.copy_(nb)
                self._counters.copy_(nc)
        return out


_FROZEN = re.compile(r"(^|\.)A$")
_SEP_EDGE = re.compile(r"^stream_(pos|mot)\.[12]\.edge$")


def grad_is_none(name, dropblock_active):
    """True for the parameters whose .grad the reference leaves None after backward.
    * The graphs `A` (requires_grad False): always.
    * The SepTemporal blocks' `edge` (musa_model.py:184-198): it enters the graph only through
      Randomized_DropBlock_Ske's M = matmul(M_seed, A * edge), whose every element the masked writes
      `M[M > 0.001] = 1.0; M[M < 0.5] = 0.0` (musa_model.py:66-69) then overwrite with a constant.
      With DropBlock active (training, keep_prob < 1: the driver's 0.9, musa_model.py:510) autograd
      therefore gives edge an all-ZERO gradient tensor - so weight-decaying optimizers (the
      reference's SGD / Adam / AdamW builders) still move it and keep state for it. Without DropBlock
      (keep_prob 1, eval) edge is unused and its gradient stays None. f3_musa_backward zero-fills
      these slots either way."""
    if _FROZEN.search(name):
        return True
    return bool(_SEP_EDGE.search(name)) and not dropblock_active


class MusaStep:
    """Fused musa_model training step: forward -> soft-target CE -> backward -> RMSprop on one HIP
    stream with preallocated buffers (main.py's train loop body with RMSprop(lr=1e-3))."""

    def __init__(self, model: Model, batch, lr=1e-3, alpha=0.99, eps=1e-8):
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
        self.last_seed = None
        # A (frozen) has no gradient; the SepTemporal blocks' edges get the zero gradient the
        # reference's DropBlock gives them (None without DropBlock). RMSprop maps a zero gradient
        # to a zero update (square_avg stays 0), as torch.optim.RMSprop (no weight decay) does
        for (name, shape, off), p in zip(model.param_views(), model.parameters()):
            if not grad_is_none(name, model.dropblock):
                p.grad = self.grads[off:off + int(np.prod(shape))].view(shape)

    def forward_backward(self, x, label, seed=None):
        m = self.model
        m.check_inputs(x)
        if x.shape[0] != self.N or not x.is_contiguous() or x.dtype != torch.float32:
            raise ValueError(f"MusaStep: x must be contiguous fp32 with batch {self.N}")
        if tuple(label.shape) != (self.N, m.num_classes) or label.dtype != torch.float32 or not label.is_contiguous():
            raise ValueError(f"MusaStep: label must be contiguous fp32 [{self.N},{m.num_classes}]")
        seed = m.draw_seed() if seed is None else int(seed)
        self.last_seed = seed
        st = stream_handle()
        m.native_forward(x, self.out, self.ws, True, seed, stream=st)
        check(lib().f3_soft_ce(ptr(self.out), ptr(label), self.N, m.num_classes, ptr(self.loss), ptr(self.dout), st),
              "soft ce")
        m.native_backward(self.N, self.dout, self.grads, self.ws, st)

    def __call__(self, x, label, seed=None):
        self.forward_backward(x, label, seed)
        check(lib().f3_rmsprop_step(ptr(self.model.flat_parameters()), ptr(self.square_avg), ptr(self.grads),
                                    self.grads.numel(), self.lr, self.alpha, self.eps, 1.0, stream_handle()),
              "rmsprop")
        return self.loss
