"""PyTorch custom ops (torch.library) over the C ABI: the boundary SURVEY §8(b) names
(`TORCH_LIBRARY(fall3, m)`-style ops with fake kernels and autograd), so the native step works
under torch.compile / FakeTensor tracing and composes with the rest of an autograd graph.

  fall3::net_forward(net, params, buffers, counters, skel?, sensor?, training)
        -> (out, workspace, new running buffers, new counters)
        model(data, sensor), Multimodal_Fall3/model/main.py:112 (combination.py:37-46)
  fall3::net_backward(net, params, dout, workspace) -> grads (flat, params layout)
        loss.backward(), main.py:115
  fall3::targcn_forward(net, params, buffers, source) -> (out, workspace)
        model(pts.permute(0,2,3,1)), TARGCN_HAR_conv_10kfold.ipynb cell 3 (TRAGCN.py:207-224)
  fall3::targcn_backward(net, params, buffers, dout, workspace) -> grads
  fall3::sktr_forward(net, params, buffers, counters, x, training, sd, seed)
        -> (out, workspace, new running buffers, new counters)
        model(x), skeleton_transformer.py:418-435 (BASELINE config 5)
  fall3::sktr_backward(net, params, dout, workspace) -> grads
  fall3::musa_forward(net, params, buffers, counters, x, training, seed) -> (out, workspace, buffers, counters)
        model(data), Multimodal_Fall3/model/musa_model.py:561-589 (root main.py:97-99)
  fall3::musa_backward(net, params, dout, workspace) -> grads
  fall3::rmsprop_(param!, square_avg!, grad, lr, alpha, eps, scale)
        optimizer.step(), model/optimizer.py:21 (torch.optim.RMSprop semantics)

`net` is the integer id of a live native model (its f3_net / f3_targcn handle); `params` is the
module's parameter list (views of one flat buffer, which the native call reads through). The ops
are functional (an op that mutates its inputs cannot carry an autograd formula): net_forward
returns the updated BatchNorm running statistics / counters, which the module copies back as
nn.BatchNorm updates them in place. Fake kernels return outputs of the right shapes without
touching the device; the workspace size comes from the host-side plan (f3_*_workspace_bytes).
"""
from __future__ import annotations

import weakref
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from ._lib import check, lib, ptr, stream_handle

_NETS: "weakref.WeakValueDictionary[int, object]" = weakref.WeakValueDictionary()


def register(module) -> int:
    """Make a native-backed module reachable from the ops; returns its id."""
    key = id(module)
    _NETS[key] = module
    return key


def _module(net: int):
    m = _NETS.get(net)
    if m is None:
        raise RuntimeError(f"fall3 op: no live native model with id {net}")
    return m


# ---------------------------------------------------------------------------------------------
# 3-stream / 2-stream / single-stream / sensor models (f3_net)
# ---------------------------------------------------------------------------------------------
@torch.library.custom_op("fall3::net_forward", mutates_args=())
def net_forward(net: int, params: List[Tensor], buffers: Tensor, counters: Tensor, skel: Optional[Tensor],
                sensor: Optional[Tensor], training: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Functional: returns (out, workspace, new running buffers, new counters); the module copies the
    new BatchNorm running statistics back (a mutating op could not carry an autograd formula)."""
    m = _module(net)
    ref = skel if skel is not None else sensor
    N = ref.shape[0]
    ws = torch.empty(m._native.workspace_bytes(N), dtype=torch.uint8, device=ref.device)
    out = torch.empty(N, m.spec.num_class, dtype=torch.float32, device=ref.device)
    nb, nc = buffers.clone(), counters.clone()
    m.native_forward(skel, sensor, out, ws, training, buffers=nb, counters=nc)
    return out, ws, nb, nc


@net_forward.register_fake
def _(net, params, buffers, counters, skel, sensor, training):
    m = _module(net)
    ref = skel if skel is not None else sensor
    N = ref.shape[0]
    return (ref.new_empty(N, m.spec.num_class, dtype=torch.float32),
            ref.new_empty(m._native.workspace_bytes(N), dtype=torch.uint8), torch.empty_like(buffers),
            torch.empty_like(counters))


@torch.library.custom_op("fall3::net_backward", mutates_args=())
def net_backward(net: int, params: List[Tensor], dout: Tensor, workspace: Tensor) -> Tensor:
    m = _module(net)
    grads = torch.empty(m._native.nparam, dtype=torch.float32, device=dout.device)
    m.native_backward(dout.shape[0], dout.contiguous(), grads, workspace)
    return grads


@net_backward.register_fake
def _(net, params, dout, workspace):
    return dout.new_empty(_module(net)._native.nparam, dtype=torch.float32)


def _no_grad_outputs(ctx, output):
    """The workspace and the new running buffers / counters carry no gradient. Without this autograd
    materialises a zero gradient for each of them before calling backward: for the ~9 GB workspace
    that is a 1 ms fill per step (4 x 245 us `FillFunctor<unsigned char>` launches in the rocprof
    trace of the unchanged main.py loop)."""
    ctx.set_materialize_grads(False)
    ctx.mark_non_differentiable(*output[1:])


def _net_setup(ctx, inputs, output):
    net, params, buffers, counters, skel, sensor, training = inputs
    ctx.net, ctx.training = net, training
    ctx.save_for_backward(output[1])
    _no_grad_outputs(ctx, output)


def _split_grads(m, grads):
    """Views of the flat gradient in parameter order (the (shape, stride, offset) table is built once
    per module; as_strided is the cheapest per-view call, ~1.3 us against ~3 us for slice + view)."""
    table = getattr(m, "_f3_grad_table", None)
    if table is None:
        table = []
        for _, shape, off in m.param_views():
            shape = tuple(int(d) for d in shape)
            stride, acc = [], 1
            for d in reversed(shape):
                stride.append(acc)
                acc *= d
            table.append((shape, tuple(reversed(stride)), int(off)))
        object.__setattr__(m, "_f3_grad_table", table)
    o0 = grads.storage_offset()
    return [grads.as_strided(shape, stride, o0 + off) for shape, stride, off in table]


def _net_backward(ctx, dout, dws, dbuf, dcnt):
    if not ctx.training:
        raise RuntimeError("fall3: backward through an eval-mode forward is not supported")
    (ws,) = ctx.saved_tensors
    m = _module(ctx.net)
    grads = torch.ops.fall3.net_backward(ctx.net, list(m.parameters()), dout.float(), ws)
    return None, _split_grads(m, grads), None, None, None, None, None


net_forward.register_autograd(_net_backward, setup_context=_net_setup)


# ---------------------------------------------------------------------------------------------
# TARGCN (f3_targcn)
# ---------------------------------------------------------------------------------------------
@torch.library.custom_op("fall3::targcn_forward", mutates_args=())
def targcn_forward(net: int, params: List[Tensor], buffers: Tensor, source: Tensor) -> Tuple[Tensor, Tensor]:
    m = _module(net)
    N = source.shape[0]
    ws = torch.empty(m._native.workspace_bytes(N), dtype=torch.uint8, device=source.device)
    out = torch.empty(N, m.num_class, dtype=torch.float32, device=source.device)
    m.native_forward(source, out, ws)
    return out, ws


@targcn_forward.register_fake
def _(net, params, buffers, source):
    m = _module(net)
    N = source.shape[0]
    return (source.new_empty(N, m.num_class, dtype=torch.float32),
            source.new_empty(m._native.workspace_bytes(N), dtype=torch.uint8))


@torch.library.custom_op("fall3::targcn_backward", mutates_args=())
def targcn_backward(net: int, params: List[Tensor], buffers: Tensor, dout: Tensor, workspace: Tensor) -> Tensor:
    m = _module(net)
    grads = torch.empty(m._native.nparam, dtype=torch.float32, device=dout.device)
    m.native_backward(dout.shape[0], dout.contiguous(), grads, workspace)
    return grads


@targcn_backward.register_fake
def _(net, params, buffers, dout, workspace):
    return dout.new_empty(_module(net)._native.nparam, dtype=torch.float32)


def _tg_setup(ctx, inputs, output):
    ctx.net = inputs[0]
    ctx.save_for_backward(inputs[2], output[1])
    _no_grad_outputs(ctx, output)


def _tg_backward(ctx, dout, dws):
    buffers, ws = ctx.saved_tensors
    m = _module(ctx.net)
    grads = torch.ops.fall3.targcn_backward(ctx.net, list(m.parameters()), buffers, dout.float(), ws)
    return None, _split_grads(m, grads), None, None


targcn_forward.register_autograd(_tg_backward, setup_context=_tg_setup)


# ---------------------------------------------------------------------------------------------
# SkeletonTransformer (f3_sktr)
# ---------------------------------------------------------------------------------------------
@torch.library.custom_op("fall3::sktr_forward", mutates_args=())
def sktr_forward(net: int, params: List[Tensor], buffers: Tensor, counters: Tensor, x: Tensor, training: bool,
                 sd: List[float], seed: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Functional like net_forward: returns the new BatchNorm3d running statistics / counters."""
    m = _module(net)
    N = x.shape[0]
    ws = torch.empty(m._native.workspace_bytes(N), dtype=torch.uint8, device=x.device)
    out = torch.empty(N, m.num_classes, dtype=torch.float32, device=x.device)
    nb, nc = buffers.clone(), counters.clone()
    m.native_forward(x, out, ws, training, sd, seed, buffers=nb, counters=nc)
    return out, ws, nb, nc


@sktr_forward.register_fake
def _(net, params, buffers, counters, x, training, sd, seed):
    m = _module(net)
    N = x.shape[0]
    return (x.new_empty(N, m.num_classes, dtype=torch.float32),
            x.new_empty(m._native.workspace_bytes(N), dtype=torch.uint8), torch.empty_like(buffers),
            torch.empty_like(counters))


@torch.library.custom_op("fall3::sktr_backward", mutates_args=())
def sktr_backward(net: int, params: List[Tensor], dout: Tensor, workspace: Tensor) -> Tensor:
    m = _module(net)
    grads = torch.empty(m._native.nparam, dtype=torch.float32, device=dout.device)
    m.native_backward(dout.shape[0], dout.contiguous(), grads, workspace)
    return grads


@sktr_backward.register_fake
def _(net, params, dout, workspace):
    return dout.new_empty(_module(net)._native.nparam, dtype=torch.float32)


def _sk_setup(ctx, inputs, output):
    ctx.net, ctx.training = inputs[0], inputs[5]
    ctx.save_for_backward(output[1])
    _no_grad_outputs(ctx, output)


def _sk_backward(ctx, dout, dws, dbuf, dcnt):
    if not ctx.training:
        raise RuntimeError("fall3: backward through an eval-mode forward is not supported")
    (ws,) = ctx.saved_tensors
    m = _module(ctx.net)
    grads = torch.ops.fall3.sktr_backward(ctx.net, list(m.parameters()), dout.float(), ws)
    return None, _split_grads(m, grads), None, None, None, None, None, None


sktr_forward.register_autograd(_sk_backward, setup_context=_sk_setup)


# ---------------------------------------------------------------------------------------------
# musa_model.Model (f3_musa)
# ---------------------------------------------------------------------------------------------
@torch.library.custom_op("fall3::musa_forward", mutates_args=())
def musa_forward(net: int, params: List[Tensor], buffers: Tensor, counters: Tensor, x: Tensor, training: bool,
                 seed: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    m = _module(net)
    N = x.shape[0]
    ws = torch.empty(m._native.workspace_bytes(N), dtype=torch.uint8, device=x.device)
    out = torch.empty(N, m.num_classes, dtype=torch.float32, device=x.device)
    nb, nc = buffers.clone(), counters.clone()
    m.native_forward(x, out, ws, training, seed, buffers=nb, counters=nc)
    return out, ws, nb, nc


@musa_forward.register_fake
def _(net, params, buffers, counters, x, training, seed):
    m = _module(net)
    N = x.shape[0]
    return (x.new_empty(N, m.num_classes, dtype=torch.float32),
            x.new_empty(m._native.workspace_bytes(N), dtype=torch.uint8), torch.empty_like(buffers),
            torch.empty_like(counters))


@torch.library.custom_op("fall3::musa_backward", mutates_args=())
def musa_backward(net: int, params: List[Tensor], dout: Tensor, workspace: Tensor) -> Tensor:
    m = _module(net)
    grads = torch.empty(m._native.nparam, dtype=torch.float32, device=dout.device)
    m.native_backward(dout.shape[0], dout.contiguous(), grads, workspace)
    return grads


@musa_backward.register_fake
def _(net, params, dout, workspace):
    return dout.new_empty(_module(net)._native.nparam, dtype=torch.float32)


def _mu_backward(ctx, dout, dws, dbuf, dcnt):
    if not ctx.training:
        raise RuntimeError("fall3: backward through an eval-mode forward is not supported")
    (ws,) = ctx.saved_tensors
    m = _module(ctx.net)
    grads = torch.ops.fall3.musa_backward(ctx.net, list(m.parameters()), dout.float(), ws)
    from .musa import grad_is_none
    # None where the reference's autograd leaves None: A (frozen) always, the SepTemporal edges
    # unless DropBlock ran (then the reference gives them a zero tensor; musa.grad_is_none)
    gl = [None if grad_is_none(name, m.dropblock) else g for g, (name, _, _) in zip(_split_grads(m, grads), m.param_views())]
    return None, gl, None, None, None, None, None


musa_forward.register_autograd(_mu_backward, setup_context=_sk_setup)


# ---------------------------------------------------------------------------------------------
# RMSprop update (in place)
# ---------------------------------------------------------------------------------------------
@torch.library.custom_op("fall3::rmsprop_", mutates_args=("param", "square_avg"))
def rmsprop_(param: Tensor, square_avg: Tensor, grad: Tensor, lr: float, alpha: float, eps: float,
             scale: float) -> None:
    if not (param.is_contiguous() and square_avg.is_contiguous() and grad.is_contiguous()):
        raise RuntimeError("fall3 rmsprop_: contiguous tensors required")
    check(lib().f3_rmsprop_step(ptr(param), ptr(square_avg), ptr(grad), param.numel(), lr, alpha, eps, scale,
                                stream_handle()), "rmsprop")


@rmsprop_.register_fake
def _(param, square_avg, grad, lr, alpha, eps, scale):
    return None
