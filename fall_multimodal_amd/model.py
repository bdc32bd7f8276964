"""Drop-in modules for the reference's model factory, backed by the gfx950 HIP library.

Reference interface mirrored here:
  build_model(config) -> nn.Module                  Multimodal_Fall3/model/build_model.py:5-19
  TwoStreamSTGCAN_BiLSTM.forward(skel, sensor)      Multimodal_Fall3/model/combination.py:37-46
  TwoStreamSTGCAN.forward(skel, sensor)             combination.py:9-25 (its missing-argument
                                                    bug, §0.7 of SURVEY.md, is fixed)
  STGCAN.forward(skel, sensor)                      Multimodal_Fall3/model/stgcan.py:210-228
  BiLSTM.forward(skel, sensor)                      Multimodal_Fall3/model/bilstm.py:41-59
  TwoStreamSpatialTemporalGraph.forward((pts, mot, ser)) -> softmax
                                                    GSTCAN_HAR_conv_10kfold.ipynb:424-444,
                                                    GSTCAN_UR_conv.ipynb (CNN_BiLSTM sensor)

Every module's state_dict has the reference's exact keys, order and shapes (the table
comes from the native plan, f3_net_entry). Parameters are views into one flat fp32
buffer and gradients come back as views into one flat gradient buffer, so the optimizer
and the data-parallel all-reduce each touch one contiguous array. The whole model's
forward is one native call and its backward another: the custom ops fall3::net_forward /
fall3::net_backward (ops.py, torch.library, with fake kernels and autograd registration).
"""
from __future__ import annotations

import ctypes
import math
import os
import sys
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn as nn

from . import _lib, ops
from ._lib import ENTRY_BUFFER, ENTRY_COUNTER, ENTRY_PARAM, check, lib, ptr, require_device, stream_handle
from .graph import STRATEGY_PARTITIONS, Graph

MODEL_IDS = {"two_stgcan_bilstm": 0, "two_stgcan": 1, "stgcn": 2, "bilstm": 3}
SENSOR_IDS = {"none": 0, "bilstm": 1, "cnn_bilstm": 2}
PRECISION_IDS = {"fp32": 0, "bf16": 1, "bf16x3": 4}


def default_precision():
    """The skeleton streams' GEMM arithmetic when a constructor is given none: "bf16x3" (fp32
    activations, split-bf16 products on bf16 MFMA; meets the north star's 1e-3 logits / identical
    argmax gate), so the reference's own `build_model(config)` call
    (model/main.py:277) trains in the benchmarked mode. F3_PRECISION=fp32|bf16 selects another."""
    p = os.environ.get("F3_PRECISION", "bf16x3")
    if p not in PRECISION_IDS:
        raise ValueError(f"F3_PRECISION must be one of {sorted(PRECISION_IDS)}, got {p!r}")
    return p


_PRECISION_LOGGED = set()


def _log_precision_once(prec, defaulted):
    """One stderr line per process and precision when a net is built: the default moved from fp32
    to bf16x3 in round 5, so a caller that relied on the old default is told."""
    if prec in _PRECISION_LOGGED or os.environ.get("F3_QUIET"):
        return
    _PRECISION_LOGGED.add(prec)
    how = "default; F3_PRECISION or precision= selects fp32 / bf16" if defaulted else "requested"
    print(f"fall_multimodal_amd: skeleton GEMMs in {prec} ({how})", file=sys.stderr)


@dataclass
class NetSpec:
    model: str = "two_stgcan_bilstm"
    layout: str = "coco_cut"
    strategy: str = "spatial"
    num_class: int = 11
    in_channels: int = 3
    sensor: str = "bilstm"
    sensor_dim: int = 15
    sensor_classes: int | None = None
    softmax_output: bool = False
    naming: str = "package"
    frames: int = 30
    sensor_frames: int = 30
    precision: str | None = None  # None: default_precision(); "fp32": exact fp32 MFMA; "bf16": bf16
    #                               operands, fp32 accumulate; "bf16x3": fp32 activations, split-bf16 GEMMs
    extra: dict = field(default_factory=dict)


class NativeNet:
    """Owner of one f3_net handle and its state_dict table."""

    def __init__(self, spec: NetSpec, K: int, V: int):
        L = lib()
        c = _lib.F3Config()
        c.model = MODEL_IDS[spec.model]
        c.num_node, c.num_partition, c.num_class = V, K, spec.num_class
        c.in_channels = spec.in_channels
        c.sensor = SENSOR_IDS[spec.sensor if spec.model in ("two_stgcan_bilstm", "bilstm") else "none"]
        c.sensor_dim = spec.sensor_dim
        c.sensor_classes = spec.sensor_classes or 0
        c.softmax_output = int(spec.softmax_output)
        c.naming = 1 if spec.naming == "notebook" else 0
        c.frames, c.sensor_frames = spec.frames, spec.sensor_frames
        # resolved here, not written back into the caller's spec
        prec = spec.precision if spec.precision is not None else default_precision()
        if prec not in PRECISION_IDS:
            raise ValueError(f"precision must be one of {sorted(PRECISION_IDS)}, got {prec!r}")
        _log_precision_once(prec, spec.precision is None)
        c.precision = PRECISION_IDS[prec]
        h = ctypes.c_void_p()
        check(L.f3_net_create(ctypes.byref(c), ctypes.byref(h)), "f3_net_create")
        self.h = h
        self.entries = []
        name, kind, nd = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_int()
        shape, off = (ctypes.c_int64 * 8)(), ctypes.c_int64()
        for i in range(L.f3_net_num_entries(h)):
            check(L.f3_net_entry(h, i, ctypes.byref(name), ctypes.byref(kind), ctypes.byref(nd), shape,
                                 ctypes.byref(off)), "f3_net_entry")
            self.entries.append((name.value.decode(), kind.value, tuple(shape[d] for d in range(nd.value)),
                                 off.value))
        self.precision = prec
        self.nparam = L.f3_net_param_count(h)
        self.nbuf = L.f3_net_buffer_count(h)
        self.ncnt = L.f3_net_counter_count(h)
        self._ws_bytes = {}

    def workspace_bytes(self, batch):
        if batch not in self._ws_bytes:
            self._ws_bytes[batch] = int(lib().f3_net_workspace_bytes(self.h, batch))
        return self._ws_bytes[batch]

    def __del__(self):
        try:
            if getattr(self, "h", None):
                lib().f3_net_destroy(self.h)
        except Exception:
            pass


def _default_value(name, shape, A):
    """PyTorch default initialisation of the reference modules (no custom init on this path)."""
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "A":
        return torch.from_numpy(A.astype(np.float32))
    if leaf == "running_mean":
        return torch.zeros(shape)
    if leaf == "running_var":
        return torch.ones(shape)
    if leaf == "num_batches_tracked":
        return torch.zeros((), dtype=torch.long)
    if "edge_importance" in name:
        return torch.ones(shape)  # stgcan.py:198-201
    if leaf.startswith(("weight_ih", "weight_hh", "bias_ih", "bias_hh")):
        b = 1.0 / math.sqrt(shape[0] // 4)  # nn.LSTM: U(+-1/sqrt(H))
        return torch.empty(shape).uniform_(-b, b)
    return None


class Fall3Net(nn.Module):
    """Generic native-backed module; the reference-named classes below configure it."""

    def __init__(self, spec: NetSpec, device=None):
        super().__init__()
        object.__setattr__(self, "spec", spec)
        graph = Graph(spec.layout, spec.strategy)
        A = graph.A
        object.__setattr__(self, "_native", NativeNet(spec, A.shape[0], A.shape[1]))
        object.__setattr__(self, "_op_id", ops.register(self))
        object.__setattr__(self, "num_node", A.shape[1])
        if device is None:
            device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        dev = torch.device(device)
        nat = self._native
        flat_p = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        flat_b = torch.zeros(max(nat.nbuf, 1), dtype=torch.float32, device=dev)
        flat_c = torch.zeros(max(nat.ncnt, 1), dtype=torch.int64, device=dev)
        self._set_flats(flat_p, flat_b, flat_c)
        shapes = {n: s for n, k, s, o in nat.entries}
        with torch.no_grad():
            for name, kind, shape, off in nat.entries:
                t = self._view(kind, shape, off)
                v = _default_value(name, shape, A)
                if v is None:
                    leaf = name.rsplit(".", 1)[-1]
                    if len(shape) >= 2:          # Conv/Linear weight: kaiming_uniform(a=sqrt 5)
                        fan_in = int(np.prod(shape[1:]))
                    elif leaf == "weight":       # BatchNorm gamma
                        t.fill_(1.0)
                        fan_in = None
                    else:                        # bias: U(+-1/sqrt(fan_in of its weight)); BN beta 0
                        w = shapes.get(name[: -len("bias")] + "weight")
                        fan_in = int(np.prod(w[1:])) if w is not None and len(w) >= 2 else None
                        if fan_in is None:
                            t.zero_()
                    if fan_in:
                        b = 1.0 / math.sqrt(fan_in)
                        t.copy_(torch.empty(shape).uniform_(-b, b))
                else:
                    t.copy_(v)
                self._register(name, kind, t)

    # -- flat storage ----------------------------------------------------------
    def _set_flats(self, p, b, c):
        object.__setattr__(self, "_flat_params", p)
        object.__setattr__(self, "_flat_buffers", b)
        object.__setattr__(self, "_flat_counters", c)

    def _view(self, kind, shape, off):
        n = int(np.prod(shape)) if len(shape) else 1
        flat = {ENTRY_PARAM: self._flat_params, ENTRY_BUFFER: self._flat_buffers,
                ENTRY_COUNTER: self._flat_counters}[kind]
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

    def _tensor(self, name):
        mod, leaf = self._owner(name)
        return mod._parameters[leaf] if leaf in mod._parameters else mod._buffers[leaf]

    def _reflatten(self):
        """Re-alias every parameter/buffer into fresh flat arrays (after .to()/.cuda())."""
        nat = self._native
        first = next(iter(self.parameters()))
        dev = first.device
        p = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        b = torch.zeros(max(nat.nbuf, 1), dtype=torch.float32, device=dev)
        c = torch.zeros(max(nat.ncnt, 1), dtype=torch.int64, device=dev)
        self._set_flats(p, b, c)
        with torch.no_grad():
            for name, kind, shape, off in nat.entries:
                cur = self._tensor(name)
                view = self._view(kind, shape, off)
                view.copy_(cur.detach().to(view.dtype))
                if kind == ENTRY_PARAM:
                    cur.data = view
                else:
                    mod, leaf = self._owner(name)
                    mod._buffers[leaf] = view

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        self._reflatten()
        return self

    def flat_parameters(self):
        return self._flat_params

    @property
    def precision(self):
        """The precision the native net was built with (spec.precision, or the default it resolved to)."""
        return self._native.precision

    def device_status(self, wait=True):
        """Raise if a device-side check of the last training forward / backward failed (F3_EDEVICE:
        the sensor branch's cooperative CNN1D group barrier timed out and wrote NaN into its outputs);
        wait=False checks only copies that have completed. The next forward / backward also raises."""
        check(lib().f3_net_status(self._native.h, 1 if wait else 0), "fall3 device status")

    def param_views(self):
        return [(name, shape, off) for name, kind, shape, off in self._native.entries if kind == ENTRY_PARAM]

    # -- forward ---------------------------------------------------------------
    def _inputs(self, args, kwargs):
        spec = self.spec
        if len(args) == 1 and isinstance(args[0], (tuple, list)):  # notebook form (pts, mot, ser)
            inp = args[0]
            return inp[0], (inp[2] if len(inp) > 2 else None)
        skel = args[0] if len(args) > 0 else kwargs.get("skel")
        sensor = args[1] if len(args) > 1 else kwargs.get("sensor")
        if spec.model == "bilstm" and sensor is None and skel is not None and len(args) == 1:
            sensor, skel = skel, None
        return skel, sensor

    def forward(self, *args, **kwargs):
        """One fall3::net_forward custom op (its autograd calls fall3::net_backward)."""
        skel, sensor = self._inputs(args, kwargs)
        skel, sensor = _prep(skel), _prep(sensor)
        self.check_inputs(skel, sensor)
        out, _, buffers, counters = torch.ops.fall3.net_forward(self._op_id, list(self.parameters()),
                                                                self._flat_buffers, self._flat_counters, skel,
                                                                sensor, self.training)
        if self.training:  # BatchNorm running statistics / num_batches_tracked (nn.BatchNorm semantics)
            with torch.no_grad():
                self._flat_buffers.copy_(buffers)
                self._flat_counters.copy_(counters)
        return out

    def native_forward(self, skel, sensor, out, workspace, training, stream=None, buffers=None, counters=None):
        nat = self._native
        N = (skel if skel is not None else sensor).shape[0]
        st = stream if stream is not None else stream_handle()
        buffers = self._flat_buffers if buffers is None else buffers
        counters = self._flat_counters if counters is None else counters
        check(lib().f3_net_forward(nat.h, N, int(training), ptr(self._flat_params), ptr(buffers), ptr(counters),
                                   ptr(skel), ptr(sensor), ptr(out), ptr(workspace), st), "fall3 forward")

    def native_backward(self, N, dout, grads, workspace, stream=None):
        st = stream if stream is not None else stream_handle()
        check(lib().f3_net_backward(self._native.h, N, ptr(self._flat_params), ptr(dout), ptr(grads),
                                    ptr(workspace), st), "fall3 backward")

    def check_inputs(self, skel, sensor):
        spec = self.spec
        if spec.model != "bilstm":
            if skel is None:
                raise ValueError("skeleton input is required")
            require_device(skel, "skel")
            cin = spec.in_channels if spec.model == "stgcn" else 3
            V = self.num_node
            if skel.dim() != 4 or skel.shape[1] != cin or skel.shape[2] != spec.frames or skel.shape[3] != V:
                raise ValueError(f"skel must be [N,{cin},{spec.frames},{V}], got {tuple(skel.shape)}")
        if spec.model in ("two_stgcan_bilstm", "bilstm"):
            if sensor is None:
                raise ValueError("sensor input is required")
            require_device(sensor, "sensor")
            if sensor.dim() != 3 or sensor.shape[1] != spec.sensor_frames or sensor.shape[2] != spec.sensor_dim:
                raise ValueError(f"sensor must be [N,{spec.sensor_frames},{spec.sensor_dim}], got {tuple(sensor.shape)}")


def _prep(t):
    return None if t is None else t.detach().contiguous().float()


# ----------------------------------------------------------------------------
# reference-named classes
# ----------------------------------------------------------------------------
def _graph_args(graph_args):
    graph_args = dict(graph_args or {})
    return graph_args.get("layout", "coco_cut"), graph_args.get("strategy", "uniform")


class STGCAN(Fall3Net):
    """stgcan.py:147-228 with a classifier (build_model 'stgcn')."""

    def __init__(self, in_channels, graph_args, num_class, device=None, frames=30, precision=None):
        layout, strategy = _graph_args(graph_args)
        super().__init__(NetSpec(model="stgcn", layout=layout, strategy=strategy, num_class=num_class,
                                 in_channels=in_channels, sensor="none", frames=frames, precision=precision),
                         device)


class BiLSTM(Fall3Net):
    """bilstm.py:21-59, feature='mean' (build_model 'bilstm')."""

    def __init__(self, input_size, hidden_size=64, num_layers=1, dropout_prob=0.3, num_classes=1,
                 feature="mean", device=None, sensor_frames=30):
        if hidden_size != 64 or num_layers != 1 or feature != "mean":
            raise NotImplementedError("fall3 implements the reference configuration: H=64, 1 layer, mean feature")
        super().__init__(NetSpec(model="bilstm", num_class=num_classes, sensor="bilstm", sensor_dim=input_size,
                                 sensor_frames=sensor_frames), device)


class CNN_BiLSTM(Fall3Net):
    """Sensor-only CNN1D -> BiLSTM (GSTCAN_UR_sensor.ipynb:493-586; BASELINE config 1): the notebook's
    class takes (hidden_size, num_layers, dropout_prob, num_classes, feature) but builds a fixed
    BiLSTM(input_size=32, hidden_size=64, num_classes=2, feature='mean') on CNN1D(4) (:577-578), so
    the module always has 2 outputs; the same arguments are accepted and ignored here."""

    def __init__(self, hidden_size=16, num_layers=1, dropout_prob=0.3, num_classes=1, feature="last", device=None,
                 sensor_dim=4, sensor_frames=30):
        super().__init__(NetSpec(model="bilstm", num_class=2, sensor="cnn_bilstm", sensor_dim=sensor_dim,
                                 sensor_frames=sensor_frames), device)

    def forward(self, x):
        return super().forward(None, x)


class TwoStreamSTGCAN(Fall3Net):
    """combination.py:9-25 (forward fixed to pass the sensor argument)."""

    def __init__(self, in_channels, graph_args, num_class, device=None, frames=30, precision=None):
        layout, strategy = _graph_args(graph_args)
        super().__init__(NetSpec(model="two_stgcan", layout=layout, strategy=strategy, num_class=num_class,
                                 sensor="none", frames=frames, precision=precision), device)


class TwoStreamSTGCAN_BiLSTM(Fall3Net):
    """combination.py:27-46."""

    def __init__(self, in_channels, graph_args, num_class, bilstm_input_size=15, device=None, frames=30,
                 sensor_frames=30, precision=None):
        layout, strategy = _graph_args(graph_args)
        super().__init__(NetSpec(model="two_stgcan_bilstm", layout=layout, strategy=strategy,
                                 num_class=num_class, sensor="bilstm", sensor_dim=bilstm_input_size,
                                 frames=frames, sensor_frames=sensor_frames, precision=precision), device)


class TwoStreamSpatialTemporalGraph(Fall3Net):
    """Notebook 3-stream form: forward((pts, mot, ser)) -> softmax.

    sensor='bilstm' is GSTCAN_HAR_conv_10kfold.ipynb (BiLSTM(15,64), head = num_class);
    sensor='cnn_bilstm' is GSTCAN_UR_conv.ipynb (CNN1D(4) -> BiLSTM(32,64), head = 2).
    The motion stream is recomputed on device from pts exactly as the notebook does
    (mot = pts[:, :2, 1:] - pts[:, :2, :-1], :1086), so `mot` is accepted and ignored.
    """

    def __init__(self, graph_args, num_class, sensor="bilstm", sensor_dim=None, sensor_classes=None,
                 device=None, frames=30, sensor_frames=30, precision=None):
        layout, strategy = _graph_args(graph_args)
        if sensor_dim is None:
            sensor_dim = 4 if sensor == "cnn_bilstm" else 15
        if sensor_classes is None:
            sensor_classes = 2 if sensor == "cnn_bilstm" else num_class
        super().__init__(NetSpec(model="two_stgcan_bilstm", layout=layout, strategy=strategy,
                                 num_class=num_class, sensor=sensor, sensor_dim=sensor_dim,
                                 sensor_classes=sensor_classes, softmax_output=True, naming="notebook",
                                 frames=frames, sensor_frames=sensor_frames, precision=precision), device)


def build_model(config, device=None, precision=None):
    """build_model.py:5-19: MODEL.NAME in {stgcn, bilstm, two_stgcan, two_stgcan_bilstm}.
    `precision` ("fp32" | "bf16" | "bf16x3") selects the GEMM arithmetic of the skeleton streams;
    None (the reference's one-argument call) is default_precision(), i.e. bf16x3."""
    name = config.MODEL.NAME
    graph_args = {"layout": config.GRAPH.LAYOUT, "strategy": config.GRAPH.STRATEGY}
    if name == "stgcn":
        return STGCAN(config.DATA.IN_CHANNELS, graph_args, num_class=config.DATA.NUM_CLASSES, device=device,
                      precision=precision)
    if name == "bilstm":
        return BiLSTM(input_size=config.DATA.SENSOR_DIM, hidden_size=64, num_layers=1, dropout_prob=0.3,
                      num_classes=config.DATA.NUM_CLASSES, feature="mean", device=device)
    if name == "two_stgcan":
        return TwoStreamSTGCAN(config.DATA.IN_CHANNELS, graph_args, num_class=config.DATA.NUM_CLASSES,
                               device=device, precision=precision)
    if name == "two_stgcan_bilstm":
        return TwoStreamSTGCAN_BiLSTM(config.DATA.IN_CHANNELS, graph_args, num_class=config.DATA.NUM_CLASSES,
                                      bilstm_input_size=config.DATA.SENSOR_DIM, device=device, precision=precision)
    raise RuntimeError(f"Model name [{name}] is not implemented.")


def spec_partitions(strategy):
    return STRATEGY_PARTITIONS[strategy]
