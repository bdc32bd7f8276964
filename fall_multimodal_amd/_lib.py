"""ctypes binding of the C ABI in include/fall3.h (libfall3.so, built for gfx950).

There is no CPU fallback: if the library is missing or no HIP device is visible the
product path raises. torch is imported first so the process uses torch's HIP runtime
(libamdhip64.so.7) and the library's kernels share torch's device context and streams.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("F3_LIB") or os.path.join(HERE, "libfall3.so")  # F3_LIB: A/B of two builds (tools only)

# every symbol declared in include/fall3.h
EXPORTS = (
    "f3_net_create", "f3_net_destroy", "f3_net_num_entries", "f3_net_entry", "f3_net_param_count",
    "f3_net_buffer_count", "f3_net_counter_count", "f3_net_workspace_bytes", "f3_net_forward",
    "f3_net_loss", "f3_net_backward", "f3_rmsprop_step", "f3_conv_forward", "f3_status_string",
    "f3_net_debug_tensor", "f3_conv_backward_data", "f3_conv_backward_weight", "f3_conv_wgrad_packed", "f3_split_x3cat",
    "f3_conv_forward_x3cat", "f3_conv_backward_data_x3cat", "f3_conv_backward_weight_x3cat", "f3_conv_step_x3cat", "f3_graph_mix_forward",
    "f3_graph_mix_backward", "f3_graph_mix_forward_ex", "f3_graph_mix_backward_ex", "f3_net_backward_phase",
    "f3_net_grad_split", "f3_net_wait_phase1", "f3_net_backward_rmsprop", "f3_net_fused_rmsprop", "f3_net_precision", "f3_net_status",
    "f3_targcn_create", "f3_targcn_destroy", "f3_targcn_num_entries", "f3_targcn_entry", "f3_targcn_param_count",
    "f3_targcn_buffer_count", "f3_targcn_workspace_bytes", "f3_targcn_forward", "f3_targcn_backward", "f3_targcn_stage_times", "f3_targcn_status", "f3_net_sensor_times", "f3_soft_ce",
    "f3_sktr_create", "f3_sktr_destroy", "f3_sktr_num_entries", "f3_sktr_entry", "f3_sktr_param_count",
    "f3_sktr_buffer_count", "f3_sktr_counter_count", "f3_sktr_workspace_bytes", "f3_sktr_forward", "f3_sktr_backward",
    "f3_musa_create", "f3_musa_destroy", "f3_musa_num_entries", "f3_musa_entry", "f3_musa_param_count",
    "f3_musa_buffer_count", "f3_musa_counter_count", "f3_musa_workspace_bytes", "f3_musa_forward", "f3_musa_backward",
    "f3_musa_guards",
    "f3_dwconv_t_forward", "f3_pointwise_conv", "f3_rgb_scratch_floats", "f3_rgb_forward", "f3_rgb_backward",
)

F3_OK, F3_EINVAL, F3_EBATCH, F3_EHIP, F3_ESTATE, F3_EDEVICE = 0, 1001, 1002, 1003, 1004, 1005
ENTRY_PARAM, ENTRY_BUFFER, ENTRY_COUNTER = 0, 1, 2


class F3TargcnConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("num_node", "num_class", "precision")]


class F3MusaConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("num_point", "frames", "num_class", "precision")]


class F3SktrConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("num_joint", "frames", "persons", "num_class", "precision")]


class F3Config(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "model", "num_node", "num_partition", "num_class", "in_channels", "sensor", "sensor_dim",
        "sensor_classes", "softmax_output", "naming", "frames", "sensor_frames", "precision")]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"fall3: {LIB_PATH} is not built (run `make` or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P, I, I64, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
    sig = {
        "f3_net_create": (I, [ctypes.POINTER(F3Config), ctypes.POINTER(P)]),
        "f3_net_destroy": (None, [P]),
        "f3_net_num_entries": (I, [P]),
        "f3_net_entry": (I, [P, I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(I), ctypes.POINTER(I),
                             ctypes.POINTER(I64), ctypes.POINTER(I64)]),
        "f3_net_param_count": (I64, [P]),
        "f3_net_buffer_count": (I64, [P]),
        "f3_net_counter_count": (I64, [P]),
        "f3_net_workspace_bytes": (I64, [P, I]),
        "f3_net_forward": (I, [P, I, I, P, P, P, P, P, P, P, P]),
        "f3_net_loss": (I, [P, I, P, P, P, P, P]),
        "f3_net_backward": (I, [P, I, P, P, P, P, P]),
        "f3_net_backward_phase": (I, [P, I, P, P, P, P, I, P]),
        "f3_net_grad_split": (I64, [P]),
        "f3_net_wait_phase1": (I, [P, P]),
        "f3_net_backward_rmsprop": (I, [P, I, P, P, P, P, P, F, F, F, P]),
        "f3_net_fused_rmsprop": (I, [P]),
        "f3_net_precision": (I, [P]),
        "f3_net_status": (I, [P, I]),
        "f3_rmsprop_step": (I, [P, P, P, I64, F, F, F, F, P]),
        "f3_conv_forward": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, I, P]),
        "f3_status_string": (ctypes.c_char_p, [I]),
        "f3_net_debug_tensor": (P, [P, I, P, I, I, ctypes.c_char_p]),
        "f3_conv_backward_data": (I, [P, P, P, P, I, I, I, I, I, I, I, I, I, P]),
        "f3_conv_backward_weight": (I, [P, P, P, P, I, I, I, I, I, I, I, I, I, P]),
        "f3_conv_wgrad_packed": (I, [P, P, P, ctypes.c_longlong, I, I, I, I, I, I, I, I, P]),
        "f3_split_x3cat": (I, [P, P, ctypes.c_int64, I, P]),
        "f3_conv_forward_x3cat": (I, [P, P, P, P, P, I, I, I, I, I, I, I, I, P]),
        "f3_conv_backward_data_x3cat": (I, [P, P, P, P, I, I, I, I, I, I, I, I, P]),
        "f3_conv_backward_weight_x3cat": (I, [P, P, P, P, I, I, I, I, I, I, I, I, P]),
        "f3_conv_step_x3cat": (I, [I, P, P, P, P, P, P, P, P, P, P, F, P, P, I, I, I, I, I, P]),
        "f3_graph_mix_forward": (I, [P, P, P, I, I, I, I, P]),
        "f3_graph_mix_backward": (I, [P, P, P, P, P, I, I, I, I, P]),
        "f3_graph_mix_forward_ex": (I, [P, P, P, I, I, I, I, I, P]),
        "f3_graph_mix_backward_ex": (I, [P, P, P, P, P, I, I, I, I, I, P]),
        "f3_targcn_create": (I, [ctypes.POINTER(F3TargcnConfig), ctypes.POINTER(P)]),
        "f3_targcn_destroy": (None, [P]),
        "f3_targcn_num_entries": (I, [P]),
        "f3_targcn_entry": (I, [P, I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(I), ctypes.POINTER(I),
                                ctypes.POINTER(I64), ctypes.POINTER(I64)]),
        "f3_targcn_param_count": (I64, [P]),
        "f3_targcn_buffer_count": (I64, [P]),
        "f3_targcn_workspace_bytes": (I64, [P, I]),
        "f3_targcn_stage_times": (I, [P, I, P]),
        "f3_targcn_status": (I, [P, I]),
        "f3_net_sensor_times": (I, [P, I, P]),
        "f3_targcn_forward": (I, [P, I, P, P, P, P, P, P]),
        "f3_targcn_backward": (I, [P, I, P, P, P, P, P, P]),
        "f3_soft_ce": (I, [P, P, I, I, P, P, P]),
        "f3_sktr_create": (I, [ctypes.POINTER(F3SktrConfig), ctypes.POINTER(P)]),
        "f3_sktr_destroy": (None, [P]),
        "f3_sktr_num_entries": (I, [P]),
        "f3_sktr_entry": (I, [P, I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(I), ctypes.POINTER(I),
                              ctypes.POINTER(I64), ctypes.POINTER(I64)]),
        "f3_sktr_param_count": (I64, [P]),
        "f3_sktr_buffer_count": (I64, [P]),
        "f3_sktr_counter_count": (I64, [P]),
        "f3_sktr_workspace_bytes": (I64, [P, I]),
        "f3_sktr_forward": (I, [P, I, I, P, P, P, P, P, P, P, ctypes.c_uint, F, P]),
        "f3_sktr_backward": (I, [P, I, P, P, P, P, P, P]),
        "f3_musa_create": (I, [ctypes.POINTER(F3MusaConfig), ctypes.POINTER(P)]),
        "f3_musa_destroy": (None, [P]),
        "f3_musa_num_entries": (I, [P]),
        "f3_musa_entry": (I, [P, I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(I), ctypes.POINTER(I),
                              ctypes.POINTER(I64), ctypes.POINTER(I64)]),
        "f3_musa_param_count": (I64, [P]),
        "f3_musa_buffer_count": (I64, [P]),
        "f3_musa_counter_count": (I64, [P]),
        "f3_musa_workspace_bytes": (I64, [P, I]),
        "f3_musa_guards": (I, [P, I, ctypes.POINTER(I64), I]),
        "f3_musa_forward": (I, [P, I, I, P, P, P, P, P, P, ctypes.c_uint, I, P]),
        "f3_musa_backward": (I, [P, I, P, P, P, P, P, P]),
        "f3_dwconv_t_forward": (I, [P, P, P, P, P, I, I, I, I, I, I, I, P]),
        "f3_pointwise_conv": (I, [P, P, P, P, I, P, P, I, I, I, I, I, I, I, I, I, P]),
        "f3_rgb_scratch_floats": (ctypes.c_longlong, [I, I]),
        "f3_rgb_forward": (I, [P, P, P, P, I, I, P]),
        "f3_rgb_backward": (I, [P, P, P, P, P, P, P, ctypes.c_longlong, I, I, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int, what: str):
    if status == F3_OK:
        return
    msg = lib().f3_status_string(status).decode()
    if status == F3_EBATCH:
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what}: {msg} (status {status})")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"fall3: {what} must be on the HIP device (MI355X); there is no CPU path")
