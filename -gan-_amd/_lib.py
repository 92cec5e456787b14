"""ctypes binding of libganamd.so (the C ABI declared in include/ganamd.h).

The product path has no fallback: if the shared library is missing or was built for another
target, importing this module raises.  Every wrapper checks dtype/device/contiguity before
handing raw pointers to the ABI and launches on torch's current HIP stream, so the calls are
captured by ``torch.cuda.graph`` like any other kernel.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
SO_PATH = os.environ.get("GANAMD_SO") or os.path.join(_HERE, "libganamd.so")   # GANAMD_SO: A/B builds

c_int = ctypes.c_int
c_long = ctypes.c_long
c_float = ctypes.c_float
c_size_t = ctypes.c_size_t
vp = ctypes.c_void_p

PAD_ZERO, PAD_REPLICATE = 0, 1
EPI_STORE, EPI_BIAS, EPI_DEMOD, EPI_ACCUM, EPI_SCALE = 0, 1, 2, 3, 4
CONV_FWD, CONV_DGRAD, CONV_WGRAD = 0, 1, 2
ACT_SIGMOID, ACT_TANH, ACT_LEAKY = 0, 1, 2
MATH_F32, MATH_BF16 = 0, 1
KERNEL_PATCH_FWD, KERNEL_PATCH_DGRAD, KERNEL_WGRAD_ROW, KERNEL_SMALL = 1, 2, 4, 8   # ganamd_conv_desc.kernel_off bits


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("B", "Cin", "H", "W", "Cout", "OH", "OW", "KH", "KW", "stride", "pad", "pad_mode", "transposed",
                 "packed_w", "math", "kernel_off")]


class GTile(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("a_off", "lda", "b_off", "ldb", "c_off", "ldc", "rows", "cols", "K", "epi", "bias_off")] + \
               [("scale", ctypes.c_float)]


class PackJob(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("out", ctypes.c_void_p)] + \
               [(n, ctypes.c_int32) for n in ("sm", "sc", "st", "M", "Ck", "T", "Mpad", "Ckp", "ps", "pk", "ppad", "x3")] + \
               [("chunk0", ctypes.c_int64)]


class CriticOp(ctypes.Structure):
    """ganamd_critic_op (include/ganamd.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("ins", ctypes.c_int32 * 3)] + \
               [(n, ctypes.c_int32) for n in ("cout", "k", "stride", "pad", "pad_mode", "n_out", "kr", "akr",
                                              "group")] + \
               [("alpha", ctypes.c_float)] + \
               [(n, ctypes.c_void_p) for n in ("w", "w_fwd", "w_dgrad", "bias", "ri", "rw", "ari", "arw")]


class CriticGrads(ctypes.Structure):
    _fields_ = [("gw", ctypes.c_void_p), ("gb", ctypes.c_void_p)]


COP = {k: i for i, k in enumerate(("swap", "conv", "prelu", "resample", "pmean", "sigmoid", "scale_add", "mbstd",
                                   "flatten"))}

ROUTE_MAX = 8          # GANAMD_ROUTE_MAX

# name -> (restype, argtypes)
_SIGS = {
    "ganamd_version": (ctypes.c_char_p, []),
    "ganamd_stream_capture_id": (c_int, [vp, ctypes.POINTER(ctypes.c_ulonglong)]),
    "ganamd_conv_workspace": (c_int, [ctypes.POINTER(ConvDesc), c_int, ctypes.POINTER(c_size_t)]),
    "ganamd_conv_plan_info": (c_int, [ctypes.POINTER(ConvDesc), c_int, c_int, ctypes.POINTER(ctypes.c_int)]),
    "ganamd_conv_pack_bytes": (c_int, [ctypes.POINTER(ConvDesc), c_int, ctypes.POINTER(c_size_t)]),
    "ganamd_conv_pack_job": (c_int, [ctypes.POINTER(ConvDesc), c_int, vp, vp, ctypes.POINTER(PackJob)]),
    "ganamd_pack_job_chunks": (ctypes.c_int64, [ctypes.POINTER(PackJob)]),
    "ganamd_conv_pack_batch": (c_int, [vp, c_int, ctypes.c_int64, vp]),
    "ganamd_conv_pack": (c_int, [ctypes.POINTER(ConvDesc), c_int, vp, vp, vp]),
    "ganamd_conv_fwd_ex": (c_int, [ctypes.POINTER(ConvDesc), vp, vp, vp, vp, vp, c_float, vp, vp, vp, vp, vp, c_size_t,
                                   vp]),
    "ganamd_mix_fwd": (c_int, [c_int, vp, vp, vp, vp, vp, c_long, c_long, vp, vp]),
    "ganamd_mix_bwd": (c_int, [c_int, vp, vp, vp, vp, vp, c_long, c_long, vp, vp, vp, vp, vp, vp, vp]),
    "ganamd_gp_workspace": (c_size_t, [c_int, c_long]),
    "ganamd_gp_fwd": (c_int, [vp, c_int, c_long, c_float, c_float, c_int, vp, vp, vp, c_size_t, vp]),
    "ganamd_gp_bwd": (c_int, [vp, vp, vp, c_int, c_long, c_float, c_float, c_int, vp, vp]),
    "ganamd_add_prelu": (c_int, [vp, vp, vp, c_int, c_long, vp, vp]),
    "ganamd_modconv_sd_bwd": (c_int, [vp, vp, vp, vp, vp, c_int, c_int, c_long, vp, vp, vp, vp]),
    "ganamd_route_bwd": (c_int, [c_int, vp, vp, vp, c_int, c_long, vp, vp]),
    "ganamd_scale_add": (c_int, [vp, vp, vp, c_long, c_long, vp, vp]),
    "ganamd_conv_fwd": (c_int, [ctypes.POINTER(ConvDesc), vp, vp, vp, vp, vp, c_float, vp, vp, c_size_t, vp]),
    "ganamd_conv_dgrad": (c_int, [ctypes.POINTER(ConvDesc), vp, vp, vp, c_float, vp, vp, c_size_t, vp]),
    "ganamd_conv_wgrad": (c_int, [ctypes.POINTER(ConvDesc), vp, vp, vp, vp, c_float, vp, c_int, vp, c_size_t, vp]),
    "ganamd_conv_wgrad2": (c_int, [ctypes.POINTER(ConvDesc), vp, vp, vp, vp, c_float, vp, c_int, vp, c_size_t, vp]),
    "ganamd_rowreduce_workspace": (c_size_t, [c_int, c_long]),
    "ganamd_bn_act_fwd": (c_int, [vp, c_int, c_long, vp, vp, vp, vp, vp, c_float, c_float, vp, vp, vp, vp, c_size_t, vp]),
    "ganamd_bn_act_fwd_seg": (c_int, [vp, c_int, c_long, c_int, vp, vp, vp, vp, vp, c_float, c_float, vp, vp, vp, vp,
                                      vp, c_size_t, vp]),
    "ganamd_bn_act_bwd": (c_int, [vp, vp, c_int, c_long, vp, vp, vp, vp, vp, vp, vp, vp, vp, c_int, vp, c_size_t, vp]),
    "ganamd_prelu_fwd": (c_int, [vp, vp, c_int, c_long, vp, vp]),
    "ganamd_prelu_bwd": (c_int, [vp, vp, vp, c_int, c_long, vp, vp, c_int, vp, c_size_t, vp]),
    "ganamd_prelu_bwd_bwd": (c_int, [vp, vp, vp, vp, vp, c_int, c_long, vp, vp, vp, vp, c_size_t, vp]),
    "ganamd_resample2d": (c_int, [vp, c_long, c_int, c_int, vp, c_int, c_int, vp, vp, c_int, vp, vp, c_int, vp]),
    "ganamd_resample2d_add": (c_int, [vp, c_long, c_int, c_int, vp, c_int, c_int, vp, vp, c_int, vp, vp, c_int,
                                      vp, vp, vp, vp]),
    "ganamd_resample2d_sum": (c_int, [vp, vp, c_long, c_int, c_int, vp, c_int, c_int, vp, vp, c_int, vp, vp, c_int,
                                      vp]),
    "ganamd_plane_dot_pair": (c_int, [vp, vp, vp, c_long, c_long, vp, vp, vp]),
    "ganamd_plane_dot": (c_int, [vp, vp, c_long, c_long, c_float, vp, vp]),
    "ganamd_row_dot": (c_int, [vp, vp, c_int, c_long, vp, c_int, vp, c_size_t, vp]),
    "ganamd_segment_sumsq": (c_int, [vp, c_long, c_int, vp, vp]),
    "ganamd_adamw": (c_int, [vp, vp, vp, vp, c_long, vp, c_float, c_float, c_float, c_float, c_float, vp]),
    "ganamd_grouped_gemm": (c_int, [vp, vp, vp, vp, vp, c_int, c_int, c_int, c_int, vp]),
    "ganamd_prelu_tangent": (c_int, [vp, vp, vp, vp, c_int, c_long, vp, vp, c_int, vp, c_size_t, vp]),
    "ganamd_act_fwd": (c_int, [c_int, vp, c_long, c_float, vp, vp]),
    "ganamd_act_bwd": (c_int, [c_int, vp, vp, c_long, c_float, vp, vp]),
    "ganamd_act_adjoint": (c_int, [c_int, vp, vp, vp, vp, c_long, c_float, vp, vp]),
    "ganamd_scale_add2": (c_int, [vp, vp, vp, vp, vp, c_long, c_long, vp, vp]),
    "ganamd_plane_dot2": (c_int, [vp, vp, vp, vp, c_long, c_long, vp, vp]),
    "ganamd_axpy": (c_int, [c_long, c_float, vp, vp, vp]),
    "ganamd_bce_fwd": (c_int, [vp, vp, c_int, vp, vp]),
    "ganamd_bce_bwd": (c_int, [vp, vp, c_int, vp, vp, vp]),
    "ganamd_softmax_m": (c_int, [c_int, vp, c_long, vp, vp]),
    "ganamd_softmax_m_bwd": (c_int, [c_int, vp, vp, c_long, vp, vp]),
    "ganamd_mbstd_workspace": (c_size_t, [c_int]),
    "ganamd_mbstd_fwd": (c_int, [vp, c_long, c_int, c_int, c_int, c_int, c_int, vp, c_long, vp, vp, c_size_t, vp]),
    "ganamd_mbstd_bwd": (c_int, [vp, c_long, vp, c_long, c_int, c_int, c_int, c_int, c_int, vp, vp, c_size_t, vp]),
    "ganamd_mbstd_tangent": (c_int, [vp, vp, c_long, c_int, c_int, c_int, c_int, c_int, vp, c_long, vp, c_size_t, vp]),
    "ganamd_mbstd_adjoint": (c_int, [vp, vp, c_long, vp, vp, c_long, c_int, c_int, c_int, c_int, c_int, vp, vp, c_size_t,
                                     vp]),
    "ganamd_linear_bn_act": (c_int, [ctypes.POINTER(ConvDesc), vp, vp, vp, c_float, vp, vp, vp, vp, vp, c_float, c_float,
                                     vp, vp, c_size_t, vp]),
    "ganamd_philox_uniform": (c_int, [vp, c_long, ctypes.c_uint64, vp, vp]),
    "ganamd_philox_normal": (c_int, [vp, c_long, ctypes.c_uint64, vp, vp]),
    "ganamd_philox_draw": (c_int, [vp, c_long, ctypes.c_uint64, vp, ctypes.c_uint32, c_int, c_int, vp]),
    "ganamd_philox_draw_keyed": (c_int, [vp, c_long, vp, vp, ctypes.c_uint32, c_int, c_int, vp]),
    "ganamd_philox_advance": (c_int, [vp, vp]),
    "ganamd_critic_create": (vp, [ctypes.POINTER(CriticOp), c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    "ganamd_critic_destroy": (None, [vp]),
    "ganamd_critic_workspace": (c_int, [vp, ctypes.POINTER(c_size_t)]),
    "ganamd_critic_value": (c_int, [vp, c_int, c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "ganamd_critic_region_bytes": (c_int, [vp, c_int, ctypes.POINTER(c_size_t)]),
    "ganamd_critic_bind": (c_int, [vp, c_int, vp, c_size_t]),
    "ganamd_critic_forward": (c_int, [vp, vp, vp, vp, c_size_t, vp]),
    "ganamd_critic_backward": (c_int, [vp, vp, vp, vp, vp, c_size_t, vp]),
    "ganamd_critic_tangent": (c_int, [vp, vp, vp, vp, c_size_t, vp]),
    "ganamd_critic_adjoint": (c_int, [vp, vp, vp, vp, vp, c_size_t, vp]),
    "ganamd_critic_gp_step": (c_int, [vp, vp, c_float, c_float, c_int, vp, vp, vp, vp, vp, vp, c_size_t, vp]),
    "ganamd_image_batch_workspace": (c_size_t, [c_int, c_int, c_int]),
    "ganamd_image_batch": (c_int, [vp, c_int, c_int, c_int, vp, vp, vp, c_int, c_int, vp, vp, c_int, c_int, vp, vp,
                                   vp, vp, c_size_t, vp]),
}

EXPORTS = tuple(_SIGS)


def _load():
    if not os.path.exists(SO_PATH):
        raise ImportError(f"{SO_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(SO_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


LIB = _load()


class GanAmdError(RuntimeError):
    pass


def check(rc: int, what: str):
    if rc != 0:
        raise GanAmdError(f"{what} failed with code {rc}")


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    """Raw device pointer of a contiguous fp32 CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
        raise GanAmdError(f"expected contiguous float32 HIP tensor, got {t.dtype} {t.device} "
                          f"contiguous={t.is_contiguous()} shape={tuple(t.shape)}")
    return t.data_ptr()


def iptr(t):
    if t is None:
        return None
    if not (t.is_cuda and t.dtype == torch.int32 and t.is_contiguous()):
        raise GanAmdError("expected contiguous int32 HIP tensor")
    return t.data_ptr()


def workspace(nbytes: int, device) -> torch.Tensor:
    """Caller-provided scratch from torch's caching allocator (graph-capture safe)."""
    return torch.empty(max(int(nbytes), 4) // 4 + 1, dtype=torch.float32, device=device)


def ws(t):
    """(pointer, bytes) of a workspace tensor (None -> NULL, 0): the two workspace arguments of the ABI."""
    if t is None:
        return None, 0
    return ptr(t), t.numel() * t.element_size()


def capture_id() -> int:
    """Id of the HIP graph capture in progress on torch's current stream (0: not capturing)."""
    v = ctypes.c_ulonglong(0)
    check(LIB.ganamd_stream_capture_id(stream(), ctypes.byref(v)), "stream_capture_id")
    return int(v.value)


def version() -> str:
    return LIB.ganamd_version().decode()


_HIP = []


def graph_node_counts(raw_graph: int) -> dict:
    """Nodes of a captured HIP graph by type (``torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()``):
    ``kernel`` = the kernel dispatches one replay issues.  Measurement only (bench.py)."""
    if not _HIP:
        _HIP.append(ctypes.CDLL("libamdhip64.so"))
    hip = _HIP[0]
    g = ctypes.c_void_p(raw_graph)
    n = ctypes.c_size_t(0)
    check(hip.hipGraphGetNodes(g, None, ctypes.byref(n)), "hipGraphGetNodes")
    nodes = (ctypes.c_void_p * max(n.value, 1))()
    check(hip.hipGraphGetNodes(g, nodes, ctypes.byref(n)), "hipGraphGetNodes")
    names = {0: "kernel", 1: "memcpy", 2: "memset"}
    out = {"kernel": 0, "memcpy": 0, "memset": 0, "other": 0}
    t = ctypes.c_int(0)
    for i in range(n.value):
        check(hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t)), "hipGraphNodeGetType")
        out[names.get(t.value, "other")] += 1
    return out
