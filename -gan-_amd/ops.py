"""Autograd operators of the hot path, each backed by libganamd.so kernels.

Tensors are CNHW: a feature map is [C, B, H, W]; a per-sample feature vector (linear layers,
styles, SE/SK attention) is [C, B].

Closure under differentiation.  The critic's gradient penalty calls
``autograd.grad(create_graph=True)`` and then ``backward()`` through it (wgangp.py:45-54,69),
so every operator the critic uses has a backward made of differentiable operators:
  conv forward / dgrad / wgrad        -> each other's backward (bilinear family)
  PReLU  -> PReLUBackward -> prelu double-backward kernel
  resample (smooth, bicubic, pools)   -> the same kernel with the transposed tap table
Generator-only operators (fused BatchNorm+PReLU, the modulated conv) are first-order.
"""
from __future__ import annotations

import contextlib
import os
import weakref

from dataclasses import dataclass

import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable
from torch.autograd.graph import get_gradient_edge

from . import _lib
from ._lib import LIB, check, iptr, ptr, stream, workspace
from ._lib import ws as wsarg
from . import tables

# ------------------------------------------------------------------------------------------
# convolution geometry
# ------------------------------------------------------------------------------------------


@dataclass(frozen=True)
class Geo:
    B: int
    Cin: int
    H: int
    W: int
    Cout: int
    OH: int
    OW: int
    K: int
    stride: int = 1
    pad: int = 0
    pad_mode: int = _lib.PAD_REPLICATE
    transposed: bool = False

    def desc(self, packed=False):
        key = (self, packed, _MATH[0], _KOFF[0])
        d = _DESC_CACHE.get(key)
        if d is None:
            d = _lib.ConvDesc(self.B, self.Cin, self.H, self.W, self.Cout, self.OH, self.OW, self.K, self.K,
                              self.stride, self.pad, self.pad_mode, int(self.transposed), int(packed), _MATH[0],
                              _KOFF[0])
            _DESC_CACHE[key] = d
        return d

    def ws_bytes(self, op, packed=False):
        key = (self, op, packed, _MATH[0], _KOFF[0])
        v = _WS_CACHE.get(key)
        if v is None:
            n = _lib.c_size_t(0)
            check(LIB.ganamd_conv_workspace(self.desc(packed), op, n), "conv_workspace")
            v = _WS_CACHE[key] = n.value
        return v

    def pack_key(self, op):
        """What the packed weight operand depends on (not the batch or the spatial size)."""
        return (op, self.Cin, self.Cout, self.K, self.transposed, self.H, self.W, self.stride, self.pad)


_DESC_CACHE: dict = {}
_WS_CACHE: dict = {}
_MATH = [_lib.MATH_F32]      # arithmetic of the conv GEMMs launched now (math_mode)
_KOFF = [0]                  # ganamd_conv_desc.kernel_off of the convs launched now (patch_conv)


@contextlib.contextmanager
def math_mode(mode: str):
    """Run the conv / linear GEMMs issued inside the block in ``"fp32"`` (exact fp32 MFMA, the
    default) or ``"bf16"`` (operands rounded to bf16, fp32 accumulation and storage).  Applies to
    the launches made while the block is active -- wrap the backward too."""
    prev = _MATH[0]
    _MATH[0] = {"fp32": _lib.MATH_F32, "bf16": _lib.MATH_BF16}[mode]
    try:
        yield
    finally:
        _MATH[0] = prev


PLAN_FIELDS = ("bm", "bn", "gx", "gy", "nfull_t", "S", "kt_per_split", "blocks", "occupancy", "cus", "kernel")


def set_patch(mask: int = 15) -> int:
    """Which convs this process's layers send to the specialised kernels (bit 0: stride-1 forwards
    to the split6 LDS-patch conv, bit 1: their dgrads, bit 2: the row-blocked weight gradient, bit 3:
    the direct conv of Cout <= 4 forwards; default 15 = all; 0 = the gather GEMMs, for A/B and
    tests).  It only sets the ``kernel_off`` field of the descriptors this module builds (and of
    critic plans created afterwards): the library itself keeps no such state.  Like ``math_mode`` it
    is read by the backward too (autograd runs it on its own threads), so it is process-wide for the
    Python layers.  Returns the previous mask."""
    prev = (~_KOFF[0]) & 15
    _KOFF[0] = (~int(mask)) & 15
    return prev


@contextlib.contextmanager
def patch_conv(mask: int = 15):
    """``set_patch(mask)`` inside the block."""
    prev = set_patch(mask)
    try:
        yield
    finally:
        set_patch(prev)


def plan_info(geo: "Geo", op: int, scaled: bool = False) -> dict:
    """The block schedule ganamd_conv_fwd / _dgrad launches for this geometry (ganamd_conv_plan_info)."""
    info = (_lib.c_int * 11)()
    check(LIB.ganamd_conv_plan_info(geo.desc(), op, int(scaled), info), "conv_plan_info")
    return dict(zip(PLAN_FIELDS, list(info)))


def conv_geo(B, cin, h, w, cout, k, stride=1, pad=0, pad_mode=_lib.PAD_REPLICATE):
    oh = (h + 2 * pad - k) // stride + 1
    ow = (w + 2 * pad - k) // stride + 1
    return Geo(B, cin, h, w, cout, oh, ow, k, stride, pad, pad_mode, False)


def convT_geo(B, cin, h, w, cout, k, stride, pad):
    oh = (h - 1) * stride - 2 * pad + k
    ow = (w - 1) * stride - 2 * pad + k
    return Geo(B, cin, h, w, cout, oh, ow, k, stride, pad, _lib.PAD_ZERO, True)


def linear_geo(B, cin, cout):
    return Geo(B, cin, 1, 1, cout, 1, 1, 1, 1, 0, _lib.PAD_ZERO, False)


class FlopCounter:
    """Counts the conv-GEMM FLOPs issued through the conv wrappers while ``enabled`` (host side;
    used by bench.py on an eager iteration to report executed vs algorithmic work).

    ``flops`` is what the MFMAs execute: a stride-s transposed conv's forward runs as s^2 phase
    GEMMs over only the taps that reach each output phase (the algorithmic work; a geometry the
    phase split does not cover runs the transposed gather, every tap at every OUTPUT pixel), the
    stride-1 transposed-gather dgrad runs over the padded frame; ``algo_flops`` is the algorithmic
    count 2 * MACs.  ``flops_bf16`` is the part issued in bf16 math."""

    enabled = False
    flops = 0
    algo_flops = 0
    flops_bf16 = 0
    launches = 0
    record = None          # optional list receiving (op, geo, has_xscale, has_yscale, math)

    @staticmethod
    def algorithmic(geo: "Geo") -> int:
        sp = geo.H * geo.W if geo.transposed else geo.OH * geo.OW
        return 2 * geo.B * sp * geo.Cout * geo.Cin * geo.K * geo.K

    @staticmethod
    def issued(geo: "Geo", op: str) -> int:
        macs_per_px = geo.Cout * geo.Cin * geo.K * geo.K
        if op == "fwd" and geo.transposed:
            s = geo.stride
            if s > 1 and geo.K % s == 0 and geo.OH % s == 0 and geo.OW % s == 0:
                # phase-decomposed (csrc/conv_gemm.hip kPhase): s^2 GEMMs of (K/s)^2 taps each
                return 2 * geo.B * geo.OH * geo.OW * macs_per_px // (s * s)
            return 2 * geo.B * geo.OH * geo.OW * macs_per_px
        if op == "dgrad" and not geo.transposed and geo.K > 1 and not (geo.stride > 1 or geo.H * geo.W <= 100):
            # transposed gather into the padded frame (csrc/conv_gemm.hip dgrad_gemm)
            return 2 * geo.B * (geo.H + 2 * geo.pad) * (geo.W + 2 * geo.pad) * macs_per_px
        return FlopCounter.algorithmic(geo)

    @classmethod
    def add(cls, geo: "Geo", op: str = "", xs=False, ys=False):
        if cls.record is not None:
            cls.record.append((op, geo, xs, ys, "bf16" if _MATH[0] == _lib.MATH_BF16 else "fp32"))
        if cls.enabled:
            f = cls.issued(geo, op)
            cls.flops += f
            cls.algo_flops += cls.algorithmic(geo)
            if _MATH[0] == _lib.MATH_BF16:
                cls.flops_bf16 += f
            cls.launches += 1


# ------------------------------------------------------------------------------------------
# packed weight operands (ganamd_conv_pack), cached per parameter between optimizer steps
# ------------------------------------------------------------------------------------------


class PackCache:
    """GEMM-order copies of parameter weights, reused by every conv call on the same weight
    (forward, input-gradient backward, the gradient penalty's double backward) until the weight
    changes.  A weight changes through (a) the fused optimizer, which bumps the epoch of its flat
    buffer (``FlatParams.epoch``; parameters outside one follow the global ``invalidate()``), or
    (b) torch in-place ops on the Parameter (``load_state_dict``, ``p.copy_``), which bump its
    version counter.  Only weights that are Parameters (or views of one) are cached.

    Weights living in an optimizer's flat buffer get a PERSISTENT copy (allocated eagerly, kept
    for the life of the model) registered with that buffer (``PackRegistry``): the optimizer
    refreshes every registered copy with one batched launch right after its update, so in the
    steady state no conv call packs anything.  Other weights, and copies first needed inside a
    HIP graph capture, are packed where the cache misses (under capture: captured there, so
    replays repack at the same points; such a copy is only reused within that one capture)."""

    epoch = 0
    entries: dict = {}

    @classmethod
    def invalidate(cls):
        cls.epoch += 1

    @classmethod
    def clear(cls):
        cls.entries.clear()
        cls.epoch += 1

    @classmethod
    def _pack(cls, geo, op, w, packed):
        check(LIB.ganamd_conv_pack(geo.desc(), op, ptr(w), ptr(packed), stream()), "conv_pack")

    @classmethod
    def _alloc(cls, geo, op, w):
        n = _lib.c_size_t(0)
        check(LIB.ganamd_conv_pack_bytes(geo.desc(), op, n), "conv_pack_bytes")
        return torch.empty(n.value // 4, device=w.device, dtype=torch.float32)

    @classmethod
    def get(cls, geo: "Geo", op: int, w):
        root = w if w._base is None else w._base
        if not isinstance(root, torch.nn.Parameter):
            return None
        base_key = (id(root), w.data_ptr(), geo.pack_key(op))
        flat = getattr(root, "_gan_flat", None)
        cap = _lib.capture_id()
        if flat is not None:
            reg = flat.packs
            e = reg.entries.get(base_key)
            if e is not None and e.root is root:
                if e.version == root._version and reg.valid(e):
                    return e.packed
                if cap == 0:          # reloaded / modified in place: refresh this copy now
                    cls._pack(geo, op, w, e.packed)
                    e.version, e.epoch = root._version, flat.epoch
                    return e.packed
            elif cap == 0:            # first use: a persistent copy, refreshed by the optimizer
                packed = cls._alloc(geo, op, w)
                cls._pack(geo, op, w, packed)
                reg.add(base_key, root, geo, op, w, packed, flat.epoch)
                return packed
        # A capture-local (or non-flat) copy: only reused inside the execution context that made
        # it: eager code, or ONE graph capture (its buffer lives in that graph's memory and is
        # refreshed only when that graph replays).
        key = base_key + (cap,)
        epoch = (id(flat), flat.epoch) if flat is not None else cls.epoch
        e = cls.entries.get(key)
        if e is not None and e[0]() is root and e[1] == root._version and e[2] == epoch:
            return e[3]
        packed = cls._alloc(geo, op, w)
        cls._pack(geo, op, w, packed)
        # the weight is held weakly and its copies leave with it: a process that builds model after
        # model (the GPU test suite: 25 GB of packed copies of dead models) keeps only live ones
        entries = cls.entries
        cls.entries[key] = (weakref.ref(root, lambda _r, k=key: entries.pop(k, None)), root._version, epoch, packed)
        return packed


class _PackEntry:
    __slots__ = ("root", "version", "epoch", "packed", "job")

    def __init__(self, root, version, epoch, packed, job):
        self.root, self.version, self.epoch, self.packed, self.job = root, version, epoch, packed, job


class PackRegistry:
    """The persistent GEMM-order weight copies of one flat parameter buffer and the batched
    repack (ganamd_conv_pack_batch) its optimizer launches after every update."""

    def __init__(self, flat):
        self.flat = flat
        self.entries: dict = {}
        self.table = None          # device copy of the job array
        self.total_chunks = 0
        self.dirty = False
        self.batch_epoch = -1      # flat epoch at which the last batched repack was issued
        self.retired = []

    def add(self, key, root, geo, op, w, packed, epoch):
        job = _lib.PackJob()
        check(LIB.ganamd_conv_pack_job(geo.desc(), op, ptr(w), ptr(packed), job), "conv_pack_job")
        self.entries[key] = _PackEntry(root, root._version, epoch, packed, job)
        self.dirty = True

    def valid(self, e) -> bool:
        return e.epoch == self.flat.epoch or (self.batch_epoch == self.flat.epoch and e.epoch <= self.batch_epoch)

    def repack(self):
        """After the optimizer update (flat.epoch already bumped): refresh every copy, one launch."""
        if not self.entries:
            return
        if self.dirty:
            if _lib.capture_id():
                raise _lib.GanAmdError("packed-weight table changed during graph capture (run one eager step first)")
            jobs = (_lib.PackJob * len(self.entries))()
            c0 = 0
            for i, e in enumerate(self.entries.values()):
                jobs[i] = e.job
                jobs[i].chunk0 = c0
                c0 += LIB.ganamd_pack_job_chunks(e.job)
            raw = torch.frombuffer(bytearray(jobs), dtype=torch.uint8)
            if self.table is not None:        # a captured graph may still launch with the old table
                self.retired.append(self.table)
            self.table = raw.to(self.flat.data.device)
            self.total_chunks = c0
            self.dirty = False
        check(LIB.ganamd_conv_pack_batch(self.table.data_ptr(), len(self.entries), self.total_chunks, stream()),
              "conv_pack_batch")
        self.batch_epoch = self.flat.epoch
        for e in self.entries.values():       # every copy now reflects the current weights
            e.version, e.epoch = e.root._version, self.flat.epoch


def invalidate_packed():
    PackCache.invalidate()


def _need(t, n, what):
    """Host-side operand check before any launch: a wrong size must raise, never fault."""
    if t is not None and n is not None and t.numel() != n:
        raise _lib.GanAmdError(f"{what}: expected {n} elements, got {tuple(t.shape)}")


def small_fwd(geo: Geo) -> bool:
    """Does ganamd_conv_fwd run this geometry as the direct conv of Cout <= 4 (csrc/conv_small.hip,
    ToRGB)?  It takes the weights as stored, so the layers pass them unpacked."""
    return (not geo.transposed and 1 <= geo.Cout <= 4 and geo.stride == 1 and geo.K in (1, 3, 5) and
            geo.pad == (geo.K - 1) // 2 and geo.OH == geo.H and geo.OW == geo.W and geo.W == 64 and
            geo.H % 8 == 0 and _MATH[0] == _lib.MATH_F32 and not (_KOFF[0] & _lib.KERNEL_SMALL))


def _w_numel(geo):
    return geo.Cin * geo.Cout * geo.K * geo.K


def _conv_fwd(geo: Geo, x, w, bias=None, xs=None, ys=None, alpha=1.0, out=None):
    _need(x, geo.Cin * geo.B * geo.H * geo.W, "conv_fwd x")
    _need(w, _w_numel(geo), "conv_fwd w")
    _need(bias, geo.Cout, "conv_fwd bias")
    _need(xs, geo.Cin * geo.B, "conv_fwd x_scale")
    _need(ys, geo.Cout * geo.B, "conv_fwd y_scale")
    FlopCounter.add(geo, "fwd", xs is not None, ys is not None)
    if out is not None:
        _need(out, geo.Cout * geo.B * geo.OH * geo.OW, "conv_fwd out")
    y = out if out is not None else torch.empty((geo.Cout, geo.B, geo.OH, geo.OW), device=x.device,
                                                dtype=torch.float32)
    pw = None if small_fwd(geo) else PackCache.get(geo, _lib.CONV_FWD, w)
    packed = pw is not None
    nb = geo.ws_bytes(_lib.CONV_FWD, packed)
    ws = workspace(nb, x.device) if nb else None
    check(LIB.ganamd_conv_fwd(geo.desc(packed), ptr(x), ptr(pw if packed else w), ptr(bias), ptr(xs), ptr(ys),
                              float(alpha), ptr(y), *wsarg(ws), stream()), "conv_fwd")
    return y


def _conv_dgrad(geo: Geo, gy, w, gys=None, alpha=1.0):
    _need(gy, geo.Cout * geo.B * geo.OH * geo.OW, "conv_dgrad gy")
    _need(w, _w_numel(geo), "conv_dgrad w")
    _need(gys, geo.Cout * geo.B, "conv_dgrad gy_scale")
    FlopCounter.add(geo, "dgrad", gys is not None, False)
    gx = torch.empty((geo.Cin, geo.B, geo.H, geo.W), device=gy.device, dtype=torch.float32)
    pw = PackCache.get(geo, _lib.CONV_DGRAD, w)
    packed = pw is not None
    nb = geo.ws_bytes(_lib.CONV_DGRAD, packed)
    ws = workspace(nb, gy.device) if nb else None
    check(LIB.ganamd_conv_dgrad(geo.desc(packed), ptr(gy), ptr(pw if packed else w), ptr(gys), float(alpha), ptr(gx),
                                *wsarg(ws), stream()), "conv_dgrad")
    return gx


def _conv_wgrad(geo: Geo, x, gy, xs=None, gys=None, alpha=1.0, out=None, accumulate=False):
    _need(x, geo.Cin * geo.B * geo.H * geo.W, "conv_wgrad x")
    _need(gy, geo.Cout * geo.B * geo.OH * geo.OW, "conv_wgrad gy")
    _need(xs, geo.Cin * geo.B, "conv_wgrad x_scale")
    _need(gys, geo.Cout * geo.B, "conv_wgrad gy_scale")
    _need(out, _w_numel(geo), "conv_wgrad out")
    FlopCounter.add(geo, "wgrad", xs is not None, gys is not None)
    shape = (geo.Cin, geo.Cout, geo.K, geo.K) if geo.transposed else (geo.Cout, geo.Cin, geo.K, geo.K)
    gw = out if out is not None else torch.empty(shape, device=x.device, dtype=torch.float32)
    nb = geo.ws_bytes(_lib.CONV_WGRAD)
    ws = workspace(nb, x.device) if nb else None
    check(LIB.ganamd_conv_wgrad(geo.desc(), ptr(x), ptr(gy), ptr(xs), ptr(gys), float(alpha), ptr(gw),
                                int(accumulate), *wsarg(ws), stream()), "conv_wgrad")
    return gw


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def flat_grad(p):
    """During a FIRST-order backward, the pre-bound flat-buffer gradient of parameter ``p`` (or of
    the Parameter a view ``p`` comes from): the backward then accumulates into it with its own
    kernel and returns None to autograd -- no per-parameter AccumulateGrad add launch (10k of them
    per generator step otherwise).  None when autograd has to handle it (create_graph backward,
    parameters outside an optimizer's flat buffer, plain tensors)."""
    if p is None or torch.is_grad_enabled():
        return None
    root = p if p._base is None else p._base
    if not isinstance(root, torch.nn.Parameter) or getattr(root, "_gan_flat", None) is None:
        return None
    g = root.grad
    if g is None or not g.is_contiguous() or g.numel() != p.numel():
        return None
    return g


def wanted(t) -> bool:
    """Will the backward pass now running use a gradient for ``t``?  False for the critic's
    weights inside the gradient penalty's ``autograd.grad(d_out.sum(), x_hat, create_graph=True)``
    (wgangp.py:47): only the input gradient is asked for there, so weight / bias / slope gradients
    are dead work -- the engine would drop them (torch's own convolution backward skips them by
    the same test).  They ARE computed in the penalty's second backward, where they are used."""
    if t is None or not t.requires_grad:
        return False
    try:
        return bool(torch._C._will_engine_execute_node(get_gradient_edge(t).node))
    except RuntimeError:       # not inside an engine call (a direct .backward() of this node)
        return True


def row_sum_acc(a, out):
    """out[c] += sum over the row c of a (a conv bias gradient into the flat gradient buffer)."""
    a = _c(a)
    C, L = _rows(a)
    _need(out, C, "row_sum out")
    ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), a.device)
    check(LIB.ganamd_row_dot(ptr(a), None, C, L, ptr(out), 1, *wsarg(ws), stream()), "row_dot")


class ConvFwd(Function):
    """y = alpha * conv(x, w) + bias   (any order of derivative)."""

    @staticmethod
    def forward(ctx, x, w, bias, geo, alpha):
        ctx.w_arg, ctx.b_arg = w, bias
        x, w = _c(x), _c(w)
        ctx.save_for_backward(x, w)
        ctx.geo, ctx.alpha, ctx.has_bias = geo, alpha, bias is not None
        return _conv_fwd(geo, x, w, None if bias is None else _c(bias), alpha=alpha)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        geo, alpha = ctx.geo, ctx.alpha
        wv = ctx.w_arg if ctx.w_arg.is_contiguous() else w     # the Parameter itself where possible
        gx = ConvDgrad.apply(gy, wv, geo, alpha) if ctx.needs_input_grad[0] else None
        gw = gb = None
        if ctx.needs_input_grad[1] and wanted(ctx.w_arg):
            tgt = flat_grad(ctx.w_arg)
            if tgt is not None:
                _conv_wgrad(geo, x, _c(gy), alpha=alpha, out=tgt, accumulate=True)
            else:
                gw = ConvWgrad.apply(x, gy, geo, alpha)
        if ctx.has_bias and ctx.needs_input_grad[2] and wanted(ctx.b_arg):
            tgt = flat_grad(ctx.b_arg)
            if tgt is not None:
                row_sum_acc(gy, tgt)
            else:
                gb = gy.sum(dim=(1, 2, 3))
        return gx, gw, gb, None, None


class ConvDgrad(Function):
    """gx = alpha * conv^T(gy, w)."""

    @staticmethod
    def forward(ctx, gy, w, geo, alpha):
        ctx.w_arg = w
        gy, w = _c(gy), _c(w)
        ctx.save_for_backward(gy, w)
        ctx.geo, ctx.alpha = geo, alpha
        return _conv_dgrad(geo, gy, w, alpha=alpha)

    @staticmethod
    def backward(ctx, ggx):
        gy, w = ctx.saved_tensors
        geo, alpha = ctx.geo, ctx.alpha
        g_gy = ConvFwd.apply(ggx, w, None, geo, alpha) if ctx.needs_input_grad[0] else None
        g_w = None
        if ctx.needs_input_grad[1] and wanted(ctx.w_arg):
            tgt = flat_grad(ctx.w_arg)
            if tgt is not None:
                _conv_wgrad(geo, _c(ggx), gy, alpha=alpha, out=tgt, accumulate=True)
            else:
                g_w = ConvWgrad.apply(ggx, gy, geo, alpha)
        return g_gy, g_w, None, None


class ConvWgrad(Function):
    """gw = alpha * d<gy, conv(x, w)>/dw."""

    @staticmethod
    def forward(ctx, x, gy, geo, alpha):
        x, gy = _c(x), _c(gy)
        ctx.save_for_backward(x, gy)
        ctx.geo, ctx.alpha = geo, alpha
        return _conv_wgrad(geo, x, gy, alpha=alpha)

    @staticmethod
    def backward(ctx, ggw):
        x, gy = ctx.saved_tensors
        geo, alpha = ctx.geo, ctx.alpha
        g_x = ConvDgrad.apply(gy, ggw, geo, alpha) if ctx.needs_input_grad[0] else None
        g_gy = ConvFwd.apply(x, ggw, None, geo, alpha) if ctx.needs_input_grad[1] else None
        return g_x, g_gy, None, None


def conv2d(x, w, bias, geo: Geo, alpha: float):
    return ConvFwd.apply(x, w, bias, geo, alpha)


def linear(x, w, bias, alpha: float, out=None):
    """EqualizedLinear on [Cin, B] -> [Cout, B] (a 1x1 conv at H = W = 1).  ``out`` (no autograd
    only): a contiguous [Cout, B] destination, e.g. one slice of a stacked buffer."""
    cin, B = x.shape
    cout = w.shape[0]
    geo = linear_geo(B, cin, cout)
    if out is not None:
        if torch.is_grad_enabled():
            raise _lib.GanAmdError("linear(out=...) is a no-grad form")
        _conv_fwd(geo, _c(x), w.reshape(cout, cin, 1, 1), bias, None, None, alpha, out=out)
        return out
    return ConvFwd.apply(x.reshape(cin, B, 1, 1), w.reshape(cout, cin, 1, 1), bias, geo, alpha).reshape(cout, B)


# ------------------------------------------------------------------------------------------
# PReLU (twice differentiable)
# ------------------------------------------------------------------------------------------


def _rows(x):
    C = x.shape[0]
    return C, x.numel() // C


class PReLU(Function):
    @staticmethod
    def forward(ctx, x, a):
        ctx.a_arg = a
        x = _c(x)
        C, L = _rows(x)
        _need(a, C, "prelu alpha")
        y = torch.empty_like(x)
        check(LIB.ganamd_prelu_fwd(ptr(x), ptr(a), C, L, ptr(y), stream()), "prelu_fwd")
        ctx.save_for_backward(x, a)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, a = ctx.saved_tensors
        tgt = flat_grad(ctx.a_arg) if ctx.needs_input_grad[1] else None
        if tgt is not None:   # first order: the slope gradient goes straight into the flat buffer
            C, L = _rows(x)
            gx = torch.empty_like(x)
            ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device)
            check(LIB.ganamd_prelu_bwd(ptr(_c(gy)), ptr(x), ptr(a), C, L, ptr(gx), ptr(tgt), 1, *wsarg(ws), stream()),
                  "prelu_bwd")
            return gx, None
        av = ctx.a_arg if ctx.a_arg.is_contiguous() else a
        if ctx.needs_input_grad[1] and wanted(ctx.a_arg):
            gx, ga = PReLUBackward.apply(gy, x, av)
            return gx, ga
        return PReLUBackwardX.apply(gy, x, av), None


class PReLUBackward(Function):
    @staticmethod
    def forward(ctx, gy, x, a):
        ctx.a_arg = a
        gy = _c(gy)
        C, L = _rows(x)
        gx = torch.empty_like(x)
        ga = torch.empty_like(a)
        ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device)
        check(LIB.ganamd_prelu_bwd(ptr(gy), ptr(x), ptr(a), C, L, ptr(gx), ptr(ga), 0, *wsarg(ws), stream()),
              "prelu_bwd")
        ctx.save_for_backward(gy, x, a)
        return gx, ga

    @staticmethod
    @once_differentiable
    def backward(ctx, ggx, gga):
        gy, x, a = ctx.saved_tensors
        C, L = _rows(x)
        ggx = None if ggx is None else _c(ggx)
        gga = None if gga is None else _c(gga)
        need_gy, need_x, need_a = ctx.needs_input_grad
        g_gy = torch.empty_like(x) if need_gy else None
        g_x = torch.empty_like(x) if (need_x and gga is not None) else None
        tgt = flat_grad(ctx.a_arg) if need_a else None     # (once_differentiable: first order here)
        g_a = torch.empty_like(a) if need_a else None
        if g_gy is None and g_x is None and g_a is None:
            return None, None, None
        ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device)
        check(LIB.ganamd_prelu_bwd_bwd(ptr(ggx), ptr(gga), ptr(gy), ptr(x), ptr(a), C, L, ptr(g_gy), ptr(g_x),
                                       ptr(g_a), *wsarg(ws), stream()), "prelu_bwd_bwd")
        if tgt is not None:
            tgt.add_(g_a)          # one tiny add; the kernel has no accumulate form
            g_a = None
        return g_gy, g_x, g_a


class PReLUBackwardX(Function):
    """gx of PReLU alone (the slope gradient is not wanted, see ``wanted``); differentiable in
    gy (the same op) and in the slope (prelu_bwd_bwd), its x-derivative is 0 almost everywhere."""

    @staticmethod
    def forward(ctx, gy, x, a):
        ctx.a_arg = a
        gy = _c(gy)
        C, L = _rows(x)
        gx = torch.empty_like(x)
        check(LIB.ganamd_prelu_bwd(ptr(gy), ptr(x), ptr(a), C, L, ptr(gx), None, 0, None, 0, stream()), "prelu_bwd")
        ctx.save_for_backward(gy, x, a)
        return gx

    @staticmethod
    def backward(ctx, ggx):
        gy, x, a = ctx.saved_tensors
        need_gy, need_x, need_a = ctx.needs_input_grad
        g_gy = PReLUBackwardX.apply(ggx, x, ctx.a_arg) if need_gy else None
        g_a = None
        if need_a and wanted(ctx.a_arg):
            C, L = _rows(x)
            g_a = torch.empty_like(a)
            tgt = flat_grad(ctx.a_arg)
            ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device)
            check(LIB.ganamd_prelu_bwd_bwd(ptr(_c(ggx)), None, ptr(gy), ptr(x), ptr(a), C, L, None, None, ptr(g_a),
                                           *wsarg(ws), stream()), "prelu_bwd_bwd")
            if tgt is not None:
                tgt.add_(g_a)
                g_a = None
        return g_gy, None, g_a


def prelu(x, a):
    return PReLU.apply(x, a)


# ------------------------------------------------------------------------------------------
# BatchNorm (train mode) fused with an optional PReLU -- generator only (first order)
# ------------------------------------------------------------------------------------------


class BNAct(Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, alpha, running_mean, running_var, momentum, eps):
        if BN_SEGMENTS[0] > 1:
            raise _lib.GanAmdError("BNAct under bn_segments: use bn_act (the segmented no-grad forward)")
        x = _c(x)
        C, L = _rows(x)
        for t, nm in ((gamma, "gamma"), (beta, "beta"), (alpha, "alpha"), (running_mean, "running_mean"),
                      (running_var, "running_var")):
            _need(t, C, f"bn_act {nm}")
        y = torch.empty_like(x)
        mean = torch.empty(C, device=x.device, dtype=torch.float32)
        invstd = torch.empty_like(mean)
        ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device)
        check(LIB.ganamd_bn_act_fwd(ptr(x), C, L, ptr(gamma), ptr(beta), ptr(alpha), ptr(running_mean),
                                    ptr(running_var), float(momentum), float(eps), ptr(y), ptr(mean), ptr(invstd),
                                    *wsarg(ws), stream()), "bn_act_fwd")
        ctx.save_for_backward(x, gamma, beta, alpha, mean, invstd)
        ctx.has_alpha = alpha is not None
        ctx.args = (gamma, beta, alpha)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        x, gamma, beta, alpha, mean, invstd = ctx.saved_tensors
        gy = _c(gy)
        C, L = _rows(x)
        gx = torch.empty_like(x)
        # parameter gradients straight into the flat buffer when all of them live there
        tg = [flat_grad(a) if (a is not None and ctx.needs_input_grad[1 + i]) else None
              for i, a in enumerate(ctx.args)]
        direct = tg[0] is not None and tg[1] is not None and (not ctx.has_alpha or tg[2] is not None)
        if direct:
            gg, gb, ga = tg
        else:
            gg = torch.empty_like(gamma)
            gb = torch.empty_like(beta)
            ga = torch.empty_like(alpha) if ctx.has_alpha else None
        ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device)
        check(LIB.ganamd_bn_act_bwd(ptr(gy), ptr(x), C, L, ptr(gamma), ptr(beta), ptr(alpha), ptr(mean), ptr(invstd),
                                    ptr(gx), ptr(gg), ptr(gb), ptr(ga), int(direct), *wsarg(ws), stream()), "bn_act_bwd")
        if direct:
            return gx, None, None, None, None, None, None, None
        return gx, gg, gb, ga, None, None, None, None


# Segmented BatchNorm (no-grad forwards only): the batch is BN_SEGMENTS[0] independent mini-batches
# stacked along it, each normalised by its own statistics (ganamd_bn_act_fwd_seg) -- one generator
# forward makes the fake batches of all n_critic critic steps (wgangp.Train.generate_fakes).
BN_SEGMENTS = [1]


@contextlib.contextmanager
def bn_segments(n: int):
    old = BN_SEGMENTS[0]
    BN_SEGMENTS[0] = int(n)
    try:
        yield
    finally:
        BN_SEGMENTS[0] = old


def bn_fwd_raw(x, C, L, gamma, beta, alpha, running_mean, running_var, momentum, eps):
    """Train-mode BatchNorm (+ PReLU) forward of [C][L] rows; honours BN_SEGMENTS.  Returns
    (y, save_mean, save_invstd) -- per (channel, segment) statistics when segmented."""
    seg = BN_SEGMENTS[0]
    if seg > 1 and torch.is_grad_enabled():
        raise _lib.GanAmdError("segmented BatchNorm is a no-grad forward")
    if L % seg:
        raise _lib.GanAmdError(f"BatchNorm: {L} elements per channel do not split into {seg} segments")
    y = torch.empty_like(x)
    mean = torch.empty(C * seg, device=x.device, dtype=torch.float32)
    invstd = torch.empty_like(mean)
    uvar = torch.empty_like(mean) if seg > 1 else None
    ws = workspace(LIB.ganamd_rowreduce_workspace(C * seg, L // seg), x.device)
    check(LIB.ganamd_bn_act_fwd_seg(ptr(x), C, L, seg, ptr(gamma), ptr(beta), ptr(alpha), ptr(running_mean),
                                    ptr(running_var), float(momentum), float(eps), ptr(y), ptr(mean), ptr(invstd),
                                    ptr(uvar), *wsarg(ws), stream()), "bn_act_fwd_seg")
    return y, mean, invstd


def linear_bn_act_ok(x, w) -> bool:
    """Whether ``linear_bn_act`` takes this linear: no autograd, fp32 math (bf16 mode keeps its bf16
    linears), an unsegmented batch, [Cin, B] with 2 <= B <= 64 and at most 4 M weights
    (ganamd_linear_bn_act's domain)."""
    return (not torch.is_grad_enabled() and _MATH[0] == _lib.MATH_F32 and BN_SEGMENTS[0] == 1 and x.dim() == 2
            and 2 <= x.shape[1] <= 64 and w.shape[0] * w.shape[1] <= (4 << 20))


def linear_bn_act(x, w, bias, alpha: float, bn, act=None):
    """``act(bn(linear(x)))`` in train mode as ONE kernel (no-grad forward only, see linear_bn_act_ok):
    the linear's epilogue computes each row's batch statistics (ganamd_linear_bn_act)."""
    cin, B = x.shape
    cout = w.shape[0]
    geo = linear_geo(B, cin, cout)
    x = _c(x)
    for t, n, nm in ((bias, cout, "bias"), (bn.weight, cout, "gamma"), (bn.bias, cout, "beta"),
                     (bn.running_mean, cout, "running_mean"), (bn.running_var, cout, "running_var"),
                     (None if act is None else act.weight, cout, "prelu alpha")):
        _need(t, n, f"linear_bn_act {nm}")
    FlopCounter.add(geo, "fwd", False, False)
    y = torch.empty((cout, B), device=x.device, dtype=torch.float32)
    wv = w.reshape(cout, cin, 1, 1)
    pw = PackCache.get(geo, _lib.CONV_FWD, wv)
    packed = pw is not None
    nb = geo.ws_bytes(_lib.CONV_FWD, packed)
    ws = workspace(nb, x.device) if (nb and not packed) else None
    check(LIB.ganamd_linear_bn_act(geo.desc(packed), ptr(x), ptr(pw if packed else wv), ptr(bias), float(alpha),
                                   ptr(bn.weight), ptr(bn.bias), ptr(None if act is None else act.weight),
                                   ptr(bn.running_mean), ptr(bn.running_var), float(bn.momentum), float(bn.eps),
                                   ptr(y), *wsarg(ws), stream()), "linear_bn_act")
    return y


def bn_act(x, bn: torch.nn.modules.batchnorm._BatchNorm, act: torch.nn.PReLU | None = None):
    """Train-mode ``act(bn(x))`` with the module's parameters and running buffers."""
    if BN_SEGMENTS[0] > 1:
        x = _c(x)
        C, L = _rows(x)
        return bn_fwd_raw(x, C, L, bn.weight, bn.bias, None if act is None else act.weight, bn.running_mean,
                          bn.running_var, bn.momentum, bn.eps)[0]
    return BNAct.apply(x, bn.weight, bn.bias, None if act is None else act.weight, bn.running_mean, bn.running_var,
                       bn.momentum, bn.eps)


# ------------------------------------------------------------------------------------------
# separable resampling (linear; its backward is the same kernel with the adjoint table)
# ------------------------------------------------------------------------------------------


def _resample(x, n_in, n_out, tab):
    idx, w, k = tab
    C, B = x.shape[0], x.shape[1]
    if x.dim() != 4 or x.shape[2] != n_in or x.shape[3] != n_in or idx.shape[0] != n_out:
        raise _lib.GanAmdError(f"resample: input {tuple(x.shape)} vs table {n_in}->{n_out}")
    y = torch.empty((C, B, n_out, n_out), device=x.device, dtype=torch.float32)
    check(LIB.ganamd_resample2d(ptr(x), C * B, n_in, n_in, ptr(y), n_out, n_out, iptr(idx), ptr(w), k, iptr(idx),
                                ptr(w), k, stream()), "resample2d")
    return y


class Resample(Function):
    @staticmethod
    def forward(ctx, x, table, adjoint):
        ctx.table, ctx.adjoint = table, adjoint
        if adjoint:
            return _resample(_c(x), table.n_out, table.n_in, table.adj)
        return _resample(_c(x), table.n_in, table.n_out, table.fwd)

    @staticmethod
    def backward(ctx, gy):
        return Resample.apply(gy, ctx.table, not ctx.adjoint), None, None


def resample(x, kind: str):
    return Resample.apply(x, tables.table(kind, x.shape[2], x.device), False)


def resample_sum(x1, x2, kind: str):
    """``resample(x1 + x2, kind)`` without materialising the sum (no autograd: the sum is formed
    while the kernel stages its input planes, ganamd_resample2d_sum)."""
    if torch.is_grad_enabled():
        raise _lib.GanAmdError("resample_sum is a no-grad form")
    x1, x2 = _c(x1), _c(x2)
    if x1.shape != x2.shape:
        raise _lib.GanAmdError(f"resample_sum: {tuple(x1.shape)} vs {tuple(x2.shape)}")
    t = tables.table(kind, x1.shape[2], x1.device)
    idx, w, k = t.fwd
    C, B, n_in = x1.shape[0], x1.shape[1], t.n_in
    if x1.dim() != 4 or x1.shape[2] != n_in or x1.shape[3] != n_in:
        raise _lib.GanAmdError(f"resample_sum: input {tuple(x1.shape)} vs table {n_in}->{t.n_out}")
    y = torch.empty((C, B, t.n_out, t.n_out), device=x1.device, dtype=torch.float32)
    check(LIB.ganamd_resample2d_sum(ptr(x1), ptr(x2), C * B, n_in, n_in, ptr(y), t.n_out, t.n_out, iptr(idx), ptr(w),
                                    k, iptr(idx), ptr(w), k, stream()), "resample2d_sum")
    return y


class PoolSumFanout(Function):
    """(t, f0', f1') = (R(f0 + f1), f0, f1): SK attention's pool of the branch sum
    (generator_13_5.py:82-84) with the branches passed through as aliases for the mixing that
    follows.  Forward: one resample of the sum formed while staging (ganamd_resample2d_sum) -- the sum
    is never stored.  Backward: each branch's gradient = R^T(g_t) + its mixing gradient, both written
    by ONE launch (ganamd_resample2d_add) -- instead of an R^T(g_t) tensor plus one add per branch."""

    @staticmethod
    def forward(ctx, f0, f1, table):
        ctx.set_materialize_grads(False)
        ctx.table, ctx.shape = table, f0.shape
        idx, w, k = table.fwd
        f0, f1 = _c(f0), _c(f1)
        C, B = f0.shape[0], f0.shape[1]
        t = torch.empty((C, B, table.n_out, table.n_out), device=f0.device, dtype=torch.float32)
        check(LIB.ganamd_resample2d_sum(ptr(f0), ptr(f1), C * B, table.n_in, table.n_in, ptr(t), table.n_out,
                                        table.n_out, iptr(idx), ptr(w), k, iptr(idx), ptr(w), k, stream()),
              "resample2d_sum")
        return t, f0.view_as(f0), f1.view_as(f1)

    @staticmethod
    @once_differentiable
    def backward(ctx, gt, g0, g1):
        if gt is None:
            return g0, g1, None
        tab = ctx.table
        idx, w, k = tab.adj
        C, B = ctx.shape[0], ctx.shape[1]
        y0 = torch.empty(ctx.shape, device=gt.device, dtype=torch.float32)
        y1 = torch.empty_like(y0)
        check(LIB.ganamd_resample2d_add(ptr(_c(gt)), C * B, tab.n_out, tab.n_out, ptr(y0), tab.n_in, tab.n_in,
                                        iptr(idx), ptr(w), k, iptr(idx), ptr(w), k,
                                        ptr(None if g0 is None else _c(g0)), ptr(y1),
                                        ptr(None if g1 is None else _c(g1)), stream()), "resample2d_add")
        return y0, y1, None


def pool_sum_fanout(f0, f1, kind: str):
    """(resample(f0 + f1, kind), f0, f1) with the fused backward of PoolSumFanout (autograd form of
    resample_sum for two branches that are also used elsewhere)."""
    if f0.shape != f1.shape or f0.dim() != 4 or f0.shape[2] != f0.shape[3]:
        raise _lib.GanAmdError(f"pool_sum_fanout: {tuple(f0.shape)} vs {tuple(f1.shape)}")
    return PoolSumFanout.apply(f0, f1, tables.table(kind, f0.shape[2], f0.device))


# ------------------------------------------------------------------------------------------
# per-plane mean (AdaptiveAvgPool2d(1)) -> [C, B]
# ------------------------------------------------------------------------------------------


class PlaneMean(Function):
    @staticmethod
    def forward(ctx, x):
        x = _c(x)
        C, B, H, W = x.shape
        out = torch.empty((C, B), device=x.device, dtype=torch.float32)
        check(LIB.ganamd_plane_dot(ptr(x), None, C * B, H * W, 1.0 / (H * W), ptr(out), stream()), "plane_dot")
        ctx.hw = (H, W)
        return out

    @staticmethod
    def backward(ctx, g):
        H, W = ctx.hw
        return (g / (H * W))[:, :, None, None].expand(-1, -1, H, W)


def plane_mean(x):
    if x.shape[2] == 1 and x.shape[3] == 1:
        return x.reshape(x.shape[0], x.shape[1])
    return PlaneMean.apply(x)


def plane_dot(a, b, scale=1.0):
    a, b = _c(a), _c(b)
    C, B, H, W = a.shape
    out = torch.empty((C, B), device=a.device, dtype=torch.float32)
    check(LIB.ganamd_plane_dot(ptr(a), ptr(b), C * B, H * W, float(scale), ptr(out), stream()), "plane_dot")
    return out


def plane_dot_pair(a, b1, b2):
    """(<a, b1>, <a, b2>) per plane in one pass over a (ganamd_plane_dot_pair), or None when the
    planes do not suit its 16-byte loads (the caller then takes two plane_dot launches)."""
    a, b1, b2 = _c(a), _c(b1), _c(b2)
    C, B, H, W = a.shape
    if (H * W) % 4 or any(t.data_ptr() % 16 for t in (a, b1, b2)):
        return None
    o1 = torch.empty((C, B), device=a.device, dtype=torch.float32)
    o2 = torch.empty_like(o1)
    check(LIB.ganamd_plane_dot_pair(ptr(a), ptr(b1), ptr(b2), C * B, H * W, ptr(o1), ptr(o2), stream()),
          "plane_dot_pair")
    return o1, o2


# ------------------------------------------------------------------------------------------
# weight-modulated conv (StyleGAN2 demodulation) -- generator only
# ------------------------------------------------------------------------------------------


class ModConv(Function):
    """y[co,b] = c * d[co,b] * conv(x * s[ci,b], W)   (generator_13_5.py:234-248, batch-shared form).

    ``d`` is an input (computed by ``demod`` with differentiable ops) so that autograd carries
    its gradient back into s and W.
    """

    @staticmethod
    def forward(ctx, x, s, d, w, geo, c, noise_scale=None, noise=None):
        """``noise_scale``/``noise``: the StyleConv noise term ``+ noise_scale[co] * noise`` fused in
        the GEMM epilogue (generator_13_5.py:265); its gradients come from one plane reduction."""
        ctx.w_arg = w
        x, s, d, w = _c(x), _c(s), _c(d), _c(w)
        if noise is None:
            y = _conv_fwd(geo, x, w, None, s, d, c)
            ctx.save_for_backward(x, s, d, w, y)
        else:
            noise = _c(noise)
            y = _conv_fwd_ex(geo, x, w, s, d, c, noise, _c(noise_scale))
            ctx.save_for_backward(x, s, d, w, y, noise_scale, noise)
        ctx.geo, ctx.c, ctx.noisy = geo, c, noise is not None
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        if ctx.noisy:
            x, s, d, w, y, ns, noise = ctx.saved_tensors
        else:
            (x, s, d, w, y), ns, noise = ctx.saved_tensors, None, None
        geo, c = ctx.geo, ctx.c
        gy = _c(gy)
        gx = gs = gd = gw = gns = None
        want_d, want_ns = ctx.needs_input_grad[2], noise is not None and ctx.needs_input_grad[6]
        if want_d or want_ns:
            # dL/dd = <gy, conv> = (<gy, y> - ns <gy, noise>) / d and the noise scale's gradient
            # sum_b <gy, noise> (into the flat buffer when it has one): one pass (modconv_sd_bwd)
            tgt = flat_grad(ns) if want_ns else None
            r = modconv_sd_bwd(gy, y, noise, d, ns, tgt)
            if r is not None:
                gd, pdn = r
                if want_ns and tgt is None:
                    gns = pdn.sum(1)
            else:                                            # unaligned planes: plane dots
                pdn = plane_dot(gy, noise) if noise is not None else None
                if want_ns:
                    gns = pdn.sum(1)
                pdy = plane_dot(gy, y)
                if pdn is not None:
                    pdy = pdy - ns[:, None] * pdn
                gd = pdy / d
            if not want_d:
                gd = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            gxs = _conv_dgrad(geo, gy, w, d, c)             # d/d(x*s)
            # one pass: gx = gxs * s, gs = <gxs, x> per plane (ganamd_mix_bwd with M = 1)
            gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
            gs = torch.empty_like(s) if ctx.needs_input_grad[1] else None
            P, HW = _planes(x)
            check(LIB.ganamd_mix_bwd(1, ptr(x), None, None, None, ptr(s), P, HW, ptr(gxs), ptr(gx), None, None, None,
                                     ptr(gs), stream()), "mix_bwd")
        if ctx.needs_input_grad[3]:
            tgt = flat_grad(ctx.w_arg)
            if tgt is not None:
                _conv_wgrad(geo, x, gy, s, d, c, out=tgt, accumulate=True)
            else:
                gw = _conv_wgrad(geo, x, gy, s, d, c)
        return gx, gs, gd, gw, None, None, gns, None


def modconv_sd_bwd(gy, y, noise, d, ns, gns_acc=None):
    """(gd, pdn) of the modulated conv (ganamd_modconv_sd_bwd): gd = dL/dd [C, B], pdn = <gy, noise>
    per plane (None without noise); ``gns_acc`` [C] (optional) += sum_b pdn.  None when the planes do
    not suit the kernel's 16-byte loads."""
    C, B, H, W = gy.shape
    if (H * W) % 4 or any(t is not None and t.data_ptr() % 16 for t in (gy, y, noise)):
        return None
    gd = torch.empty((C, B), device=gy.device, dtype=torch.float32)
    pdn = torch.empty_like(gd) if noise is not None else None
    check(LIB.ganamd_modconv_sd_bwd(ptr(gy), ptr(_c(y)), ptr(None if noise is None else _c(noise)), ptr(_c(d)),
                                    ptr(None if ns is None else _c(ns)), C, B, H * W, ptr(gd), ptr(pdn),
                                    ptr(gns_acc), stream()), "modconv_sd_bwd")
    return gd, pdn


def demod(s, w, c, eps=1e-8):
    """d[co,b] = rsqrt(c^2 * sum_ci s[ci,b]^2 * sum_k W[co,ci,k]^2 + eps)."""
    wsq = w.pow(2).sum(dim=(2, 3))                       # [Cout, Cin]
    return torch.rsqrt((c * c) * (wsq @ (s * s)) + eps)  # [Cout, B]


def modconv(x, s, w, geo, c):
    return ModConv.apply(x, s, demod(s, w, c), w, geo, c)


# ------------------------------------------------------------------------------------------
# gradient penalty on the critic's input gradient (csrc/fused.hip)
# ------------------------------------------------------------------------------------------


class GradPenalty(Function):
    """lambda * mean_b (||g_b|| - center)^2 (mode 0: WGAN-GP, train/wgangp.py:34-54) or
    lambda * mean_b ||g_b||^2 (mode 1: R1/R2, train/wganlazygpR2.py:57-70) of g = grad_x D [B, ...].
    The penalty and its gradient w.r.t. g come from two fused kernels (ganamd_gp_fwd/_bwd) in
    closed form; the double backward then continues through the critic's backward operators."""

    @staticmethod
    def forward(ctx, g, center, lam, mode):
        g = _c(g)
        B = g.shape[0]
        n = g.numel() // B
        norms = torch.empty(B, device=g.device, dtype=torch.float32)
        out = torch.empty((), device=g.device, dtype=torch.float32)
        ws = workspace(LIB.ganamd_gp_workspace(B, n), g.device)
        check(LIB.ganamd_gp_fwd(ptr(g), B, n, float(center), float(lam), int(mode), ptr(norms), ptr(out), *wsarg(ws),
                                stream()), "gp_fwd")
        ctx.save_for_backward(g, norms)
        ctx.args = (B, n, float(center), float(lam), int(mode))
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, gout):
        g, norms = ctx.saved_tensors
        B, n, center, lam, mode = ctx.args
        dg = torch.empty_like(g)
        check(LIB.ganamd_gp_bwd(ptr(g), ptr(norms), ptr(_c(gout.reshape(1))), B, n, center, lam, mode, ptr(dg),
                                stream()), "gp_bwd")
        return dg, None, None, None


def grad_penalty(g, center=1.0, lam=1.0, mode=0):
    return GradPenalty.apply(g, center, lam, mode)


# ------------------------------------------------------------------------------------------
# fused per-plane elementwise ops (csrc/fused.hip)
# ------------------------------------------------------------------------------------------


def _planes(x):
    C, B = x.shape[0], x.shape[1]
    return C * B, x.numel() // (C * B)


def _scale_rows(x, s, r=None):
    x, s = _c(x), _c(s)
    P, HW = _planes(x)
    _need(s, P, "scale_rows s")
    _need(r, x.numel(), "scale_add r")
    y = torch.empty_like(x)
    check(LIB.ganamd_scale_add(ptr(x), ptr(s), ptr(None if r is None else _c(r)), P, HW, ptr(y), stream()),
          "scale_add")
    return y


class ScaleRows(Function):
    """y[c,b,:] = x[c,b,:] * s[c,b]   (any order of derivative, with PlaneDot)."""

    @staticmethod
    def forward(ctx, x, s):
        ctx.save_for_backward(x, s)
        return _scale_rows(x, s)

    @staticmethod
    def backward(ctx, g):
        x, s = ctx.saved_tensors
        gx = ScaleRows.apply(g, s) if ctx.needs_input_grad[0] else None
        gs = PlaneDot.apply(g, x) if ctx.needs_input_grad[1] else None
        return gx, gs


class PlaneDot(Function):
    """z[c,b] = sum_hw a[c,b,:] * b[c,b,:]   (any order of derivative, with ScaleRows)."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return plane_dot(a, b)

    @staticmethod
    def backward(ctx, gz):
        a, b = ctx.saved_tensors
        ga = ScaleRows.apply(b, gz) if ctx.needs_input_grad[0] else None
        gb = ScaleRows.apply(a, gz) if ctx.needs_input_grad[1] else None
        return ga, gb


class ScaleAdd(Function):
    """y = r + x * s[c,b]: the SE-gated residual of both networks (generator_13_5.py:455-466,
    discriminator_9_4.py:158-161); differentiable to any order (the critic's GP)."""

    @staticmethod
    def forward(ctx, x, s, r):
        ctx.save_for_backward(x, s)
        return _scale_rows(x, s, r)

    @staticmethod
    def backward(ctx, g):
        x, s = ctx.saved_tensors
        gx = ScaleRows.apply(g, s) if ctx.needs_input_grad[0] else None
        gs = PlaneDot.apply(g, x) if ctx.needs_input_grad[1] else None
        return gx, gs, g


def scale_add(x, s, r):
    return ScaleAdd.apply(x, s, r)


class Mix(Function):
    """y = sum_m att[m] * f_m   (selective-kernel mixing; generator only, first order)."""

    @staticmethod
    def forward(ctx, att, *feas):
        feas = [_c(f) for f in feas]
        att = _c(att)
        M = len(feas)
        P, HW = _planes(feas[0])
        _need(att, M * P, "mix att")
        y = torch.empty_like(feas[0])
        fp = [ptr(f) for f in feas] + [None] * (4 - M)
        check(LIB.ganamd_mix_fwd(M, *fp, ptr(att), P, HW, ptr(y), stream()), "mix_fwd")
        ctx.save_for_backward(att, *feas)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        att, *feas = ctx.saved_tensors
        gy = _c(gy)
        M = len(feas)
        P, HW = _planes(feas[0])
        gfs = [torch.empty_like(f) if ctx.needs_input_grad[1 + i] else None for i, f in enumerate(feas)]
        gatt = torch.empty_like(att) if ctx.needs_input_grad[0] else None
        fp = [ptr(f) for f in feas] + [None] * (4 - M)
        gp = [ptr(g) for g in gfs] + [None] * (4 - M)
        check(LIB.ganamd_mix_bwd(M, *fp, ptr(att), P, HW, ptr(gy), *gp, ptr(gatt), stream()), "mix_bwd")
        return (gatt, *gfs)


def mix(feas, att):
    """feas: M tensors [C,B,H,W]; att: [M,C,B]."""
    return Mix.apply(att, *feas)


class AddPReLU(Function):
    """y = PReLU(a + b)   (generator only, first order)."""

    @staticmethod
    def forward(ctx, a, b, alpha):
        ctx.alpha_arg = alpha
        a, b = _c(a), _c(b)
        C, L = _rows(a)
        _need(alpha, C, "add_prelu alpha")
        y = torch.empty_like(a)
        check(LIB.ganamd_add_prelu(ptr(a), ptr(b), ptr(alpha), C, L, ptr(y), stream()), "add_prelu")
        ctx.save_for_backward(a, b, alpha)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, gy):
        a, b, alpha = ctx.saved_tensors
        z = a + b
        C, L = _rows(z)
        gz = torch.empty_like(z)
        tgt = flat_grad(ctx.alpha_arg) if ctx.needs_input_grad[2] else None
        ga = tgt if tgt is not None else torch.empty_like(alpha)
        ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), z.device)
        check(LIB.ganamd_prelu_bwd(ptr(_c(gy)), ptr(z), ptr(alpha), C, L, ptr(gz), ptr(ga), int(tgt is not None),
                                   *wsarg(ws), stream()), "prelu_bwd")
        return gz, gz, (None if tgt is not None else ga)


def add_prelu(a, b, alpha):
    return AddPReLU.apply(a, b, alpha)


class Route(Function):
    """Channel-range views x[lo:hi] of a CNHW tensor (each contiguous), one per use.  The backward
    writes x's gradient in ONE pass (ganamd_route_bwd: each row the sum of the views covering it, in
    view order; 0 where none does) -- autograd's own slice backward makes a zero-filled full-size
    tensor per view and then adds them (the dual-path blocks of generator_13_5.py:448-467, 496-564
    take 3-5 views of every block input).  Generator only, first order."""

    @staticmethod
    def forward(ctx, x, bounds):
        ctx.set_materialize_grads(False)
        ctx.bounds, ctx.shape = bounds, x.shape
        return tuple(x[lo:hi] for lo, hi in bounds)

    @staticmethod
    @once_differentiable
    def backward(ctx, *gs):
        import ctypes
        C = ctx.shape[0]
        L = 1
        for s in ctx.shape[1:]:
            L *= s
        parts = [(_c(g), lo, hi) for g, (lo, hi) in zip(gs, ctx.bounds) if g is not None and hi > lo]
        if not parts:
            return None, None
        gx = torch.empty(ctx.shape, device=parts[0][0].device, dtype=torch.float32)
        n = len(parts)
        arr = (ctypes.c_void_p * n)(*[ptr(g) for g, _, _ in parts])
        lo = (ctypes.c_int32 * n)(*[lo for _, lo, _ in parts])
        hi = (ctypes.c_int32 * n)(*[hi for _, _, hi in parts])
        check(LIB.ganamd_route_bwd(n, arr, lo, hi, C, L, ptr(gx), stream()), "route_bwd")
        return gx, None


def route(x, bounds):
    """``[x[lo:hi] for lo, hi in bounds]`` with a one-pass backward (Route); at most
    GANAMD_ROUTE_MAX views.  Without autograd it is plain slicing."""
    if len(bounds) > _lib.ROUTE_MAX:
        raise _lib.GanAmdError(f"route: {len(bounds)} views > {_lib.ROUTE_MAX}")
    bounds = tuple((int(lo), int(hi)) for lo, hi in bounds)
    if not (torch.is_grad_enabled() and x.requires_grad):
        return tuple(x[lo:hi] for lo, hi in bounds)
    return Route.apply(x, bounds)


def modconv_fused(x, s, d, w, geo, c, noise=None, noise_scale=None, act=None):
    """No-grad modulated conv with the StyleConv noise and the following PReLU in the GEMM
    epilogue (ganamd_conv_fwd_ex): y = PReLU(c*d*conv(x*s, W) + noise_scale*noise)."""
    x, s, d = _c(x), _c(s), _c(d)
    _need(d, geo.Cout * geo.B, "conv_fwd y_scale")
    _need(x, geo.Cin * geo.B * geo.H * geo.W, "conv_fwd x")
    _need(s, geo.Cin * geo.B, "conv_fwd x_scale")
    _need(noise, geo.Cout * geo.B * geo.OH * geo.OW, "conv_fwd noise")
    _need(noise_scale, geo.Cout if noise is not None else None, "conv_fwd noise_scale")
    _need(act, geo.Cout, "conv_fwd act")
    return _conv_fwd_ex(geo, x, w, s, d, c, noise, noise_scale, act)


def _conv_fwd_ex(geo, x, w, xs, ys, alpha, noise=None, noise_scale=None, act=None):
    FlopCounter.add(geo, "fwd", xs is not None, ys is not None)
    y = torch.empty((geo.Cout, geo.B, geo.OH, geo.OW), device=x.device, dtype=torch.float32)
    pw = PackCache.get(geo, _lib.CONV_FWD, w)
    packed = pw is not None
    nb = geo.ws_bytes(_lib.CONV_FWD, packed)
    ws = workspace(nb, x.device) if nb else None
    check(LIB.ganamd_conv_fwd_ex(geo.desc(packed), ptr(x), ptr(pw if packed else _c(w)), None, ptr(xs), ptr(ys),
                                 float(alpha), ptr(None if noise is None else _c(noise)), ptr(noise_scale),
                                 ptr(act), ptr(y), *wsarg(ws), stream()), "conv_fwd_ex")
    return y


# ------------------------------------------------------------------------------------------
# layout helpers at the module boundary
# ------------------------------------------------------------------------------------------


class _SwapNC(Function):
    """Contiguous [N,C,H,W] <-> [C,N,H,W] swap whose gradient is again contiguous (callers of the
    reference view input gradients, e.g. ``grad.view(B, -1)`` at wgangp.py:53)."""

    @staticmethod
    def forward(ctx, x):
        return x.permute(1, 0, 2, 3).contiguous()

    @staticmethod
    def backward(ctx, g):
        return _SwapNC.apply(g)


def nchw_to_cnhw(x):
    return _SwapNC.apply(x)


def cnhw_to_nchw(x):
    return _SwapNC.apply(x)


# ------------------------------------------------------------------------------------------
# pointwise activations and BCE (the vanilla pair of config 1: generator_1.py, discriminator_1.py,
# train/gan.py)
# ------------------------------------------------------------------------------------------


class Act(Function):
    """Sigmoid / Tanh / LeakyReLU(slope) over a contiguous tensor (csrc/act.hip).  The backward
    reads the forward OUTPUT for sigmoid / tanh and the forward INPUT for leaky."""

    @staticmethod
    def forward(ctx, x, kind, slope):
        x = _c(x)
        y = torch.empty_like(x)
        check(LIB.ganamd_act_fwd(int(kind), ptr(x), x.numel(), float(slope), ptr(y), stream()), "act_fwd")
        ctx.save_for_backward(x if kind == _lib.ACT_LEAKY else y)
        ctx.kind, ctx.slope = int(kind), float(slope)
        return y

    @staticmethod
    def backward(ctx, gy):
        (v,) = ctx.saved_tensors
        gy = _c(gy)
        gx = torch.empty_like(v)
        check(LIB.ganamd_act_bwd(ctx.kind, ptr(v), ptr(gy), v.numel(), ctx.slope, ptr(gx), stream()), "act_bwd")
        return gx, None, None


def sigmoid(x):
    return Act.apply(x, _lib.ACT_SIGMOID, 0.0)


def tanh(x):
    return Act.apply(x, _lib.ACT_TANH, 0.0)


def leaky_relu(x, slope):
    return Act.apply(x, _lib.ACT_LEAKY, slope)


class BCELoss(Function):
    """torch.nn.BCELoss() (mean reduction, logs clamped at -100) of probabilities p against
    targets (train/gan.py:21); the gradient reaches p only (targets are constants there)."""

    @staticmethod
    def forward(ctx, p, target):
        p, target = _c(p), _c(target)
        if p.shape != target.shape:
            raise ValueError(f"BCELoss: input {tuple(p.shape)} vs target {tuple(target.shape)}")
        out = torch.empty((), device=p.device, dtype=torch.float32)
        check(LIB.ganamd_bce_fwd(ptr(p), ptr(target), p.numel(), ptr(out), stream()), "bce_fwd")
        ctx.save_for_backward(p, target)
        return out

    @staticmethod
    def backward(ctx, gout):
        p, target = ctx.saved_tensors
        gout = _c(gout.reshape(1))
        gp = torch.empty_like(p)
        check(LIB.ganamd_bce_bwd(ptr(p), ptr(target), p.numel(), ptr(gout), ptr(gp), stream()), "bce_bwd")
        return gp, None


def bce_loss(p, target):
    return BCELoss.apply(p, target)


class SoftmaxM(Function):
    """softmax over the M branch axis of x[M][P] (the SK attention heads, generator_13_5.py:88,131:
    softmax(dim=1) of [B, M, C, 1, 1]); backward gx = y (gy - <y, gy>_M)."""

    @staticmethod
    def forward(ctx, x):
        x = _c(x)
        M = x.shape[0]
        y = torch.empty_like(x)
        check(LIB.ganamd_softmax_m(M, ptr(x), x.numel() // M, ptr(y), stream()), "softmax_m")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        gy = _c(gy)
        M = y.shape[0]
        gx = torch.empty_like(y)
        check(LIB.ganamd_softmax_m_bwd(M, ptr(y), ptr(gy), y.numel() // M, ptr(gx), stream()), "softmax_m_bwd")
        return gx


def softmax_m(x):
    return SoftmaxM.apply(x)


# ------------------------------------------------------------------------------------------
# independent branches on their own HIP streams
# ------------------------------------------------------------------------------------------

BRANCH_STREAMS = [os.environ.get("GANAMD_BRANCHES", "1") != "0"]   # A/B: GANAMD_BRANCHES=0 runs branches inline
_STREAM_POOL: dict = {}


class Branches:
    """``with Branches(dev, n) as br: with br[i]: ...`` -- each branch body runs on its own pooled
    HIP stream, forked from the current stream on entry and joined back into it on exit (a captured
    graph gets parallel branches).  Tensors a branch allocates are consumed on the current stream
    only after the join, and every later branch forks after that consumer, so the caching allocator
    never hands a branch's memory to work that could overlap its readers.

    Branch sets do not nest: inside a branch a further set runs inline.  (A nested set would need
    streams of its own per enclosing branch -- one shared pool per nesting depth, as an earlier
    build had, makes sibling branches fork and join through the same inner streams, serialising
    them and letting the allocator recycle one sibling's inner blocks while the other still reads
    them; the k3/k5 split inside the parallel StyleBlocks also measured slower, 37.9 vs 39.8
    img/s.)  On the CPU, or with BRANCH_STREAMS[0] False, the bodies run inline.

    Current-stream tensors the branches read must be passed to ``share`` (or ``branch_share``):
    the branches' backward nodes release them from their own streams."""

    _depth = [0]

    def __init__(self, device, n):
        dev = torch.device(device)
        self.on = BRANCH_STREAMS[0] and dev.type == "cuda" and n > 1 and Branches._depth[0] == 0
        self.n = n
        if self.on:
            key = dev.index if dev.index is not None else torch.cuda.current_device()
            pool = _STREAM_POOL.setdefault(key, [])
            while len(pool) < n:
                pool.append(torch.cuda.Stream(device=dev))
            self.streams = pool[:n]

    def __enter__(self):
        if self.on:
            Branches._depth[0] += 1
            self.main = torch.cuda.current_stream()
            for s in self.streams:
                s.wait_stream(self.main)
        return self

    def __exit__(self, *exc):
        if self.on:
            Branches._depth[0] -= 1
            for s in self.streams:
                self.main.wait_stream(s)
        return False

    def __getitem__(self, i):
        return torch.cuda.stream(self.streams[i]) if self.on else contextlib.nullcontext()

    def share(self, *tensors):
        """Tensors made on the current stream that the branches read: see ``branch_share``."""
        if self.on:
            _record(tensors, self.streams)

    def out(self, i, t):
        """Branch ``i``'s output ``t``: its gradient is made on the current stream (the consumer's
        backward) and read by branch ``i``'s backward on ``i``'s stream, which releases it when the
        read is ISSUED -- so the gradient is recorded on that stream (a hook on ``t``), or the caching
        allocator could hand its block to current-stream work while the branch's weight gradient
        still reads it (measured: four conv3 weight gradients of the 64x64 StyleBlocks differing
        between two runs of the same generator step, none with the branches inline)."""
        if self.on and t.requires_grad:
            s = self.streams[i]
            t.register_hook(lambda g, s=s: _record((g,), (s,)))
        return t


def _record(tensors, streams):
    for t in tensors:
        if t is not None and t.is_cuda:
            for s in streams:
                t.record_stream(s)


def branch_share(*tensors):
    """Mark current-stream tensors that branch-stream work reads -- in the forward, or in the
    backward through a branch op's saved tensors -- as used by every pooled branch stream.

    The backward of a branch op runs on that branch's stream (autograd keeps the forward's stream)
    and releases its saved tensors when it has been ISSUED, not when its kernels have run: without
    this, a block allocated on the main stream (a branch's input, a view of the forward's bulk noise
    draw) could be handed by the caching allocator to a main-stream kernel while a branch kernel still
    reads it -- a race whose outcome depends on timing (under graph capture: a missing edge in the
    graph).  With the streams recorded, the allocator reuses such a block only after the branch
    streams' work queued at the free has finished (during a capture: after the capture)."""
    if not BRANCH_STREAMS[0]:
        return
    for t in tensors:
        if t is not None and t.is_cuda:
            pool = _STREAM_POOL.get(t.device.index if t.device.index is not None else torch.cuda.current_device())
            if pool:
                _record((t,), pool)
