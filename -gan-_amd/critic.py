"""The critic as an explicit program: forward, first-order backward and the gradient penalty's
double backward as kernel sequences over saved activations -- no autograd graph.

Reference: the critic step's gradient penalty (train/wgangp.py:34-54, 68-69) differentiates the
critic's input gradient ``g = grad_x sum D(x_hat)`` with ``autograd.grad(create_graph=True)`` and
then ``backward()``; autograd materialises the graph of the backward and walks it.  Here the
same derivative is computed by four explicit sweeps over the layer program of D9_4
(discriminators/discriminator_9_4.py:163-199), each a sequence of libganamd.so kernels:

  forward   x_v  for every value v of the program (saved)
  backward  g_v  = d sum(D)/d x_v  (seed 1 at the output)          -> g = g_input
  penalty   P(g) and v = dP/dg  (ganamd_gp_fwd / _bwd)
  tangent   xd_v = directional derivative of x_v along v            (forward-mode, seed xd_in = v)
  adjoint   a_v  = d h / d x_v for h(theta) = <v, g(theta)> (+ sum_b w_b D_b when first-order
            loss weights w are folded in), reverse sweep with the second-order terms:
              conv      a_in += W^T a_out;  dW += wgrad(x_in, a_out) + wgrad(xd_in, g_out)
              PReLU     a_in  = a_out * prelu'(x);  dalpha += sum a_out*min(x,0) + sum g_out*xd[x<=0]
              sigmoid   a_in  = a_out s(1-s) + g_out xd s(1-s)(1-2s)
              x*s + r   a_x = a_out s + g_out sd;  a_s = <a_out, x> + <g_out, xd>;  a_r = a_out
              MiniBatchStdDev: ganamd_mbstd_adjoint (the cross-sample second-order term)
  dP/dtheta = dh/dtheta, accumulated straight into the parameters' gradient buffers.

The FLOPs are those of the reference's double backward (one forward, one input-gradient
backward, one tangent forward, one adjoint backward and two weight-gradient GEMMs per conv), but
nothing is taped at run time beyond the saved activations, no per-layer autograd nodes run, and
dead work (weight gradients inside ``autograd.grad``) is never issued.

Entry points:
  * ``critic_forward(D, x, segments)`` -- the drop-in ``Discriminator.forward``: one autograd
    node (``_CriticFn``) whose backward is the explicit backward sweep and is itself
    differentiable (``_CriticGrad``: its backward is the tangent + adjoint sweeps), so the
    reference's ``autograd.grad(..., create_graph=True)`` + ``backward()`` protocol still works.
  * ``gradient_penalty(D, x_hat, center, lam, mode)`` -- what ``Train.gradient_penalty`` calls:
    forward, backward, fused penalty; ``.backward()`` on the result runs tangent + adjoint.
  * ``regularised_step(D, x, segments, loss_w, specs)`` -- the lazy-GP trainer's critic step
    (real/fake losses + R1/R2/GP on three segments) in one pass of each sweep.
"""
from __future__ import annotations

import torch
from torch import nn
from torch.autograd import Function

from . import _lib, ops, tables
from ._lib import LIB, check, ptr, stream, workspace

# ------------------------------------------------------------------------------------------
# program
# ------------------------------------------------------------------------------------------


class Op:
    __slots__ = ("kind", "ins", "out", "mod", "arg")

    def __init__(self, kind, ins, out, mod=None, arg=None):
        self.kind, self.ins, self.out, self.mod, self.arg = kind, ins, out, mod, arg


class Program:
    """Straight-line layer program of a critic: values are integers, value 0 is the NCHW input."""

    def __init__(self):
        self.ops: list[Op] = []
        self.n = 1
        self.out = 0
        self.params: list[nn.Parameter] = []

    def op(self, kind, ins, mod=None, arg=None):
        o = self.n
        self.n += 1
        self.ops.append(Op(kind, list(ins), o, mod, arg))
        return o


def _d94_se(P, m, y):
    from .discriminator_9_4 import SEBlock_conv
    if isinstance(m, SEBlock_conv):        # discriminator_9_4.py:83-109 (pool5, 5->3->1 convs)
        c = m.convs
        t = P.op("resample", [y], arg="pool5")
        t = P.op("prelu", [P.op("conv", [t], c[0])], c[1])
        t = P.op("prelu", [P.op("conv", [t], c[2])], c[3])
        z = P.op("pmean", [t])
        z = P.op("prelu", [P.op("linear", [z], m.fcs[0])], m.fcs[1])
    else:                                  # discriminator_9_4.py:111-128
        f = m.fcs
        z = P.op("pmean", [y])
        z = P.op("prelu", [P.op("linear", [z], f[0])], f[1])
        z = P.op("prelu", [P.op("linear", [z], f[2])], f[3])
    return P.op("sigmoid", [P.op("linear", [z], m.fc_out)])


def _d94_block(P, m, x):
    """DiscriminatorBlock.forward (discriminator_9_4.py:147-161)."""
    if m.downsample:
        r = P.op("conv", [P.op("resample", [x], arg="smooth_down2")], m.residual[1])
    else:
        r = x
    b = m.block
    y = P.op("prelu", [P.op("conv", [x], b[0])], b[1])
    y = P.op("prelu", [P.op("conv", [y], b[2])], b[3])
    if m.downsample:
        d = m.down_sample
        y = P.op("prelu", [P.op("conv", [P.op("resample", [y], arg="smooth")], d[1])], d[2])
    s = _d94_se(P, m.se, y)
    return P.op("scale_add", [y, s, r])


def build_d94(D) -> Program:
    """The layer program of D9_4 (Discriminator.forward, discriminator_9_4.py:195-199)."""
    from .discriminator_9_4 import DiscriminatorBlock, EqualizedConv2d, MiniBatchStdDev
    P = Program()
    v = P.op("swap", [0])
    for mod in D.conv:
        if isinstance(mod, EqualizedConv2d):
            v = P.op("conv", [v], mod)
        elif isinstance(mod, nn.PReLU):
            v = P.op("prelu", [v], mod)
        elif isinstance(mod, DiscriminatorBlock):
            v = _d94_block(P, mod, v)
        elif isinstance(mod, MiniBatchStdDev):
            v = P.op("mbstd", [v], mod)
        else:
            raise TypeError(type(mod))
    v = P.op("flatten", [v])
    v = P.op("prelu", [P.op("linear", [v], D.fc[0])], D.fc[1])
    P.out = P.op("linear", [v], D.fc[2])
    P.params = list(D.parameters())
    return P


def program_of(D) -> Program:
    prog = D.__dict__.get("_critic_program")
    if prog is None:
        prog = build_d94(D)
        D.__dict__["_critic_program"] = prog
    return prog


# ------------------------------------------------------------------------------------------
# kernels of one op (thin wrappers; all launch on torch's current stream)
# ------------------------------------------------------------------------------------------


def _conv_parts(mod):
    """(weight, bias, alpha, k, stride, pad) of an EqualizedConv2d / EqualizedLinear."""
    w = mod.weight.weight
    return w, mod.bias, mod.weight.c


def _geo(op, x):
    m = op.mod
    if op.kind == "linear":
        cin, B = x.shape
        return ops.linear_geo(B, cin, m.weight.weight.shape[0])
    C, B, H, W = x.shape
    return ops.conv_geo(B, C, H, W, m.bias.shape[0], m.k, m.stride, m.padding)


def _w4(op):
    w = op.mod.weight.weight
    return w if w.dim() == 4 else w.view(w.shape[0], w.shape[1], 1, 1)


def _as4(op, t, geo, out=False):
    if op.kind != "linear":
        return t
    c = geo.Cout if out else geo.Cin
    return t.view(c, geo.B, 1, 1)


def _as2(op, t):
    return t.view(t.shape[0], t.shape[1]) if op.kind == "linear" else t


def _rows(t):
    return t.shape[0], t.numel() // t.shape[0]


def _planes(t):
    return t.shape[0] * t.shape[1], t.numel() // (t.shape[0] * t.shape[1])


def _grad_buf(p):
    """p.grad, created as zeros when absent (engine sweeps accumulate into it)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    g = p.grad
    if not g.is_contiguous():
        raise _lib.GanAmdError("critic engine: parameter gradients must be contiguous")
    return g


def _prelu_fwd(x, a):
    C, L = _rows(x)
    y = torch.empty_like(x)
    check(LIB.ganamd_prelu_fwd(ptr(x), ptr(a), C, L, ptr(y), stream()), "prelu_fwd")
    return y


def _prelu_bwd(gy, x, a, galpha):
    C, L = _rows(x)
    gx = torch.empty_like(x)
    ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device) if galpha is not None else None
    check(LIB.ganamd_prelu_bwd(ptr(gy), ptr(x), ptr(a), C, L, ptr(gx), ptr(galpha), 1, ptr(ws), stream()),
          "prelu_bwd")
    return gx


def _prelu_tangent(xd, gy, x, a, galpha):
    C, L = _rows(x)
    yd = torch.empty_like(x)
    ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device) if galpha is not None else None
    check(LIB.ganamd_prelu_tangent(ptr(xd), ptr(gy), ptr(x), ptr(a), C, L, ptr(yd), ptr(galpha), 1, ptr(ws),
                                   stream()), "prelu_tangent")
    return yd


def _resample(x, kind):
    tab = tables.table(kind, x.shape[2], x.device)
    return ops._resample(x, tab.n_in, tab.n_out, tab.fwd)


def _resample_adj(gy, kind, n_in):
    """adjoint (backward) of resampler ``kind`` whose forward input was n_in x n_in"""
    tab = tables.table(kind, n_in, gy.device)
    return ops._resample(gy, tab.n_out, tab.n_in, tab.adj)


def _pmean(x):
    C, B, H, W = x.shape
    if H * W == 1:
        return x.reshape(C, B)
    out = torch.empty((C, B), device=x.device, dtype=torch.float32)
    check(LIB.ganamd_plane_dot(ptr(x), None, C * B, H * W, 1.0 / (H * W), ptr(out), stream()), "plane_dot")
    return out


def _pmean_adj(g, shape):
    C, B, H, W = shape
    if H * W == 1:
        return g.reshape(C, B, 1, 1)
    return (g * (1.0 / (H * W))).reshape(C, B, 1, 1).expand(C, B, H, W).contiguous()


def _act(kind, x):
    y = torch.empty_like(x)
    check(LIB.ganamd_act_fwd(kind, ptr(x), x.numel(), 0.0, ptr(y), stream()), "act_fwd")
    return y


def _act_bwd(kind, v, gy):
    gx = torch.empty_like(v)
    check(LIB.ganamd_act_bwd(kind, ptr(v), ptr(gy), v.numel(), 0.0, ptr(gx), stream()), "act_bwd")
    return gx


def _act_adjoint(kind, v, ay, gy, xd):
    ax = torch.empty_like(v)
    check(LIB.ganamd_act_adjoint(kind, ptr(v), ptr(ay), ptr(gy), ptr(xd), v.numel(), 0.0, ptr(ax), stream()),
          "act_adjoint")
    return ax


def _scale_add2(x1, s1, x2=None, s2=None, r=None):
    P, HW = _planes(x1)
    y = torch.empty_like(x1)
    check(LIB.ganamd_scale_add2(ptr(x1), ptr(s1), ptr(x2), ptr(s2), ptr(r), P, HW, ptr(y), stream()), "scale_add2")
    return y


def _plane_dot2(a1, b1, a2=None, b2=None):
    P, HW = _planes(a1)
    out = torch.empty(a1.shape[:2], device=a1.device, dtype=torch.float32)
    check(LIB.ganamd_plane_dot2(ptr(a1), ptr(b1), ptr(a2), ptr(b2), P, HW, ptr(out), stream()), "plane_dot2")
    return out


def _axpy(x, y, a=1.0):
    check(LIB.ganamd_axpy(y.numel(), float(a), ptr(x), ptr(y), stream()), "axpy")


def _swap(x):
    return x.permute(1, 0, 2, 3).contiguous()


def _flatten(x):
    """[C,B,H,W] -> [(c,h,w), B]: the NCHW .view(B, -1) feature order of discriminator_9_4.py:197."""
    C, B, H, W = x.shape
    return x.permute(0, 2, 3, 1).reshape(C * H * W, B).contiguous()


def _unflatten(z, shape):
    C, B, H, W = shape
    return z.view(C, H, W, B).permute(0, 3, 1, 2).contiguous()


# ------------------------------------------------------------------------------------------
# one run of the program on one input batch
# ------------------------------------------------------------------------------------------


class Run:
    """Saved activations (X), first-order gradients (G), tangents (XD) and adjoints (A) of one
    critic evaluation, and the sweeps over them."""

    def __init__(self, prog: Program, segments: int = 1):
        self.prog = prog
        self.segments = segments
        self.X: dict = {}
        self.G: dict = {}
        self.XD: dict = {}
        self.borrowed: set = set()

    # ---------------------------------------------------------------- forward
    def forward(self, x_nchw):
        X = self.X
        X[0] = x_nchw
        for op in self.prog.ops:
            X[op.out] = self._fwd(op, [X[i] for i in op.ins])
        return X[self.prog.out]

    def _fwd(self, op, xs):
        k = op.kind
        x = xs[0]
        if k == "swap":
            return _swap(x)
        if k in ("conv", "linear"):
            geo = _geo(op, x)
            w, b, c = _conv_parts(op.mod)
            y = ops._conv_fwd(geo, _as4(op, x, geo), _w4(op), b, alpha=c)
            return _as2(op, y)
        if k == "prelu":
            return _prelu_fwd(x, op.mod.weight)
        if k == "resample":
            return _resample(x, op.arg)
        if k == "pmean":
            return _pmean(x)
        if k == "sigmoid":
            return _act(_lib.ACT_SIGMOID, x)
        if k == "scale_add":
            return _scale_add2(xs[0], xs[1], r=xs[2])
        if k == "mbstd":
            C, B, H, W = x.shape
            y = torch.empty((C + 1, B, H, W), device=x.device, dtype=torch.float32)
            ws = workspace(LIB.ganamd_mbstd_workspace(self.segments), x.device)
            check(LIB.ganamd_mbstd_fwd(ptr(x), B * H * W, C, B, H * W, self.segments, 4, ptr(y), B * H * W, None,
                                       ptr(ws), stream()), "mbstd_fwd")
            return y
        if k == "flatten":
            return _flatten(x)
        raise _lib.GanAmdError(f"unknown critic op {k}")

    # ---------------------------------------------------------------- accumulation
    def _acc(self, D, v, t, borrowed=False):
        """D[v] += t.  A tensor that is also another value's gradient (an identity pass-through)
        is held 'borrowed' and never written in place."""
        if v not in D:
            D[v] = t
            if borrowed:
                self.borrowed.add((id(D), v))
            return
        key = (id(D), v)
        if key in self.borrowed:
            if borrowed:        # both borrowed: materialise a sum
                s = t.clone()
                _axpy(D[v], s)
                D[v] = s
            else:
                _axpy(D[v], t)  # t is fresh: add the borrowed one into it
                D[v] = t
            self.borrowed.discard(key)
            return
        _axpy(t, D[v])

    # ---------------------------------------------------------------- first-order backward
    def backward(self, seed, params: bool, need_input: bool):
        """g_v for every value from g_out = seed; parameter gradients accumulated into .grad when
        ``params``; the input gradient (NCHW) returned when ``need_input``."""
        G = self.G
        G.clear()
        self.borrowed.clear()
        G[self.prog.out] = seed
        X = self.X
        for op in reversed(self.prog.ops):
            gy = G.get(op.out)
            if gy is None:
                continue
            k = op.kind
            x = X[op.ins[0]]
            first = op.ins[0] == 1 and k in ("conv",)   # the stem conv reads the swapped input
            if k == "swap":
                if need_input:
                    G[0] = _swap(gy)
            elif k in ("conv", "linear"):
                geo = _geo(op, x)
                w, b, c = _conv_parts(op.mod)
                if not first or need_input:
                    gx = ops._conv_dgrad(geo, _as4(op, gy, geo, out=True), _w4(op), alpha=c)
                    self._acc(G, op.ins[0], _as2(op, gx))
                if params and w.requires_grad:
                    ops._conv_wgrad(geo, _as4(op, x, geo), _as4(op, gy, geo, out=True), alpha=c,
                                    out=_grad_buf(w), accumulate=True)
                    ops.row_sum_acc(gy, _grad_buf(b))
            elif k == "prelu":
                a = op.mod.weight
                self._acc(G, op.ins[0], _prelu_bwd(gy, x, a, _grad_buf(a) if params and a.requires_grad else None))
            elif k == "resample":
                self._acc(G, op.ins[0], _resample_adj(gy, op.arg, x.shape[2]))
            elif k == "pmean":
                self._acc(G, op.ins[0], _pmean_adj(gy, x.shape), borrowed=x.shape[2] * x.shape[3] == 1)
            elif k == "sigmoid":
                self._acc(G, op.ins[0], _act_bwd(_lib.ACT_SIGMOID, X[op.out], gy))
            elif k == "scale_add":
                xv, s, r = op.ins
                self._acc(G, xv, _scale_add2(gy, X[s]))
                self._acc(G, s, _plane_dot2(gy, X[xv]))
                self._acc(G, r, gy, borrowed=True)
            elif k == "mbstd":
                C, B, H, W = x.shape
                gx = torch.empty_like(x)
                ws = workspace(LIB.ganamd_mbstd_workspace(self.segments), x.device)
                check(LIB.ganamd_mbstd_bwd(ptr(x), B * H * W, ptr(gy), B * H * W, C, B, H * W, self.segments, 4,
                                           ptr(gx), ptr(ws), stream()), "mbstd_bwd")
                self._acc(G, op.ins[0], gx)
            elif k == "flatten":
                self._acc(G, op.ins[0], _unflatten(gy, x.shape))
        return G.get(0)

    # ---------------------------------------------------------------- tangent (forward-mode)
    def tangent(self, v_nchw, params: bool):
        """xd_v along the input direction v; the PReLU slopes' second-order term (needs G)
        accumulates into their gradients when ``params``."""
        XD, X, G = self.XD, self.X, self.G
        XD.clear()
        XD[0] = v_nchw
        for op in self.prog.ops:
            k = op.kind
            xd = XD[op.ins[0]]
            x = X[op.ins[0]]
            if k == "swap":
                XD[op.out] = _swap(xd)
            elif k in ("conv", "linear"):
                geo = _geo(op, x)
                w, b, c = _conv_parts(op.mod)
                XD[op.out] = _as2(op, ops._conv_fwd(geo, _as4(op, xd, geo), _w4(op), None, alpha=c))
            elif k == "prelu":
                a = op.mod.weight
                XD[op.out] = _prelu_tangent(xd, G[op.out], x, a, _grad_buf(a) if params and a.requires_grad else None)
            elif k == "resample":
                XD[op.out] = _resample(xd, op.arg)
            elif k == "pmean":
                XD[op.out] = _pmean(xd)
            elif k == "sigmoid":
                XD[op.out] = _act_bwd(_lib.ACT_SIGMOID, X[op.out], xd)
            elif k == "scale_add":
                xv, s, r = op.ins
                XD[op.out] = _scale_add2(XD[xv], X[s], X[xv], XD[s], XD[r])
            elif k == "mbstd":
                C, B, H, W = x.shape
                yd = torch.empty((C + 1, B, H, W), device=x.device, dtype=torch.float32)
                ws = workspace(LIB.ganamd_mbstd_workspace(self.segments), x.device)
                check(LIB.ganamd_mbstd_tangent(ptr(x), ptr(xd), B * H * W, C, B, H * W, self.segments, 4, ptr(yd),
                                               B * H * W, ptr(ws), stream()), "mbstd_tangent")
                XD[op.out] = yd
            elif k == "flatten":
                XD[op.out] = _flatten(xd)
        return XD[self.prog.out]

    # ---------------------------------------------------------------- adjoint (second-order reverse)
    def adjoint(self, a_seed, params: bool, need_input: bool = False):
        """Reverse sweep of h = <v, g> (+ <a_seed, D(x)>): accumulates dh/dtheta into the
        parameters' gradients; returns dh/dx (NCHW) when ``need_input``.  a_seed may be None
        (pure penalty)."""
        A: dict = {}
        X, G, XD = self.X, self.G, self.XD
        self.borrowed.clear()
        if a_seed is not None:
            A[self.prog.out] = a_seed
        for op in reversed(self.prog.ops):
            k = op.kind
            ay = A.pop(op.out, None)
            gy = G.get(op.out)
            x = X[op.ins[0]]
            if k == "swap":
                if need_input and ay is not None:
                    A[0] = _swap(ay)
            elif k in ("conv", "linear"):
                geo = _geo(op, x)
                w, b, c = _conv_parts(op.mod)
                first = op.ins[0] == 1
                if ay is not None and (not first or need_input):
                    gx = ops._conv_dgrad(geo, _as4(op, ay, geo, out=True), _w4(op), alpha=c)
                    self._acc(A, op.ins[0], _as2(op, gx))
                if params and w.requires_grad:
                    gw = _grad_buf(w)
                    if ay is not None:
                        ops._conv_wgrad(geo, _as4(op, x, geo), _as4(op, ay, geo, out=True), alpha=c, out=gw,
                                        accumulate=True)
                        ops.row_sum_acc(ay, _grad_buf(b))
                    if gy is not None:
                        ops._conv_wgrad(geo, _as4(op, XD[op.ins[0]], geo), _as4(op, gy, geo, out=True), alpha=c,
                                        out=gw, accumulate=True)
            elif k == "prelu":
                if ay is not None:
                    a = op.mod.weight
                    self._acc(A, op.ins[0],
                              _prelu_bwd(ay, x, a, _grad_buf(a) if params and a.requires_grad else None))
            elif k == "resample":
                if ay is not None:
                    self._acc(A, op.ins[0], _resample_adj(ay, op.arg, x.shape[2]))
            elif k == "pmean":
                if ay is not None:
                    self._acc(A, op.ins[0], _pmean_adj(ay, x.shape), borrowed=x.shape[2] * x.shape[3] == 1)
            elif k == "sigmoid":
                if ay is None:
                    ay = torch.zeros_like(x)
                self._acc(A, op.ins[0], _act_adjoint(_lib.ACT_SIGMOID, X[op.out], ay, gy, XD[op.ins[0]]))
            elif k == "scale_add":
                xv, s, r = op.ins
                if ay is None:
                    self._acc(A, xv, _scale_add2(gy, XD[s]))
                    self._acc(A, s, _plane_dot2(gy, XD[xv]))
                else:
                    self._acc(A, xv, _scale_add2(ay, X[s], gy, XD[s]))
                    self._acc(A, s, _plane_dot2(ay, X[xv], gy, XD[xv]))
                    self._acc(A, r, ay, borrowed=True)
            elif k == "mbstd":
                C, B, H, W = x.shape
                if ay is None:
                    ay = torch.zeros_like(gy)
                ax = torch.empty_like(x)
                ws = workspace(LIB.ganamd_mbstd_workspace(self.segments), x.device)
                check(LIB.ganamd_mbstd_adjoint(ptr(x), ptr(XD[op.ins[0]]), B * H * W, ptr(gy), ptr(ay), B * H * W, C,
                                               B, H * W, self.segments, 4, ptr(ax), ptr(ws), stream()),
                      "mbstd_adjoint")
                self._acc(A, op.ins[0], ax)
            elif k == "flatten":
                if ay is not None:
                    self._acc(A, op.ins[0], _unflatten(ay, x.shape))
        return A.get(0)


# ------------------------------------------------------------------------------------------
# the penalty on the input gradient
# ------------------------------------------------------------------------------------------


def _penalty(g, center, lam, mode):
    """(value, norms) of lam * mean_b (||g_b|| - center)^2 (mode 0) / lam * mean_b ||g_b||^2 (mode 1)."""
    B = g.shape[0]
    n = g.numel() // B
    norms = torch.empty(B, device=g.device, dtype=torch.float32)
    out = torch.empty((), device=g.device, dtype=torch.float32)
    ws = workspace(LIB.ganamd_gp_workspace(B, n), g.device)
    check(LIB.ganamd_gp_fwd(ptr(g), B, n, float(center), float(lam), int(mode), ptr(norms), ptr(out), ptr(ws),
                            stream()), "gp_fwd")
    return out, norms


def _penalty_grad(g, norms, gout, center, lam, mode, out=None):
    B = g.shape[0]
    n = g.numel() // B
    dg = out if out is not None else torch.empty_like(g)
    check(LIB.ganamd_gp_bwd(ptr(g), ptr(norms), ptr(gout), B, n, float(center), float(lam), int(mode), ptr(dg),
                            stream()), "gp_bwd")
    return dg


def _params_wanted(params):
    return any(ops.wanted(p) for p in params)


# ------------------------------------------------------------------------------------------
# autograd surface
# ------------------------------------------------------------------------------------------


class _CriticFn(Function):
    """D(x) as one autograd node.  backward = the explicit backward sweep; it is differentiable
    (create_graph) through _CriticGrad."""

    @staticmethod
    def forward(ctx, x, run, *params):
        ctx.run = run
        ctx.n_params = len(params)
        ctx.params = params
        out = run.forward(x.detach().contiguous())
        return out.t()                                       # [1, B] -> [B, 1]

    @staticmethod
    def backward(ctx, gout):
        run = ctx.run
        seed = gout.t().contiguous()
        want_p = any(ctx.needs_input_grad[2:]) and _params_wanted(ctx.params)
        if torch.is_grad_enabled():                          # create_graph: keep it differentiable
            gx = _CriticGrad.apply(seed, run, want_p, *ctx.params)
            return (gx, None) + (None,) * ctx.n_params
        gx = run.backward(seed, params=want_p, need_input=ctx.needs_input_grad[0])
        return (gx, None) + (None,) * ctx.n_params


class _CriticGrad(Function):
    """g = dD/dx (for the seed); its backward, given v = dR/dg, is the tangent + adjoint sweeps
    (parameter gradients accumulated into .grad)."""

    @staticmethod
    def forward(ctx, seed, run, first_order_params, *params):
        ctx.run, ctx.params = run, params
        gx = run.backward(seed, params=first_order_params, need_input=True)
        run.G.pop(0, None)     # the run must not hold this node's output (ctx -> run -> output cycle)
        return gx

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, v):
        run = ctx.run
        want_p = _params_wanted(ctx.params)
        run.tangent(v.contiguous(), params=want_p)
        run.adjoint(None, params=want_p)
        return (None, None, None) + (None,) * len(ctx.params)


def critic_forward(D, x, segments: int = 1):
    """The drop-in Discriminator.forward: [B,3,64,64] -> [B,1] through the explicit program."""
    prog = program_of(D)
    run = Run(prog, segments)
    params = [p for p in prog.params if p.requires_grad]
    if not torch.is_grad_enabled() or not (x.requires_grad or params):
        with torch.no_grad():
            return run.forward(x.detach().contiguous()).t()
    return _CriticFn.apply(x, run, *params)


class _PenaltyFn(Function):
    """The penalty value; its backward (scaled by the incoming gradient) is the tangent +
    adjoint sweeps of the run."""

    @staticmethod
    def forward(ctx, anchor, run, g, center, lam, mode):
        value, norms = _penalty(g, center, lam, mode)
        ctx.run, ctx.g, ctx.norms, ctx.args = run, g, norms, (center, lam, mode)
        ctx.anchor_param = anchor
        return value

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gout):
        run = ctx.run
        center, lam, mode = ctx.args
        v = _penalty_grad(ctx.g, ctx.norms, gout.reshape(1).contiguous(), center, lam, mode)
        want_p = ops.wanted(ctx.anchor_param)
        run.tangent(v, params=want_p)
        run.adjoint(None, params=want_p)
        return (None,) * 6


def gradient_penalty(D, x_hat, center=1.0, lam=1.0, mode=0):
    """lam * mean_b (||grad_x sum D(x_hat)||_b - center)^2 (train/wgangp.py:34-54) -- or, mode 1,
    lam * mean_b ||.||^2 (R1/R2) -- with forward, input-gradient backward and the fused penalty
    run now; ``.backward()`` on the result runs the double backward (tangent + adjoint sweeps)."""
    prog = program_of(D)
    run = Run(prog, 1)
    x_hat = x_hat.detach().contiguous()
    run.forward(x_hat)
    B = x_hat.shape[0]
    seed = torch.ones((1, B), device=x_hat.device, dtype=torch.float32)
    g = run.backward(seed, params=False, need_input=True)
    params = [p for p in prog.params if p.requires_grad]
    if not params or not torch.is_grad_enabled():
        return _penalty(g, center, lam, mode)[0]
    return _PenaltyFn.apply(params[0], run, g, center, lam, mode)


def regularised_step(D, x, segments, loss_w, specs):
    """One pass of every sweep over a batch of ``segments`` equal segments (the lazy trainer's
    real / fake / interpolated batches, train/wganlazygpR2.py:48-77): returns (pred [N,1],
    penalties).  Objective: sum_b loss_w[b] * D(x)_b + sum_s penalty_s(grad_x of segment s),
    specs[s] = (center, lam, mode) or None.  Its gradient is accumulated into D's .grad."""
    prog = program_of(D)
    run = Run(prog, segments)
    x = x.detach().contiguous()
    pred = run.forward(x)                                     # [1, N]
    N = x.shape[0]
    Bs = N // segments
    seed = torch.ones((1, N), device=x.device, dtype=torch.float32)
    g = run.backward(seed, params=False, need_input=True)
    v = torch.zeros_like(g)
    one = torch.ones(1, device=x.device, dtype=torch.float32)
    vals = []
    for s, spec in enumerate(specs):
        if spec is None:
            vals.append(None)
            continue
        center, lam, mode = spec
        gs = g[s * Bs:(s + 1) * Bs]
        val, norms = _penalty(gs, center, lam, mode)
        _penalty_grad(gs, norms, one, center, lam, mode, out=v[s * Bs:(s + 1) * Bs])
        vals.append(val)
    run.tangent(v, params=True)
    run.adjoint(loss_w.reshape(1, N).contiguous(), params=True)
    return pred.t(), vals
