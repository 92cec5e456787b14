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

The sweeps run inside libganamd.so (csrc/critic.hip, the ganamd_critic_* C ABI; one
ganamd_critic_gp_step call is the whole GP double backward for a non-Python host, INTEGRATION.md
§4).  This module builds the program of a Discriminator, hands the engine its op table (weights,
GEMM-order packed copies from ops.PackCache, resampling tables) and one workspace per evaluation,
and puts the reference's autograd protocol on top.

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
from ._lib import ws as wsarg

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
# the op table of the C-ABI engine (include/ganamd.h "Critic program engine", csrc/critic.hip)
# ------------------------------------------------------------------------------------------


def _grad_buf(p):
    """p.grad, created as zeros when absent (engine sweeps accumulate into it)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    g = p.grad
    if not g.is_contiguous():
        raise _lib.GanAmdError("critic engine: parameter gradients must be contiguous")
    return g


def _w4(op):
    w = op.mod.weight.weight
    return w if w.dim() == 4 else w.view(w.shape[0], w.shape[1], 1, 1)


def _shapes(prog, C0, H0, W0):
    """(C, H, W) per value (value 0: the NCHW input), as ganamd_critic_create derives them."""
    sh = {0: (C0, H0, W0)}
    for op in prog.ops:
        C, H, W = sh[op.ins[0]]
        k = op.kind
        if k == "conv":
            m = op.mod
            sh[op.out] = (m.bias.shape[0], (H + 2 * m.padding - m.k) // m.stride + 1,
                          (W + 2 * m.padding - m.k) // m.stride + 1)
        elif k == "linear":
            sh[op.out] = (op.mod.weight.weight.shape[0], 1, 1)
        elif k == "resample":
            sh[op.out] = (C, tables.table(op.arg, H, "cpu").n_out, tables.table(op.arg, H, "cpu").n_out)
        elif k == "pmean":
            sh[op.out] = (C, 1, 1)
        elif k == "mbstd":
            sh[op.out] = (C + 1, H, W)
        elif k == "flatten":
            sh[op.out] = (C * H * W, 1, 1)
        else:
            sh[op.out] = (C, H, W)
    return sh


def _geo_of(op, B, shape_in):
    C, H, W = shape_in
    m = op.mod
    if op.kind == "linear":
        return ops.linear_geo(B, C, m.weight.weight.shape[0])
    return ops.conv_geo(B, C, H, W, m.bias.shape[0], m.k, m.stride, m.padding)


def _op_table(prog, B, sh, device, keep):
    """ctypes ganamd_critic_op[] of the program at batch B (packed weight copies from the cache)."""
    t = (_lib.CriticOp * len(prog.ops))()
    for i, op in enumerate(prog.ops):
        e = t[i]
        e.kind = _lib.COP["conv" if op.kind == "linear" else op.kind]
        ins = list(op.ins) + [-1] * (3 - len(op.ins))
        for j in range(3):
            e.ins[j] = ins[j]
        if op.kind in ("conv", "linear"):
            m = op.mod
            geo = _geo_of(op, B, sh[op.ins[0]])
            w = _w4(op)
            pf = ops.PackCache.get(geo, _lib.CONV_FWD, w)
            pd = ops.PackCache.get(geo, _lib.CONV_DGRAD, w)
            keep += [w, pf, pd, m.bias]
            e.cout, e.k, e.stride, e.pad, e.pad_mode = geo.Cout, geo.K, geo.stride, geo.pad, geo.pad_mode
            e.alpha = float(m.weight.c)
            e.w, e.w_fwd, e.w_dgrad, e.bias = ptr(w), ptr(pf), ptr(pd), ptr(m.bias)
        elif op.kind == "prelu":
            e.w = ptr(op.mod.weight)
            keep.append(op.mod.weight)
        elif op.kind == "resample":
            tab = tables.table(op.arg, sh[op.ins[0]][1], device)
            (fi, fw, fk), (ai, aw, ak) = tab.fwd, tab.adj
            keep.append(tab)
            e.n_out, e.kr, e.akr = tab.n_out, fk, ak
            e.ri, e.rw, e.ari, e.arw = _lib.iptr(fi), ptr(fw), _lib.iptr(ai), ptr(aw)
        elif op.kind == "mbstd":
            e.group = op.mod.group_size
    return t


# ------------------------------------------------------------------------------------------
# one run of the program on one input batch
# ------------------------------------------------------------------------------------------


class _Values:
    """Read access to one sweep's values (0 X, 1 G, 2 XD, 3 A) as views of the run's workspace."""

    def __init__(self, run, which):
        self.run, self.which = run, which

    def __getitem__(self, v):
        run = self.run
        p = _lib.ctypes.c_void_p()
        check(LIB.ganamd_critic_value(run.plan, self.which, int(v), _lib.ctypes.byref(p)), "critic_value")
        if not p.value:
            raise KeyError(v)
        if v == 0:
            return run.x if self.which == 0 else run.v
        C, H, W = run.sh[v]
        n = C * run.B * H * W
        for reg in run.regions:
            off = (p.value - reg.data_ptr()) // 4 if reg is not None else -1
            if 0 <= off and off + n <= reg.numel():
                t = reg[off:off + n]
                break
        else:
            raise _lib.GanAmdError(f"critic value {v} outside the run's workspace")
        # per-sample vectors (linear / pool / flatten outputs and activations of them) are [C, B];
        # maps (a 1x1 conv output included) [C, B, H, W]
        return t.view(C, run.B) if run.vec[v] else t.view(C, run.B, H, W)

    def get(self, v, default=None):
        try:
            return self[v]
        except KeyError:
            return default


class Run:
    """One critic evaluation through the C-ABI engine (ganamd_critic_*): the plan of the program
    at this batch, the workspace regions holding the saved activations (X), gradients (G),
    tangents (XD) and adjoints (A) -- each allocated when the sweep that fills it starts, so a
    first-order evaluation holds X and G only -- and the sweeps.  ``X`` / ``G`` / ``XD`` read
    values back (tests, tools)."""

    def __init__(self, prog: Program, segments: int = 1):
        self.prog = prog
        self.segments = segments
        self.plan = None
        self.regions = [None] * 4       # scratch + X, G, XD, A: allocated by the sweep that fills them
        self.keep = []
        self.x = self.v = None

    # read access to the values (views made on access: holding _Values objects here would make a
    # Run <-> _Values reference cycle, and a cycle keeps the run's workspace -- ~10 GiB at B = 64 --
    # alive until the cyclic GC happens to run: peak HBM then grew with every eager iteration)
    X = property(lambda self: _Values(self, 0))
    G = property(lambda self: _Values(self, 1))
    XD = property(lambda self: _Values(self, 2))

    def __del__(self):
        if self.plan:
            LIB.ganamd_critic_destroy(self.plan)
            self.plan = None

    def _setup(self, x):
        B, C, H, W = x.shape
        if self.plan:                   # a new evaluation on this Run: nothing of the old one is reused
            LIB.ganamd_critic_destroy(self.plan)
            self.plan = None
            self.regions = [None] * 4
            self.keep = []
        self.B = B
        self.sh = _shapes(self.prog, C, H, W)
        self.vec = {0: False}
        for op in self.prog.ops:
            self.vec[op.out] = op.kind in ("linear", "pmean", "flatten") or (
                op.kind in ("prelu", "sigmoid") and self.vec[op.ins[0]])
        self.table = _op_table(self.prog, B, self.sh, x.device, self.keep)
        self.plan = LIB.ganamd_critic_create(self.table, len(self.prog.ops), B, C, H, W, self.segments, ops._MATH[0],
                                             ops._KOFF[0])
        if not self.plan:
            raise _lib.GanAmdError(f"critic program rejected by ganamd_critic_create (B={B}, segments={self.segments})")
        self._region(0, x.device)

    def _region(self, which, device):
        """Allocate and bind workspace region ``which`` (ganamd_critic_region_bytes / _bind)."""
        if self.regions[which] is None:
            n = _lib.c_size_t(0)
            check(LIB.ganamd_critic_region_bytes(self.plan, which, _lib.ctypes.byref(n)), "critic_region_bytes")
            self.regions[which] = workspace(n.value, device)
            check(LIB.ganamd_critic_bind(self.plan, which, *wsarg(self.regions[which])), "critic_bind")

    def _grads(self):
        """ganamd_critic_grads[] of the parameters that want a gradient (created as zeros)."""
        g = (_lib.CriticGrads * len(self.prog.ops))()
        for i, op in enumerate(self.prog.ops):
            if op.kind in ("conv", "linear"):
                w, b = op.mod.weight.weight, op.mod.bias
                if w.requires_grad:
                    g[i].gw = ptr(_grad_buf(w))
                if b is not None and b.requires_grad:
                    g[i].gb = ptr(_grad_buf(b))
            elif op.kind == "prelu" and op.mod.weight.requires_grad:
                g[i].gw = ptr(_grad_buf(op.mod.weight))
        return g

    def _count(self, sweep, params=False, need_input=False, seeded=False):
        """The sweep's conv GEMMs into ops.FlopCounter (host-side bookkeeping of the bench)."""
        if not ops.FlopCounter.enabled and ops.FlopCounter.record is None:
            return
        convs = [op for op in self.prog.ops if op.kind in ("conv", "linear")]
        if sweep in ("forward", "tangent"):
            for op in convs:
                ops.FlopCounter.add(_geo_of(op, self.B, self.sh[op.ins[0]]), "fwd")
            return
        # which values carry an adjoint (the backward: all; the adjoint: from the seed and the
        # second-order sources -- sigmoid, the SE product, MiniBatchStdDev -- downwards)
        has = {self.prog.out} if (sweep == "backward" or seeded) else set()
        for op in reversed(self.prog.ops):
            live = op.out in has or (sweep == "adjoint" and op.kind in ("sigmoid", "mbstd"))
            if op.kind in ("conv", "linear"):
                geo = _geo_of(op, self.B, self.sh[op.ins[0]])
                first = self.prog.ops[op.ins[0] - 1].kind == "swap" if op.ins[0] > 0 else True
                if op.out in has and (not first or need_input):
                    ops.FlopCounter.add(geo, "dgrad")
                if params and op.mod.weight.weight.requires_grad:
                    for _ in range((op.out in has) + (sweep == "adjoint")):
                        ops.FlopCounter.add(geo, "wgrad")
            if live:
                has.update(op.ins)
            elif sweep == "adjoint" and op.kind == "scale_add":     # G-terms only: x and the gate
                has.update(op.ins[:2])

    # ---------------------------------------------------------------- sweeps
    def forward(self, x_nchw):
        self.x = x_nchw
        self._setup(x_nchw)
        self._count("forward")
        check(LIB.ganamd_critic_forward(self.plan, ptr(x_nchw), None, None, 0, stream()), "critic_forward")
        return self.X[self.prog.out].clone()               # [1, B], not a view of the workspace

    def backward(self, seed, params: bool, need_input: bool):
        """g_v for every value from g_out = seed ([1, B]); parameter gradients accumulated into
        .grad when ``params``; the input gradient (NCHW) returned when ``need_input``."""
        self._count("backward", params, need_input)
        self.seed = seed.contiguous()
        gx = torch.empty_like(self.x) if need_input else None
        self._region(1, self.x.device)
        check(LIB.ganamd_critic_backward(self.plan, ptr(self.seed), self._grads() if params else None, ptr(gx),
                                         None, 0, stream()), "critic_backward")
        return gx

    def tangent(self, v_nchw, params: bool):
        """xd_v along the input direction v; the PReLU slopes' second-order term accumulates into
        their gradients when ``params``."""
        self._count("tangent")
        self.v = v_nchw.contiguous()
        self._region(2, self.x.device)
        check(LIB.ganamd_critic_tangent(self.plan, ptr(self.v), self._grads() if params else None, None, 0,
                                        stream()), "critic_tangent")
        return self.XD[self.prog.out]

    def adjoint(self, a_seed, params: bool, need_input: bool = False):
        """Reverse sweep of h = <v, g> (+ <a_seed, D(x)>): accumulates dh/dtheta into the
        parameters' gradients; returns dh/dx (NCHW) when ``need_input``.  a_seed may be None."""
        self._count("adjoint", params, need_input, seeded=a_seed is not None)
        self.a_seed = None if a_seed is None else a_seed.contiguous()
        ax = torch.empty_like(self.x) if need_input else None
        self._region(3, self.x.device)
        check(LIB.ganamd_critic_adjoint(self.plan, ptr(self.a_seed), self._grads() if params else None, ptr(ax),
                                        None, 0, stream()), "critic_adjoint")
        return ax

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
    check(LIB.ganamd_gp_fwd(ptr(g), B, n, float(center), float(lam), int(mode), ptr(norms), ptr(out), *wsarg(ws),
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
        return run.backward(seed, params=first_order_params, need_input=True)   # not kept by the run

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


def penalty_sweeps(D, x_hat):
    """The part of the gradient penalty that depends on x_hat only: the forward and the input-gradient
    sweep of D at x_hat (no autograd node)."""
    run = Run(program_of(D), 1)
    x_hat = x_hat.detach().contiguous()
    run.forward(x_hat)
    seed = torch.ones((1, x_hat.shape[0]), device=x_hat.device, dtype=torch.float32)
    return run, run.backward(seed, params=False, need_input=True)


def penalty_value(D, run, g, center=1.0, lam=1.0, mode=0):
    """The fused penalty on the input gradient g of ``penalty_sweeps``; its ``.backward()`` runs the
    double backward (tangent + adjoint sweeps)."""
    params = [p for p in program_of(D).params if p.requires_grad]
    if not params or not torch.is_grad_enabled():
        return _penalty(g, center, lam, mode)[0]
    return _PenaltyFn.apply(params[0], run, g, center, lam, mode)


def gradient_penalty(D, x_hat, center=1.0, lam=1.0, mode=0):
    """lam * mean_b (||grad_x sum D(x_hat)||_b - center)^2 (train/wgangp.py:34-54) -- or, mode 1,
    lam * mean_b ||.||^2 (R1/R2) -- with forward, input-gradient backward and the fused penalty
    run now; ``.backward()`` on the result runs the double backward (tangent + adjoint sweeps)."""
    run, g = penalty_sweeps(D, x_hat)
    return penalty_value(D, run, g, center, lam, mode)


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
