"""Float64 emulation of one conv-GEMM launch of libganamd.so (test infrastructure).

``emulate(op, geo, ...)`` recomputes what ``ops._conv_fwd`` / ``_conv_fwd_ex`` / ``_conv_dgrad`` /
``_conv_wgrad`` returned for the same operands, in float64 with torch autograd on the host:

  fwd    y  = alpha * conv(pad(x * xs), W) * ys + bias (+ noise_scale * noise)
  dgrad  gx = alpha * conv^T(gy * gys, W)           (the adjoint of the padded conv)
  wgrad  gW = alpha * sum_n (gy * gys) x gather(x * xs)

with CNHW activations ([C][B][H][W]) and [C][B] scales as the kernels take them.  ``bf16=True``
rounds both GEMM operands to bf16 (RNE) at the kernels' rounding points (GANAMD_MATH_BF16: the
fp32 product x * xs, resp. gy * gys, is rounded, and the UNSCALED weight), so the only remaining
difference to the kernel is its fp32 accumulation order.
"""
import torch
import torch.nn.functional as F

from gan_amd import _lib


_DT = [torch.float64]     # the emulation's dtype (emulate(dtype=...)): float64, or float32 for fp32's own error


def _bf(t, bf16):
    return t.float().to(torch.bfloat16).to(_DT[0]) if bf16 else t.to(_DT[0])


def _scaled(t, s, bf16):
    """t [C][B][H][W] * s [C][B] in fp32 (the kernel's staging product), rounded when bf16, as NCHW."""
    t = t.float()
    if s is not None:
        t = t * s.float()[:, :, None, None]
    return _bf(t, bf16).permute(1, 0, 2, 3)


def _conv(geo, x, w):
    """The launch's convolution on NCHW float64 operands."""
    if geo.transposed:
        return F.conv_transpose2d(x, w, stride=geo.stride, padding=geo.pad)
    if geo.pad:
        mode = "replicate" if geo.pad_mode == _lib.PAD_REPLICATE else "constant"
        x = F.pad(x, (geo.pad,) * 4, mode=mode)
    return F.conv2d(x, w, stride=geo.stride)


def _wshape(geo):
    return (geo.Cin, geo.Cout, geo.K, geo.K) if geo.transposed else (geo.Cout, geo.Cin, geo.K, geo.K)


def emulate(op, geo, x=None, w=None, gy=None, xs=None, ys=None, alpha=1.0, bias=None, noise=None, noise_scale=None,
            bf16=False, dtype=torch.float64):
    """float64 result (CPU): fwd / dgrad in CNHW, wgrad in the weight's layout.  dtype=float32: the
    same convolution evaluated in float32 on the host (fp32's own rounding, for error bars)."""
    _DT[0] = dtype
    try:
        return _emulate(op, geo, x, w, gy, xs, ys, alpha, bias, noise, noise_scale, bf16).double()
    finally:
        _DT[0] = torch.float64


def _emulate(op, geo, x, w, gy, xs, ys, alpha, bias, noise, noise_scale, bf16):
    dt = _DT[0]
    cpu = lambda t: None if t is None else t.detach().cpu()   # noqa: E731
    x, w, gy, xs, ys, bias = map(cpu, (x, w, gy, xs, ys, bias))
    if op == "fwd":
        wr = _bf(w.reshape(_wshape(geo)), bf16)
        y = _conv(geo, _scaled(x.reshape(geo.Cin, geo.B, geo.H, geo.W), xs, bf16), wr) * alpha
        y = y.permute(1, 0, 2, 3)
        if ys is not None:
            y = y * ys.to(dt)[:, :, None, None]
        if bias is not None:
            y = y + bias.to(dt)[:, None, None, None]
        if noise is not None:
            y = y + noise_scale.detach().cpu().to(dt)[:, None, None, None] * noise.detach().cpu().to(dt)
        return y
    if op == "dgrad":
        wr = _bf(w.reshape(_wshape(geo)), bf16)
        x_ = torch.zeros(geo.B, geo.Cin, geo.H, geo.W, dtype=dt, requires_grad=True)
        g = _scaled(gy.reshape(geo.Cout, geo.B, geo.OH, geo.OW), ys, bf16)
        gx, = torch.autograd.grad(_conv(geo, x_, wr), x_, g)
        return (gx * alpha).permute(1, 0, 2, 3)
    if op == "wgrad":
        w_ = torch.zeros(_wshape(geo), dtype=dt, requires_grad=True)
        xin = _scaled(x.reshape(geo.Cin, geo.B, geo.H, geo.W), xs, bf16)
        g = _scaled(gy.reshape(geo.Cout, geo.B, geo.OH, geo.OW), ys, bf16)
        gw, = torch.autograd.grad(_conv(geo, xin, w_), w_, g)
        return gw * alpha
    raise ValueError(op)


def max_rel(got, ref):
    """max |got - ref| / max |ref| (float64)."""
    got = got.detach().cpu().double().reshape(-1)
    ref = ref.detach().double().reshape(-1)
    return float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-300))


class Recorder:
    """Records (a sample of) the conv launches made through gan_amd.ops while active: every
    ``every``-th launch of each kind, at most ``cap`` in total, with clones of its operands and
    result, for ``emulate``.  Use as a context manager."""

    def __init__(self, every=1, cap=10 ** 9, kinds=("fwd", "dgrad", "wgrad")):
        self.every, self.cap, self.kinds = every, cap, kinds
        self.calls = []
        self.seen = {k: 0 for k in ("fwd", "dgrad", "wgrad")}

    def _take(self, kind):
        if kind not in self.kinds or len(self.calls) >= self.cap:
            return False
        self.seen[kind] += 1
        return (self.seen[kind] - 1) % self.every == 0

    def __enter__(self):
        from gan_amd import ops
        self.ops = ops
        self.orig = (ops._conv_fwd, ops._conv_fwd_ex, ops._conv_dgrad, ops._conv_wgrad)
        f_fwd, f_ex, f_dg, f_wg = self.orig
        rec = self
        clone = lambda t: None if t is None else t.detach().clone()   # noqa: E731

        def conv_fwd(geo, x, w, bias=None, xs=None, ys=None, alpha=1.0, out=None):
            y = f_fwd(geo, x, w, bias, xs, ys, alpha, out)
            if rec._take("fwd"):
                rec.calls.append(dict(op="fwd", geo=geo, x=clone(x), w=clone(w), bias=clone(bias), xs=clone(xs),
                                      ys=clone(ys), alpha=alpha, got=clone(y), math=ops._MATH[0]))
            return y

        def conv_fwd_ex(geo, x, w, xs, ys, alpha, noise=None, noise_scale=None, act=None):
            y = f_ex(geo, x, w, xs, ys, alpha, noise, noise_scale, act)
            if act is None and rec._take("fwd"):
                rec.calls.append(dict(op="fwd", geo=geo, x=clone(x), w=clone(w), xs=clone(xs), ys=clone(ys),
                                      alpha=alpha, noise=clone(noise), noise_scale=clone(noise_scale), got=clone(y),
                                      math=ops._MATH[0]))
            return y

        def conv_dgrad(geo, gy, w, gys=None, alpha=1.0):
            gx = f_dg(geo, gy, w, gys, alpha)
            if rec._take("dgrad"):
                rec.calls.append(dict(op="dgrad", geo=geo, gy=clone(gy), w=clone(w), ys=clone(gys), alpha=alpha,
                                      got=clone(gx), math=ops._MATH[0]))
            return gx

        def conv_wgrad(geo, x, gy, xs=None, gys=None, alpha=1.0, out=None, accumulate=False):
            take = rec._take("wgrad")
            before = clone(out) if take and accumulate and out is not None else None
            gw = f_wg(geo, x, gy, xs, gys, alpha, out, accumulate)
            if take:
                got = gw.detach().clone() if before is None else gw.detach() - before
                rec.calls.append(dict(op="wgrad", geo=geo, x=clone(x), gy=clone(gy), xs=clone(xs), ys=clone(gys),
                                      alpha=alpha, got=got, accumulated=before is not None, math=ops._MATH[0]))
            return gw

        ops._conv_fwd, ops._conv_fwd_ex, ops._conv_dgrad, ops._conv_wgrad = conv_fwd, conv_fwd_ex, conv_dgrad, conv_wgrad
        return self

    def __exit__(self, *exc):
        ops = self.ops
        ops._conv_fwd, ops._conv_fwd_ex, ops._conv_dgrad, ops._conv_wgrad = self.orig
        return False

    def check(self, bf16, bars, log=print):
        """Emulate every recorded launch; returns {kind: worst max_rel} and asserts the bars."""
        worst = {}
        for c in self.calls:
            ref = emulate(c["op"], c["geo"], x=c.get("x"), w=c.get("w"), gy=c.get("gy"), xs=c.get("xs"),
                          ys=c.get("ys"), alpha=c["alpha"], bias=c.get("bias"), noise=c.get("noise"),
                          noise_scale=c.get("noise_scale"), bf16=bf16)
            e = max_rel(c["got"], ref)
            g = c["geo"]
            key = c["op"]
            if e > worst.get(key, (0, None))[0]:
                worst[key] = (e, f"B={g.B} {g.Cin}->{g.Cout} {g.H}x{g.W} k{g.K} s{g.stride}{' T' if g.transposed else ''}"
                                 f"{' scaled' if c.get('xs') is not None or c.get('ys') is not None else ''}")
            c.clear()
        log(f"{len(self.calls)} launches emulated: worst {worst}")
        for k, (e, where) in worst.items():
            assert e <= bars[k], (k, e, where, bars[k])
        return worst


def seq_fp32(op, geo, x=None, w=None, gy=None, xs=None, ys=None, alpha=1.0):
    """The launch's convolution as a plain fp32 FMA loop on the device: ONE accumulator per output,
    K = Cin*K*K (fwd) or Cout*K*K (dgrad) fp32 multiply-adds in tap order -- what a textbook fp32
    GPU convolution does.  Its error against float64 is the yardstick of "fp32-class" for launches
    whose outputs number in the millions (the max-error tail of any fp32 accumulation grows with
    them).  fwd / dgrad of stride-1 replicate- or zero-padded convs; CNHW in and out."""
    dev = (x if x is not None else gy).device
    k, p = geo.K, geo.pad
    W = w.detach().float().reshape(geo.Cout, geo.Cin, k, k)
    mode = "replicate" if geo.pad_mode == _lib.PAD_REPLICATE else "constant"
    if op == "fwd":
        xin = x.float().reshape(geo.Cin, geo.B, geo.H, geo.W)
        if xs is not None:
            xin = xin * xs.float()[:, :, None, None]
        xp = F.pad(xin, (p,) * 4, mode=mode) if p else xin
        acc = torch.zeros(geo.Cout, geo.B, geo.OH, geo.OW, device=dev, dtype=torch.float32)
        for ci in range(geo.Cin):
            for kh in range(k):
                for kw in range(k):
                    acc.addcmul_(W[:, ci, kh, kw][:, None, None, None], xp[ci, :, kh:kh + geo.OH, kw:kw + geo.OW][None])
        acc = acc * alpha
        if ys is not None:
            acc = acc * ys.float()[:, :, None, None]
        return acc
    if op == "dgrad":
        g = gy.float().reshape(geo.Cout, geo.B, geo.OH, geo.OW)
        if ys is not None:
            g = g * ys.float()[:, :, None, None]
        Hp, Wp = geo.H + 2 * p, geo.W + 2 * p
        acc = torch.zeros(geo.Cin, geo.B, Hp, Wp, device=dev, dtype=torch.float32)
        for co in range(geo.Cout):
            for kh in range(k):
                for kw in range(k):
                    acc[:, :, kh:kh + geo.OH, kw:kw + geo.OW].addcmul_(W[co, :, kh, kw][:, None, None, None], g[co][None])
        if p and mode == "replicate":      # the padding's adjoint: the ring folds onto the edge pixels
            gx = torch.zeros(geo.Cin, geo.B, geo.H, geo.W, device=dev, dtype=torch.float32)
            ih = torch.arange(Hp, device=dev).sub(p).clamp(0, geo.H - 1)
            iw = torch.arange(Wp, device=dev).sub(p).clamp(0, geo.W - 1)
            idx = (ih[:, None] * geo.W + iw[None, :]).reshape(-1)
            gx.view(geo.Cin, geo.B, -1).index_add_(2, idx, acc.reshape(geo.Cin, geo.B, -1))
        else:
            gx = acc[:, :, p:p + geo.H, p:p + geo.W]
        return gx * alpha
    raise ValueError(op)
