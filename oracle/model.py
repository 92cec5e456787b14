"""CPU oracle: a functional fp32 restatement of G13_5, D9_4 and the WGAN-GP step.

TEST INFRASTRUCTURE ONLY (the checker, never the product): imported by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg.

Parity is PINNED: ``tests/test_oracle_golden.py`` checks this restatement against the golden
fixtures that ``tests/golden/make_golden.py`` produced by importing the reference itself.

Differences of form (not of value) from the reference:
  * parameters live in a flat ``name -> tensor`` dict keyed by the reference's
    ``named_parameters()`` names instead of an ``nn.Module`` tree;
  * the weight-modulated conv uses the batch-shared form
    ``y = d[b,co] * conv(pad(x * s[b,ci]), W*c)`` with ``d = rsqrt(sum_ci s^2 sum_k (W*c)^2 + eps)``
    instead of materialising per-sample weights with ``groups=B``
    (generator_13_5.py:234-248); equal to <=1e-6 relative.
Everything else follows the reference op for op (file:line cited per function).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


class Params:
    """name -> leaf tensor.  In ``lazy`` mode a missing name is created with reference-like init."""

    def __init__(self, tensors=None, lazy=False, generator=None):
        self.t = dict(tensors or {})
        self.buffers = {}
        self.lazy = lazy
        self.gen = generator
        self.used = set()

    def __call__(self, name, shape, init="randn"):
        self.used.add(name)
        if name not in self.t:
            if not self.lazy:
                raise KeyError(name)
            if init == "randn":
                v = torch.randn(shape, generator=self.gen)
            elif init == "zeros":
                v = torch.zeros(shape)
            elif init == "ones":
                v = torch.ones(shape)
            elif init == "prelu":
                v = torch.full(shape, 0.25)
            elif init == "noise":
                v = torch.rand(shape, generator=self.gen) * 0.1 + 0.2
            elif init == "convt":
                v = (torch.rand(shape, generator=self.gen) * 2 - 1) / math.sqrt(shape[1] * shape[2] * shape[3])
            else:
                raise KeyError(init)
            self.t[name] = v.requires_grad_(True)
        t = self.t[name]
        assert tuple(t.shape) == tuple(shape), (name, tuple(t.shape), tuple(shape))
        return t

    def bn_buffers(self, name, c):
        if name not in self.buffers:
            self.buffers[name] = (torch.zeros(c), torch.ones(c))
        return self.buffers[name]


# ----------------------------------------------------------------------------------------------
# shared primitives
# ----------------------------------------------------------------------------------------------

# bf16 emulation of the build's GANAMD_MATH_BF16 GEMMs (test infrastructure for config 4, which
# the reference does not have): when set, the two GEMM operands of every equalized conv / linear
# -- the (padded) input and the UNSCALED weight -- are rounded to bf16 (RNE) before the product;
# the equalized-LR scale and the bias apply after it, in the working precision.
BF16_GEMM = [False]


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype) if BF16_GEMM[0] else t


def eq_linear(P, pre, x, cin, cout, wname="weights", bias_init="randn"):
    """EqualizedLinear: generator_13_5.py:19-26 / discriminator_9_4.py:20-27."""
    w = P(f"{pre}.weight.{wname}", (cout, cin))
    b = P(f"{pre}.bias", (cout,), bias_init)
    if BF16_GEMM[0]:
        return F.linear(_bf(x), _bf(w)) * (1.0 / math.sqrt(cin)) + b
    return F.linear(x, w * (1.0 / math.sqrt(cin)), b)


def eq_conv(P, pre, x, cin, cout, k, pad, stride=1, wname="weights"):
    """EqualizedConv2d with ReplicationPad2d: generator_13_5.py:29-38 / discriminator_9_4.py:30-40."""
    w = P(f"{pre}.weight.{wname}", (cout, cin, k, k))
    b = P(f"{pre}.bias", (cout,))
    if pad:
        x = F.pad(x, (pad, pad, pad, pad), mode="replicate")
    if BF16_GEMM[0]:
        return F.conv2d(_bf(x), _bf(w), None, stride=stride) * (1.0 / math.sqrt(cin * k * k)) + b.view(1, -1, 1, 1)
    return F.conv2d(x, w * (1.0 / math.sqrt(cin * k * k)), b, stride=stride)


def prelu(P, pre, x, c):
    """nn.PReLU(c): per-channel slope."""
    return F.prelu(x, P(f"{pre}.weight", (c,), "prelu"))


def bn(P, pre, x, c):
    """nn.BatchNorm1d/2d in train mode (batch statistics, running stats momentum 0.1)."""
    rm, rv = P.bn_buffers(pre, c)
    return F.batch_norm(x, rm, rv, P(f"{pre}.weight", (c,), "ones"), P(f"{pre}.bias", (c,), "zeros"),
                        training=True, momentum=0.1, eps=1e-5)


_SMOOTH = torch.tensor([[1.0, 2.0, 1.0], [2.0, 4.0, 2.0], [1.0, 2.0, 1.0]]) / 16.0


def smooth(x):
    """Smooth: depthwise binomial 3x3 with replication pad (generator_13_5.py:134-150)."""
    b, c, h, w = x.shape
    y = F.pad(x.reshape(b * c, 1, h, w), (1, 1, 1, 1), mode="replicate")
    return F.conv2d(y, _SMOOTH.to(x.dtype).view(1, 1, 3, 3)).reshape(b, c, h, w)


def softmax_mix(feas, att):
    return (feas * att).sum(dim=1)


# ----------------------------------------------------------------------------------------------
# G13_5 (generators/generator_13_5.py)
# ----------------------------------------------------------------------------------------------

class GCtx:
    def __init__(self, P, w, randn):
        self.P, self.w, self.randn = P, w, randn


def g_mapping(P, pre, x, planes, layers):
    """MappingNetwork: [EqLinear, BN1d, PReLU] x n (generator_13_5.py:205-216)."""
    for i in range(layers):
        x = eq_linear(P, f"{pre}.net.{3 * i}", x, planes, planes)
        x = bn(P, f"{pre}.net.{3 * i + 1}", x, planes)
        x = prelu(P, f"{pre}.net.{3 * i + 2}", x, planes)
    return x


def g_modconv(C, pre, x, cin, cout, k):
    """Conv2dWeightModulate (generator_13_5.py:219-248) in the batch-shared form."""
    P = C.P
    s = g_mapping(P, f"{pre}.to_style.0", C.w, 256, 1)
    s = eq_linear(P, f"{pre}.to_style.1", s, 256, cin)
    s = bn(P, f"{pre}.to_style.2", s, cin)                           # [B, cin]
    wt = P(f"{pre}.weight.weights", (cout, cin, k, k)) * (1.0 / math.sqrt(cin * k * k))
    wsq = (wt * wt).sum(dim=(2, 3))                                  # [cout, cin]
    d = torch.rsqrt((s * s) @ wsq.t() + 1e-8)                        # [B, cout]
    xs = x * s[:, :, None, None]
    p = (k - 1) // 2
    if p:
        xs = F.pad(xs, (p, p, p, p), mode="replicate")
    return F.conv2d(xs, wt) * d[:, :, None, None]


def g_styleconv(C, pre, x, cin, cout, k, noise):
    """StyleConv (generator_13_5.py:251-266); its bias add is a no-op in the reference."""
    y = g_modconv(C, f"{pre}.conv", x, cin, cout, k)
    C.P(f"{pre}.bias", (cout,))  # exists, never used
    if noise:
        sn = C.P(f"{pre}.scale_noise", (cout,), "noise")
        y = y + sn[None, :, None, None] * C.randn(tuple(y.shape))
    return y


def g_sk_attention(C, pre, feas, planes, m, img):
    """SKAttention_conv / SKAttention_fc (generator_13_5.py:41-131)."""
    P = C.P
    b, s, c = feas.shape[:3]
    u = feas.sum(dim=1)
    if img > 4:
        assert u.shape[2] >= 8
        t = F.adaptive_avg_pool2d(u, 5)
        for i in range(2):
            t = eq_conv(P, f"{pre}.conv_main.{3 * i}", t, planes, planes, 3, 1)
            t = bn(P, f"{pre}.conv_main.{3 * i + 1}", t, planes)
            t = prelu(P, f"{pre}.conv_main.{3 * i + 2}", t, planes)
        z = F.adaptive_avg_pool2d(t, 1).view(b, c)
        nfc = 1
    else:
        z = F.adaptive_avg_pool2d(u, 1).view(b, c)
        nfc = 2
    for i in range(nfc):
        z = eq_linear(P, f"{pre}.fc_main.{3 * i}", z, planes, planes)
        z = bn(P, f"{pre}.fc_main.{3 * i + 1}", z, planes)
        z = prelu(P, f"{pre}.fc_main.{3 * i + 2}", z, planes)
    vecs = []
    for i in range(m):
        v = eq_linear(P, f"{pre}.fc_sub_{i}.0", z, planes, planes)
        v = bn(P, f"{pre}.fc_sub_{i}.1", v, planes)
        v = prelu(P, f"{pre}.fc_sub_{i}.2", v, planes)
        vecs.append(eq_linear(P, f"{pre}.fc_sub_{i}.3", v, planes, planes))
    att = torch.softmax(torch.stack(vecs, dim=1), dim=1)
    return att.view(b, s, c, 1, 1)


def g_stylebl(C, pre, x, last, inp, out, dense, k, m, img):
    """StyleBlock (generator_13_5.py:298-322)."""
    x = g_styleconv(C, f"{pre}.conv1", x, last, inp, 1, False)
    x = prelu(C.P, f"{pre}.activation1", x, inp)
    if m == 1:
        x = g_styleconv(C, f"{pre}.conv2", x, inp, inp, k, True)
        x = prelu(C.P, f"{pre}.activation2", x, inp)
    else:  # SKStyleConv (generator_13_5.py:269-295)
        feas = []
        for i in range(m):
            f = g_styleconv(C, f"{pre}.skconv.conv_{i}", x, inp, inp, 3 + 2 * i, True)
            feas.append(prelu(C.P, f"{pre}.skconv.nonlinear_{i}", f, inp))
        feas = torch.stack(feas, dim=1)
        x = softmax_mix(feas, g_sk_attention(C, f"{pre}.skconv.sk_attention", feas, inp, m, img))
    return g_styleconv(C, f"{pre}.conv3", x, inp, out + dense, 3, False)


def g_se(C, pre, x, planes, img):
    """SEBlock_conv / SEBlock_fc of G (generator_13_5.py:352-405), returns the sigmoid gate."""
    P = C.P
    b, c = x.shape[:2]
    if img > 4:
        assert x.shape[2] >= 8
        t = F.adaptive_avg_pool2d(x, 5)
        for i in range(2):
            t = eq_conv(P, f"{pre}.convs.{3 * i}", t, planes, planes, 3, 1)
            t = bn(P, f"{pre}.convs.{3 * i + 1}", t, planes)
            t = prelu(P, f"{pre}.convs.{3 * i + 2}", t, planes)
        z = F.adaptive_avg_pool2d(t, 1).view(b, c)
        nfc = 1
    else:
        z = F.adaptive_avg_pool2d(x, 1).view(b, c)
        nfc = 2
    for i in range(nfc):
        z = eq_linear(P, f"{pre}.fcs.{3 * i}", z, planes, planes)
        z = bn(P, f"{pre}.fcs.{3 * i + 1}", z, planes)
        z = prelu(P, f"{pre}.fcs.{3 * i + 2}", z, planes)
    z = eq_linear(P, f"{pre}.fc_out", z, planes, planes)
    z = bn(P, f"{pre}.fc_bn", z, planes)
    return torch.sigmoid(z).view(b, c, 1, 1)


def g_block_out(last, out, dense, root, unify):
    """BasicBlock.get_out_planes (generator_13_5.py:410-417)."""
    return 2 * out + 2 * dense if (unify or root) else last + dense


def g_basic(C, pre, x, last, inp, out, dense, root, unify, m, img):
    """BasicBlock.forward (generator_13_5.py:448-467) incl. ResnetInit (325-349)."""
    P, dd = C.P, out
    if unify:
        x = g_stylebl(C, f"{pre}.unify", x, last, inp, 2 * out, dense, 3, m, img)
        x = prelu(P, f"{pre}.activation_unify", x, 2 * out + dense)
        rlast = out + dense
    else:
        rlast = last - out
    xr = torch.cat([x[:, :dd], x[:, 2 * dd:]], 1)
    xt = x[:, dd:]
    r = f"{pre}.rir_3"
    rr = g_stylebl(C, f"{r}.residual", xr, rlast, inp, out, dense, 3, m, img)
    rt = g_stylebl(C, f"{r}.residual_across", xr, rlast, inp, out, 0, 3, m, img)
    tt = g_stylebl(C, f"{r}.transient", xt, rlast, inp, out, 0, 3, m, img)
    tr = g_stylebl(C, f"{r}.transient_across", xt, rlast, inp, out, dense, 3, m, img)
    x_res3 = prelu(P, f"{r}.activation_residual", rr + tr, out + dense)
    x_tr3 = prelu(P, f"{r}.activation_transient", rt + tt, out)
    head = x_res3[:, :dd]
    feas_res = x[:, :dd] + head * g_se(C, f"{pre}.se_attention_residual", head, out, img)
    if root:
        sc = g_stylebl(C, f"{pre}.shortcut", x, last, inp, 0, dense, 3, m, img)
        sc = prelu(P, f"{pre}.activation_shortcut", sc, dense)
        return torch.cat([feas_res, x_tr3, sc, x_res3[:, dd:]], 1)
    return torch.cat([feas_res, x_tr3, x[:, 2 * dd:], x_res3[:, dd:]], 1)


def g_to_rgb(C, pre, x, planes, m, img):
    """ToRGB (generator_13_5.py:470-493) incl. SKConv (173-202)."""
    P = C.P
    if m == 1:
        x = eq_conv(P, f"{pre}.pre_conv", x, planes, planes, 3, 1)
        x = bn(P, f"{pre}.pre_bn", x, planes)
        x = prelu(P, f"{pre}.pre_activation", x, planes)
    else:
        feas = []
        for i in range(m):
            k = 3 + 2 * i
            f = eq_conv(P, f"{pre}.skconv.conv_{i}", x, planes, planes, k, (k - 1) // 2)
            f = bn(P, f"{pre}.skconv.BatchNorm_{i}", f, planes)
            feas.append(prelu(P, f"{pre}.skconv.nonlinear_{i}", f, planes))
        feas = torch.stack(feas, dim=1)
        x = softmax_mix(feas, g_sk_attention(C, f"{pre}.skconv.sk_attention", feas, planes, m, img))
    x = eq_conv(P, f"{pre}.conv", x, planes, 3, 5, 2)
    return bn(P, f"{pre}.bn", x, 3)


def g_tree_out(last, out, dense, level, bnum):
    return 2 * out + 2 * dense  # every Tree ends in a root BasicBlock


def g_tree(C, pre, x, rgb, last, inp, out, dense, level, bnum, m, img):
    """Tree (generator_13_5.py:496-564): construction bookkeeping + forward."""
    xs = []
    if level > 1:
        prev_unify = last < 2 * out
        xs.append(g_basic(C, f"{pre}.prev_root", x, last, inp, out, dense, False, prev_unify, m, img))
        cur_last = last
        for i in reversed(range(1, level)):
            x, rgb = g_tree(C, f"{pre}.level_{i}", x, rgb, cur_last, inp, out, dense, i, bnum, m, img)
            cur_last = g_tree_out(cur_last, out, dense, i, bnum)
            xs.append(x)
        unify0 = False
    else:
        cur_last = last
        unify0 = last < 2 * out
    for i in range(bnum):
        uni = unify0 if i == 0 else False
        x = g_basic(C, f"{pre}.block_{i}", x, cur_last, inp, out, dense, False, uni, m, img)
        cur_last = g_block_out(cur_last, out, dense, False, uni)
        xs.append(x[:, :2 * out])
    xs.append(x[:, 2 * out:])
    xs = torch.cat(xs, 1)
    y = g_basic(C, f"{pre}.root", xs, xs.shape[1], inp * bnum, out, dense, True, False, m, img)
    rgb = g_to_rgb(C, f"{pre}.to_rgb", y, 2 * out + 2 * dense, m, img) + rgb
    return y, rgb


def g_skconvt(C, pre, x, planes):
    """SKConvT (generator_13_5.py:153-170): ConvT k4 s2 p1 | bicubic x2 + smooth, SK-mixed."""
    P = C.P
    a = F.conv_transpose2d(x, P(f"{pre}.convT.weight", (planes, planes, 4, 4), "convt"),
                           P(f"{pre}.convT.bias", (planes,), "zeros"), stride=2, padding=1)
    a = prelu(P, f"{pre}.activation_convT", bn(P, f"{pre}.bn", a, planes), planes)
    b = smooth(F.interpolate(x, scale_factor=2, mode="bicubic", align_corners=False))
    feas = torch.stack([a, b], dim=1)
    return softmax_mix(feas, g_sk_attention(C, f"{pre}.sk_attention", feas, planes, 2, 8))


G_STAGES = [  # (in_planes, out_planes, level, blocks, m, image)  for planes=48
    (384, 192, 1, 2, 1, 4),
    (192, 192, 2, 2, 2, 8),
    (96, 96, 2, 2, 2, 16),
    (48, 48, 2, 2, 2, 32),
    (48, 48, 2, 2, 2, 64),
]
DENSE = 6


def generator(P, z, randn):
    """Generator.forward (generator_13_5.py:610-631) -> rgb [B,3,64,64] (no tanh)."""
    C = GCtx(P, None, randn)
    pre = "block0"
    C.w = g_mapping(P, f"{pre}.mapping_network", torch.squeeze(z), 256, 12)
    x = F.conv_transpose2d(z, P(f"{pre}.convT.weight", (256, 384, 4, 4), "convt"),
                           P(f"{pre}.convT.bias", (384,), "zeros"), stride=1, padding=0)
    x = prelu(P, f"{pre}.activation", bn(P, f"{pre}.bn", x, 384), 384)
    rgb = g_to_rgb(C, f"{pre}.to_rgb", x, 384, 1, 4)
    inp, out, level, bnum, m, img = G_STAGES[0]
    x, rgb = g_tree(C, f"{pre}.tree", x, rgb, 384, inp, out, DENSE, level, bnum, m, img)
    last = 2 * out + 2 * DENSE
    for i in range(1, 5):
        inp, out, level, bnum, m, img = G_STAGES[i]
        pre = f"block{i}"
        rgb = g_skconvt(C, f"{pre}.upsample_rgb", rgb, 3)
        x = g_skconvt(C, f"{pre}.upsample", x, last)
        x, rgb = g_tree(C, f"{pre}.tree", x, rgb, last, inp, out, DENSE, level, bnum, m, img)
        last = 2 * out + 2 * DENSE
    return rgb


# ----------------------------------------------------------------------------------------------
# D9_4 (discriminators/discriminator_9_4.py)
# ----------------------------------------------------------------------------------------------

D_BLOCKS = [  # (seq index, in, out, downsample, image_size)  discriminator_9_4.py:168-187
    (2, 64, 64, False, 64), (3, 64, 64, False, 64), (4, 64, 128, True, 32),
    (5, 128, 128, False, 32), (6, 128, 128, False, 32), (7, 128, 256, True, 16),
    (8, 256, 256, False, 16), (9, 256, 256, False, 16), (10, 256, 512, True, 8),
    (11, 512, 512, False, 8), (12, 512, 512, False, 8), (13, 512, 1024, True, 4),
    (15, 1025, 1025, False, 4), (16, 1025, 1025, False, 4), (17, 1025, 1025, True, 2),
]


def d_se(P, pre, x, c, img):
    """D's SEBlock_conv (no pad, 5->3->1) / SEBlock_fc (discriminator_9_4.py:83-128)."""
    b = x.shape[0]
    if img > 4:
        assert x.shape[2] >= 8
        t = F.adaptive_avg_pool2d(x, 5)
        for i in range(2):
            t = eq_conv(P, f"{pre}.convs.{2 * i}", t, c, c, 3, 0, wname="weight")
            t = prelu(P, f"{pre}.convs.{2 * i + 1}", t, c)
        z = F.adaptive_avg_pool2d(t, 1).view(b, c)
        nfc = 1
    else:
        z = F.adaptive_avg_pool2d(x, 1).view(b, c)
        nfc = 2
    for i in range(nfc):
        z = eq_linear(P, f"{pre}.fcs.{2 * i}", z, c, c, wname="weight")
        z = prelu(P, f"{pre}.fcs.{2 * i + 1}", z, c)
    z = eq_linear(P, f"{pre}.fc_out", z, c, c, wname="weight")
    return torch.sigmoid(z).view(b, c, 1, 1)


def d_block(P, pre, x, cin, cout, down, img):
    """DiscriminatorBlock.forward (discriminator_9_4.py:131-161)."""
    if down:
        h, w = x.shape[2] // 2, x.shape[3] // 2
        r = F.interpolate(smooth(x), (h, w), mode="bicubic", align_corners=False)
        res = eq_conv(P, f"{pre}.residual.1", r, cin, cout, 1, 0, wname="weight")
    else:
        res = x
    y = eq_conv(P, f"{pre}.block.0", x, cin, cin, 3, 1, wname="weight")
    y = prelu(P, f"{pre}.block.1", y, cin)
    y = eq_conv(P, f"{pre}.block.2", y, cin, cout, 3, 1, wname="weight")
    y = prelu(P, f"{pre}.block.3", y, cout)
    if down:
        y = eq_conv(P, f"{pre}.down_sample.1", smooth(y), cout, cout, 3, 1, stride=2, wname="weight")
        y = prelu(P, f"{pre}.down_sample.2", y, cout)
    return y * d_se(P, f"{pre}.se", y, cout, img) + res


def minibatch_stddev(x, group=4):
    """MiniBatchStdDev (discriminator_9_4.py:42-54)."""
    assert x.shape[0] % group == 0
    std = torch.sqrt(x.reshape(group, -1).var(dim=0) + 1e-8).mean().view(1, 1, 1, 1)
    b, _, h, w = x.shape
    return torch.cat([x, std.expand(b, -1, h, w)], dim=1)


def discriminator(P, x):
    """Discriminator.forward (discriminator_9_4.py:163-199) -> [B,1]."""
    y = eq_conv(P, "conv.0", x, 3, 64, 3, 1, wname="weight")
    y = prelu(P, "conv.1", y, 64)
    for idx, cin, cout, down, img in D_BLOCKS:
        if idx == 15:
            y = minibatch_stddev(y)
        y = d_block(P, f"conv.{idx}", y, cin, cout, down, img)
    y = y.reshape(y.shape[0], -1)
    y = eq_linear(P, "fc.0", y, 4100, 4100, wname="weight", bias_init="zeros")
    y = prelu(P, "fc.1", y, 4100)
    return eq_linear(P, "fc.2", y, 4100, 1, wname="weight", bias_init="zeros")


# ----------------------------------------------------------------------------------------------
# progan pair (generators/generator_3_progan.py, discriminators/discriminator_3_wgangp_progan.py)
# ----------------------------------------------------------------------------------------------

def progan_stages(ngf):
    """(cin, cout, stride, pad) of the five ConvT k4 stages (generator_3_progan.py:43-50)."""
    return [(None, ngf * 8, 1, 0), (ngf * 8, ngf * 4, 2, 1), (ngf * 4, ngf * 2, 2, 1),
            (ngf * 2, ngf, 2, 1), (ngf, 3, 2, 1)]


def progan_generator(P, z, randn=None, ngf=256):
    """Generator.forward (generator_3_progan.py:33-54): [ConvT k4, BN2d, PReLU(1)] x 5, Tanh."""
    x = z
    for i, (cin, cout, s, p) in enumerate(progan_stages(ngf)):
        cin = x.shape[1]
        w = P(f"main.{i}.0.weight", (cin, cout, 4, 4), "convt")
        b = P(f"main.{i}.0.bias", (cout,), "zeros")
        x = F.conv_transpose2d(x, w, b, stride=s, padding=p)
        x = bn(P, f"main.{i}.1", x, cout)
        x = F.prelu(x, P(f"main.{i}.2.weight", (1,), "prelu"))
    return torch.tanh(x)


def progan_stddev(x):
    """StandardDeviation (discriminator_3_wgangp_progan.py:7-16): batch std, eps 10e-8."""
    b, _, h, w = x.shape
    o = x - x.mean(dim=0, keepdim=True)
    o = torch.sqrt(o.pow(2.0).mean(dim=0, keepdim=False) + 10e-8).mean().view(1, 1, 1, 1)
    return torch.cat([x, o.repeat(b, 1, h, w)], 1)


def progan_d_layers(ndf, nc=3):
    """(cin, cout, k, stride, pad) of the EqualizedConv2d stack (discriminator_3_wgangp_progan.py:35-66);
    None marks StandardDeviation."""
    return [(nc, ndf, 1, 1, 0), (ndf, ndf, 3, 1, 1), (ndf, ndf, 3, 2, 1), (ndf, 2 * ndf, 3, 1, 1),
            (2 * ndf, 2 * ndf, 3, 2, 1), (2 * ndf, 4 * ndf, 3, 1, 1), (4 * ndf, 4 * ndf, 3, 2, 1),
            (4 * ndf, 8 * ndf, 3, 1, 1), (8 * ndf, 8 * ndf, 3, 2, 1), None, (8 * ndf + 1, 8 * ndf, 3, 1, 1),
            (8 * ndf, 8 * ndf, 4, 1, 0), (8 * ndf, 1, 1, 1, 0)]


def progan_discriminator(P, x, ndf=64):
    """Discriminator.forward (discriminator_3_wgangp_progan.py:31-70): zero-padded
    EqualizedConv2d (input scaled by sqrt(2)/sqrt(k*k*cin), :22,28-29), single-slope PReLU."""
    idx = 0
    layers = progan_d_layers(ndf)
    for j, l in enumerate(layers):
        if l is None:
            x = progan_stddev(x)
            idx += 1
            continue
        cin, cout, k, s, p = l
        w = P(f"main.{idx}.conv.weight", (cout, cin, k, k))
        b = P(f"main.{idx}.bias", (cout,))
        scale = math.sqrt(2) / math.sqrt(k * k * cin)
        x = F.conv2d(x * scale, w, None, stride=s, padding=p) + b.view(1, cout, 1, 1)
        idx += 1
        if j < len(layers) - 1:
            x = F.prelu(x, P(f"main.{idx}.weight", (1,), "prelu"))
            idx += 1
    return x.view(x.shape[0], -1)


# ----------------------------------------------------------------------------------------------
# WGAN-GP steps (train/wgangp.py)
# ----------------------------------------------------------------------------------------------

class WGANGP:
    """The oracle counterpart of ``train/wgangp.py:Train``: one D-step and one G-step.

    ``draw`` supplies randomness in the reference's order: ``draw.randn(shape)`` for z and the
    in-forward noise, ``draw.rand(shape)`` for eps.
    """

    def __init__(self, GP: Params, DP: Params, nz=256, gen=None, disc=None):
        self.GP, self.DP, self.nz = GP, DP, nz
        self.gen = gen or generator          # (P, z, randn) -> images
        self.disc = disc or discriminator    # (P, x) -> [B, 1]
        # torch.optim.AdamW defaults (weight_decay 0.01, eps 1e-8) as wgangp.py:17-18
        self.g_order = list(GP.t.keys())
        self.d_order = list(DP.t.keys())
        self.opt_G = torch.optim.AdamW([GP.t[k] for k in self.g_order], lr=1e-4, betas=(0.5, 0.999))
        self.opt_D = torch.optim.AdamW([DP.t[k] for k in self.d_order], lr=4e-4, betas=(0.5, 0.999))

    def generator_trainstep(self, b, draw):
        """wgangp.py:20-27."""
        self.opt_G.zero_grad()
        z = draw.randn((b, self.nz, 1, 1))
        gen = self.gen(self.GP, z, draw.randn)
        g_loss = -torch.mean(self.disc(self.DP, gen))
        g_loss.backward()
        self.opt_G.step()
        return gen, g_loss

    def gradient_penalty(self, x_real, x_fake, b, draw, center=1.0):
        """wgangp.py:34-54."""
        eps = draw.rand((b,)).view(b, 1, 1, 1)
        xi = ((1 - eps) * x_real + eps * x_fake).detach().requires_grad_()
        d_out = self.disc(self.DP, xi)
        g = torch.autograd.grad(d_out.sum(), xi, create_graph=True, retain_graph=True, only_inputs=True)[0]
        g2 = g.pow(2).view(b, -1).sum(1)
        return (g2.sqrt() - center).pow(2).mean()

    def discriminator_trainstep(self, images, b, draw):
        """wgangp.py:56-71."""
        self.opt_D.zero_grad()
        z = draw.randn((b, self.nz, 1, 1))
        with torch.no_grad():
            gen = self.gen(self.GP, z, draw.randn)
        gen.requires_grad_()
        real_loss = -torch.mean(self.disc(self.DP, images))
        real_loss.backward()
        fake_loss = torch.mean(self.disc(self.DP, gen))
        fake_loss.backward()
        gp = 10 * self.gradient_penalty(images, gen, b, draw)
        gp.backward()
        self.opt_D.step()
        return real_loss, fake_loss, gp


class WGANLazyR2(WGANGP):
    """The oracle counterpart of ``train/wganlazygpR2.py:Train`` with the optimizers of
    ``train/trainunits.py:18-19`` (Adam, G lr 1e-4 betas (0.5, 0.99), D lr 4e-4 betas (0.0, 0.99)).
    Follows the reference's call sequence literally: separate real / fake passes, one backward per
    term (gradients accumulate)."""

    def __init__(self, GP: Params, DP: Params, nz=256, gen=None, disc=None):
        super().__init__(GP, DP, nz, gen, disc)
        self.opt_G = torch.optim.Adam([GP.t[k] for k in self.g_order], lr=1e-4, betas=(0.5, 0.99))
        self.opt_D = torch.optim.Adam([DP.t[k] for k in self.d_order], lr=4e-4, betas=(0.0, 0.99))

    def compute_grad2(self, d_out, x_in):
        """wganlazygpR2.py:37-46."""
        g = torch.autograd.grad(d_out.sum(), x_in, create_graph=True, retain_graph=True, only_inputs=True)[0]
        return g.pow(2).view(x_in.shape[0], -1).sum(1)

    def discriminator_trainstep(self, images, b, idx, draw):
        """wganlazygpR2.py:48-77."""
        self.opt_D.zero_grad()
        z = draw.randn((b, self.nz, 1, 1))
        with torch.no_grad():
            gen = self.gen(self.GP, z, draw.randn)
        gen.requires_grad_()
        images = images.detach().requires_grad_()
        reg = idx % 5 == 0
        pred_r = self.disc(self.DP, images)
        real_loss = -torch.mean(pred_r)
        r1 = torch.zeros(1)
        real_loss.backward(retain_graph=reg)
        if reg:
            r1 = 5 * self.compute_grad2(pred_r, images).mean()
            r1.backward()
        pred_f = self.disc(self.DP, gen)
        fake_loss = torch.mean(pred_f)
        r2 = torch.zeros(1)
        fake_loss.backward(retain_graph=reg)
        if reg:
            r2 = 5 * self.compute_grad2(pred_f, gen).mean()
            r2.backward()
        gp = torch.zeros(1)
        if reg:
            gp = 10 * self.gradient_penalty(images, gen, b, draw) * 5
            gp.backward()
        self.opt_D.step()
        return real_loss, fake_loss, gp, r1, r2


# ----------------------------------------------------------------------------------------------
# Vanilla pair + BCE trainer (config 1: generators/generator_1.py, discriminators/discriminator_1.py,
# train/gan.py)
# ----------------------------------------------------------------------------------------------

def vanilla_generator(P, z, randn=None, image=(3, 64, 64)):
    """generator_1.py:16-29: Linear z->256, LeakyReLU(0.2), Linear 256->512, LeakyReLU(0.2),
    Linear 512->3*64*64, Tanh, viewed as [B, 3, 64, 64]."""
    x = z.reshape(z.shape[0], -1)
    dims = [x.shape[1], 256, 512, image[0] * image[1] * image[2]]
    for j, i in enumerate((0, 2, 4)):
        x = F.linear(x, P(f"generator.{i}.weight", (dims[j + 1], dims[j])), P(f"generator.{i}.bias", (dims[j + 1],)))
        x = F.leaky_relu(x, 0.2) if i < 4 else torch.tanh(x)
    return x.view(z.shape[0], *image)


def vanilla_discriminator(P, x):
    """discriminator_1.py:14-25: Linear 12288->256, LeakyReLU(0.2), Linear 256->64, LeakyReLU(0.2),
    Linear 64->1, Sigmoid."""
    h = x.reshape(x.shape[0], -1)
    dims = [h.shape[1], 256, 64, 1]
    for j, i in enumerate((0, 2, 4)):
        h = F.linear(h, P(f"discriminator.{i}.weight", (dims[j + 1], dims[j])),
                     P(f"discriminator.{i}.bias", (dims[j + 1],)))
        h = F.leaky_relu(h, 0.2) if i < 4 else torch.sigmoid(h)
    return h


class GAN(WGANGP):
    """The oracle counterpart of ``train/gan.py:Train`` (BCE with noisy labels) with the Adam
    optimizers of ``train/trainunits.py:18-19``."""

    def __init__(self, GP: Params, DP: Params, nz=256):
        super().__init__(GP, DP, nz, vanilla_generator, vanilla_discriminator)
        self.opt_G = torch.optim.Adam([GP.t[k] for k in self.g_order], lr=1e-4, betas=(0.5, 0.99))
        self.opt_D = torch.optim.Adam([DP.t[k] for k in self.d_order], lr=4e-4, betas=(0.0, 0.99))

    def generator_trainstep(self, b, draw):
        """gan.py:26-35: targets 0.95 + 0.05 U[0,1)."""
        valid = 0.95 + 0.05 * draw.rand((b, 1))
        self.opt_G.zero_grad()
        z = draw.randn((b, self.nz, 1, 1))
        gen = self.gen(self.GP, z)
        g_loss = F.binary_cross_entropy(self.disc(self.DP, gen), valid)
        g_loss.backward()
        self.opt_G.step()
        return gen, g_loss

    def discriminator_trainstep(self, images, b, draw):
        """gan.py:37-53: real targets 0.95 + 0.05 U, fake targets 0.05 U (drawn in that order),
        then z."""
        valid = 0.95 + 0.05 * draw.rand((b, 1))
        fake = 0.0 + 0.05 * draw.rand((b, 1))
        z = draw.randn((b, self.nz, 1, 1))
        self.opt_D.zero_grad()
        with torch.no_grad():
            gen = self.gen(self.GP, z)
        real_loss = F.binary_cross_entropy(self.disc(self.DP, images), valid)
        real_loss.backward()
        fake_loss = F.binary_cross_entropy(self.disc(self.DP, gen), fake)
        fake_loss.backward()
        self.opt_D.step()
        return real_loss, fake_loss


class Draw:
    """Randomness replayed from one CPU generator in call order (the reference's global-RNG order)."""

    def __init__(self, seed):
        self.g = torch.Generator().manual_seed(seed)
        self.log = []

    def randn(self, shape):
        self.log.append(("randn", tuple(shape)))
        return torch.randn(shape, generator=self.g)

    def rand(self, shape):
        self.log.append(("rand", tuple(shape)))
        return torch.rand(shape, generator=self.g)


def params_from_plan(plan_params, seed):
    """Params filled by the documented rule (oracle/params.py) in the reference's order."""
    from oracle.params import fill_value
    t = {}
    for i, (name, kind, shape) in enumerate(plan_params):
        v = fill_value(seed, i, kind, tuple(shape))
        if v is None:  # frozen Smooth kernel
            continue
        t[name] = v.requires_grad_(True)
    return Params(t)
