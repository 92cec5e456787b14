"""Drop-in G13_5 generator (reference: generators/generator_13_5.py).

Surface kept from the reference: ``Generator(z_dim, planes=48)``, ``forward(z[B,256,1,1]) ->
[B,3,64,64]`` (NCHW), module/attribute names (so ``named_parameters()`` / ``state_dict()`` keys
and their order are identical), parameter init distributions and construction order (so a
seeded construction reproduces the reference's weights), train-mode BatchNorm running-stat
updates, the no-op StyleConv bias (generator_13_5.py:263), and one N(0,1) noise draw per noisy
StyleConv per forward in the reference's call order.

What differs is underneath: activations are CNHW, every conv / convT / linear is an MFMA
implicit GEMM from libganamd.so, the weight-modulated conv runs batch-shared (x*s, conv, *d)
instead of materialising B per-sample weight sets, BatchNorm is fused with the PReLU that
follows it, and Smooth / bicubic / adaptive pooling are tap-table resamples.
"""
from __future__ import annotations

import math
import os
from typing import List

import torch
from torch import nn

from . import ops
from .ops import bn_act, prelu

# A/B: GANAMD_SHORTCUT_BRANCH=0 runs a root BasicBlock's shortcut after rir_3 instead of beside it
SHORTCUT_BRANCH = [os.environ.get("GANAMD_SHORTCUT_BRANCH", "1") != "0"]


def _normal(shape):
    return nn.Parameter(nn.init.normal_(torch.empty(shape), mean=0, std=1))


class EqualizedWeight(nn.Module):
    """N(0,1) parameter used at runtime times 1/sqrt(fan_in) (generator_13_5.py:8-16)."""

    def __init__(self, shape: List[int]):
        super().__init__()
        self.shape = shape
        self.scale = 1.0 / math.sqrt(math.prod(shape[1:]))
        self.weights = _normal(shape)

    def forward(self):
        return self.weights * self.scale


class EqualizedLinear(nn.Module):
    """generator_13_5.py:19-26; forward on feature-major [in, B]."""

    def __init__(self, in_planes: int, out_planes: int):
        super().__init__()
        self.weight = EqualizedWeight([out_planes, in_planes])
        self.bias = _normal(out_planes)

    def forward(self, x):
        return ops.linear(x, self.weight.weights, self.bias, self.weight.scale)


class EqualizedConv2d(nn.Module):
    """ReplicationPad2d((k-1)//2) + conv (generator_13_5.py:29-38); forward on CNHW."""

    def __init__(self, in_planes: int, out_planes: int, kernel_size: int):
        super().__init__()
        self.weight = EqualizedWeight([out_planes, in_planes, kernel_size, kernel_size])
        self.bias = _normal(out_planes)
        self.k = kernel_size

    def forward(self, x):
        C, B, H, W = x.shape
        geo = ops.conv_geo(B, C, H, W, self.bias.shape[0], self.k, 1, (self.k - 1) // 2)
        return ops.conv2d(x, self.weight.weights, self.bias, geo, self.weight.scale)


def _conv_bn_act(conv, bn, act, x):
    return bn_act(conv(x), bn, act)


def _lin_bn_act(lin, bn, act, x):
    # no-grad forwards (the critic steps' fake batches): linear + BatchNorm1d + PReLU in one launch
    if ops.linear_bn_act_ok(x, lin.weight.weights):
        return ops.linear_bn_act(x, lin.weight.weights, lin.bias, lin.weight.scale, bn, act)
    return bn_act(lin(x), bn, act)


def _mix(feas, att):
    """sum_m att[m] * feas[m] (att: [M, C, B]) -- one fused kernel (ops.mix)."""
    return ops.mix(feas, att)


def _sk_mix(attn, feas):
    """SK mixing of the branches by their attention (generator_13_5.py:80-89, 165-170, 196-202).  With
    autograd on two branches of an SKAttention_conv the pool of the branch sum and the branches'
    pass-through to the mix are one op (ops.pool_sum_fanout): the sum is never stored and each branch's
    gradient (mix + pool) is written in one pass."""
    if len(feas) == 2 and isinstance(attn, SKAttention_conv) and torch.is_grad_enabled() and \
            (feas[0].requires_grad or feas[1].requires_grad):
        t, f0, f1 = ops.pool_sum_fanout(feas[0], feas[1], "pool5")
        return _mix([f0, f1], attn.head(t))
    return _mix(feas, attn(feas))


def _heads(attn, z):
    if not torch.is_grad_enabled():   # each head's last linear writes its slice of [M, C, B] (no stack copy)
        out = torch.empty((attn.M,) + tuple(z.shape), device=z.device, dtype=torch.float32)
        for i in range(attn.M):
            sub = getattr(attn, f"fc_sub_{i}")
            v = _lin_bn_act(sub[0], sub[1], sub[2], z)
            ops.linear(v, sub[3].weight.weights, sub[3].bias, sub[3].weight.scale, out=out[i])
        return ops.softmax_m(out)
    vecs = []
    for i in range(attn.M):
        sub = getattr(attn, f"fc_sub_{i}")
        v = _lin_bn_act(sub[0], sub[1], sub[2], z)
        vecs.append(sub[3](v))
    return ops.softmax_m(torch.stack(vecs, 0))          # [M, C, B], softmax over M


class SKAttention_conv(nn.Module):
    """Selective-kernel attention on maps >= 8x8 (generator_13_5.py:41-89)."""

    def __init__(self, planes: int, m: int):
        super().__init__()
        mods = []
        for _ in range(2):
            mods += [EqualizedConv2d(planes, planes, 3), nn.BatchNorm2d(planes), nn.PReLU(planes)]
        self.conv_main = nn.Sequential(*mods)
        self.fc_main = nn.Sequential(EqualizedLinear(planes, planes), nn.BatchNorm1d(planes), nn.PReLU(planes))
        self.M = m
        for i in range(m):
            setattr(self, f"fc_sub_{i}", nn.Sequential(EqualizedLinear(planes, planes), nn.BatchNorm1d(planes),
                                                      nn.PReLU(planes), EqualizedLinear(planes, planes)))

    def forward(self, feas):
        if len(feas) == 2 and not torch.is_grad_enabled():   # pool of the branch sum, the sum never stored
            assert feas[0].shape[2] >= 8
            t = ops.resample_sum(feas[0], feas[1], "pool5")
        else:
            u = feas[0]
            for f in feas[1:]:
                u = u + f
            assert u.shape[2] >= 8
            t = ops.resample(u, "pool5")
        return self.head(t)

    def head(self, t):
        """The attention from the pooled branch sum t [C, B, 5, 5]."""
        cm = self.conv_main
        t = _conv_bn_act(cm[0], cm[1], cm[2], t)
        t = _conv_bn_act(cm[3], cm[4], cm[5], t)
        z = _lin_bn_act(self.fc_main[0], self.fc_main[1], self.fc_main[2], ops.plane_mean(t))
        return _heads(self, z)


class SKAttention_fc(nn.Module):
    """Selective-kernel attention on 4x4 maps (generator_13_5.py:92-131)."""

    def __init__(self, planes: int, m: int):
        super().__init__()
        mods = []
        for _ in range(2):
            mods += [EqualizedLinear(planes, planes), nn.BatchNorm1d(planes), nn.PReLU(planes)]
        self.fc_main = nn.Sequential(*mods)
        self.M = m
        for i in range(m):
            setattr(self, f"fc_sub_{i}", nn.Sequential(EqualizedLinear(planes, planes), nn.BatchNorm1d(planes),
                                                      nn.PReLU(planes), EqualizedLinear(planes, planes)))

    def forward(self, feas):
        u = feas[0]
        for f in feas[1:]:
            u = u + f
        fm = self.fc_main
        z = _lin_bn_act(fm[0], fm[1], fm[2], ops.plane_mean(u))
        z = _lin_bn_act(fm[3], fm[4], fm[5], z)
        return _heads(self, z)


class Smooth(nn.Module):
    """Binomial 3x3 blur, replication pad (generator_13_5.py:134-150).  The frozen kernel is
    kept as a parameter for checkpoint compatibility; the forward uses the equal tap table."""

    def __init__(self):
        super().__init__()
        k = torch.tensor([[[[1.0, 2.0, 1.0], [2.0, 4.0, 2.0], [1.0, 2.0, 1.0]]]])
        self.kernel = nn.Parameter(k / k.sum(), requires_grad=False)

    def forward(self, x):
        return ops.resample(x, "smooth")


class SKConvT(nn.Module):
    """ConvT(k4,s2,p1)+BN+PReLU  ||  bicubic x2 + Smooth, SK-mixed (generator_13_5.py:153-170)."""

    def __init__(self, planes: int):
        super().__init__()
        self.convT = nn.ConvTranspose2d(planes, planes, kernel_size=4, stride=2, padding=1)
        self.bn = nn.BatchNorm2d(planes)
        self.activation_convT = nn.PReLU(planes)
        self.smooth = Smooth()
        self.sk_attention = SKAttention_conv(planes, 2)

    def forward(self, x):
        C, B, H, W = x.shape
        geo = ops.convT_geo(B, C, H, W, C, 4, 2, 1)
        a = bn_act(ops.conv2d(x, self.convT.weight, self.convT.bias, geo, 1.0), self.bn, self.activation_convT)
        b = ops.resample(x, "up2_smooth")
        return _sk_mix(self.sk_attention, [a, b])


class SKConv(nn.Module):
    """k3 || k5 dense conv + BN + PReLU, SK-mixed (generator_13_5.py:173-202)."""

    def __init__(self, in_planes: int, out_planes: int, m: int, image_size: int):
        super().__init__()
        assert m > 0
        self.M = m
        for i in range(m):
            setattr(self, f"conv_{i}", EqualizedConv2d(in_planes, out_planes, kernel_size=3 + i * 2))
            setattr(self, f"BatchNorm_{i}", nn.BatchNorm2d(out_planes))
            setattr(self, f"nonlinear_{i}", nn.PReLU(out_planes))
        self.sk_attention = (SKAttention_conv if image_size > 4 else SKAttention_fc)(out_planes, m)

    def forward(self, x):
        feas = [_conv_bn_act(getattr(self, f"conv_{i}"), getattr(self, f"BatchNorm_{i}"),
                             getattr(self, f"nonlinear_{i}"), x) for i in range(self.M)]
        return _sk_mix(self.sk_attention, feas)


class MappingNetwork(nn.Module):
    """[EqLinear, BN1d, PReLU] x n (generator_13_5.py:205-216)."""

    def __init__(self, planes: int, n_layers: int):
        super().__init__()
        mods = []
        for _ in range(n_layers):
            mods += [EqualizedLinear(planes, planes), nn.BatchNorm1d(planes), nn.PReLU(planes)]
        self.net = nn.Sequential(*mods)

    def forward(self, z):
        n = self.net
        for i in range(0, len(n), 3):
            z = _lin_bn_act(n[i], n[i + 1], n[i + 2], z)
        return z


class Conv2dWeightModulate(nn.Module):
    """StyleGAN2 modulated/demodulated conv (generator_13_5.py:219-248), batch-shared form."""

    def __init__(self, d_latent: int, in_planes: int, out_planes: int, kernel_size: int, demodulate: bool = True,
                 eps: float = 1e-8):
        super().__init__()
        self.to_style = nn.Sequential(MappingNetwork(d_latent, 1), EqualizedLinear(d_latent, in_planes),
                                      nn.BatchNorm1d(in_planes))
        self.out_planes = out_planes
        self.demodulate = demodulate
        self.weight = EqualizedWeight([out_planes, in_planes, kernel_size, kernel_size])
        self.eps = eps
        self.k = kernel_size
        assert demodulate, "G13_5 always demodulates"

    _bank_sd = None      # (s, d) handed over by the Generator's style bank for this forward

    def forward(self, x, w, noise=None, noise_scale=None, act=None):
        """``noise``/``noise_scale``/``act``: the owning StyleConv's noise and the PReLU that follows
        it (slopes); without autograd they run in the GEMM epilogue, with autograd as separate ops."""
        C, B, H, W = x.shape
        geo = ops.conv_geo(B, C, H, W, self.out_planes, self.k, 1, (self.k - 1) // 2)
        if self._bank_sd is not None:
            s, d = self._bank_sd
        else:
            s = _lin_bn_act(self.to_style[1], self.to_style[2], None, self.to_style[0](w))   # [Cin, B]
            d = ops.demod(s, self.weight.weights, self.weight.scale)
        if not torch.is_grad_enabled():
            return ops.modconv_fused(x, s, d, self.weight.weights, geo, self.weight.scale, noise, noise_scale, act)
        y = ops.ModConv.apply(x, s, d, self.weight.weights, geo, self.weight.scale, noise_scale, noise)
        return y if act is None else prelu(y, act)


class StyleConv(nn.Module):
    """Modulated conv (+ per-channel-scaled N(0,1) noise); the bias is a no-op exactly as in the
    reference (generator_13_5.py:251-266: ``x + self.bias[...]`` is never assigned)."""

    def __init__(self, d_latent: int, in_planes: int, out_planes: int, kernel_size: int, use_noise: bool = False):
        super().__init__()
        self.conv = Conv2dWeightModulate(d_latent, in_planes, out_planes, kernel_size=kernel_size)
        self.use_noise = use_noise
        if use_noise:
            self.scale_noise = nn.Parameter(nn.init.uniform_(torch.empty(out_planes), a=0.2, b=0.3))
        self.bias = _normal(out_planes)
        self._hub = None

    def forward(self, x, w, act=None):
        """``act``: slopes of the PReLU applied to this conv's output by the caller (fused)."""
        noise = None
        if self.use_noise:
            C, B = self.conv.out_planes, x.shape[1]
            noise = self._hub.noise((B, C, x.shape[2], x.shape[3]))   # CNHW draw of an NCHW-shaped randn
        return self.conv(x, w, noise, self.scale_noise if self.use_noise else None, act)


class SKStyleConv(nn.Module):
    """k3 || k5 StyleConv + noise + PReLU, SK-mixed (generator_13_5.py:269-295)."""

    def __init__(self, d_latent: int, in_planes: int, out_planes: int, m: int, image_size: int, use_noise: bool):
        super().__init__()
        assert m > 0
        self.M = m
        for i in range(m):
            setattr(self, f"conv_{i}", StyleConv(d_latent, in_planes, out_planes, kernel_size=3 + i * 2,
                                                 use_noise=use_noise))
            setattr(self, f"nonlinear_{i}", nn.PReLU(out_planes))
        self.sk_attention = (SKAttention_conv if image_size > 4 else SKAttention_fc)(out_planes, m)

    def forward(self, x, w):
        # the k3 / k5 branches run in order on the current stream: the stream-level parallelism
        # is ResnetInit's four StyleBlocks (ops.Branches does not nest)
        feas = [getattr(self, f"conv_{i}")(x, w, getattr(self, f"nonlinear_{i}").weight) for i in range(self.M)]
        return _sk_mix(self.sk_attention, feas)


class StyleBlock(nn.Module):
    """1x1 StyleConv -> PReLU -> (k StyleConv | SKStyleConv) -> 3x3 StyleConv (generator_13_5.py:298-322)."""

    def __init__(self, d_latent: int, last_planes: int, in_planes: int, out_planes: int, dense_depth: int,
                 kernel_size: int, m: int, image_size: int):
        super().__init__()
        assert m > 0
        self.conv1 = StyleConv(d_latent, last_planes, in_planes, kernel_size=1)
        self.activation1 = nn.PReLU(in_planes)
        self.m = m
        if m == 1:
            self.conv2 = StyleConv(d_latent, in_planes, in_planes, kernel_size, True)
            self.activation2 = nn.PReLU(in_planes)
        else:
            self.skconv = SKStyleConv(d_latent, in_planes, in_planes, m, image_size, True)
        self.conv3 = StyleConv(d_latent, in_planes, out_planes + dense_depth, kernel_size=3)

    def forward(self, x, w):
        x = self.conv1(x, w, self.activation1.weight)
        if self.m == 1:
            x = self.conv2(x, w, self.activation2.weight)
        else:
            x = self.skconv(x, w)
        return self.conv3(x, w)


class ResnetInit(nn.Module):
    """Dual-path (residual / transient) cross block (generator_13_5.py:325-349)."""

    def __init__(self, d_latent: int, last_planes: int, in_planes: int, out_planes: int, dense_depth: int,
                 kernel_size: int, m: int, image_size: int):
        super().__init__()
        args = (d_latent, last_planes, in_planes, out_planes)
        self.residual = StyleBlock(*args, dense_depth, kernel_size, m, image_size)
        self.transient = StyleBlock(*args, 0, kernel_size, m, image_size)
        self.residual_across = StyleBlock(*args, 0, kernel_size, m, image_size)
        self.transient_across = StyleBlock(*args, dense_depth, kernel_size, m, image_size)
        self.activation_residual = nn.PReLU(out_planes + dense_depth)
        self.activation_transient = nn.PReLU(out_planes)

    def forward(self, x, w, extra=None):
        """``extra = (block, x_e)``: one more independent StyleBlock -- a root BasicBlock's shortcut --
        run as a fifth branch; its output is returned third."""
        x_res, x_tr = x
        # the four StyleBlocks are independent: on a GPU each runs on its own HIP stream (their
        # hundreds of small, launch-bound kernels overlap; a captured graph keeps the branches),
        # issued in the reference's order so the noise draws keep theirs (the shortcut's draws
        # follow the four blocks', as in the reference's BasicBlock)
        with ops.Branches(x_res.device, 4 + (extra is not None)) as br:
            br.share(x_res, x_tr, None if extra is None else extra[1])
            with br[0]:
                r_r = br.out(0, self.residual(x_res, w))
            with br[1]:
                r_t = br.out(1, self.residual_across(x_res, w))
            with br[2]:
                t_t = br.out(2, self.transient(x_tr, w))
            with br[3]:
                t_r = br.out(3, self.transient_across(x_tr, w))
            if extra is not None:
                with br[4]:
                    e = br.out(4, extra[0](extra[1], w))
        out = (ops.add_prelu(r_r, t_r, self.activation_residual.weight),
               ops.add_prelu(r_t, t_t, self.activation_transient.weight))
        return out if extra is None else out + (e,)


class SEBlock_conv(nn.Module):
    """Channel gate from pooled 5x5 maps (generator_13_5.py:352-382); returns [C, B]."""

    def __init__(self, in_planes: int):
        super().__init__()
        mods = []
        for _ in range(2):
            mods += [EqualizedConv2d(in_planes, in_planes, 3), nn.BatchNorm2d(in_planes), nn.PReLU(in_planes)]
        self.convs = nn.Sequential(*mods)
        self.fcs = nn.Sequential(EqualizedLinear(in_planes, in_planes), nn.BatchNorm1d(in_planes), nn.PReLU(in_planes))
        self.fc_out = EqualizedLinear(in_planes, in_planes)
        self.fc_bn = nn.BatchNorm1d(in_planes)

    def forward(self, x):
        assert x.shape[2] >= 8
        c = self.convs
        t = _conv_bn_act(c[0], c[1], c[2], ops.resample(x, "pool5"))
        t = _conv_bn_act(c[3], c[4], c[5], t)
        z = _lin_bn_act(self.fcs[0], self.fcs[1], self.fcs[2], ops.plane_mean(t))
        return ops.sigmoid(_lin_bn_act(self.fc_out, self.fc_bn, None, z))


class SEBlock_fc(nn.Module):
    """Channel gate on 4x4 maps (generator_13_5.py:385-405); returns [C, B]."""

    def __init__(self, in_planes: int):
        super().__init__()
        mods = []
        for _ in range(2):
            mods += [EqualizedLinear(in_planes, in_planes), nn.BatchNorm1d(in_planes), nn.PReLU(in_planes)]
        self.fcs = nn.Sequential(*mods)
        self.fc_out = EqualizedLinear(in_planes, in_planes)
        self.fc_bn = nn.BatchNorm1d(in_planes)

    def forward(self, x):
        f = self.fcs
        z = _lin_bn_act(f[0], f[1], f[2], ops.plane_mean(x))
        z = _lin_bn_act(f[3], f[4], f[5], z)
        return ops.sigmoid(_lin_bn_act(self.fc_out, self.fc_bn, None, z))


class BasicBlock(nn.Module):
    """Dual-path-network block with channel split/concat (generator_13_5.py:408-467)."""

    def get_out_planes(self):
        if self.is_unify or self.root:
            return 2 * self.out_planes + 2 * self.dense_depth
        return self.last_planes + self.dense_depth

    def __init__(self, d_latent: int, last_planes: int, in_planes: int, out_planes: int, dense_depth: int, root: bool,
                 is_unify: bool, m: int, image_size: int):
        super().__init__()
        self.root = root
        self.last_planes = last_planes
        self.out_planes = out_planes
        self.dense_depth = dense_depth
        self.is_unify = is_unify
        if is_unify:
            self.unify = StyleBlock(d_latent, last_planes, in_planes, 2 * out_planes, dense_depth, 3, m, image_size)
            self.activation_unify = nn.PReLU(2 * out_planes + dense_depth)
            rir_last = out_planes + dense_depth
        else:
            rir_last = last_planes - out_planes
        self.rir_3 = ResnetInit(d_latent, rir_last, in_planes, out_planes, dense_depth, 3, m, image_size)
        if root:
            self.shortcut = StyleBlock(d_latent, last_planes, in_planes, 0, dense_depth, 3, m, image_size)
            self.activation_shortcut = nn.PReLU(dense_depth)
        self.se_attention_residual = (SEBlock_conv if image_size > 4 else SEBlock_fc)(out_planes)

    def forward(self, x, w):
        d = self.out_planes
        if self.is_unify:
            x = prelu(self.unify(x, w), self.activation_unify.weight)
        C = x.shape[0]
        # the channel ranges of x, one view per use: x's gradient is then ONE pass (ops.route)
        # instead of a zero-filled full-size tensor per slice plus the adds that sum them
        if self.root:
            x_a, x_c, x_tr, x_skip, x_sc = ops.route(x, [(0, d), (2 * d, C), (d, C), (0, d), (0, C)])
        else:
            x_a, x_c, x_tr, x_skip, x_tail = ops.route(x, [(0, d), (2 * d, C), (d, C), (0, d), (2 * d, C)])
        x_res = torch.cat([x_a, x_c], 0)
        if self.root and SHORTCUT_BRANCH[0]:     # the shortcut StyleBlock beside the four of rir_3
            r3, t3, sc = self.rir_3((x_res, x_tr), w, extra=(self.shortcut, x_sc))
        else:
            r3, t3 = self.rir_3((x_res, x_tr), w)
            sc = self.shortcut(x_sc, w) if self.root else None
        head_se, head, r_tail = ops.route(r3, [(0, d), (0, d), (d, r3.shape[0])])
        feas_res = ops.scale_add(head, self.se_attention_residual(head_se), x_skip)
        if self.root:
            sc = prelu(sc, self.activation_shortcut.weight)
            return torch.cat([feas_res, t3, sc, r_tail], 0)
        return torch.cat([feas_res, t3, x_tail, r_tail], 0)


class ToRGB(nn.Module):
    """generator_13_5.py:470-493 (no tanh anywhere in G13_5)."""

    def __init__(self, planes: int, m: int, image_size: int):
        super().__init__()
        assert m > 0
        self.m = m
        if m == 1:
            self.pre_conv = EqualizedConv2d(planes, planes, 3)
            self.pre_bn = nn.BatchNorm2d(planes)
            self.pre_activation = nn.PReLU(planes)
        else:
            self.skconv = SKConv(planes, planes, m, image_size)
        self.conv = EqualizedConv2d(planes, 3, kernel_size=5)
        self.bn = nn.BatchNorm2d(3)

    def forward(self, x):
        if self.m == 1:
            x = _conv_bn_act(self.pre_conv, self.pre_bn, self.pre_activation, x)
        else:
            x = self.skconv(x)
        return bn_act(self.conv(x), self.bn, None)


class Tree(nn.Module):
    """DLA-style recursive aggregation (generator_13_5.py:496-564)."""

    def get_out_planes(self):
        return self.root.get_out_planes()

    def __init__(self, d_latent: int, last_planes: int, in_planes: int, out_planes: int, dense_depth: int, level: int,
                 block_num: int, m: int, image_size: int):
        super().__init__()
        assert block_num > 0
        self.level = level
        self.block_num = block_num
        self.out_planes = out_planes
        self.dense_depth = dense_depth
        root_last = 2 * out_planes * (block_num - 1)
        cur = last_planes
        if level == 1:
            first_unify = last_planes < 2 * out_planes
        else:
            self.prev_root = BasicBlock(d_latent, last_planes, in_planes, out_planes, dense_depth, False,
                                        last_planes < 2 * out_planes, m, image_size)
            root_last += self.prev_root.get_out_planes()
            for i in reversed(range(1, level)):
                sub = Tree(d_latent, cur, in_planes, out_planes, dense_depth, i, block_num, m, image_size)
                cur = sub.get_out_planes()
                root_last += cur
                setattr(self, f"level_{i}", sub)
            first_unify = False
        for i in range(block_num):
            blk = BasicBlock(d_latent, cur, in_planes, out_planes, dense_depth, False, first_unify and i == 0, m,
                             image_size)
            cur = blk.get_out_planes()
            setattr(self, f"block_{i}", blk)
        root_last += cur
        self.root_last_planes = root_last
        self.root = BasicBlock(d_latent, root_last, in_planes * block_num, out_planes, dense_depth, True, False, m,
                               image_size)
        self.to_rgb = ToRGB(self.get_out_planes(), m, image_size)

    def forward(self, x, w, rgb):
        d2 = 2 * self.out_planes
        xs = []
        if self.level > 1:
            x_prev, x = ops.route(x, [(0, x.shape[0])] * 2)
            xs.append(self.prev_root(x_prev, w))
        for i in reversed(range(1, self.level)):
            x, rgb = getattr(self, f"level_{i}")(x, w, rgb)
            x_keep, x = ops.route(x, [(0, x.shape[0])] * 2)
            xs.append(x_keep)
        for i in range(self.block_num):
            x = getattr(self, f"block_{i}")(x, w)
            if i + 1 < self.block_num:
                x_head, x = ops.route(x, [(0, d2), (0, x.shape[0])])
                xs.append(x_head)
        xs.append(x)                            # the last block's x[:d2] and x[d2:], in order
        out = self.root(torch.cat(xs, 0), w)
        out, out_rgb = ops.route(out, [(0, out.shape[0])] * 2)
        return out, self.to_rgb(out_rgb) + rgb


class GeneratorBlock(nn.Module):
    """x2 upsampling stage (generator_13_5.py:567-583)."""

    def get_out_planes(self):
        return self.tree.get_out_planes()

    def __init__(self, d_latent: int, last_planes: int, in_planes: int, out_planes: int, dense_depth: int, level: int,
                 block_num: int, m: int, image_size: int):
        super().__init__()
        self.upsample = SKConvT(last_planes)
        self.tree = Tree(d_latent, last_planes, in_planes, out_planes, dense_depth, level, block_num, m, image_size)
        self.upsample_rgb = SKConvT(3)

    def forward(self, x, w, rgb):
        rgb = self.upsample_rgb(rgb)
        x = self.upsample(x)
        return self.tree(x, w, rgb)


class GeneratorStart(nn.Module):
    """Mapping network, 1->4 ConvT, first ToRGB and tree (generator_13_5.py:586-607)."""

    def get_out_planes(self):
        return self.tree.get_out_planes()

    def __init__(self, z_dim: int, mapping_layer: int, in_planes: int, out_planes: int, dense_depth: int, level: int,
                 block_num: int, m: int):
        super().__init__()
        self.mapping_network = MappingNetwork(z_dim, mapping_layer)
        self.convT = nn.ConvTranspose2d(z_dim, out_planes, kernel_size=4, stride=1, padding=0)
        self.bn = nn.BatchNorm2d(out_planes)
        self.activation = nn.PReLU(out_planes)
        self.to_rgb = ToRGB(out_planes, m, 4)
        self.tree = Tree(z_dim, out_planes, in_planes, out_planes // 2, dense_depth, level, block_num, m, 4)

    def forward(self, z):
        B, zd = z.shape[0], z.shape[1]
        zc = z.reshape(B, zd).t().contiguous()                   # [256, B]
        w = self.mapping_network(zc)
        hook = self.__dict__.get("_w_hook")
        if hook is not None:
            hook(w)
        geo = ops.convT_geo(B, zd, 1, 1, self.convT.out_channels, 4, 1, 0)
        x = ops.conv2d(zc.reshape(zd, B, 1, 1), self.convT.weight, self.convT.bias, geo, 1.0)
        x = bn_act(x, self.bn, self.activation)
        rgb = self.to_rgb(x)
        x, rgb = self.tree(x, w, rgb)
        return x, w, rgb


class _NoiseHub:
    """Where StyleConv gets its N(0,1) noise; a Generator-wide hook so callers can replay draws.

    A forward makes 253 noise draws (generator_13_5.py:265).  When the source can draw in bulk
    (DeviceRNG.noise_bulk) and a previous forward at the same batch recorded the draw shapes,
    the hub draws ALL of a forward's noise with one launch at its start and hands out views in
    the same order (one launch instead of 253; inside a captured graph the bulk draw is captured
    too, so every replay gets fresh noise).  Otherwise, with an indexed source
    (DeviceRNG.noise_at), draw i of the forward reads the generator's offset without advancing it
    and carries i in its counter, and the forward advances the offset once at its end: the draws
    made inside ResnetInit's parallel branch streams never race on the offset word.  A replaying
    source (ReplayRNG) keeps the per-draw path and the reference's draw order."""

    def __init__(self):
        self.source = None          # shape -> tensor: per-draw, advancing (ReplayRNG.noise)
        self.bulk_source = None     # numel -> flat N(0,1) tensor, or None (per-draw only)
        self.indexed_source = None  # (shape, i >= 1) -> tensor at the current offset, no advance
        self.advance = None         # advances the indexed source's offset (end of the forward)
        self.shapes = {}            # batch -> the draw shapes of one forward
        self._rec = None
        self._bulk = None
        self._idx = 0

    def attach(self, rng):
        """Draw from ``rng`` (DeviceRNG: bulk / indexed; ReplayRNG: per draw in call order)."""
        self.source = rng.noise
        self.bulk_source = getattr(rng, "noise_bulk", None)
        self.indexed_source = getattr(rng, "noise_at", None)
        self.advance = getattr(rng, "advance", None) if self.indexed_source is not None else None

    def begin(self, batch):
        self._rec, self._bulk, self._idx = [], None, 0
        bulk = self.bulk_source if self.source is not None else None
        shapes = self.shapes.get(batch)
        if bulk is not None and shapes:
            total = sum(C * B * H * W for B, C, H, W in shapes)
            buf = bulk(total)
            ops.branch_share(buf)       # its views are saved by ops on the branch streams
            self._bulk = (buf, list(shapes), 0, 0)

    def end(self, batch):
        if self._rec is not None:
            self.shapes[batch] = self._rec
        if self._idx and self.advance is not None:   # on the forward's stream, after the joins
            self.advance()
        self._rec, self._bulk, self._idx = None, None, 0

    def noise(self, shape_nchw):
        if self._rec is not None:
            self._rec.append(tuple(shape_nchw))
        if self._bulk is not None:
            buf, shapes, i, off = self._bulk
            if i < len(shapes) and shapes[i] == tuple(shape_nchw):
                B, C, H, W = shape_nchw
                n = C * B * H * W
                self._bulk = (buf, shapes, i + 1, off + n)
                return buf[off:off + n].view(C, B, H, W)
            self._bulk = None           # the draw sequence changed: per-draw from here on
        if self.indexed_source is not None:
            self._idx += 1
            return self.indexed_source(shape_nchw, self._idx)
        if self.source is not None:
            return self.source(shape_nchw)
        B, C, H, W = shape_nchw
        return torch.randn((C, B, H, W), device=torch.cuda.current_device())


class Generator(nn.Module):
    """G13_5: z [B,256,1,1] -> rgb [B,3,64,64] (generator_13_5.py:610-631)."""

    def __init__(self, z_dim, planes=48):
        super().__init__()
        self.block0 = GeneratorStart(z_dim, 12, planes * 8, planes * 8, planes // 8, 1, 2, 1)
        self.block1 = GeneratorBlock(z_dim, self.block0.get_out_planes(), planes * 4, planes * 4, planes // 8, 2, 2, 2,
                                     8)
        self.block2 = GeneratorBlock(z_dim, self.block1.get_out_planes(), planes * 2, planes * 2, planes // 8, 2, 2, 2,
                                     16)
        self.block3 = GeneratorBlock(z_dim, self.block2.get_out_planes(), planes * 1, planes * 1, planes // 8, 2, 2, 2,
                                     32)
        self.block4 = GeneratorBlock(z_dim, self.block3.get_out_planes(), planes * 1, planes * 1, planes // 8, 2, 2, 2,
                                     64)
        hub = _NoiseHub()
        object.__setattr__(self, "noise_hub", hub)
        for mod in self.modules():
            if isinstance(mod, StyleConv):
                object.__setattr__(mod, "_hub", hub)

    # ---- style bank (stylebank.py) ----------------------------------------------------------
    use_bank = True

    def flat_layout(self):
        """Parameter order for optim.FlatParams: the style bank's parameters first, contiguous."""
        from .stylebank import bank_param_order
        first = bank_param_order(self)
        ids = {id(p) for p in first}
        return first + [p for p in self.parameters() if id(p) not in ids]

    def _bank(self):
        if not self.use_bank:
            return None
        flat = self.__dict__.get("_flat")
        if flat is None:
            return None
        bank = self.__dict__.get("_style_bank")
        if bank is None or bank.flat is not flat or not bank.valid():
            from .stylebank import StyleBank
            try:
                bank = StyleBank(self, flat)
            except RuntimeError:
                return None
            self.__dict__["_style_bank"] = bank
        return bank

    def _run_bank(self, w):
        s_list, d_list = self.__dict__["_style_bank"](w)
        for m, s, d in zip(self.__dict__["_style_bank"].mods, s_list, d_list):
            m.__dict__["_bank_sd"] = (s, d)

    def _tracked(self):
        lst = getattr(self, "_nbt", None)
        if lst is None or (lst and lst[0].device != self.block0.bn.weight.device):
            lst = [m.num_batches_tracked for m in self.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
            object.__setattr__(self, "_nbt", lst)
        return lst

    def forward(self, x):
        if not self.training:
            raise NotImplementedError("G13_5 is only ever run in train mode (batch statistics)")
        bank = self._bank()
        self.block0.__dict__["_w_hook"] = self._run_bank if bank is not None else None
        self.noise_hub.begin(x.shape[0])
        try:
            h, w, rgb = self.block0(x)
            h, rgb = self.block1(h, w, rgb)
            h, rgb = self.block2(h, w, rgb)
            h, rgb = self.block3(h, w, rgb)
            h, rgb = self.block4(h, w, rgb)
        finally:
            self.noise_hub.end(x.shape[0])
            if bank is not None:
                for m in bank.mods:
                    m.__dict__["_bank_sd"] = None
        with torch.no_grad():
            torch._foreach_add_(self._tracked(), ops.BN_SEGMENTS[0])   # segmented: one update per segment
        return ops.cnhw_to_nchw(rgb)
