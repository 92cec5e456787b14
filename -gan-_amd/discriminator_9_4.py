"""Drop-in D9_4 critic (reference: discriminators/discriminator_9_4.py).

Surface kept: ``Discriminator()``, ``forward(x[B,3,64,64]) -> [B,1]`` (NCHW), module and
parameter names/order, init distributions, ``B % 4 == 0`` assertion of MiniBatchStdDev, and full
support for ``torch.autograd.grad(..., create_graph=True)`` followed by ``backward()`` (the
gradient penalty of train/wgangp.py:34-54): every operator used here is closed under
differentiation (see ops.py).

Underneath: CNHW activations, MFMA implicit-GEMM convs (replication padding folded into the
gather, stride 2 included), PReLU kernels with first/second derivatives, Smooth /
bicubic-downsample / adaptive-pool as tap-table resamples (DownSample's smooth+bicubic is one
composed table), MiniBatchStdDev and the SE sigmoid as kernels.  ``forward`` runs the layer
program of critic.py (explicit backward and gradient-penalty double backward);
``forward_autograd`` keeps the per-layer autograd formulation for A/B tests.
"""
from __future__ import annotations

import math
from typing import List

import torch
from torch import nn

from . import critic, ops
from .ops import prelu


class EqualizedWeight(nn.Module):
    """discriminator_9_4.py:9-17 (parameter spelled ``weight`` here)."""

    def __init__(self, shape: List[int]):
        super().__init__()
        self.shape = shape
        self.c = 1.0 / math.sqrt(math.prod(shape[1:]))
        self.weight = nn.Parameter(nn.init.normal_(torch.empty(shape), mean=0, std=1))

    def forward(self):
        return self.weight * self.c


class EqualizedLinear(nn.Module):
    """discriminator_9_4.py:20-27 (bias initialised as N(0,1) * bias, i.e. zeros by default)."""

    def __init__(self, in_planes: int, out_planes: int, bias: float = 0.0):
        super().__init__()
        self.weight = EqualizedWeight([out_planes, in_planes])
        self.bias = nn.Parameter(nn.init.normal_(torch.empty(out_planes), mean=0, std=1) * bias)

    def forward(self, x):
        return ops.linear(x, self.weight.weight, self.bias, self.weight.c)


class EqualizedConv2d(nn.Module):
    """ReplicationPad2d(padding) + strided conv (discriminator_9_4.py:30-40); CNHW forward."""

    def __init__(self, in_features: int, out_features: int, kernel_size: int, padding: int = 0, stride: int = 1):
        super().__init__()
        self.stride = stride
        self.weight = EqualizedWeight([out_features, in_features, kernel_size, kernel_size])
        self.bias = nn.Parameter(nn.init.normal_(torch.empty(out_features), mean=0, std=1))
        self.padding = padding
        self.k = kernel_size

    def forward(self, x):
        C, B, H, W = x.shape
        geo = ops.conv_geo(B, C, H, W, self.bias.shape[0], self.k, self.stride, self.padding)
        return ops.conv2d(x, self.weight.weight, self.bias, geo, self.weight.c)


class MiniBatchStdDev(nn.Module):
    """discriminator_9_4.py:42-54.  The reference groups NCHW ``x.view(4, -1)``: element
    (b, c, h, w) belongs to group b // (B/4); in CNHW that is ``x.view(C, 4, B/4, H, W)``."""

    segments = 1     # set by Discriminator.forward: the batch is this many independent mini-batches

    def __init__(self, group_size: int = 4):
        super().__init__()
        self.group_size = group_size

    def forward(self, x):
        C, B, H, W = x.shape
        S = self.segments
        assert B % S == 0 and (B // S) % self.group_size == 0
        Bs = B // S
        g = x.reshape(C, S, self.group_size, Bs // self.group_size, H, W)
        std = torch.sqrt(g.var(dim=2) + 1e-8).mean(dim=(0, 2, 3, 4))          # one value per segment
        feat = std.view(1, S, 1, 1, 1).expand(1, S, Bs, H, W).reshape(1, B, H, W)
        return torch.cat([x, feat], dim=0)


class Smooth(nn.Module):
    """discriminator_9_4.py:56-72 (frozen kernel kept for checkpoint compatibility)."""

    def __init__(self):
        super().__init__()
        k = torch.tensor([[[[1.0, 2.0, 1.0], [2.0, 4.0, 2.0], [1.0, 2.0, 1.0]]]])
        self.kernel = nn.Parameter(k / k.sum(), requires_grad=False)

    def forward(self, x):
        return ops.resample(x, "smooth")


class DownSample(nn.Module):
    """Smooth then bicubic to H//2 (discriminator_9_4.py:74-81), one composed tap table."""

    def __init__(self):
        super().__init__()
        self.smooth = Smooth()

    def forward(self, x):
        return ops.resample(x, "smooth_down2")


class SEBlock_conv(nn.Module):
    """pool5 -> 2x (3x3 conv, no pad, PReLU) -> fc -> PReLU -> fc -> sigmoid (discriminator_9_4.py:83-109)."""

    def __init__(self, in_planes: int):
        super().__init__()
        self.convs = nn.Sequential(EqualizedConv2d(in_planes, in_planes, 3), nn.PReLU(in_planes),
                                   EqualizedConv2d(in_planes, in_planes, 3), nn.PReLU(in_planes))
        self.fcs = nn.Sequential(EqualizedLinear(in_planes, in_planes), nn.PReLU(in_planes))
        self.fc_out = EqualizedLinear(in_planes, in_planes)

    def forward(self, x):
        assert x.shape[2] >= 8
        c = self.convs
        t = prelu(c[0](ops.resample(x, "pool5")), c[1].weight)
        t = prelu(c[2](t), c[3].weight)
        z = prelu(self.fcs[0](ops.plane_mean(t)), self.fcs[1].weight)
        return ops.sigmoid(self.fc_out(z))


class SEBlock_fc(nn.Module):
    """GAP -> 2x (fc, PReLU) -> fc -> sigmoid (discriminator_9_4.py:111-128)."""

    def __init__(self, in_planes: int):
        super().__init__()
        self.fcs = nn.Sequential(EqualizedLinear(in_planes, in_planes), nn.PReLU(in_planes),
                                 EqualizedLinear(in_planes, in_planes), nn.PReLU(in_planes))
        self.fc_out = EqualizedLinear(in_planes, in_planes)

    def forward(self, x):
        f = self.fcs
        z = prelu(f[0](ops.plane_mean(x)), f[1].weight)
        z = prelu(f[2](z), f[3].weight)
        return ops.sigmoid(self.fc_out(z))


class DiscriminatorBlock(nn.Module):
    """Residual block with optional Smooth + stride-2 downsampling (discriminator_9_4.py:131-161)."""

    def __init__(self, in_features, out_features, downsample, image_size):
        super().__init__()
        self.residual = nn.Sequential()
        self.block = nn.Sequential(
            EqualizedConv2d(in_features, in_features, kernel_size=3, padding=1), nn.PReLU(in_features),
            EqualizedConv2d(in_features, out_features, kernel_size=3, padding=1), nn.PReLU(out_features))
        self.se = SEBlock_conv(out_features) if image_size > 4 else SEBlock_fc(out_features)
        self.down_sample = nn.Sequential()
        self.downsample = downsample
        if downsample:
            self.residual = nn.Sequential(DownSample(), EqualizedConv2d(in_features, out_features, kernel_size=1))
            self.down_sample = nn.Sequential(
                Smooth(), EqualizedConv2d(out_features, out_features, kernel_size=3, padding=1, stride=2),
                nn.PReLU(out_features))

    def forward(self, x):
        if self.downsample:
            res = self.residual[1](self.residual[0](x))
        else:
            res = x
        b = self.block
        y = prelu(b[0](x), b[1].weight)
        y = prelu(b[2](y), b[3].weight)
        if self.downsample:
            d = self.down_sample
            y = prelu(d[1](d[0](y)), d[2].weight)
        return ops.scale_add(y, self.se(y), res)


class Discriminator(nn.Module):
    """D9_4: x [B,3,64,64] -> [B,1] (discriminator_9_4.py:163-199)."""

    def __init__(self):
        super().__init__()
        f = 64
        self.conv = nn.Sequential(
            EqualizedConv2d(3, f, 3, 1), nn.PReLU(f),
            DiscriminatorBlock(f, f, False, 64), DiscriminatorBlock(f, f, False, 64),
            DiscriminatorBlock(f, 2 * f, True, 32),
            DiscriminatorBlock(2 * f, 2 * f, False, 32), DiscriminatorBlock(2 * f, 2 * f, False, 32),
            DiscriminatorBlock(2 * f, 4 * f, True, 16),
            DiscriminatorBlock(4 * f, 4 * f, False, 16), DiscriminatorBlock(4 * f, 4 * f, False, 16),
            DiscriminatorBlock(4 * f, 8 * f, True, 8),
            DiscriminatorBlock(8 * f, 8 * f, False, 8), DiscriminatorBlock(8 * f, 8 * f, False, 8),
            DiscriminatorBlock(8 * f, 16 * f, True, 4),
            MiniBatchStdDev(),
            DiscriminatorBlock(16 * f + 1, 16 * f + 1, False, 4), DiscriminatorBlock(16 * f + 1, 16 * f + 1, False, 4),
            DiscriminatorBlock(16 * f + 1, 16 * f + 1, True, 2),
        )
        n = 2 * 2 * (16 * f + 1)
        self.fc = nn.Sequential(EqualizedLinear(n, n), nn.PReLU(n), EqualizedLinear(n, 1))

    def forward(self, input, segments: int = 1):
        """``segments`` > 1: ``input`` is that many independent mini-batches stacked along the
        batch (the critic step runs its real and fake batches as one pass); every layer is
        per-sample except MiniBatchStdDev, which is computed per segment, so the output equals
        the per-segment calls concatenated.

        Runs the critic as the explicit layer program of critic.py: one autograd node whose
        backward (and, under create_graph, double backward) are kernel sweeps over the saved
        activations -- no per-layer autograd graph.

        Parameter gradients: the sweeps accumulate them straight into each parameter's ``.grad``
        (the optimizer's flat gradient buffer) and hand autograd None for the parameters, which
        is what ``loss.backward()`` -- the only way train/wgangp.py:20-71 uses them -- needs.  A
        consequence: ``torch.autograd.grad(loss, D.parameters())`` finds no gradient (it raises
        "appears to not have been used in the graph", or returns None with allow_unused=True;
        the result is ALSO added to ``.grad``), and hooks registered on D's parameters do not
        fire.  Use ``forward_autograd`` for per-parameter autograd semantics."""
        return critic.critic_forward(self, input, segments)

    def forward_autograd(self, input, segments: int = 1):
        """The same forward as per-layer autograd Functions (ops.py), every one of them closed
        under differentiation: the A/B reference for the explicit program in the GPU tests."""
        B = input.shape[0]
        for mod in self.conv:
            if isinstance(mod, MiniBatchStdDev):
                mod.segments = segments
        x = ops.nchw_to_cnhw(input)
        for mod in self.conv:
            x = prelu(x, mod.weight) if isinstance(mod, nn.PReLU) else mod(x)
        C, _, H, W = x.shape
        z = x.permute(0, 2, 3, 1).reshape(C * H * W, B)         # NCHW .view(B, -1) feature order
        z = prelu(self.fc[0](z), self.fc[1].weight)
        return self.fc[2](z).t()
