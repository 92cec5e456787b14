"""Drop-in progan critic (reference: discriminators/discriminator_3_wgangp_progan.py:31-70).

Surface kept: ``Discriminator(ngpu, ndf, nc)``, ``forward(x[B,nc,64,64]) -> [B,1]``, module tree
(``main.{i}`` = EqualizedConv2d / PReLU() / StandardDeviation), parameter names and order
(``main.{i}.bias`` before ``main.{i}.conv.weight``), N(0,1) inits, and support for
``torch.autograd.grad(..., create_graph=True)`` then ``backward()`` (the gradient penalty).

Underneath: CNHW activations; EqualizedConv2d = zero-padded implicit-GEMM conv with the input
scale sqrt(2)/sqrt(k*k*cin) (:22,28-29) folded into the GEMM's alpha and the bias in its
epilogue; single-slope PReLU on the twice-differentiable PReLU kernels; StandardDeviation
(:7-16) over the batch in CNHW (per segment when the critic step stacks its real and fake
batches, as Discriminator.forward of discriminator_9_4 does).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _lib, ops
from .ops import prelu


class StandardDeviation(nn.Module):
    """discriminator_3_wgangp_progan.py:7-16 on CNHW [C, B, H, W]; ``segments`` independent batches."""

    segments = 1

    def forward(self, x):
        C, B, H, W = x.shape
        S = self.segments
        assert B % S == 0
        g = x.reshape(C, S, B // S, H, W)
        o = g - g.mean(dim=2, keepdim=True)
        std = torch.sqrt(o.pow(2.0).mean(dim=2) + 10e-8).mean(dim=(0, 2, 3))      # one value per segment
        feat = std.view(1, S, 1, 1, 1).expand(1, S, B // S, H, W).reshape(1, B, H, W)
        return torch.cat([x, feat], dim=0)


class EqualizedConv2d(nn.Module):
    """discriminator_3_wgangp_progan.py:19-29: conv(x * sqrt(2)/sqrt(k*k*cin)) + bias, zero padding."""

    def __init__(self, in_planes, out_planes, kernel_size, stride=1, padding=0, groups=1):
        super().__init__()
        assert groups == 1
        self.conv = nn.Conv2d(in_planes, out_planes, kernel_size, stride, padding, groups=groups)
        self.scale = math.sqrt(2) / math.sqrt(kernel_size * kernel_size * in_planes)
        self.bias = self.conv.bias
        self.conv.bias = None
        nn.init.normal_(self.conv.weight)
        nn.init.normal_(self.bias)

    def forward(self, x):
        C, B, H, W = x.shape
        c = self.conv
        geo = ops.conv_geo(B, C, H, W, c.out_channels, c.kernel_size[0], c.stride[0], c.padding[0], _lib.PAD_ZERO)
        return ops.conv2d(x, c.weight, self.bias, geo, self.scale)


class Discriminator(nn.Module):
    def __init__(self, ngpu, ndf, nc):
        super().__init__()
        self.ngpu = ngpu
        self.main = nn.Sequential(
            EqualizedConv2d(nc, ndf, 1, 1, 0), nn.PReLU(),
            EqualizedConv2d(ndf, ndf, 3, 1, 1), nn.PReLU(),
            EqualizedConv2d(ndf, ndf, 3, 2, 1), nn.PReLU(),
            EqualizedConv2d(ndf, ndf * 2, 3, 1, 1), nn.PReLU(),
            EqualizedConv2d(ndf * 2, ndf * 2, 3, 2, 1), nn.PReLU(),
            EqualizedConv2d(ndf * 2, ndf * 4, 3, 1, 1), nn.PReLU(),
            EqualizedConv2d(ndf * 4, ndf * 4, 3, 2, 1), nn.PReLU(),
            EqualizedConv2d(ndf * 4, ndf * 8, 3, 1, 1), nn.PReLU(),
            EqualizedConv2d(ndf * 8, ndf * 8, 3, 2, 1), nn.PReLU(),
            StandardDeviation(),
            EqualizedConv2d(ndf * 8 + 1, ndf * 8, 3, 1, 1), nn.PReLU(),
            EqualizedConv2d(ndf * 8, ndf * 8, 4, 1, 0), nn.PReLU(),
            EqualizedConv2d(ndf * 8, 1, 1, 1, 0),
        )

    def forward(self, input, segments: int = 1):
        B = input.shape[0]
        x = ops.nchw_to_cnhw(input)
        for mod in self.main:
            if isinstance(mod, nn.PReLU):
                x = prelu(x, mod.weight.expand(x.shape[0]).contiguous())
            else:
                if isinstance(mod, StandardDeviation):
                    mod.segments = segments
                x = mod(x)
        return x.reshape(1, B).t()           # [1, B, 1, 1] -> out.view(B, -1)
