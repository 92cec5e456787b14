"""Drop-in progan generator (reference: generators/generator_3_progan.py:33-54).

Surface kept: ``Generator(ngpu, nz, ngf, nc)``, ``forward(z[B,nz,1,1]) -> [B,3,64,64]`` (NCHW),
module tree ``main.{0..4}.{0: ConvTranspose2d, 1: BatchNorm2d, 2: PReLU()}`` + ``main.5: Tanh``,
parameter names/order, PyTorch default inits.  ``nc`` is accepted and unused, as in the
reference (the last stage is hard-wired to 3 channels, :50).

Underneath: CNHW activations; each ConvTranspose2d (k4: s1 p0 from 1x1, then s2 p1) is one
implicit-GEMM launch in transposed-gather mode (ops.conv2d with a convT geometry); BatchNorm2d
(train mode) + the single-slope PReLU are one fused kernel (ops.BNAct; the slope is broadcast
over channels and its gradient summed back by autograd).
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops


class Generator(nn.Module):
    def get_upsample(self, planes, out_planes, kernel_size, stride, padding):
        return nn.Sequential(nn.ConvTranspose2d(planes, out_planes, kernel_size=kernel_size, stride=stride,
                                                padding=padding),
                             nn.BatchNorm2d(out_planes), nn.PReLU())

    def __init__(self, ngpu, nz, ngf, nc):
        super().__init__()
        self.ngpu = ngpu
        self.main = nn.Sequential(
            self.get_upsample(nz, ngf * 8, 4, 1, 0),
            self.get_upsample(ngf * 8, ngf * 4, 4, 2, 1),
            self.get_upsample(ngf * 4, ngf * 2, 4, 2, 1),
            self.get_upsample(ngf * 2, ngf * 1, 4, 2, 1),
            self.get_upsample(ngf * 1, 3, 4, 2, 1),
            nn.Tanh(),
        )

    def forward(self, input):
        if not self.training:
            raise NotImplementedError("the progan generator is run in train mode (batch statistics)")
        x = ops.nchw_to_cnhw(input)
        for stage in list(self.main)[:-1]:
            convT, bn, act = stage
            C, B, H, W = x.shape
            cout = convT.out_channels
            geo = ops.convT_geo(B, C, H, W, cout, convT.kernel_size[0], convT.stride[0], convT.padding[0])
            y = ops.conv2d(x, convT.weight, convT.bias, geo, 1.0)
            x = ops.BNAct.apply(y, bn.weight, bn.bias, act.weight.expand(cout).contiguous(), bn.running_mean,
                                bn.running_var, bn.momentum, bn.eps)
            with torch.no_grad():
                bn.num_batches_tracked.add_(1)
        return ops.cnhw_to_nchw(torch.tanh(x))
