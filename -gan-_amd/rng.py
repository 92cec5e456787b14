"""Sources of the hot path's randomness: z, eps and the in-forward StyleConv noise.

The reference draws all three from the unseeded global RNG in a fixed call order
(train/wgangp.py:22,35,58; generator_13_5.py:265).  ``DeviceRNG`` draws on the GPU (the
production path); ``ReplayRNG`` reproduces a seeded CPU draw sequence in the reference's order
and shapes so results can be compared with the golden fixtures element for element.
"""
from __future__ import annotations

import torch


class DeviceRNG:
    def __init__(self, device, seed: int | None = None):
        self.device = torch.device(device)
        if seed is not None:
            torch.cuda.manual_seed(seed)

    def randn(self, shape):
        return torch.randn(shape, device=self.device)

    def rand(self, shape):
        return torch.rand(shape, device=self.device)

    def noise(self, shape_nchw):
        B, C, H, W = shape_nchw
        return torch.randn((C, B, H, W), device=self.device)

    def noise_bulk(self, numel):
        """All of one generator forward's noise in one draw (generator_13_5._NoiseHub)."""
        return torch.randn(numel, device=self.device)


class ReplayRNG:
    """Draws from one CPU generator in call order, returns device tensors (CNHW for noise)."""

    def __init__(self, seed: int, device):
        self.g = torch.Generator().manual_seed(seed)
        self.device = torch.device(device)
        self.log = []

    def randn(self, shape):
        self.log.append(("randn", tuple(shape)))
        return torch.randn(shape, generator=self.g).to(self.device)

    def rand(self, shape):
        self.log.append(("rand", tuple(shape)))
        return torch.rand(shape, generator=self.g).to(self.device)

    def noise(self, shape_nchw):
        self.log.append(("randn", tuple(shape_nchw)))
        return torch.randn(shape_nchw, generator=self.g).permute(1, 0, 2, 3).contiguous().to(self.device)
