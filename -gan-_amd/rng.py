"""Sources of the hot path's randomness: z, eps and the in-forward StyleConv noise.

The reference draws all three from the unseeded global RNG in a fixed call order
(train/wgangp.py:22,35,58; generator_13_5.py:265).  ``DeviceRNG`` draws on the GPU (the
production path); ``ReplayRNG`` reproduces a seeded CPU draw sequence in the reference's order
and shapes so results can be compared with the golden fixtures element for element.
"""
from __future__ import annotations

import torch

from . import _lib


class DeviceRNG:
    """Philox4x32-10 draws on the device (csrc/rng.hip, ganamd_philox_*).

    The stream offset is a device-resident counter that every draw advances on the stream, so
    draws issued inside a captured HIP graph are fresh on every replay.  The seed defaults to
    torch's initial seed, so ``torch.manual_seed`` makes a run repeatable as in the reference.
    """

    def __init__(self, device, seed: int | None = None):
        self.device = torch.device(device)
        self.seed = int(torch.initial_seed() if seed is None else seed) & 0xFFFFFFFFFFFFFFFF
        self.offset = torch.zeros(1, dtype=torch.int64, device=self.device)

    def _draw(self, fn, shape):
        out = torch.empty(shape, dtype=torch.float32, device=self.device)
        n = out.numel()
        if n:
            _lib.check(fn(out.data_ptr(), n, self.seed, self.offset.data_ptr(), _lib.stream()), fn.__name__)
        return out

    def randn(self, shape):
        return self._draw(_lib.LIB.ganamd_philox_normal, shape)

    def rand(self, shape):
        return self._draw(_lib.LIB.ganamd_philox_uniform, shape)

    def noise(self, shape_nchw):
        B, C, H, W = shape_nchw
        return self.randn((C, B, H, W))

    def noise_bulk(self, numel):
        """All of one generator forward's noise in one draw (generator_13_5._NoiseHub)."""
        return self.randn((numel,))


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
