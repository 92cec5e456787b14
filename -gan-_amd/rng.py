"""Sources of the hot path's randomness: z, eps and the in-forward StyleConv noise.

The reference draws all three from the unseeded global RNG in a fixed call order
(train/wgangp.py:22,35,58; generator_13_5.py:265).  ``DeviceRNG`` draws on the GPU (the
production path); ``ReplayRNG`` reproduces a seeded CPU draw sequence in the reference's order
and shapes so results can be compared with the golden fixtures element for element.
"""
from __future__ import annotations

import torch

from . import _lib


def _signed64(v: int) -> int:
    """A uint64 key as the int64 with the same bits (the key tensor's dtype)."""
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= 1 << 63 else v


class DeviceRNG:
    """Philox4x32-10 draws on the device (csrc/rng.hip, ganamd_philox_*).

    The stream offset is a device-resident counter that every draw advances on the stream, so
    draws issued inside a captured HIP graph are fresh on every replay.  The seed defaults to the
    device generator's seed (``torch.cuda.initial_seed()``), so ``torch.cuda.manual_seed`` -- per
    rank in data-parallel runs -- makes a run repeatable; pass ``seed=`` to be explicit.

    Consumers that may run CONCURRENTLY (on different HIP streams) must not share an offset word:
    the draw reads it and a later launch advances it, unordered across streams.  ``fork(s)`` gives
    a generator with the same key and its own word starting at ``s * 2**40`` (stream s of the
    seed), so its counters never meet this one's.  The trainers draw the generator's z and noise
    from ``fork(1)`` and the critic's eps from the base stream (the pipelined iteration replays
    the next fake batch on a side stream while the critic step draws eps, bench.py), and the
    synthetic real batches come from ``fork(2)``.  Inside one generator forward the per-draw noise
    of ResnetInit's parallel branches reads the offset without advancing it and carries the draw
    index in counter word 1 (``noise_at``); the forward advances once at its end (``advance``).
    """

    STREAM_SHIFT = 40

    def __init__(self, device, seed: int | None = None, stream: int = 0, _key=None):
        self.device = torch.device(device)
        if seed is None:
            seed = torch.cuda.initial_seed() if self.device.type == "cuda" else torch.initial_seed()
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.stream = int(stream)
        self.offset = torch.full((1,), self.stream << self.STREAM_SHIFT, dtype=torch.int64, device=self.device)
        # the Philox key in device memory (ganamd_philox_draw_keyed), shared with every fork: a
        # re-key is one in-place write that graphs captured before it see on their next replay
        self.key = _key if _key is not None else torch.full((1,), _signed64(self.seed), dtype=torch.int64,
                                                            device=self.device)
        self.log = None              # list: record (stream, offset, sub, n) of eager draws (tests)
        self._forks = {}

    def fork(self, stream: int) -> "DeviceRNG":
        """Stream ``stream`` of this seed (one per (parent, stream): the same object every call)."""
        r = self._forks.get(stream)
        if r is None:
            r = self._forks[stream] = DeviceRNG(self.device, self.seed, self.stream + stream, _key=self.key)
        return r

    def _draw(self, normal, shape, sub=0, advance=True):
        out = torch.empty(shape, dtype=torch.float32, device=self.device)
        n = out.numel()
        if n:
            if self.log is not None:
                self.log.append((self.stream, int(self.offset.item()), sub, n))
            _lib.check(_lib.LIB.ganamd_philox_draw_keyed(out.data_ptr(), n, self.key.data_ptr(), self.offset.data_ptr(),
                                                         sub, int(normal), int(advance), _lib.stream()), "philox_draw")
        return out

    def randn(self, shape):
        return self._draw(True, shape)

    def rand(self, shape):
        return self._draw(False, shape)

    def noise(self, shape_nchw):
        B, C, H, W = shape_nchw
        return self.randn((C, B, H, W))

    def noise_at(self, shape_nchw, index: int):
        """Draw ``index`` (>= 1) of a set that shares the current offset (no advance)."""
        B, C, H, W = shape_nchw
        return self._draw(True, (C, B, H, W), sub=index, advance=False)

    def advance(self):
        _lib.check(_lib.LIB.ganamd_philox_advance(self.offset.data_ptr(), _lib.stream()), "philox_advance")

    def noise_bulk(self, numel):
        """All of one generator forward's noise in one draw (generator_13_5._NoiseHub)."""
        return self.randn((numel,))

    def state(self):
        """Offsets of this generator and its forks (device tensors, cloned): restore with set_state."""
        return {s: r.offset.clone() for s, r in [(self.stream, self)] + [(f.stream, f) for f in self._forks.values()]}

    def set_seed(self, seed: int):
        """Re-key this generator and its forks (a resumed run continues the SAVED seed's sequence).
        The key is written in place on the device, so graphs captured before this draw with the new
        key from their next replay on, as the eager path does."""
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.key.fill_(_signed64(self.seed))
        for f in self._forks.values():
            f.set_seed(self.seed)

    def set_state(self, st):
        """Restore offsets saved by state() (forks missing here are created)."""
        self.offset.copy_(st[self.stream])
        for s in st:
            if s != self.stream:
                self.fork(s - self.stream)
        for f in self._forks.values():
            if f.stream in st:
                f.offset.copy_(st[f.stream])


class ReplayRNG:
    """Draws from one CPU generator in call order, returns device tensors (CNHW for noise).
    One sequence in the reference's call order: every fork is the generator itself."""

    def fork(self, stream: int) -> "ReplayRNG":
        return self

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
