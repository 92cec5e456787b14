"""CPU restatement of the device RNG (csrc/rng.hip, ganamd_philox_*) -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; the product path draws on the device.

Philox4x32-10 as published by Salmon, Moraes, Dror & Shaw, "Parallel random numbers: as easy
as 1, 2, 3" (SC'11) and its Random123 reference release (the generator behind torch.randn on
CUDA/HIP): round multipliers 0xD2511F53 / 0xCD9E8D57, Weyl key bumps 0x9E3779B9 / 0xBB67AE85,
10 rounds.  Pinned by the Random123 known-answer vectors (tests/test_rng.py).  The reference
draws z / eps / noise from torch's unseeded global generator (train/wgangp.py:22,35,58;
generator_13_5.py:265), so its exact stream is not a parity target; the mapping from words to
floats below is this framework's own and is pinned bit-exact against the device.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr: np.ndarray, key: tuple[int, int]) -> np.ndarray:
    """ctr: (n, 4) uint32 counters; key: two uint32 words.  Returns (n, 4) uint32."""
    c = [ctr[:, i].astype(np.uint64) for i in range(4)]
    k0, k1 = key[0] & 0xFFFFFFFF, key[1] & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return np.stack(c, 1).astype(np.uint32)


def words(n: int, seed: int, offset: int, sub: int = 0) -> np.ndarray:
    """The first n words of a draw at stream offset `offset` (element 4g+i = word i of group g);
    `sub` is the draw index added to counter word 1 (csrc/rng.hip ganamd_philox_draw)."""
    g = np.arange((n + 3) // 4, dtype=np.uint64)
    ctr = np.stack([g & _MASK, (g >> np.uint64(32)) + np.uint64(sub), np.full_like(g, offset & 0xFFFFFFFF),
                    np.full_like(g, (offset >> 32) & 0xFFFFFFFF)], 1).astype(np.uint32)
    return philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)).reshape(-1)[:n]


def uniform(n: int, seed: int, offset: int, sub: int = 0) -> np.ndarray:
    return ((words(n, seed, offset, sub) >> 8).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)


def normal(n: int, seed: int, offset: int, sub: int = 0) -> np.ndarray:
    w = words(4 * ((n + 3) // 4), seed, offset, sub).reshape(-1, 2)
    u1 = ((w[:, 0] >> 8).astype(np.float64) + 1.0) * 2.0 ** -24
    u2 = (w[:, 1] >> 8).astype(np.float64) * 2.0 ** -24
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.stack([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)], 1).reshape(-1)
    return z[:n].astype(np.float32)
