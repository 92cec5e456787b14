"""Tap tables for the separable resampling kernel (ganamd_resample2d).

Every fixed linear resampler on the hot path acts separably on H and W with clamped indices,
so it is a small dense 1-D matrix per axis.  We build those matrices once on the host (float64,
then stored fp32), compose them where the reference applies two in a row, and ship them as
ELL tables (K taps per output index).  The adjoint (backward) is the transposed matrix, so the
same kernel runs forward and backward and the pair is closed under differentiation, which the
critic's double backward needs.

Reference operators restated here:
  * Smooth: binomial [1,2,1]/4 per axis, ReplicationPad2d(1)  (generator_13_5.py:134-150,
    discriminator_9_4.py:56-72)
  * nn.Upsample(scale_factor=2, mode='bicubic', align_corners=False)  (generator_13_5.py:160):
    src = (dst + 0.5) * 0.5 - 0.5, 4 taps at floor(src)-1..+2 clamped to [0, H-1], A = -0.75
  * F.interpolate(size=H//2, mode='bicubic', align_corners=False)  (discriminator_9_4.py:81):
    src = 2*dst + 0.5, taps {-0.09375, 0.59375, 0.59375, -0.09375}
  * AdaptiveAvgPool2d(5): window [floor(i*H/5), ceil((i+1)*H/5))  (generator_13_5.py:44,
    discriminator_9_4.py:86)
"""
from __future__ import annotations

import math

import numpy as np
import torch

A_CUBIC = -0.75


def _cc1(x):  # |x| <= 1
    return ((A_CUBIC + 2) * x - (A_CUBIC + 3)) * x * x + 1


def _cc2(x):  # 1 < |x| < 2
    return ((A_CUBIC * x - 5 * A_CUBIC) * x + 8 * A_CUBIC) * x - 4 * A_CUBIC


def smooth_1d(n):
    m = np.zeros((n, n))
    for i in range(n):
        for a, k in enumerate((0.25, 0.5, 0.25)):
            m[i, min(max(i + a - 1, 0), n - 1)] += k
    return m


def _bicubic_1d(n_in, n_out, scale):
    m = np.zeros((n_out, n_in))
    for o in range(n_out):
        src = scale * (o + 0.5) - 0.5
        i0 = math.floor(src)
        t = src - i0
        ws = (_cc2(t + 1.0), _cc1(t), _cc1(1.0 - t), _cc2(2.0 - t))
        for a, w in enumerate(ws):
            m[o, min(max(i0 - 1 + a, 0), n_in - 1)] += w
    return m


def bicubic_up2_1d(n):
    return _bicubic_1d(n, 2 * n, 0.5)


def bicubic_down2_1d(n):
    return _bicubic_1d(n, n // 2, 2.0)


def adaptive_pool_1d(n, out):
    m = np.zeros((out, n))
    for o in range(out):
        s = (o * n) // out
        e = -((-(o + 1) * n) // out)
        m[o, s:e] = 1.0 / (e - s)
    return m


def _aa_cubic(x, a=-0.5):
    """Keys cubic with a = -0.5: the filter of torch's antialiased bicubic (as PIL's)."""
    x = abs(x)
    if x < 1.0:
        return ((a + 2) * x - (a + 3)) * x * x + 1
    if x < 2.0:
        return ((a * x - 5 * a) * x + 8 * a) * x - 4 * a
    return 0.0


def bicubic_aa_1d(n_in, n_out):
    """F.interpolate(mode='bicubic', antialias=True, align_corners=False) along one axis, the
    Resize of torchvision's tensor path (units/dataloader.py:11): for scale = n_in/n_out >= 1 the
    cubic is stretched by the scale (support 2*scale) and every row renormalised to sum 1."""
    scale = n_in / n_out
    support = 2.0 * scale if scale >= 1.0 else 2.0
    inv = 1.0 / scale if scale >= 1.0 else 1.0
    m = np.zeros((n_out, n_in))
    for o in range(n_out):
        center = scale * (o + 0.5)
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), n_in)
        w = np.asarray([_aa_cubic((j + xmin - center + 0.5) * inv) for j in range(xmax - xmin)])
        tot = w.sum()
        m[o, xmin:xmax] = w / tot if tot != 0 else w
    return m


def operator_1d(kind: str, n: int) -> np.ndarray:
    if kind == "smooth":
        return smooth_1d(n)
    if kind == "up2":
        return bicubic_up2_1d(n)
    if kind == "up2_smooth":            # SKConvT: smooth(upsample(x))
        return smooth_1d(2 * n) @ bicubic_up2_1d(n)
    if kind == "smooth_down2":          # D's DownSample: interpolate(smooth(x), H//2)
        return bicubic_down2_1d(n) @ smooth_1d(n)
    if kind == "pool5":
        return adaptive_pool_1d(n, 5)
    raise KeyError(kind)


def ell(m: np.ndarray):
    """Dense [O][I] -> (idx int32 [O][K], w float32 [O][K])."""
    rows = [np.nonzero(r)[0] for r in m]
    k = max(1, max(len(r) for r in rows))
    idx = np.zeros((m.shape[0], k), np.int32)
    w = np.zeros((m.shape[0], k), np.float32)
    for o, r in enumerate(rows):
        idx[o, :len(r)] = r
        w[o, :len(r)] = m[o, r]
    return idx, w


class Table:
    """Device tables of one separable operator on square maps, forward and adjoint."""

    def __init__(self, kind: str, n: int, device):
        m = operator_1d(kind, n)
        self.kind, self.n_in, self.n_out = kind, m.shape[1], m.shape[0]
        fi, fw = ell(m)
        ai, aw = ell(m.T.copy())
        self.fwd = (torch.from_numpy(fi).to(device), torch.from_numpy(fw).to(device), fi.shape[1])
        self.adj = (torch.from_numpy(ai).to(device), torch.from_numpy(aw).to(device), ai.shape[1])


_CACHE: dict = {}


def table(kind: str, n: int, device) -> Table:
    key = (kind, n, str(device))
    t = _CACHE.get(key)
    if t is None:
        t = _CACHE[key] = Table(kind, n, device)
    return t
