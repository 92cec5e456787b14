"""Deterministic parameter fill rule shared by the golden-fixture generator and the tests.

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg. The product path never imports anything under ``oracle/``.

The reference initialises its parameters from the unseeded global RNG at module construction
(``generators/generator_13_5.py:8-16,19-38,257-258``, ``discriminators/discriminator_9_4.py:9-40``),
so no two runs agree.  For parity we overwrite every parameter with a documented, per-tensor-seeded
rule that depends only on (seed, index in ``named_parameters()`` order, kind, shape).  The kind of
a parameter is derived from the class of the module that owns it and its attribute name, so the
rule is identical for the reference modules and for our drop-in modules (same class names).
"""
from __future__ import annotations

import math

import torch

# (owner class name, attribute name) -> kind
_KIND = {
    ("EqualizedWeight", "weights"): "eqw",      # G13_5 spells it 'weights' (generator_13_5.py:13)
    ("EqualizedWeight", "weight"): "eqw",       # D9_4 spells it 'weight' (discriminator_9_4.py:14)
    ("EqualizedLinear", "bias"): "eqb",
    ("EqualizedConv2d", "bias"): "eqb",
    ("BatchNorm1d", "weight"): "bn_w",
    ("BatchNorm1d", "bias"): "bn_b",
    ("BatchNorm2d", "weight"): "bn_w",
    ("BatchNorm2d", "bias"): "bn_b",
    ("PReLU", "weight"): "prelu",
    ("ConvTranspose2d", "weight"): "convt_w",
    ("ConvTranspose2d", "bias"): "convt_b",
    ("StyleConv", "scale_noise"): "noise_scale",
    ("StyleConv", "bias"): "style_bias",        # a no-op in the reference (generator_13_5.py:263)
    ("Smooth", "kernel"): "smooth",             # frozen binomial kernel, requires_grad=False
    ("Conv2d", "weight"): "eqw",                # progan D: nn.Conv2d inside EqualizedConv2d, N(0,1) init
                                                # (discriminator_3_wgangp_progan.py:20-24)
    ("Linear", "weight"): "lin_w",              # vanilla pair: plain nn.Linear (generator_1.py:18-22,
    ("Linear", "bias"): "lin_b",                # discriminator_1.py:15-19)
}


def param_kinds(module: torch.nn.Module):
    """Return ``[(name, kind, shape)]`` in ``named_parameters()`` order."""
    owner = {}
    for mname, mod in module.named_modules():
        for pname, p in mod.named_parameters(recurse=False):
            full = f"{mname}.{pname}" if mname else pname
            owner[full] = (type(mod).__name__, pname)
    out = []
    for name, p in module.named_parameters():
        key = owner[name]
        if key not in _KIND:
            raise KeyError(f"unclassified parameter {name} owned by {key}")
        out.append((name, _KIND[key], tuple(p.shape)))
    return out


def fill_value(seed: int, index: int, kind: str, shape) -> torch.Tensor | None:
    """The value of parameter number ``index`` (CPU fp32), or None to leave it unchanged."""
    if kind == "smooth":
        return None
    g = torch.Generator().manual_seed(seed * 1_000_003 + index)
    n = torch.randn(shape, generator=g, dtype=torch.float32)
    if kind == "eqw":
        return n
    if kind == "eqb":
        return 0.5 * n
    if kind == "bn_w":
        return 1.0 + 0.1 * n
    if kind == "bn_b":
        return 0.1 * n
    if kind == "prelu":
        return 0.25 + 0.05 * n
    if kind == "convt_w":
        fan_in = shape[1] * shape[2] * shape[3]
        return n / math.sqrt(fan_in)
    if kind == "convt_b":
        return 0.1 * n
    if kind == "noise_scale":
        return 0.25 + 0.02 * n
    if kind == "style_bias":
        return n
    if kind == "lin_w":      # N(0, 1/fan_in): keeps the vanilla critic's sigmoid out of saturation
        return n / math.sqrt(shape[1])
    if kind == "lin_b":
        return 0.1 * n
    raise KeyError(kind)


@torch.no_grad()
def fill_module(module: torch.nn.Module, seed: int):
    """Overwrite every parameter of ``module`` with the fill rule (works for CPU or GPU modules)."""
    kinds = param_kinds(module)
    params = dict(module.named_parameters())
    for i, (name, kind, shape) in enumerate(kinds):
        v = fill_value(seed, i, kind, shape)
        if v is not None:
            params[name].copy_(v)
    return kinds


def summary_indices(numel: int, k: int = 8):
    """Fixed sample positions used by grad/delta summaries."""
    return [((j * 2654435761) + 12345) % numel for j in range(k)]


def tensor_summary(t: torch.Tensor, k: int = 8):
    """[sum, l2, absmax, s_0..s_{k-1}] of a tensor (float64 math, CPU)."""
    f = t.detach().reshape(-1).to("cpu", torch.float64)
    idx = summary_indices(f.numel(), k)
    return [float(f.sum()), float(f.norm()), float(f.abs().max())] + [float(f[i]) for i in idx]
