"""CPU: the drop-in modules expose exactly the reference's parameters (names, order, shapes,
kinds), and the resampling tap tables equal the reference's torch operators."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import gan_amd
from gan_amd import tables
from oracle.params import param_kinds
from tests._util import plan


@pytest.fixture(scope="module")
def P():
    return plan()


def test_generator_parameters(P):
    G = gan_amd.Generator(256)
    got = [[n, k, list(s)] for n, k, s in param_kinds(G)]
    assert got == P["g_params"]
    assert [n for n, _ in G.named_buffers()] == P["g_buffers"]
    assert sum(p.numel() for p in G.parameters()) == 362387256


def test_discriminator_parameters(P):
    D = gan_amd.Discriminator()
    got = [[n, k, list(s)] for n, k, s in param_kinds(D)]
    assert got == P["d_params"]
    assert sum(p.numel() for p in D.parameters()) == 152712222


def _apply_1d(kind, x):
    m = torch.from_numpy(tables.operator_1d(kind, x.shape[-1]))
    return torch.einsum("oh,pw,bchw->bcop", m, m, x.double())


@pytest.mark.parametrize("n", [4, 8, 16, 32, 64])
def test_resample_tables_match_torch(n):
    g = torch.Generator().manual_seed(n)
    x = torch.randn(2, 3, n, n, generator=g)
    k = torch.tensor([[1.0, 2.0, 1.0], [2.0, 4.0, 2.0], [1.0, 2.0, 1.0]]) / 16
    sm = lambda t: F.conv2d(F.pad(t.reshape(-1, 1, *t.shape[2:]), (1, 1, 1, 1), mode="replicate"),
                            k.view(1, 1, 3, 3)).reshape(t.shape)
    up = F.interpolate(x, scale_factor=2, mode="bicubic", align_corners=False)
    assert torch.allclose(_apply_1d("smooth", x).float(), sm(x), atol=1e-6)
    assert torch.allclose(_apply_1d("up2", x).float(), up, atol=1e-5)
    assert torch.allclose(_apply_1d("up2_smooth", x).float(), sm(up), atol=1e-5)
    if n >= 4:
        dn = F.interpolate(sm(x), (n // 2, n // 2), mode="bicubic", align_corners=False)
        assert torch.allclose(_apply_1d("smooth_down2", x).float(), dn, atol=1e-5)
    if n >= 8:
        assert torch.allclose(_apply_1d("pool5", x).float(), F.adaptive_avg_pool2d(x, 5), atol=1e-6)


def test_ell_roundtrip():
    m = tables.operator_1d("up2_smooth", 8)
    idx, w = tables.ell(m)
    dense = np.zeros_like(m)
    for o in range(m.shape[0]):
        for j in range(idx.shape[1]):
            dense[o, idx[o, j]] += w[o, j]
    assert np.allclose(dense, m, atol=1e-7)


def test_progan_plan():
    """Drop-in progan pair (config 5): module tree, parameter names / kinds / shapes / order and
    buffers equal the reference's (tests/golden/plan_progan.json, made by importing it)."""
    import json
    import os
    import gan_amd
    from oracle.params import param_kinds
    from tests._util import GOLDEN
    with open(os.path.join(GOLDEN, "plan_progan.json")) as f:
        pp = json.load(f)
    G = gan_amd.generator_3_progan.Generator(1, 256, pp["ngf"], 3)
    D = gan_amd.discriminator_3_wgangp_progan.Discriminator(1, pp["ndf"], 3)
    assert [[n, k, list(s)] for n, k, s in param_kinds(G)] == pp["g_params"]
    assert [[n, k, list(s)] for n, k, s in param_kinds(D)] == pp["d_params"]
    assert [n for n, _ in G.named_buffers()] == pp["g_buffers"]
