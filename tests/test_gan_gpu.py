"""GPU parity of the vanilla pair and its BCE trainer (config 1: generator_1.py, discriminator_1.py,
train/gan.py) against the reference's fixture (tests/golden/make_golden_gan.py), B=16.

Randomness (label noise, z) is replayed from the same seeded CPU generator in the reference's draw
order.  Bars: module outputs and losses at 1e-5 norm-relative (one fp32 GEMM chain, K <= 12288);
gradient summaries at 1e-4 of each tensor's largest element; the first Adam step moves each weight
by ~lr * sign(g), so update norms at 1e-3."""
import json
import os

import numpy as np
import pytest
import torch

from oracle.params import fill_module, tensor_summary
from tests._util import GOLDEN, fixture, rel_err, summary_check

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def pp():
    with open(os.path.join(GOLDEN, "plan_gan.json")) as f:
        return json.load(f)


def _pair(pp):
    import gan_amd
    from gan_amd.discriminator_1 import Discriminator
    from gan_amd.generator_1 import Generator
    G = Generator(pp["nz"], (3, 64, 64))
    D = Discriminator((3, 64, 64))
    assert [n for n, _, _ in pp["g_params"]] == [n for n, _ in G.named_parameters()]
    assert [n for n, _, _ in pp["d_params"]] == [n for n, _ in D.named_parameters()]
    fill_module(G, pp["g_seed"])
    fill_module(D, pp["d_seed"])
    return gan_amd, G.to(DEV), D.to(DEV)


def _rows(mod, before=None, lr=1.0):
    rows, deltas = [], []
    for i, (_, p) in enumerate(mod.named_parameters()):
        rows.append(tensor_summary(p.grad))
        if before is not None:
            deltas.append(tensor_summary((p.detach() - before[i]) / lr)[1])
    return rows, np.asarray(deltas)


def test_gan_forward(pp):
    fx = fixture("gan_b16.npz")
    _, G, D = _pair(pp)
    x = torch.randn(16, 3, 64, 64, generator=torch.Generator().manual_seed(int(fx["d_fwd_x_seed"][0])))
    with torch.no_grad():
        g = G(torch.from_numpy(fx["g_fwd_z"]).to(DEV))
        d = D(x.to(DEV))
    torch.cuda.synchronize()
    assert tuple(g.shape) == (4, 3, 64, 64) and tuple(d.shape) == (16, 1)
    assert rel_err(g.cpu().numpy(), fx["g_fwd_out"]) < 1e-5
    assert rel_err(d.cpu().numpy(), fx["d_fwd_out"]) < 1e-5


def test_gan_d_step(pp):
    from gan_amd.gan import Train
    fx = fixture("gan_b16.npz")
    gan, G, D = _pair(pp)
    tr = Train([], DEV, 1, pp["nz"], G, "G1", D, "D1", rng=gan.ReplayRNG(711, DEV))
    images = torch.randn(16, 3, 64, 64, generator=torch.Generator().manual_seed(710)).to(DEV)
    before = [p.detach().clone() for p in D.parameters()]
    losses = [float(v.detach()) for v in tr.discriminator_trainstep(images, 16)]
    torch.cuda.synchronize()
    assert [k for k, _ in tr.rng.log] == ["rand", "rand", "randn"]
    assert rel_err(losses, fx["d_losses"]) < 1e-5, (losses, fx["d_losses"])
    rows, dl = _rows(D, before, 4e-4)
    err, where = summary_check(rows, fx["d_grads"])
    assert err < 1e-4, (err, where)
    assert rel_err(dl, fx["d_deltas"][:, 1]) < 1e-3


def test_gan_g_step(pp):
    from gan_amd.gan import Train
    fx = fixture("gan_b16.npz")
    gan, G, D = _pair(pp)
    tr = Train([], DEV, 1, pp["nz"], G, "G1", D, "D1", rng=gan.ReplayRNG(721, DEV))
    before = [p.detach().clone() for p in G.parameters()]
    d_before = [p.detach().clone() for p in D.parameters()]
    gen, g_loss = tr.generator_trainstep(16)
    torch.cuda.synchronize()
    assert rel_err([float(g_loss)], fx["g_loss"]) < 1e-5
    assert rel_err(tensor_summary(gen), fx["g_gen"]) < 1e-5
    rows, dl = _rows(G, before, 1e-4)
    err, where = summary_check(rows, fx["g_grads"])
    assert err < 1e-4, (err, where)
    assert rel_err(dl, fx["g_deltas"][:, 1]) < 1e-3
    assert all(torch.equal(a, b) for a, b in zip(d_before, D.parameters()))   # the critic is not updated
