"""Golden fixtures of the progan pair under the WGAN-GP trainer (config 5 of BASELINE.json:
generators/generator_3_progan.py with ngf=256, discriminators/discriminator_3_wgangp_progan.py with
ndf=64, train/wgangp.py), made by importing the REFERENCE in this container (run here only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_progan.py

Same recipe as make_golden.py (stubs for the GUI/IO-only imports, parameters overwritten by the
rule of oracle/params.py, randomness injected by seeding the global CPU generator).  Records at
B=4: G and D outputs, one critic step and one generator step (losses, gradient summaries, AdamW
deltas), and the parameter plans.  No reference source is copied: only numbers are written.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (installs the stubs and the reference path)

import torch  # noqa: E402
from generators.generator_3_progan import Generator  # noqa: E402
from discriminators.discriminator_3_wgangp_progan import Discriminator  # noqa: E402
from train import wgangp  # noqa: E402

from oracle.params import fill_module, tensor_summary  # noqa: E402

G_SEED, D_SEED, NGF, NDF = 3, 4, 256, 64


def pair():
    G = Generator(ngpu=1, nz=256, ngf=NGF, nc=3)
    D = Discriminator(ngpu=1, ndf=NDF, nc=3)
    return G, D, fill_module(G, G_SEED), fill_module(D, D_SEED)


def main():
    t0 = time.time()
    B = 4
    G, D, gk, dk = pair()
    plan = {"g_seed": G_SEED, "d_seed": D_SEED, "ngf": NGF, "ndf": NDF,
            "g_params": [[n, k, list(s)] for n, k, s in gk], "d_params": [[n, k, list(s)] for n, k, s in dk],
            "g_buffers": [n for n, _ in G.named_buffers()]}
    out = {}
    z = torch.randn(B, 256, 1, 1, generator=torch.Generator().manual_seed(700))
    x = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(701))
    with torch.no_grad():
        out["z"], out["g_out"] = z.numpy(), G(z).numpy()
        out["x"], out["d_out"] = x.numpy(), D(x).numpy()
    out["g_buffers"] = np.asarray([[float(b.double().sum()), float(b.double().norm())] for _, b in G.named_buffers()])

    G, D, _, _ = pair()
    tr = wgangp.Train([0] * 10, torch.device("cpu"), 1, 256, G, "G3_progan", D, "D3_progan")
    images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(710))
    before = [p.detach().clone() for p in D.parameters()]
    torch.manual_seed(711)
    losses = tr.discriminator_trainstep(images, B)
    out["d_losses"] = np.asarray([float(v) for v in losses])
    out["d_grads"], out["d_has_grad"] = mg.grad_table(D)
    out["d_deltas"] = mg.delta_table(D, before, 4e-4)
    print("d step", out["d_losses"], time.time() - t0, flush=True)

    G, D, _, _ = pair()
    tr = wgangp.Train([0] * 10, torch.device("cpu"), 1, 256, G, "G3_progan", D, "D3_progan")
    torch.manual_seed(721)
    gen, g_loss = tr.generator_trainstep(B)
    out["g_loss"] = np.asarray([float(g_loss)])
    out["gen"] = np.asarray(tensor_summary(gen))
    out["g_grads"], out["g_has_grad"] = mg.grad_table(G)
    print("g step", float(g_loss), time.time() - t0, flush=True)
    np.savez_compressed(os.path.join(HERE, "progan_b4.npz"), **out)
    with open(os.path.join(HERE, "plan_progan.json"), "w") as f:
        json.dump(plan, f)
    print("done", time.time() - t0)


if __name__ == "__main__":
    main()
