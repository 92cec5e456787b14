"""Golden fixtures of the vanilla pair and its BCE trainer (config 1: generators/generator_1.py,
discriminators/discriminator_1.py, train/gan.py), made by importing the REFERENCE in this container
(run here only; /root/reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_gan.py

Same recipe as make_golden.py (no-op ``tqdm.tk`` / ``torchvision`` stubs, parameters overwritten by
the documented rule of oracle/params.py, randomness injected by seeding the global CPU generator
right before each call).  Records (``gan_b16.npz`` + ``plan_gan.json``):
  * the parameter plan of both nets (names, kinds, shapes);
  * G forward at B=4 (full output) and D forward at B=16;
  * one critic step at B=16 (gan.py:37-53): real / fake BCE losses, per-tensor gradient summaries,
    Adam deltas (lr 4e-4, betas (0.0, 0.99), trainunits.py:19);
  * one generator step at B=16 (gan.py:26-35): loss, output summary, gradient summaries, Adam
    deltas (lr 1e-4, betas (0.5, 0.99), trainunits.py:18).
No reference source is copied: only numbers are written.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (installs the stubs, puts the reference on sys.path)

import torch  # noqa: E402
from discriminators.discriminator_1 import Discriminator  # noqa: E402
from generators.generator_1 import Generator  # noqa: E402
from train import gan  # noqa: E402

from oracle.params import fill_module  # noqa: E402

G_SEED, D_SEED = 11, 12
NZ, B = 256, 16


def build_pair():
    G = Generator(NZ, (3, 64, 64))
    D = Discriminator((3, 64, 64))
    return G, D, fill_module(G, G_SEED), fill_module(D, D_SEED)


def main():
    t0 = time.time()
    G, D, gk, dk = build_pair()
    plan = {"torch": torch.__version__, "g_seed": G_SEED, "d_seed": D_SEED, "nz": NZ, "batch": B,
            "g_params": [[n, k, list(s)] for n, k, s in gk], "d_params": [[n, k, list(s)] for n, k, s in dk]}
    out = {}
    z = torch.randn(4, NZ, 1, 1, generator=torch.Generator().manual_seed(700))
    x = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(701))
    with torch.no_grad():
        out["g_fwd_z"], out["g_fwd_out"] = z.numpy(), G(z).numpy()
        out["d_fwd_x_seed"], out["d_fwd_out"] = np.asarray([701]), D(x).numpy()

    G, D, _, _ = build_pair()
    tr = gan.Train([0] * 10, torch.device("cpu"), 1, NZ, G, "G1", D, "D1")
    images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(710))
    before = [p.detach().clone() for p in D.parameters()]
    torch.manual_seed(711)
    real_loss, fake_loss = tr.discriminator_trainstep(images, B)
    gt, has = mg.grad_table(D)
    out["d_losses"] = np.asarray([float(real_loss), float(fake_loss)])
    out["d_grads"], out["d_has_grad"], out["d_deltas"] = gt, has, mg.delta_table(D, before, 4e-4)
    print("d step", out["d_losses"], time.time() - t0, flush=True)

    G, D, _, _ = build_pair()
    tr = gan.Train([0] * 10, torch.device("cpu"), 1, NZ, G, "G1", D, "D1")
    before = [p.detach().clone() for p in G.parameters()]
    torch.manual_seed(721)
    gen_imgs, g_loss = tr.generator_trainstep(B)
    gt, has = mg.grad_table(G)
    out["g_loss"] = np.asarray([float(g_loss)])
    out["g_gen"] = np.asarray(mg.tensor_summary(gen_imgs))
    out["g_grads"], out["g_has_grad"], out["g_deltas"] = gt, has, mg.delta_table(G, before, 1e-4)
    print("g step", float(g_loss), time.time() - t0, flush=True)

    np.savez_compressed(os.path.join(HERE, "gan_b16.npz"), **out)
    with open(os.path.join(HERE, "plan_gan.json"), "w") as f:
        json.dump(plan, f)
    print("done", time.time() - t0)


if __name__ == "__main__":
    main()
