"""Golden fixtures of the lazy-GP + R1/R2 trainer (train/wganlazygpR2.py), made by importing the
REFERENCE in this container (run here only; /root/reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_lazy.py

Same recipe as make_golden.py (no-op ``tqdm.tk`` / ``torchvision`` stubs, parameters overwritten
by the documented rule of oracle/params.py, randomness injected by seeding the global CPU
generator right before each call).  Records, at B=4:
  * one critic step with the regularisers (idx % 5 == 0, wganlazygpR2.py:48-77): the five
    losses (real, fake, gp, R1, R2), per-tensor gradient summaries, Adam deltas (lr 4e-4,
    betas (0.0, 0.99), trainunits.py:19);
  * one critic step without them (idx = 1);
  * one generator step (wganlazygpR2.py:17-24): loss, gradient summaries, Adam deltas (lr 1e-4,
    betas (0.5, 0.99), trainunits.py:18).
No reference source is copied: only numbers are written.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (installs the stubs, imports the reference models)

import torch  # noqa: E402
from train import wganlazygpR2  # noqa: E402


def main():
    t0 = time.time()
    B = 4
    out = {}
    for idx, img_seed, rng_seed in ((0, 500, 501), (1, 510, 511)):
        G, D, _, _ = mg.build_pair()
        tr = wganlazygpR2.Train([0] * 10, torch.device("cpu"), 1, 256, G, "G13_5", D, "D9_4")
        images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(img_seed)).requires_grad_()
        before = [p.detach().clone() for p in D.parameters()]
        torch.manual_seed(rng_seed)
        losses = tr.discriminator_trainstep(images, B, idx)
        gt, has = mg.grad_table(D)
        dt = mg.delta_table(D, before, 4e-4)
        out[f"d{idx}_losses"] = np.asarray([float(v.detach().reshape(-1)[0]) for v in losses])
        out[f"d{idx}_grads"], out[f"d{idx}_has_grad"], out[f"d{idx}_deltas"] = gt, has, dt
        print(f"d step idx={idx}", out[f"d{idx}_losses"], time.time() - t0, flush=True)
        del G, D, tr, before

    G, D, _, _ = mg.build_pair()
    tr = wganlazygpR2.Train([0] * 10, torch.device("cpu"), 1, 256, G, "G13_5", D, "D9_4")
    before = [p.detach().clone() for p in G.parameters()]
    torch.manual_seed(601)
    gen_imgs, g_loss = tr.generator_trainstep(B)
    gt, has = mg.grad_table(G)
    dt = mg.delta_table(G, before, 1e-4)
    out["g_loss"] = np.asarray([float(g_loss)])
    out["g_grads"], out["g_has_grad"], out["g_deltas"] = gt.astype(np.float32), has, dt.astype(np.float32)
    print("g step", float(g_loss), time.time() - t0, flush=True)
    np.savez_compressed(os.path.join(HERE, "lazy_b4.npz"), **out)
    print("done", time.time() - t0)


if __name__ == "__main__":
    main()
