"""Golden fixture of one WGAN-GP critic step at the HEADLINE batch (B=64, config 2), made by
importing the REFERENCE in this container (run here only; /root/reference does not exist on the
GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_b64.py

Same recipe as make_golden.py (stubs, documented parameter fill, randomness injected by seeding
the global CPU generator right before the call).  The reference's critic step runs on CPU at
B=64: its generator forward is under no_grad, so the per-sample modulated weights are transient.
Records ``d_step_b64.npz``: the three losses, the critic's output on the real batch, per-sample
norms of the critic's input gradient on the real batch (d sum D(x) / dx), per-tensor gradient
summaries of the step and the AdamW deltas.  No reference source is copied: only numbers.
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
from train import wgangp  # noqa: E402

from oracle.params import summary_indices  # noqa: E402


def main():
    t0 = time.time()
    B = 64
    G, D, _, _ = mg.build_pair()
    x = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(320)).requires_grad_()
    out = D(x)
    gx, = torch.autograd.grad(out.sum(), x)
    d_out, gx_norm = out.detach().numpy(), gx.reshape(B, -1).norm(dim=1).numpy()
    gx_samples = gx.reshape(-1)[torch.as_tensor(summary_indices(gx.numel(), 64))].numpy()
    print("d fwd/input grad", time.time() - t0, flush=True)
    del out, gx

    tr = wgangp.Train([0] * 10, torch.device("cpu"), 1, 256, G, "G13_5", D, "D9_4")
    images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(330))
    before = [p.detach().clone() for p in D.parameters()]
    torch.manual_seed(331)
    real_loss, fake_loss, gp = tr.discriminator_trainstep(images, B)
    gt, has = mg.grad_table(D)
    dt = mg.delta_table(D, before, 4e-4)
    np.savez_compressed(os.path.join(HERE, "d_step_b64.npz"),
                        losses=np.asarray([float(real_loss), float(fake_loss), float(gp)]),
                        grads=gt, has_grad=has, deltas=dt, d_out=d_out, gx_norm=gx_norm, gx_samples=gx_samples)
    print("d step b64", [float(real_loss), float(fake_loss), float(gp)], time.time() - t0, flush=True)


if __name__ == "__main__":
    main()
