"""Golden fixture of one WGAN-GP GENERATOR step above the smallest batch (B=16), made by importing
the REFERENCE in this container (run here only; /root/reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_g16.py

Same recipe as make_golden.py (stubs, documented parameter fill, randomness injected by seeding the
global CPU generator right before the call).  train/wgangp.py:20-27 at B=16 on CPU: the
reference materialises the per-sample modulated weights (B x 178.7 M floats) and keeps them for
the backward, so B=16 is the largest batch whose generator step fits this container's memory;
the headline batch B=64 is pinned through the oracle (make_f64.py --headline), which this
fixture pins in turn.  Records ``g_step_b16.npz``: the loss, a summary of the generated images,
per-tensor gradient summaries and AdamW deltas.  No reference source is copied: only numbers.
"""
from __future__ import annotations

import os
import resource
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (installs the stubs, imports the reference models)

import torch  # noqa: E402
from train import wgangp  # noqa: E402

from oracle.params import tensor_summary  # noqa: E402

B, SEED = 16, 421


def main():
    t0 = time.time()
    G, D, _, _ = mg.build_pair()
    tr = wgangp.Train([0] * 10, torch.device("cpu"), 1, 256, G, "G13_5", D, "D9_4")
    before = [p.detach().clone() for p in G.parameters()]
    torch.manual_seed(SEED)
    gen_imgs, g_loss = tr.generator_trainstep(B)
    gt, has = mg.grad_table(G)
    dt = mg.delta_table(G, before, 1e-4)
    np.savez_compressed(os.path.join(HERE, "g_step_b16.npz"), g_loss=np.asarray([float(g_loss)]),
                        gen=np.asarray(tensor_summary(gen_imgs)), grads=gt.astype(np.float32),
                        has_grad=has, deltas=dt.astype(np.float32))
    print("g step b16", float(g_loss), f"{time.time() - t0:.0f}s",
          f"peak RSS {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20:.1f} GiB", flush=True)


if __name__ == "__main__":
    main()
