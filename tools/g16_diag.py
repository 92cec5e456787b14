"""Dump the GPU generator step's per-tensor gradient summaries at B=16 (the fixture of
tests/golden/make_golden_g16.py, seed 421) to gpurun_out/g16_rows.npy for offline comparison
with the reference and float64 truth."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gan_amd  # noqa: E402
from oracle.params import fill_module, tensor_summary  # noqa: E402
from tests._util import plan  # noqa: E402

P = plan()
G = gan_amd.Generator(256)
fill_module(G, P["g_seed"])
D = gan_amd.Discriminator()
fill_module(D, P["d_seed"])
G, D = G.cuda(), D.cuda()
if "--no-bank" in sys.argv:
    G.use_bank = False
tr = gan_amd.Train([0] * 10, "cuda", 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.ReplayRNG(421, "cuda"))
gen, loss = tr.generator_backward(16)
params = dict(G.named_parameters())
rows = np.asarray([tensor_summary(params[n].grad) if params[n].grad is not None else [np.nan] * 11
                   for n, _, _ in P["g_params"]])
tag = "nobank" if "--no-bank" in sys.argv else "bank"
np.save(f"gpurun_out/g16_rows_{tag}.npy", rows)
print("loss", float(loss.detach()), tag)
