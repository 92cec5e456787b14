"""GPU fp32 rounding spread of the G13_5 forward at B=4 (companion of make_f64.g_out_spread):
distance to float64 truth with the weights perturbed by ~1 ulp, per trial, module and bank paths."""
import sys

import torch

sys.path.insert(0, ".")
import gan_amd  # noqa: E402
from gan_amd.optim import FlatParams  # noqa: E402
from oracle.params import fill_module  # noqa: E402
from tests._util import fixture, plan, rel_err  # noqa: E402

P = plan()
fx = fixture("g_fwd_b4.npz")
truth = fixture("f64_truth.npz")
for bank in (False, True):
    for t in range(6):
        G = gan_amd.Generator(256)
        fill_module(G, P["g_seed"])
        G = G.cuda()
        if bank:
            FlatParams(G)
        if t:
            g = torch.Generator().manual_seed(t)
            with torch.no_grad():
                for p in G.parameters():
                    p.mul_(1 + 6e-8 * torch.randn(p.shape, generator=g).cuda())
        G.noise_hub.source = gan_amd.ReplayRNG(101, "cuda").noise
        with torch.no_grad():
            out = G(torch.from_numpy(fx["z"]).cuda())
        print(f"bank={bank} trial={t} vs truth {rel_err(out.cpu().numpy(), truth['g_out']):.3e} "
              f"vs ref {rel_err(out.cpu().numpy(), fx['out']):.3e}", flush=True)
        del G
print("cpu fp32 spread:", truth["g_out_fp32_spread"])
