"""Style bank vs per-module path: per-parameter gradient disagreement, worst offenders by name."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import gan_amd  # noqa: E402
from gan_amd.optim import FlatParams  # noqa: E402
from oracle.params import fill_module  # noqa: E402
from tests._util import plan  # noqa: E402

P = plan()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
z = torch.randn(B, 256, 1, 1, generator=torch.Generator().manual_seed(5)).cuda()
res = []
for use in (False, True):
    G = gan_amd.Generator(256)
    fill_module(G, P["g_seed"])
    G = G.cuda()
    flat = FlatParams(G)
    G.use_bank = use
    G.noise_hub.source = gan_amd.ReplayRNG(7, "cuda").noise
    out = G(z)
    r = torch.randn(out.shape, generator=torch.Generator().manual_seed(3)).cuda()
    (out * r).sum().backward()
    torch.cuda.synchronize()
    names = {id(p): n for n, p in G.named_parameters()}
    res.append(([names[id(p)] for p in flat.trainable], [p.grad.detach().double().cpu().clone() for p in flat.trainable],
                out.detach().double().cpu()))
    del G, flat
(n0, g0, o0), (n1, g1, o1) = res
assert n0 == n1
print("out rel", float((o1 - o0).norm() / o0.norm()))
errs = []
for name, a, b in zip(n0, g0, g1):
    na = float(a.norm())
    errs.append((float((a - b).norm()) / max(na, 1e-30), name, na, float(b.norm())))
errs.sort(reverse=True)
for e in errs[:40]:
    print(f"{e[0]:.3e} {e[1]}  |ref| {e[2]:.3e} |bank| {e[3]:.3e}")
kinds = {}
for e, name, _, _ in errs:
    k = name.split(".")[-3:]
    k = ".".join(k)
    for tag in ("to_style.0.net.0.weight.weights", "to_style.0.net.0.bias", "to_style.0.net.1.weight",
                "to_style.0.net.1.bias", "to_style.0.net.2.weight", "to_style.1.weight.weights", "to_style.1.bias",
                "to_style.2.weight", "to_style.2.bias", "conv.weight.weights"):
        if name.endswith(tag):
            kinds.setdefault(tag, []).append(e)
            break
    else:
        kinds.setdefault("other", []).append(e)
for k, v in kinds.items():
    print(f"{k:36s} n={len(v):5d} median {np.median(v):.2e} max {np.max(v):.2e}")
