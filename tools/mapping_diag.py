"""Precision of G13_5's main mapping network (12 x [EqualizedLinear, BatchNorm1d(train), PReLU],
generator_13_5.py:205-216) on the GPU vs float64, forward and backward at B=16, against the same
network in fp32 torch on the CPU -- isolates where the B=16 generator step's mapping-network
gradients lose accuracy (tests/test_headline_gpu.py::test_g_step_b16)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gan_amd  # noqa: E402
from oracle.params import fill_module  # noqa: E402
from tests._util import plan  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
P = plan()
G = gan_amd.Generator(256)
fill_module(G, P["g_seed"])
mp = G.block0.mapping_network
g = torch.Generator().manual_seed(3)
z = torch.randn(256, B, generator=g)
R = torch.randn(256, B, generator=g)


def ref(dt):
    x = z.to(dt).t()          # [B, 256]
    ps = []
    n = mp.net
    for i in range(0, len(n), 3):
        lin, bn, act = n[i], n[i + 1], n[i + 2]
        W = lin.weight.weights.detach().to(dt).clone().requires_grad_()
        b = lin.bias.detach().to(dt).clone().requires_grad_()
        ga = bn.weight.detach().to(dt).clone().requires_grad_()
        be = bn.bias.detach().to(dt).clone().requires_grad_()
        al = act.weight.detach().to(dt).clone().requires_grad_()
        ps += [W, b, ga, be, al]
        x = x @ (W * (1 / math.sqrt(256))).t() + b
        mu = x.mean(0, keepdim=True)
        var = x.var(0, unbiased=False, keepdim=True)
        x = (x - mu) / torch.sqrt(var + 1e-5) * ga + be
        x = torch.where(x > 0, x, al * x)
    (x * R.to(dt).t()).sum().backward()
    return x.detach().double(), [p.grad.double() for p in ps]


y64, g64 = ref(torch.float64)
y32, g32 = ref(torch.float32)
mp = mp.cuda()
zc = z.cuda()
out = mp(zc)
(out * R.cuda()).sum().backward()
gg = []
for i in range(0, len(mp.net), 3):
    lin, bn, act = mp.net[i], mp.net[i + 1], mp.net[i + 2]
    gg += [lin.weight.weights.grad, lin.bias.grad, bn.weight.grad, bn.bias.grad, act.weight.grad]


def rel(a, b):
    return float((a.double().cpu() - b).norm() / b.norm())


print(f"B={B} out: gpu {rel(out.t(), y64):.2e} cpu-fp32 {rel(y32, y64):.2e}")
names = ["W", "b", "gamma", "beta", "alpha"]
for k in range(len(g64)):
    print(f"layer {k // 5:2d} {names[k % 5]:5s} gpu {rel(gg[k], g64[k]):.2e} cpu-fp32 {rel(g32[k], g64[k]):.2e}")
