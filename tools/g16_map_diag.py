"""The B=16 generator step's mapping-network gradients (tests/test_headline_gpu.py::test_g_step_b16):
with dL/dw fixed to its float64 truth (tools/g16_gw_f64.npy, from tools/g16_grad_diag.py cpu f64),
the exact backward of the 12-layer mapping network gives the step's mapping gradients to 8e-5 (from
the GPU's own dL/dw) -- yet the GPU step has 1.2e-3.  This runs the mapping network alone on the GPU
(z of the test's Draw(421), upstream gradient = the float64 dL/dw) and prints each layer's forward
output and parameter-gradient error against float64, next to CPU fp32."""
import math
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import gan_amd  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle.params import fill_module  # noqa: E402
from tests._util import plan  # noqa: E402

P = plan()
G = gan_amd.Generator(256)
fill_module(G, P["g_seed"])
mp = G.block0.mapping_network
z = om.Draw(421).randn((16, 256, 1, 1)).reshape(16, 256)
gw = torch.from_numpy(np.load(os.path.join(REPO, "tools", "g16_gw_f64.npy")))     # [B, 256]


def ref(dt):
    x = z.to(dt)
    ps, outs = [], []
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
        x.retain_grad()
        outs.append(x)
    x.backward(gw.to(dt))
    return [o.detach().double() for o in outs], [p.grad.double() for p in ps], [o.grad.double() for o in outs]


o64, g64, h64 = ref(torch.float64)
o32, g32, h32 = ref(torch.float32)
mp = mp.cuda()
x = z.t().contiguous().cuda()
outs = []
n = mp.net
h = x
for i in range(0, len(n), 3):
    h = gan_amd.generator_13_5._lin_bn_act(n[i], n[i + 1], n[i + 2], h)
    h.retain_grad()
    outs.append(h)
h.backward(gw.t().contiguous().float().cuda())
gg = []
for i in range(0, len(n), 3):
    lin, bn, act = n[i], n[i + 1], n[i + 2]
    gg += [lin.weight.weights.grad, lin.bias.grad, bn.weight.grad, bn.bias.grad, act.weight.grad]


def rel(a, b):
    return float((a.double().cpu() - b).norm() / b.norm().clamp_min(1e-300))


names = ["W", "b", "gamma", "beta", "alpha"]
for L in range(12):
    print(f"layer {L:2d} out: gpu {rel(outs[L].t(), o64[L]):.2e} cpu-fp32 {rel(o32[L], o64[L]):.2e}   grads: " +
          " ".join(f"{names[k]} {rel(gg[5 * L + k], g64[5 * L + k]):.1e}/{rel(g32[5 * L + k], g64[5 * L + k]):.1e}"
                   for k in (0, 2, 3, 4)) +
          f"   d/d(out): gpu {rel(outs[L].grad.t(), h64[L]):.1e} cpu-fp32 {rel(h32[L], h64[L]):.1e}", flush=True)

# the last layer's backward step by step on the GPU ops (layer 11: BN+PReLU backward, then the linear's
# input gradient), against float64 on the same saved values
L = 11
lin, bn, act = n[3 * L], n[3 * L + 1], n[3 * L + 2]
x_in = outs[L - 1].detach().double().cpu().t()          # [B, 256] the layer's input (GPU forward)
W = lin.weight.weights.detach().double().cpu() / 16.0
pre = x_in @ W.t() + lin.bias.detach().double().cpu()
mu, var = pre.mean(0), pre.var(0, unbiased=False)
xh = (pre - mu) / torch.sqrt(var + 1e-5)
z = xh * bn.weight.detach().double().cpu() + bn.bias.detach().double().cpu()
g = gw.double() * torch.where(z > 0, torch.ones_like(z), act.weight.detach().double().cpu().expand_as(z))
gbn = (g - g.mean(0) - xh * (g * xh).mean(0)) * bn.weight.detach().double().cpu() / torch.sqrt(var + 1e-5)
gin = gbn @ W
print("layer 11 input-gradient from its own saved values: gpu", f"{rel(outs[L - 1].grad.t(), gin):.2e}")
print("batch-mean of d/d(out 10) (float64 truth, gpu):", float(h64[10].mean(0).abs().max()),
      float(outs[10].grad.t().double().cpu().mean(0).abs().max()), "scale", float(h64[10].abs().max()))

# layer 10's BatchNorm + PReLU backward ALONE on the GPU (fresh autograd graph, the GPU's own input and
# upstream gradient) -- does the kernel reproduce the chain's error?
L = 10
lin, bn, act = n[3 * L], n[3 * L + 1], n[3 * L + 2]
for p_ in (bn.weight, bn.bias, act.weight):
    p_.grad = None
with torch.no_grad():
    pre10 = lin(outs[L - 1].detach())
pre10 = pre10.detach().clone().requires_grad_()
y10 = gan_amd.ops.bn_act(pre10, bn, act)
gy10 = outs[L].grad.detach().clone()
y10.backward(gy10)
pre64 = pre10.detach().double().cpu().t().clone().requires_grad_()
mu, var = pre64.mean(0), pre64.var(0, unbiased=False)
ga64 = bn.weight.detach().double().cpu().clone().requires_grad_()
be64 = bn.bias.detach().double().cpu().clone().requires_grad_()
al64 = act.weight.detach().double().cpu().clone().requires_grad_()
zz = (pre64 - mu) / torch.sqrt(var + 1e-5) * ga64 + be64
yy = torch.where(zz > 0, zz, al64 * zz)
yy.backward(gy10.double().cpu().t())
print("layer 10 BN+PReLU backward alone:  gx", f"{rel(pre10.grad.t(), pre64.grad):.2e}", " gamma",
      f"{rel(bn.weight.grad, ga64.grad):.2e}", " beta", f"{rel(bn.bias.grad, be64.grad):.2e}", " alpha",
      f"{rel(act.weight.grad, al64.grad):.2e}")
print("forward y10 vs chain out 10:", f"{rel(y10.t(), outs[L].detach().double().cpu().t()):.2e}")

# the chain again, keeping the graph: are BNAct 10's saved tensors intact after the backward?
for p_ in mp.parameters():
    p_.grad = None
h = x
outs2 = []
for i in range(0, len(n), 3):
    h = gan_amd.generator_13_5._lin_bn_act(n[i], n[i + 1], n[i + 2], h)
    outs2.append(h)
node = outs2[10].grad_fn
saved_before = [t.detach().clone() for t in node.saved_tensors]
h.backward(gw.t().contiguous().float().cuda(), retain_graph=True)
torch.cuda.synchronize()
saved_after = [t.detach().clone() for t in node.saved_tensors]
for k, (a_, b_) in enumerate(zip(saved_before, saved_after)):
    if a_ is not None:
        print(f"BNAct 10 saved tensor {k} {tuple(a_.shape)}: changed by the backward: {float((a_ - b_).abs().max()):.3e}")
print("chain again: gamma10", f"{rel(n[31].weight.grad, g64[5 * 10 + 2]):.2e}", "beta10", f"{rel(n[31].bias.grad, g64[5 * 10 + 3]):.2e}")

# what BNAct 10's backward actually receives in the chain (a pre-hook on its node)
for p_ in mp.parameters():
    p_.grad = None
h = x
outs3 = []
for i in range(0, len(n), 3):
    h = gan_amd.generator_13_5._lin_bn_act(n[i], n[i + 1], n[i + 2], h)
    outs3.append(h)
got_in = {}
outs3[10].grad_fn.register_prehook(lambda go: got_in.__setitem__("gy", [None if g is None else g.detach().clone() for g in go]))
outs3[10].register_hook(lambda g: got_in.__setitem__("tensor_hook", g.detach().clone()))
h.backward(gw.t().contiguous().float().cuda())
torch.cuda.synchronize()
gys = got_in["gy"]
print("BNAct 10 receives", len(gys), "grads:", [None if g is None else (tuple(g.shape), g.is_contiguous()) for g in gys])
print("  vs tensor hook:", f"{float((gys[0] - got_in['tensor_hook']).abs().max()):.3e}",
      " vs float64 truth:", f"{rel(gys[0].t(), h64[10]):.2e}")
print("chain with hooks: gamma10", f"{rel(n[31].weight.grad, g64[5 * 10 + 2]):.2e}")
