"""B=16 generator step: sensitivity of the mapping network's layer-10 gradients to a relative perturbation of
one layer's pre-activations in the float64 step (the PReLU kink of make_f64.py KINK); CPU only."""
import sys, math, numpy as np, torch
sys.path.insert(0, '/root/repo')
import gan_amd
from oracle import model as om
from oracle.params import fill_module
from tests._util import plan
P = plan()
G = gan_amd.Generator(256); fill_module(G, P["g_seed"])
n = G.block0.mapping_network.net
z = om.Draw(421).randn((16, 256, 1, 1)).reshape(16, 256)
gw = torch.from_numpy(np.load('/root/repo/tools/g16_gw_f64.npy'))
def chain(dt, perturb=None, seed=0):
    x = z.to(dt); ps=[]; pres=[]
    gen = torch.Generator().manual_seed(seed)
    for L, i in enumerate(range(0, len(n), 3)):
        lin, bn, act = n[i], n[i + 1], n[i + 2]
        W = lin.weight.weights.detach().to(dt); b = lin.bias.detach().to(dt)
        ga = bn.weight.detach().to(dt).clone().requires_grad_(); be = bn.bias.detach().to(dt).clone().requires_grad_(); al = act.weight.detach().to(dt).clone().requires_grad_()
        x = x @ (W * (1 / math.sqrt(256))).t() + b
        if perturb is not None and L == perturb[0]:
            x = x * (1 + perturb[1] * torch.randn(x.shape, generator=gen, dtype=dt))
        pres.append(x)
        mu = x.mean(0, keepdim=True); var = x.var(0, unbiased=False, keepdim=True)
        x = (x - mu) / torch.sqrt(var + 1e-5) * ga + be
        x = torch.where(x > 0, x, al * x)
        ps.append((ga, be, al))
    x.backward(gw.to(dt))
    return ps, pres
base, pres = chain(torch.float64)
r = lambda a, b: float((a - b).norm() / b.norm())
for L in (10, 9, 11):
    for eps in (1e-7, 1e-6):
        pp, _ = chain(torch.float64, (L, eps))
        print(f"perturb pre{L} by {eps:.0e}: gamma10 {r(pp[10][0].grad, base[10][0].grad):.2e} beta10 {r(pp[10][1].grad, base[10][1].grad):.2e} alpha10 {r(pp[10][2].grad, base[10][2].grad):.2e}")
g = base[10]
print("beta10 grad norm", float(base[10][1].grad.norm()), "gamma10", float(base[10][0].grad.norm()))
# the PReLU kink: layer-10 pre-activations z10 closest to 0
x = z.to(torch.float64)
for L, i in enumerate(range(0, len(n), 3)):
    lin, bn, act = n[i], n[i + 1], n[i + 2]
    W = lin.weight.weights.detach().double(); b = lin.bias.detach().double()
    x = x @ (W * (1 / math.sqrt(256))).t() + b
    mu = x.mean(0, keepdim=True); var = x.var(0, unbiased=False, keepdim=True)
    zz = (x - mu) / torch.sqrt(var + 1e-5) * bn.weight.detach().double() + bn.bias.detach().double()
    if L == 10:
        a = zz.abs().flatten().argsort()[:4]
        for k in a:
            bb, c = int(k) // 256, int(k) % 256
            print(f"layer 10 z[b={bb}, c={c}] = {float(zz[bb, c]):.3e}  (|z| scale {float(zz.abs().mean()):.3f})")
    x = torch.where(zz > 0, zz, act.weight.detach().double() * zz)
