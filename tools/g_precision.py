"""Where does the G13_5 forward lose precision?  Distance to float64 truth over ~1-ulp weight
perturbation trials for: the build ('ours'), the build with BatchNorm swapped for torch's
('ours_bn_torch'), and the CPU oracle's torch ops executed on the GPU ('oracle_gpu')."""
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
import gan_amd  # noqa: E402
from gan_amd import generator_13_5 as gm, ops  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle.params import fill_module  # noqa: E402
from tests._util import fixture, plan, rel_err  # noqa: E402

P = plan()
fx = fixture("g_fwd_b4.npz")
truth = fixture("f64_truth.npz")["g_out"]
TRIALS = 5


def perturb(tensors, t):
    if t:
        g = torch.Generator().manual_seed(t)
        with torch.no_grad():
            for v in tensors:
                v.mul_(1 + 6e-8 * torch.randn(v.shape, generator=g).to(v.device))


def bn_act_torch(x, bn, act=None):
    C = x.shape[0]
    y = F.batch_norm(x.reshape(C, -1).t(), bn.running_mean, bn.running_var, bn.weight, bn.bias, True, bn.momentum,
                     bn.eps)
    if act is not None:
        y = F.prelu(y, act.weight)
    return y.t().reshape(x.shape).contiguous()


def run_ours(bn_torch):
    if bn_torch:
        gm.bn_act = bn_act_torch
    errs = []
    for t in range(TRIALS):
        G = gan_amd.Generator(256)
        fill_module(G, P["g_seed"])
        G = G.cuda()
        perturb(list(G.parameters()), t)
        G.noise_hub.source = gan_amd.ReplayRNG(101, "cuda").noise
        with torch.no_grad():
            out = G(torch.from_numpy(fx["z"]).cuda())
        errs.append(rel_err(out.cpu().numpy(), truth))
    gm.bn_act = ops.bn_act
    return errs


def run_oracle_gpu():
    errs = []
    om._SMOOTH = om._SMOOTH.cuda()
    for t in range(TRIALS):
        GP = om.params_from_plan(P["g_params"], P["g_seed"])
        GP.t = {k: v.cuda() for k, v in GP.t.items()}
        GP.bn_buffers = lambda name, c, GP=GP: GP.buffers.setdefault(
            name, (torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")))
        perturb(list(GP.t.values()), t)
        d = om.Draw(101)
        with torch.no_grad():
            out = om.generator(GP, torch.from_numpy(fx["z"]).cuda(), lambda s: d.randn(s).cuda())
        errs.append(rel_err(out.cpu().numpy(), truth))
    return errs


for name, fn in (("ours", lambda: run_ours(False)), ("ours_bn_torch", lambda: run_ours(True)),
                 ("oracle_gpu", run_oracle_gpu)):
    e = fn()
    print(f"{name:14s} mean {np.mean(e):.3e}  " + " ".join(f"{v:.2e}" for v in e), flush=True)
s = truth_spread = fixture("f64_truth.npz")["g_out_fp32_spread"]
print(f"{'cpu_fp32':14s} mean {np.mean(s):.3e}  " + " ".join(f"{v:.2e}" for v in s))
