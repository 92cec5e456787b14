"""Localise the B=16 generator-step gradient excess (tests/test_headline_gpu.py::test_g_step_b16).

The gradient of the 12-layer main mapping network is dL/dw -- the latent's gradient, summed by
the style bank over the 519 style MLPs -- pushed back through 12 BatchNorm1d layers.  This dumps
the intermediate gradients on both sides so they can be compared against float64 truth:

  gw          dL/dw at the mapping network's output            [256, B]
  gS[name]    dL/ds of every modulated conv's style (after BN)  [cin, B]
  gD[name]    dL/dd of every demodulation vector                [cout, B]

  python tools/g16_grad_diag.py gpu            -> gpurun_out/g16_diag_gpu.npz   (GPU box)
  python tools/g16_grad_diag.py cpu f64|f32    -> gpurun_out/g16_diag_<dt>.npz  (host oracle)
  python tools/g16_grad_diag.py compare        -> relative errors vs f64, GPU next to fp32 CPU

Same seeds as the test (ReplayRNG(421) / Draw(421), fixture-plan weights).
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "gpurun_out")
B, SEED = 16, 421


def gpu():
    import gan_amd
    from gan_amd.generator_13_5 import Conv2dWeightModulate
    from oracle.params import fill_module, tensor_summary
    from tests._util import plan
    P = plan()
    G = gan_amd.Generator(256)
    fill_module(G, P["g_seed"])
    D = gan_amd.Discriminator()
    fill_module(D, P["d_seed"])
    G, D = G.cuda(), D.cuda()
    names = {id(m): n for n, m in G.named_modules() if isinstance(m, Conv2dWeightModulate)}
    got = {}
    orig = G._run_bank

    def run_bank(w):
        w.register_hook(lambda g: got.__setitem__("gw", g.detach().cpu().double().numpy()))
        orig(w)
        for m in G.__dict__["_style_bank"].mods:
            s, d = m.__dict__["_bank_sd"]
            n = names[id(m)]
            s.register_hook(lambda g, n=n: got.__setitem__("gS:" + n, g.detach().t().cpu().double().numpy()))
            d.register_hook(lambda g, n=n: got.__setitem__("gD:" + n, g.detach().t().cpu().double().numpy()))
    G._run_bank = run_bank
    tr = gan_amd.Train([0] * 10, "cuda", 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.ReplayRNG(SEED, "cuda"))
    if os.environ.get("G16_PATCH") is not None:        # ganamd_conv_set_patch mask (0: gather GEMM only)
        gan_amd.ops.set_patch(int(os.environ["G16_PATCH"]))
    gen, loss = tr.generator_backward(B)
    torch.cuda.synchronize()
    got["gw"] = got["gw"].T                       # [B, 256] like the oracle
    params = dict(G.named_parameters())
    got["rows"] = np.asarray([tensor_summary(params[n].grad) if params[n].grad is not None else [np.nan] * 11
                              for n, _, _ in P["g_params"]])
    got["loss"] = np.asarray([float(loss.detach())])
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"g16_diag_{os.environ.get('G16_TAG', 'gpu')}.npz"), **got)
    print("gpu: loss", float(loss.detach()), "entries", len(got))


def cpu(dt_name):
    from oracle import model as om
    from tests._util import plan
    dt = torch.float64 if dt_name == "f64" else torch.float32
    torch.set_num_threads(os.cpu_count() or 8)
    P = plan()
    got = {}

    def params(pp, seed):
        Pm = om.params_from_plan(pp, seed)
        if dt == torch.float64:
            Pm.t = {k: v.detach().to(dt).requires_grad_() for k, v in Pm.t.items()}
            Pm.bn_buffers = lambda name, c: Pm.buffers.setdefault(name, (torch.zeros(c, dtype=dt),
                                                                         torch.ones(c, dtype=dt)))
        return Pm

    class DrawT(om.Draw):
        def randn(self, shape):
            return super().randn(shape).to(dt)

        def rand(self, shape):
            return super().rand(shape).to(dt)

    orig_map, orig_mod = om.g_mapping, om.g_modconv

    def g_mapping(Pm, pre, x, planes, layers):
        y = orig_map(Pm, pre, x, planes, layers)
        if pre.endswith("block0.mapping_network") and y.requires_grad:
            y.register_hook(lambda g: got.__setitem__("gw", g.detach().double().numpy()))
        return y

    def g_modconv(C, pre, x, cin, cout, k):
        # oracle/model.py:g_modconv with hooks on s and d (the same arithmetic)
        import math
        import torch.nn.functional as F
        Pm = C.P
        s = orig_map(Pm, f"{pre}.to_style.0", C.w, 256, 1)
        s = om.eq_linear(Pm, f"{pre}.to_style.1", s, 256, cin)
        s = om.bn(Pm, f"{pre}.to_style.2", s, cin)
        wt = Pm(f"{pre}.weight.weights", (cout, cin, k, k)) * (1.0 / math.sqrt(cin * k * k))
        wsq = (wt * wt).sum(dim=(2, 3))
        d = torch.rsqrt((s * s) @ wsq.t() + 1e-8)
        if s.requires_grad:
            s.register_hook(lambda g: got.__setitem__("gS:" + pre, g.detach().double().numpy()))
            d.register_hook(lambda g: got.__setitem__("gD:" + pre, g.detach().double().numpy()))
        xs = x * s[:, :, None, None]
        p = (k - 1) // 2
        if p:
            xs = F.pad(xs, (p, p, p, p), mode="replicate")
        return F.conv2d(xs, wt) * d[:, :, None, None]

    om.g_mapping, om.g_modconv = g_mapping, g_modconv
    GP, DP = params(P["g_params"], P["g_seed"]), params(P["d_params"], P["d_seed"])
    _gen, loss = om.WGANGP(GP, DP).generator_trainstep(B, DrawT(SEED))
    got["loss"] = np.asarray([float(loss.detach())])
    os.makedirs(OUT, exist_ok=True)
    np.savez(os.path.join(OUT, f"g16_diag_{dt_name}.npz"), **got)
    print(dt_name, "loss", float(loss.detach()), "entries", len(got))


def compare():
    t = np.load(os.path.join(OUT, "g16_diag_f64.npz"))
    tags = sys.argv[2:] or ["gpu", "f32"]
    sides = {k: np.load(os.path.join(OUT, f"g16_diag_{k}.npz")) for k in tags
             if os.path.exists(os.path.join(OUT, f"g16_diag_{k}.npz"))}

    def rel(a, b):
        return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
    print(f"{'quantity':60s} " + " ".join(f"{k:>10s}" for k in sides))
    keys = ["gw"] + sorted(k for k in t.files if k.startswith("gS:")) + sorted(k for k in t.files if k.startswith("gD:"))
    agg = {k: [] for k in sides}
    for key in keys:
        errs = {k: rel(v[key], t[key]) if key in v.files else float("nan") for k, v in sides.items()}
        for k, e in errs.items():
            agg[k].append((e, key))
        if key == "gw" or max(errs.values()) > 1e-5:
            print(f"{key:60s} " + " ".join(f"{errs[k]:10.2e}" for k in sides))
    for k, lst in agg.items():
        e = np.asarray([x for x, _ in lst[1:]])
        print(k, "style/demod grads: median", np.median(e), "p99", np.percentile(e, 99), "max", e.max(),
              max(lst[1:])[1])
    # the G-step's parameter gradients (rows) against float64 truth: which tensors carry the
    # norm-vector statistic's error (tests/_util.grad_norm_stats)
    import json
    from tests._util import GOLDEN, grad_norm_stats
    truth = np.load(os.path.join(GOLDEN, "f64_g16.npz"))["g16_grads"]
    names = [n for n, _, _ in json.load(open(os.path.join(GOLDEN, "plan.json")))["g_params"]]
    for k, v in sides.items():
        if "rows" not in v.files:
            continue
        rows = v["rows"]
        print(k, "grad_norm_stats vs f64:", grad_norm_stats(rows, truth))
        g, w = rows[:, 1], truth[:, 1]
        ok = ~np.isnan(w) & ~np.isnan(g)
        d2 = np.where(ok, (g - w) ** 2, 0.0)
        tot = np.sqrt(np.nansum(np.where(ok, w ** 2, 0.0)))
        for i in np.argsort(-d2)[:12]:
            print(f"   {np.sqrt(d2[i]) / tot:.2e} of |w|  rel {abs(g[i] - w[i]) / abs(w[i]):.2e}  {names[i]}")


if __name__ == "__main__":
    {"gpu": gpu, "cpu": lambda: cpu(sys.argv[2]), "compare": compare}[sys.argv[1]]()
