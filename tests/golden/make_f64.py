"""Float64 "truth" fixtures, computed by the pinned CPU oracle (oracle/model.py) in float64.

    python tests/golden/make_f64.py

Why: the fp32 reference is itself far from exact on this path (measured here: G13_5 output
2e-4 relative; G-step gradient norms median 1.7 %, vector 1.5 % -- BatchNorm1d over B=4 samples
is ill-conditioned).  Comparing the GPU build only against the fp32 reference would mix the
reference's rounding error into the bar.  These fixtures let the tests require the GPU build to
be as close to float64 truth as the fp32 reference is (the reference's own distance to truth
is stored alongside as ``ref_*``).  The oracle is pinned to the reference by
tests/test_oracle_golden.py before it is trusted here.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import model as om  # noqa: E402
from oracle.params import tensor_summary  # noqa: E402
from tests._util import fixture, grad_norm_stats, plan, rel_err  # noqa: E402

DT = torch.float64


class Draw64(om.Draw):
    def randn(self, shape):
        return super().randn(shape).to(DT)

    def rand(self, shape):
        return super().rand(shape).to(DT)


def params64(pp, seed):
    P = om.params_from_plan(pp, seed)
    P.t = {k: v.detach().to(DT).requires_grad_() for k, v in P.t.items()}
    P.bn_buffers = lambda name, c: P.buffers.setdefault(name, (torch.zeros(c, dtype=DT), torch.ones(c, dtype=DT)))
    return P


def grad_rows(P, names):
    return np.asarray([tensor_summary(P.t[n].grad) if n in P.t and P.t[n].grad is not None else [np.nan] * 11
                       for n in names])


def g_out_spread(trials=12):
    """fp32 rounding spread of the G13_5 forward at B=4: the oracle in fp32 with every weight
    perturbed by ~1 ulp (relative N(0, 6e-8)), distance to float64 truth per trial.  One fp32
    evaluation order is one draw from this distribution (the reference's own error is one
    such draw), so the GPU bar is set on the distribution, not on that single draw."""
    pl = plan()
    fx = fixture("g_fwd_b4.npz")
    truth = fixture("f64_truth.npz")["g_out"]
    errs = []
    for t in range(1, trials + 1):
        GP = om.params_from_plan(pl["g_params"], pl["g_seed"])
        g = torch.Generator().manual_seed(t)
        with torch.no_grad():
            for v in GP.t.values():
                v.mul_(1 + 6e-8 * torch.randn(v.shape, generator=g))
            out = om.generator(GP, torch.from_numpy(fx["z"]), om.Draw(101).randn)
        errs.append(rel_err(out.numpy(), truth))
        print("spread trial", t, errs[-1], flush=True)
    return np.asarray(errs)


def step_spread(trials=6):
    """Same idea for the training steps: gradient statistics (tests/_util.grad_norm_stats) of the
    fp32 oracle with ~1-ulp perturbed weights against float64 truth, per trial."""
    pl = plan()
    truth = fixture("f64_truth.npz")
    dnames = [n for n, _, _ in pl["d_params"]]
    gnames = [n for n, _, _ in pl["g_params"]]
    res = {f"d{B}_fp32_spread": [] for B in (4, 8)}
    res["g_fp32_spread"] = []
    for t in range(1, trials + 1):
        for B, img_seed, rng_seed in ((4, 300, 301), (8, 310, 311), (4, None, 401)):
            GP = om.params_from_plan(pl["g_params"], pl["g_seed"])
            DP = om.params_from_plan(pl["d_params"], pl["d_seed"])
            g = torch.Generator().manual_seed(t)
            with torch.no_grad():
                for v in list(GP.t.values()) + list(DP.t.values()):
                    v.mul_(1 + 6e-8 * torch.randn(v.shape, generator=g))
            tr = om.WGANGP(GP, DP)
            if img_seed is None:
                tr.generator_trainstep(4, om.Draw(rng_seed))
                rows = grad_rows(GP, gnames)
                key, tkey = "g_fp32_spread", "g_grads"
            else:
                images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(img_seed))
                tr.discriminator_trainstep(images, B, om.Draw(rng_seed))
                rows = grad_rows(DP, dnames)
                key, tkey = f"d{B}_fp32_spread", f"d{B}_grads"
            res[key].append(grad_norm_stats(rows, truth[tkey]))
            print("step spread", t, key, res[key][-1], flush=True)
    return {k: np.asarray(v) for k, v in res.items()}


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    om._SMOOTH = om._SMOOTH.to(DT)
    pl = plan()
    t0 = time.time()
    out = {}

    fx = fixture("g_fwd_b4.npz")
    GP = params64(pl["g_params"], pl["g_seed"])
    d = Draw64(101)
    with torch.no_grad():
        g = om.generator(GP, torch.from_numpy(fx["z"]).to(DT), d.randn)
    out["g_out"] = g.numpy()
    out["ref_g_out_err"] = np.asarray(rel_err(fx["out"], g.numpy()))
    print("g fwd", time.time() - t0, out["ref_g_out_err"], flush=True)

    dnames = [n for n, _, _ in pl["d_params"]]
    for B, img_seed, rng_seed in ((4, 300, 301), (8, 310, 311)):
        fx = fixture(f"d_step_b{B}.npz")
        GP, DP = params64(pl["g_params"], pl["g_seed"]), params64(pl["d_params"], pl["d_seed"])
        tr = om.WGANGP(GP, DP)
        images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(img_seed)).to(DT)
        losses = [float(v.detach()) for v in tr.discriminator_trainstep(images, B, Draw64(rng_seed))]
        # torch.optim.AdamW.step already ran; grads are still in .grad
        rows = grad_rows(DP, dnames)
        out[f"d{B}_losses"] = np.asarray(losses)
        out[f"d{B}_grads"] = rows
        out[f"ref_d{B}_stats"] = np.asarray(grad_norm_stats(fx["grads"], rows))
        out[f"ref_d{B}_loss_err"] = np.asarray(rel_err(fx["losses"], losses))
        print(f"d step b{B}", time.time() - t0, out[f"ref_d{B}_stats"], flush=True)

    fx = fixture("g_step_b4.npz")
    GP, DP = params64(pl["g_params"], pl["g_seed"]), params64(pl["d_params"], pl["d_seed"])
    tr = om.WGANGP(GP, DP)
    gen, g_loss = tr.generator_trainstep(4, Draw64(401))
    gnames = [n for n, _, _ in pl["g_params"]]
    rows = grad_rows(GP, gnames)
    out["g_loss"] = np.asarray([float(g_loss.detach())])
    out["g_grads"] = rows.astype(np.float32)
    out["ref_g_stats"] = np.asarray(grad_norm_stats(fx["grads"], rows))
    print("g step", time.time() - t0, out["ref_g_stats"], flush=True)
    np.savez_compressed(os.path.join(HERE, "f64_truth.npz"), **out)
    out["g_out_fp32_spread"] = g_out_spread()
    np.savez_compressed(os.path.join(HERE, "f64_truth.npz"), **out)
    out.update(step_spread())
    np.savez_compressed(os.path.join(HERE, "f64_truth.npz"), **out)


def lazy_main(trials=4):
    """Float64 truth of the two lazy-GP + R1/R2 critic steps of tests/golden/make_golden_lazy.py
    (idx 0: with the regularisers, idx 1: without), the reference's distance to it, and the fp32
    spread (weights perturbed by ~1 ulp)."""
    torch.set_num_threads(os.cpu_count() or 8)
    pl = plan()
    fx = fixture("lazy_b4.npz")
    dnames = [n for n, _, _ in pl["d_params"]]
    out = {}
    for idx, img_seed, rng_seed in ((0, 500, 501), (1, 510, 511)):
        images = torch.randn(4, 3, 64, 64, generator=torch.Generator().manual_seed(img_seed))
        smooth32 = om._SMOOTH
        om._SMOOTH = smooth32.to(DT)
        GP, DP = params64(pl["g_params"], pl["g_seed"]), params64(pl["d_params"], pl["d_seed"])
        tr = om.WGANLazyR2(GP, DP)
        losses = [float(v.detach().reshape(-1)[0])
                  for v in tr.discriminator_trainstep(images.to(DT), 4, idx, Draw64(rng_seed))]
        om._SMOOTH = smooth32
        k = f"d{idx}"
        out[f"{k}_losses"], out[f"{k}_grads"] = np.asarray(losses), grad_rows(DP, dnames)
        out[f"ref_{k}_stats"] = np.asarray(grad_norm_stats(fx[f"{k}_grads"], out[f"{k}_grads"]))
        n = 5 if idx == 0 else 2
        out[f"ref_{k}_loss_err"] = np.asarray(rel_err(fx[f"{k}_losses"][:n], losses[:n]))
        print("lazy truth", k, out[f"ref_{k}_stats"], out[f"ref_{k}_loss_err"], flush=True)
        spread = []
        for t in range(1, trials + 1):
            GP = om.params_from_plan(pl["g_params"], pl["g_seed"])
            DP = om.params_from_plan(pl["d_params"], pl["d_seed"])
            g = torch.Generator().manual_seed(t)
            with torch.no_grad():
                for v in list(GP.t.values()) + list(DP.t.values()):
                    v.mul_(1 + 6e-8 * torch.randn(v.shape, generator=g))
            om.WGANLazyR2(GP, DP).discriminator_trainstep(images, 4, idx, om.Draw(rng_seed))
            spread.append(grad_norm_stats(grad_rows(DP, dnames), out[f"{k}_grads"]))
            print("lazy spread", k, t, spread[-1], flush=True)
        out[f"{k}_fp32_spread"] = np.asarray(spread)
    np.savez_compressed(os.path.join(HERE, "f64_lazy.npz"), **out)


def progan_main(trials=6):
    """Float64 truth of the progan pair's critic and generator steps (tests/golden/
    make_golden_progan.py), the reference's distance to it, and the fp32 spread."""
    import json
    torch.set_num_threads(os.cpu_count() or 8)
    with open(os.path.join(HERE, "plan_progan.json")) as f:
        pp = json.load(f)
    fx = fixture("progan_b4.npz")
    dn = [n for n, _, _ in pp["d_params"]]
    gn = [n for n, _, _ in pp["g_params"]]
    images = torch.randn(4, 3, 64, 64, generator=torch.Generator().manual_seed(710))

    def run(dt, perturb=None):
        if dt == DT:
            GP, DP = params64(pp["g_params"], pp["g_seed"]), params64(pp["d_params"], pp["d_seed"])
            dr, dg = Draw64(711), Draw64(721)
        else:
            GP = om.params_from_plan(pp["g_params"], pp["g_seed"])
            DP = om.params_from_plan(pp["d_params"], pp["d_seed"])
            dr, dg = om.Draw(711), om.Draw(721)
            g = torch.Generator().manual_seed(perturb)
            with torch.no_grad():
                for v in list(GP.t.values()) + list(DP.t.values()):
                    v.mul_(1 + 6e-8 * torch.randn(v.shape, generator=g))
        tr = om.WGANGP(GP, DP, gen=om.progan_generator, disc=om.progan_discriminator)
        losses = [float(v.detach()) for v in tr.discriminator_trainstep(images.to(dt), 4, dr)]
        drows = grad_rows(DP, dn)
        GP2 = params64(pp["g_params"], pp["g_seed"]) if dt == DT else om.params_from_plan(pp["g_params"], pp["g_seed"])
        DP2 = params64(pp["d_params"], pp["d_seed"]) if dt == DT else om.params_from_plan(pp["d_params"], pp["d_seed"])
        if dt != DT:
            g = torch.Generator().manual_seed(perturb)
            with torch.no_grad():
                for v in list(GP2.t.values()) + list(DP2.t.values()):
                    v.mul_(1 + 6e-8 * torch.randn(v.shape, generator=g))
        tr = om.WGANGP(GP2, DP2, gen=om.progan_generator, disc=om.progan_discriminator)
        _gen, g_loss = tr.generator_trainstep(4, dg)
        return losses + [float(g_loss.detach())], drows, grad_rows(GP2, gn)

    losses, drows, grows = run(DT)
    out = {"losses": np.asarray(losses), "d_grads": drows, "g_grads": grows,
           "ref_d_stats": np.asarray(grad_norm_stats(fx["d_grads"], drows)),
           "ref_g_stats": np.asarray(grad_norm_stats(fx["g_grads"], grows)),
           "ref_loss_err": np.asarray(rel_err(np.r_[fx["d_losses"], fx["g_loss"]], losses))}
    print("progan truth", out["ref_d_stats"], out["ref_g_stats"], out["ref_loss_err"], flush=True)
    sd, sg, sl = [], [], []
    for t in range(1, trials + 1):
        l32, d32, g32 = run(torch.float32, perturb=t)
        sd.append(grad_norm_stats(d32, drows))
        sg.append(grad_norm_stats(g32, grows))
        sl.append(rel_err(l32, losses))
        print("progan spread", t, sd[-1], sg[-1], sl[-1], flush=True)
    out["d_fp32_spread"], out["g_fp32_spread"], out["loss_fp32_spread"] = np.asarray(sd), np.asarray(sg), np.asarray(sl)
    np.savez_compressed(os.path.join(HERE, "f64_progan.npz"), **out)


def headline_main(trials=3):
    """Generator steps above B=4 (train/wgangp.py:20-27):

    * B=16: float64 truth of the reference's fixture g_step_b16.npz (make_golden_g16.py, same
      seed 421), the reference's distance to it, and the fp32 spread (oracle in fp32 with ~1-ulp
      perturbed weights) -> f64_g16.npz;
    * B=64, the headline batch: the reference's own formulation does not fit this container there
      (B x 178.7 M modulated weights kept for the backward: 47 GiB already at B=16), and neither
      does the oracle's (~100 GiB); tests/test_headline_gpu.py::test_g_step_b64_vs_oracle runs the
      fp32 oracle -- pinned to the reference at B=4 and B=16 -- on the GPU box's host instead."""
    import resource
    torch.set_num_threads(os.cpu_count() or 8)
    pl = plan()
    gnames = [n for n, _, _ in pl["g_params"]]
    fx = fixture("g_step_b16.npz")
    t0 = time.time()
    smooth32 = om._SMOOTH
    om._SMOOTH = smooth32.to(DT)
    GP, DP = params64(pl["g_params"], pl["g_seed"]), params64(pl["d_params"], pl["d_seed"])
    _gen, g_loss = om.WGANGP(GP, DP).generator_trainstep(16, Draw64(421))
    om._SMOOTH = smooth32
    rows = grad_rows(GP, gnames)
    out = {"g16_loss": np.asarray([float(g_loss.detach())]), "g16_grads": rows,
           "ref_g16_stats": np.asarray(grad_norm_stats(fx["grads"], rows)),
           "ref_g16_loss_err": np.asarray(rel_err(fx["g_loss"], [float(g_loss.detach())]))}
    del GP, DP, _gen, g_loss
    print("g16 truth", time.time() - t0, out["ref_g16_stats"], out["ref_g16_loss_err"],
          f"peak RSS {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20:.1f} GiB", flush=True)

    def fp32_step(B, seed, perturb):
        GP = om.params_from_plan(pl["g_params"], pl["g_seed"])
        DP = om.params_from_plan(pl["d_params"], pl["d_seed"])
        if perturb:
            g = torch.Generator().manual_seed(perturb)
            with torch.no_grad():
                for v in list(GP.t.values()) + list(DP.t.values()):
                    v.mul_(1 + 6e-8 * torch.randn(v.shape, generator=g))
        gen, g_loss = om.WGANGP(GP, DP).generator_trainstep(B, om.Draw(seed))
        return float(g_loss.detach()), tensor_summary(gen.detach()), grad_rows(GP, gnames)

    spread, lerr = [], []
    for t in range(1, trials + 1):
        l32, _, r32 = fp32_step(16, 421, t)
        spread.append(grad_norm_stats(r32, rows))
        lerr.append(rel_err([l32], out["g16_loss"]))
        print("g16 spread", t, spread[-1], lerr[-1], flush=True)
    out["g16_fp32_spread"], out["g16_loss_fp32_spread"] = np.asarray(spread), np.asarray(lerr)
    np.savez_compressed(os.path.join(HERE, "f64_g16.npz"), **out)

    # B=64 (the headline batch) is NOT written here: the oracle's fp32 generator step needs ~100 GiB
    # of host memory there, beyond this container; tests/test_headline_gpu.py runs it on the GPU
    # box's host inside the test, with bars from the B=16 spread above.


# The B=16 generator step's float64 forward puts ONE PReLU input on the kink: G13_5's main mapping
# network, layer 10 (block0.mapping_network.net.32), sample 11, channel 209, z = 5.24e-7 (|z| ~ 0.8
# elsewhere).  An fp32 evaluation's ~1e-6 forward rounding decides which branch of the PReLU it
# takes, and the two branches' gradients differ by 2.8e-2 in that layer's BatchNorm bias (1.5e-2
# below it): a perturbation of that layer's pre-activations by 1e-6 (relative, random) moves the
# float64 step to exactly the GPU's numbers (tools/g16_map_diag.py; no such jump at 1e-7).  The
# reference's own fp32 run lands on the float64 side, the GPU's on the other.  kink_main() adds the
# float64 truth of the OTHER branch (same step, that one PReLU derivative taken as the slope).
KINK = ("block0.mapping_network.net.32", 11, 209)


def kink_main():
    torch.set_num_threads(os.cpu_count() or 8)
    pl = plan()
    gnames = [n for n, _, _ in pl["g_params"]]
    name, kb, kc = KINK
    orig = om.prelu
    seen = {}

    def prelu(P, pre, x, c):
        if pre != name:
            return orig(P, pre, x, c)
        a = P(f"{pre}.weight", (c,), "prelu")
        seen["z"] = float(x[kb, kc])
        mask = x > 0
        mask[kb, kc] = ~mask[kb, kc]                    # the other branch at the kink element
        return torch.where(mask, x, a * x)

    om.prelu = prelu
    smooth32 = om._SMOOTH
    om._SMOOTH = smooth32.to(DT)
    GP, DP = params64(pl["g_params"], pl["g_seed"]), params64(pl["d_params"], pl["d_seed"])
    _gen, g_loss = om.WGANGP(GP, DP).generator_trainstep(16, Draw64(421))
    om._SMOOTH, om.prelu = smooth32, orig
    rows = grad_rows(GP, gnames)
    path = os.path.join(HERE, "f64_g16.npz")
    cur = dict(np.load(path))
    cur["g16_grads_kink"] = rows
    cur["g16_loss_kink"] = np.asarray([float(g_loss.detach())])
    cur["kink_z"] = np.asarray([seen["z"]])
    print("kink branch: z", seen["z"], "loss", float(g_loss.detach()), "vs", float(cur["g16_loss"][0]),
          "grads vs the float64 branch", grad_norm_stats(rows, cur["g16_grads"]), flush=True)
    np.savez_compressed(path, **cur)


if __name__ == "__main__":
    if "--kink" in sys.argv:
        kink_main()
        sys.exit(0)
    if "--headline" in sys.argv:
        headline_main()
        sys.exit(0)
    if "--progan" in sys.argv:   # --trials N: fp32 draws for the spread (default 6; the fixture uses 24)
        progan_main(int(sys.argv[sys.argv.index("--trials") + 1]) if "--trials" in sys.argv else 6)
        sys.exit(0)
    if "--lazy" in sys.argv:
        lazy_main()
        sys.exit(0)
    if "--spread-only" in sys.argv:     # add/refresh only the fp32 spread entry
        torch.set_num_threads(os.cpu_count() or 8)
        path = os.path.join(HERE, "f64_truth.npz")
        cur = dict(np.load(path))
        if "--steps" in sys.argv:
            cur.update(step_spread())
        else:
            cur["g_out_fp32_spread"] = g_out_spread()
        np.savez_compressed(path, **cur)
    else:
        main()
