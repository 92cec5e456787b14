"""Parity at the batches the benchmarks run (the B=4/8 fixtures of test_models_gpu.py exercise
other launch schedules: at B=64 the generator step runs split-K tails, frame-split dgrads, style-
bank tiles and branch streams that B=4 never reaches).

test_g_step_b16              generator step (train/wgangp.py:20-27) at B=16 against the REFERENCE's
                             own fixture (tests/golden/make_golden_g16.py: 47 GiB of host memory,
                             the largest batch its per-sample modulated weights allow) and float64
                             truth (make_f64.py --headline): gradients within 2x the fp32 spread.
test_g_step_b64_vs_oracle    the headline batch: the CPU oracle (pinned to the reference at B=4 and
                             B=16) runs the same step on the host in this test (~100 GiB, ~1 min on
                             16 threads); GPU within the bars the oracle meets against the reference.
test_lazy_critic_b128_vs_oracle  config 4's regularised critic step (R1 + R2 + GP, 3B = 384 samples
                             through the critic program) at B=128.
test_progan_steps_b64_vs_oracle  config 5's pair, critic and generator step at B=64.

Randomness: ReplayRNG(seed) on the GPU and oracle.model.Draw(seed) on the host replay the same
CPU generator in the reference's call order.
"""
import gc
import json
import os

import numpy as np
import pytest
import torch

from oracle.params import fill_module, tensor_summary
from tests._util import D_BAR, G_BAR, GOLDEN, check_grads, fixture, grad_norm_stats, plan, rel_err

# host-side oracle runs of minutes each (16 threads): longer than the suite's per-test limit
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
DEV = "cuda"


@pytest.fixture(scope="module")
def gan():
    import gan_amd
    return gan_amd


@pytest.fixture(scope="module")
def P():
    return plan()


def _rows(mod, names):
    params = dict(mod.named_parameters())
    return np.asarray([tensor_summary(params[n].grad) if params[n].grad is not None else [np.nan] * 11 for n in names])


def _pair(gan, P):
    G = gan.Generator(256)
    fill_module(G, P["g_seed"])
    D = gan.Discriminator()
    fill_module(D, P["d_seed"])
    return G.to(DEV), D.to(DEV)


def _free(*objs):
    del objs
    gc.collect()
    torch.cuda.empty_cache()


def _threads():
    torch.set_num_threads(min(16, os.cpu_count() or 8))


def test_g_step_b16(gan, P):
    fx = fixture("g_step_b16.npz")
    t64 = fixture("f64_g16.npz")
    G, D = _pair(gan, P)
    tr = gan.Train([0] * 10, DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.ReplayRNG(421, DEV))
    # The float64 forward of this step puts ONE PReLU input on the kink (make_f64.py KINK: the main
    # mapping network's layer 10 = block0.mapping_network.net.32, sample 11, channel 209, z = 5.2e-7
    # against |z| ~ 0.8): fp32's ~1e-6 forward rounding picks the branch, and the two branches'
    # gradients differ by 2.8e-2 in that layer's BatchNorm bias and ~1.5e-2 in every mapping layer
    # below it (a 1e-6 perturbation of the float64 forward there reproduces the GPU's numbers;
    # tools/g16_map_diag.py).  The test reads the branch the GPU took from the sign of that
    # layer's output element (PReLU keeps the sign: its slope there is positive) and holds the GPU
    # to the float64 truth OF THAT BRANCH (g16_grads: z > 0; g16_grads_kink: the same step with that
    # one PReLU derivative taken as the slope), at the same bars -- 2x the reference's / the fp32 spread.
    mod = gan.generator_13_5
    kink_act = G.block0.mapping_network.net[32]
    seen = []
    inner = mod._lin_bn_act

    def spy(lin, bn, act, z):
        out = inner(lin, bn, act, z)
        if act is kink_act:
            seen.append(float(out.detach()[209, 11]))           # [C][B] layout
        return out
    mod._lin_bn_act = spy
    try:
        gen, g_loss = tr.generator_trainstep(16)
    finally:
        mod._lin_bn_act = inner
    assert len(seen) == 1, seen
    assert float(kink_act.weight.detach()[209]) > 0
    names = [n for n, _, _ in P["g_params"]]
    rows = _rows(G, names)
    loss = float(g_loss.detach())
    assert rel_err([loss], fx["g_loss"]) < 1e-4, (loss, fx["g_loss"])
    assert rel_err(tensor_summary(gen), fx["gen"]) < 1e-3
    has = np.asarray([0 if np.isnan(r[0]) else 1 for r in rows])
    assert (has == fx["has_grad"]).all()
    side = "float64 branch" if seen[0] > 0 else "other branch at the kink"
    truth = t64["g16_grads"] if seen[0] > 0 else t64["g16_grads_kink"]
    got = grad_norm_stats(rows, truth)
    worst = np.maximum(t64["ref_g16_stats"], t64["g16_fp32_spread"].max(axis=0))
    bars = [2 * w + 1e-5 for w in worst]
    print(f"G-step B=16: kink element {seen[0]:.3e} -> {side}; vs its f64 truth {got}; "
          f"reference {t64['ref_g16_stats']} bars {bars}")
    assert all(g <= b for g, b in zip(got, bars)), (side, got, bars)
    assert rel_err([loss], t64["g16_loss"]) <= 2 * max(float(t64["ref_g16_loss_err"]),
                                                       float(t64["g16_loss_fp32_spread"].max())) + 1e-6


def test_g_step_b64_vs_oracle(gan, P):
    from oracle import model as om
    B, seed = 64, 431
    G, D = _pair(gan, P)
    tr = gan.Train([0] * 10, DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.ReplayRNG(seed, DEV))
    gen, g_loss = tr.generator_trainstep(B)
    names = [n for n, _, _ in P["g_params"]]
    rows, loss, gsum = _rows(G, names), float(g_loss.detach()), tensor_summary(gen)
    _free(G, D, tr, gen, g_loss)

    _threads()
    GP = om.params_from_plan(P["g_params"], P["g_seed"])
    DP = om.params_from_plan(P["d_params"], P["d_seed"])
    ogen, og_loss = om.WGANGP(GP, DP).generator_trainstep(B, om.Draw(seed))
    want = np.asarray([tensor_summary(GP.t[n].grad) if n in GP.t and GP.t[n].grad is not None else [np.nan] * 11
                       for n in names])
    oloss, osum = float(og_loss.detach()), tensor_summary(ogen.detach())
    del GP, DP, ogen, og_loss
    gc.collect()
    print("G-step B=64: loss", loss, "oracle", oloss, "grad stats vs oracle", grad_norm_stats(rows, want))
    assert rel_err([loss], [oloss]) < 1e-4
    assert rel_err(gsum, osum) < 1e-3
    # GPU and oracle are two fp32 evaluations, each about as far from float64 truth as the fp32
    # spread measured at B=16 (f64_g16.npz; BatchNorm over 64 samples conditions no worse): bars
    # = 2x that spread, and never tighter than the B=4 bars the oracle meets vs the reference
    t64 = fixture("f64_g16.npz")
    w = np.maximum(t64["ref_g16_stats"], t64["g16_fp32_spread"].max(axis=0))
    bar = {k: max(G_BAR[k], 2 * float(v)) for k, v in zip(("median", "p99", "max", "vec"), w)}
    check_grads(rows, want, bar)


def test_lazy_critic_b128_vs_oracle(gan, P):
    from oracle import model as om
    B, img_seed, seed = 128, 520, 521
    images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(img_seed))
    G, D = _pair(gan, P)
    tr = gan.wganlazygpR2.Train([0] * 10, DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.ReplayRNG(seed, DEV))
    tr.optimizer_D.zero_grad()
    out = tr.discriminator_backward(images.to(DEV), B, 0)          # R1 + R2 + GP: 3B = 384 samples
    losses = [float(v.detach().reshape(-1)[0]) for v in out]
    names = [n for n, _, _ in P["d_params"]]
    rows = _rows(D, names)
    _free(G, D, tr, out)

    _threads()
    GP = om.params_from_plan(P["g_params"], P["g_seed"])
    DP = om.params_from_plan(P["d_params"], P["d_seed"])
    want_l = [float(v.detach().reshape(-1)[0]) for v in
              om.WGANLazyR2(GP, DP).discriminator_trainstep(images, B, 0, om.Draw(seed))]
    want = np.asarray([tensor_summary(DP.t[n].grad) if n in DP.t and DP.t[n].grad is not None else [np.nan] * 11
                       for n in names])
    del GP, DP
    gc.collect()
    print("lazy critic B=128: losses", losses, "oracle", want_l, "grad stats", grad_norm_stats(rows, want))
    assert rel_err(losses, want_l) < 1e-3, (losses, want_l)
    check_grads(rows, want, D_BAR)


def test_progan_steps_b64_vs_oracle(gan):
    from oracle import model as om
    with open(os.path.join(GOLDEN, "plan_progan.json")) as f:
        pp = json.load(f)
    B = 64

    def pair():
        G = gan.generator_3_progan.Generator(1, 256, pp["ngf"], 3)
        D = gan.discriminator_3_wgangp_progan.Discriminator(1, pp["ndf"], 3)
        fill_module(G, pp["g_seed"])
        fill_module(D, pp["d_seed"])
        return G.to(DEV), D.to(DEV)

    def oracle_pair():
        return (om.params_from_plan(pp["g_params"], pp["g_seed"]), om.params_from_plan(pp["d_params"], pp["d_seed"]))

    dn, gn = [n for n, _, _ in pp["d_params"]], [n for n, _, _ in pp["g_params"]]
    images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(730))
    _threads()
    # critic step
    G, D = pair()
    tr = gan.Train([0] * 10, DEV, 1, 256, G, "G3_progan", D, "D3_progan", rng=gan.ReplayRNG(731, DEV))
    losses = [float(v.detach()) for v in tr.discriminator_backward(images.to(DEV), B)]
    drows = _rows(D, dn)
    GP, DP = oracle_pair()
    otr = om.WGANGP(GP, DP, gen=om.progan_generator, disc=om.progan_discriminator)
    want_l = [float(v.detach()) for v in otr.discriminator_trainstep(images, B, om.Draw(731))]
    dwant = np.asarray([tensor_summary(DP.t[n].grad) if n in DP.t and DP.t[n].grad is not None else [np.nan] * 11 for n in dn])
    print("progan critic B=64", losses, want_l, grad_norm_stats(drows, dwant))
    assert rel_err(losses, want_l) < 1e-3, (losses, want_l)
    check_grads(drows, dwant, D_BAR)
    # generator step
    G, D = pair()
    tr = gan.Train([0] * 10, DEV, 1, 256, G, "G3_progan", D, "D3_progan", rng=gan.ReplayRNG(741, DEV))
    _gen, g_loss = tr.generator_backward(B)
    grows = _rows(G, gn)
    def oracle_g(perturb):
        GP, DP = oracle_pair()
        if perturb:      # ~1 ulp relative on every weight: one more fp32 evaluation order
            gg = torch.Generator().manual_seed(perturb)
            with torch.no_grad():
                for v in list(GP.t.values()) + list(DP.t.values()):
                    v.mul_(1 + 6e-8 * torch.randn(v.shape, generator=gg))
        otr = om.WGANGP(GP, DP, gen=om.progan_generator, disc=om.progan_discriminator)
        _ogen, og_loss = otr.generator_trainstep(B, om.Draw(741))
        return float(og_loss.detach()), np.asarray(
            [tensor_summary(GP.t[n].grad) if n in GP.t and GP.t[n].grad is not None else [np.nan] * 11 for n in gn])

    oloss, gwant = oracle_g(0)
    # the progan generator's gradient statistics are heavy-tailed between fp32 evaluation orders
    # (its B=4 test uses 24 perturbed oracle draws): bars = 3x the distance between two oracle
    # evaluations (one perturbed by ~1 ulp), never tighter than G_BAR
    spread = grad_norm_stats(oracle_g(1)[1], gwant)
    bar = {k: max(G_BAR[k], 3 * float(v)) for k, v in zip(("median", "p99", "max", "vec"), spread)}
    print("progan generator B=64", float(g_loss.detach()), oloss, grad_norm_stats(grows, gwant), "oracle spread", spread)
    assert rel_err([float(g_loss.detach())], [oloss]) < 1e-4
    check_grads(grows, gwant, bar)


def test_lazy_bf16_b128(gan, P):
    """Config 4 as benchmarked: the bf16 plain critic step and the bf16 generator step at B=128
    (train/wganlazygpR2.py:48-77, 17-27).

    (1) Per op: a sample of the generator step's conv GEMM launches (forward with the x*s gather and
        *d / noise epilogue, dgrad, wgrad; every 11th) re-evaluated in float64 with both operands
        rounded to bf16 at the kernels' rounding points (tests/_emu.py) -- only fp32 accumulation
        order remains, bar 1e-5.  (The critic's launches at 2B = 256: test_critic_bf16_matches_emulation.)
    (2) End to end, the generator step against the same step in fp32 on the same inputs (device
        Philox draws, same seed), and the plain critic step against the fp32 CPU oracle: bf16 is
        measurably on and within bf16's reach.  Bars: losses 2e-2 (the fake loss and the
        generator loss carry G13_5's ~100 sequential layers: 8e-2, as at B=4 in
        test_models_gpu.py::test_lazy_bf16_steps); gradient-norm statistics median 2e-2, vector 5e-2
        (bf16 operands carry 2^-9 relative rounding per operand; measured values are printed)."""
    from oracle import model as om
    from tests._emu import Recorder
    B, seed = 128, 811

    def gen_step(precision, record=False):
        G, D = _pair(gan, P)
        tr = gan.wganlazygpR2.Train([0] * 10, DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.DeviceRNG(DEV, seed),
                                    precision=precision)
        rec = Recorder(every=11, cap=40) if record else None
        if rec:
            with rec:
                _gen, g_loss = tr.generator_backward(B)
        else:
            _gen, g_loss = tr.generator_backward(B)
        torch.cuda.synchronize()
        rows = _rows(G, [n for n, _, _ in P["g_params"]])
        return float(g_loss.detach()), rows, rec

    loss_bf, rows_bf, rec = gen_step("bf16", record=True)
    assert all(c["math"] == gan._lib.MATH_BF16 for c in rec.calls) and len(rec.calls) >= 30
    _threads()
    rec.check(bf16=True, bars={"fwd": 1e-5, "dgrad": 1e-5, "wgrad": 1e-5})
    del rec
    _free()
    loss_32, rows_32, _ = gen_step("fp32")
    e_loss = rel_err([loss_bf], [loss_32])
    g_stats = grad_norm_stats(rows_bf, rows_32)
    print(f"bf16 generator step B={B}: loss {loss_bf} vs fp32 {loss_32} (rel {e_loss:.2e}); grad stats vs fp32 {g_stats}")
    assert 1e-7 < e_loss < 8e-2
    assert g_stats[0] < 2e-2 and g_stats[3] < 5e-2, g_stats
    _free()

    # plain critic step (idx 1: no R1/R2/GP) in bf16 vs the fp32 CPU oracle
    img_seed, dseed = 812, 813
    images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(img_seed))
    G, D = _pair(gan, P)
    tr = gan.wganlazygpR2.Train([0] * 10, DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.ReplayRNG(dseed, DEV),
                                precision="bf16")
    tr.optimizer_D.zero_grad()
    out = tr.discriminator_backward(images.to(DEV), B, 1)
    losses = [float(v.detach().reshape(-1)[0]) for v in out[:2]]
    names = [n for n, _, _ in P["d_params"]]
    rows = _rows(D, names)
    _free(G, D, tr, out)
    GP = om.params_from_plan(P["g_params"], P["g_seed"])
    DP = om.params_from_plan(P["d_params"], P["d_seed"])
    want_l = [float(v.detach().reshape(-1)[0]) for v in
              om.WGANLazyR2(GP, DP).discriminator_trainstep(images, B, 1, om.Draw(dseed))[:2]]
    want = np.asarray([tensor_summary(DP.t[n].grad) if n in DP.t and DP.t[n].grad is not None else [np.nan] * 11
                       for n in names])
    del GP, DP
    gc.collect()
    er, ef = rel_err(losses[:1], want_l[:1]), rel_err(losses[1:], want_l[1:])
    d_stats = grad_norm_stats(rows, want)
    print(f"bf16 plain critic step B={B}: losses {losses} vs fp32 oracle {want_l} (rel {er:.2e} / {ef:.2e}); "
          f"grad stats {d_stats}")
    assert 1e-7 < er < 2e-2 and 1e-7 < ef < 8e-2
    assert d_stats[0] < 2e-2 and d_stats[3] < 5e-2, d_stats
