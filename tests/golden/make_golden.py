"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE in this container.

Run here only (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does (SURVEY.md §8(c) golden-vector plan):
  * imports ``generators/generator_13_5.py``, ``discriminators/discriminator_9_4.py`` and
    ``train/wgangp.py`` from /root/reference, with no-op stubs for the GUI/IO-only modules
    ``tqdm.tk`` and ``torchvision`` (they never touch step arithmetic);
  * overwrites the parameters with the documented rule of ``oracle/params.py``;
  * injects randomness by seeding the global CPU generator right before each call, so the
    reference's own ``torch.randn``/``torch.rand`` draws (z, the 253 in-forward noise tensors,
    eps) come out in a documented order that the build replays;
  * records the parameter plan (names/kinds/shapes), the conv trace, the noise draw order, module
    outputs, one D-step and one G-step (losses, per-tensor gradient summaries, AdamW deltas).

No reference source is copied: only numbers are written.
"""
from __future__ import annotations

import json
import os
import sys
import time
import types

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def _install_stubs():
    import matplotlib
    matplotlib.use("Agg")

    class _Bar:
        def __init__(self, *a, **k):
            pass

        def set_postfix(self, *a, **k):
            pass

        update = reset = close = set_postfix

    m = types.ModuleType("tqdm.tk")
    m.tqdm = _Bar
    sys.modules["tqdm.tk"] = m
    tv = types.ModuleType("torchvision")
    tvu = types.ModuleType("torchvision.utils")
    tvu.make_grid = lambda *a, **k: None
    tvu.save_image = lambda *a, **k: None
    tv.utils = tvu
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.utils"] = tvu


_install_stubs()
sys.path.insert(0, REF)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from generators.generator_13_5 import Generator  # noqa: E402
from discriminators.discriminator_9_4 import Discriminator  # noqa: E402
from train import wgangp  # noqa: E402

from oracle.params import fill_module, param_kinds, tensor_summary  # noqa: E402

G_SEED, D_SEED = 1, 2
torch.set_num_threads(os.cpu_count() or 8)


class Tracer:
    """Records every conv / convT the reference issues and every randn shape."""

    def __init__(self):
        self.convs, self.randn = [], []
        self.on = False

    def __enter__(self):
        self._c2, self._ct, self._rn = F.conv2d, F.conv_transpose2d, torch.randn
        tr = self

        def conv2d(x, w, bias=None, stride=1, padding=0, dilation=1, groups=1):
            if tr.on:
                s = stride if isinstance(stride, int) else stride[0]
                tr.convs.append(["conv", int(w.shape[1]), int(w.shape[0] // groups), int(w.shape[2]),
                                 int(s), int(x.shape[2]), int(x.shape[3]), int(groups)])
            return tr._c2(x, w, bias, stride, padding, dilation, groups)

        def conv_t(x, w, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1):
            if tr.on:
                s = stride if isinstance(stride, int) else stride[0]
                tr.convs.append(["convT", int(w.shape[0]), int(w.shape[1]), int(w.shape[2]), int(s),
                                 int(x.shape[2]), int(x.shape[3]), 1])
            return tr._ct(x, w, bias, stride, padding, output_padding, groups, dilation)

        def randn(*size, **kw):
            if tr.on:
                shp = size[0] if len(size) == 1 and isinstance(size[0], (tuple, list)) else size
                tr.randn.append([int(s) for s in shp])
            return tr._rn(*size, **kw)

        F.conv2d, F.conv_transpose2d, torch.randn = conv2d, conv_t, randn
        return self

    def __exit__(self, *a):
        F.conv2d, F.conv_transpose2d, torch.randn = self._c2, self._ct, self._rn


def build_pair():
    G = Generator(256)
    D = Discriminator()
    gk = fill_module(G, G_SEED)
    dk = fill_module(D, D_SEED)
    return G, D, gk, dk


def grad_table(mod):
    rows, has = [], []
    for _, p in mod.named_parameters():
        if p.grad is None:
            rows.append([np.nan] * 11)
            has.append(0)
        else:
            rows.append(tensor_summary(p.grad))
            has.append(1)
    return np.asarray(rows, np.float64), np.asarray(has, np.int8)


def delta_table(mod, before, lr):
    rows = []
    for (_, p), b in zip(mod.named_parameters(), before):
        rows.append(tensor_summary((p.detach() - b) / lr))
    return np.asarray(rows, np.float64)


def main():
    t0 = time.time()
    plan = {"torch": torch.__version__, "g_seed": G_SEED, "d_seed": D_SEED}
    G, D, gk, dk = build_pair()
    plan["g_params"] = [[n, k, list(s)] for n, k, s in gk]
    plan["d_params"] = [[n, k, list(s)] for n, k, s in dk]
    plan["g_buffers"] = [n for n, _ in G.named_buffers()]
    print("built", time.time() - t0, flush=True)

    # ---- G forward, B=4 -------------------------------------------------------------
    B = 4
    z = torch.randn(B, 256, 1, 1, generator=torch.Generator().manual_seed(100))
    stages = {}

    def hook(name):
        def f(_m, _i, out):
            outs = out if isinstance(out, tuple) else (out,)
            stages[name] = [tensor_summary(o) for o in outs]
        return f

    hs = [getattr(G, f"block{i}").register_forward_hook(hook(f"block{i}")) for i in range(5)]
    with Tracer() as tr, torch.no_grad():
        torch.manual_seed(101)
        tr.on = True
        out = G(z)
        tr.on = False
    for h in hs:
        h.remove()
    plan["g_conv_trace_b4"] = tr.convs
    plan["g_noise_shapes_b4"] = tr.randn
    buf = np.asarray([[float(b.double().sum()), float(b.double().norm())] for _, b in G.named_buffers()])
    np.savez_compressed(os.path.join(HERE, "g_fwd_b4.npz"), z=z.numpy(), out=out.numpy(), buffers=buf,
                        **{f"stage_{k}": np.asarray(v) for k, v in stages.items()})
    print("g fwd", time.time() - t0, flush=True)

    # ---- D forward, B=4 and B=8 -----------------------------------------------------
    dres = {}
    for B in (4, 8):
        x = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(200 + B))
        with Tracer() as tr, torch.no_grad():
            tr.on = True
            dres[f"out_b{B}"] = D(x).numpy()
            tr.on = False
        if B == 4:
            plan["d_conv_trace_b4"] = tr.convs
    np.savez_compressed(os.path.join(HERE, "d_fwd.npz"), **dres)
    print("d fwd", time.time() - t0, flush=True)

    # ---- one D-step (wgangp.py:56-71) at B=4 and B=8 -----------------------------------
    for B, img_seed, rng_seed in ((4, 300, 301), (8, 310, 311)):
        G, D, _, _ = build_pair()
        tr_ = wgangp.Train([0] * 10, torch.device("cpu"), 1, 256, G, "G13_5", D, "D9_4")
        images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(img_seed))
        before = [p.detach().clone() for p in D.parameters()]
        torch.manual_seed(rng_seed)
        real_loss, fake_loss, gp = tr_.discriminator_trainstep(images, B)
        gt, has = grad_table(D)
        dt = delta_table(D, before, 4e-4)
        np.savez_compressed(os.path.join(HERE, f"d_step_b{B}.npz"),
                            losses=np.asarray([float(real_loss), float(fake_loss), float(gp)]),
                            grads=gt, has_grad=has, deltas=dt)
        print(f"d step b{B}", [float(real_loss), float(fake_loss), float(gp)], time.time() - t0, flush=True)
        del G, D, tr_, before

    # ---- one G-step (wgangp.py:20-27) at B=4 -------------------------------------------
    B = 4
    G, D, _, _ = build_pair()
    tr_ = wgangp.Train([0] * 10, torch.device("cpu"), 1, 256, G, "G13_5", D, "D9_4")
    before = [p.detach().clone() for p in G.parameters()]
    torch.manual_seed(401)
    gen_imgs, g_loss = tr_.generator_trainstep(B)
    gt, has = grad_table(G)
    dt = delta_table(G, before, 1e-4)
    np.savez_compressed(os.path.join(HERE, "g_step_b4.npz"), g_loss=np.asarray([float(g_loss)]),
                        gen=np.asarray(tensor_summary(gen_imgs)), grads=gt.astype(np.float32),
                        has_grad=has, deltas=dt.astype(np.float32))
    print("g step", float(g_loss), time.time() - t0, flush=True)

    with open(os.path.join(HERE, "plan.json"), "w") as f:
        json.dump(plan, f)
    print("done", time.time() - t0)


if __name__ == "__main__":
    main()
