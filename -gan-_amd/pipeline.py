"""The measured WGAN-GP iteration (train/wgangp.py:20-71 with n_critic critic steps per generator
step) as replayed HIP graphs, and its eager twin in the same stream order.

bench.py times ``Iteration.step`` and tests/test_pipeline_gpu.py checks that one replay equals one
``Iteration.eager`` call bit for bit, so the number the bench reports comes from a tested path.

Graph mode, ``overlap=True`` (the headline schedule): the next critic step's
fake batch (no-grad generator forward, 41 % of a critic step's FLOPs) depends on G's weights only
-- G does not change during the n_critic steps -- so it is replayed on a second HIP stream while
this step's critic passes, gradient penalty, (N > 1: the RCCL all-reduce) and AdamW run on the
main stream.  Two copies of the fake-batch graph (own memory pools) double-buffer the batch: the
side stream writes buffer (i+1) % 2 while the critic reads buffer i % 2.

Randomness: every consumer that can run concurrently with another owns its Philox stream
(rng.py DeviceRNG.fork): the generator's z and noise come from ``tr.rng_g`` (stream 1), the
critic's eps from ``tr.rng`` (stream 0), the synthetic real batches from stream 2.  The per-stream
draw order is the same in the replay and in ``eager``, so both draw identical numbers.

N > 1: the flat gradient of each optimizer step is all-reduced between the backward graph and the
optimizer graph (collectives stay outside capture; ``sync``).  ``overlap=False`` captures one graph
per phase (N = 1: backward + optimizer step in one).

``batch_fakes=True``: the n_critic fake batches come from ONE generator forward over n_critic * B
samples with segmented BatchNorm (wgangp.Train.generate_fakes) -- wider launches that fill the
chip better than five B-sample forwards -- replayed before the first critic step.
"""
from __future__ import annotations

import torch

from .dist import allreduce_mean_


def _sync_none(flat):
    return flat


class Iteration:
    """``Iteration(tr, B, n_critic, world)``; ``capture()`` once after an eager warm-up, then
    ``step()`` replays one iteration.  ``eager()`` runs the same iteration without graphs.
    ``real_source``: callable returning a synthetic real batch (default: device Philox stream 2 of
    ``tr.rng``, N(0,1) [B,3,64,64], the reference's ImageNet-normalised scale)."""

    def __init__(self, tr, B, n_critic=5, world=1, overlap=True, real_source=None, allreduce=None,
                 batch_fakes=False):
        self.tr, self.B, self.n_critic, self.world, self.overlap = tr, B, n_critic, world, overlap
        self.batch_fakes = batch_fakes
        if batch_fakes and not hasattr(tr, "generate_fakes"):
            raise ValueError("batch_fakes needs a trainer with generate_fakes (wgangp.Train)")
        self.dev = tr.device
        tr.rng_g                             # create the generator's RNG stream now (snapshot sees it)
        if real_source is None:
            data = tr.rng.fork(2)
            real_source = lambda: data.randn((B, 3, 64, 64))       # noqa: E731
        self.real = real_source
        self.allreduce = allreduce if allreduce is not None else (allreduce_mean_ if world > 1 else _sync_none)
        self.graphs = {}
        self._captured = False

    # ---- eager ---------------------------------------------------------------------------
    def eager(self):
        """One iteration without graphs, in the stream order of ``step`` (fake batch, then the
        critic step on a real batch; n_critic times; then the generator step)."""
        tr, B = self.tr, self.B
        out = []
        fakes = tr.generate_fakes(self.n_critic, B) if self.batch_fakes else None
        for i in range(self.n_critic):
            fake = fakes[i] if fakes is not None else tr.generate_fake(B)
            # detached: a live penalty value would keep its node -- and the critic run with all of
            # its saved activations -- alive until the iteration returns
            out.append(tuple(v.detach() for v in tr.discriminator_backward(self.real(), B, gen_imgs=fake)))
            self.allreduce(tr.optimizer_D.flat.grad)
            tr.optimizer_D.step()
        gen = tuple(v.detach() for v in tr.generator_backward(B))
        self.allreduce(tr.optimizer_G.flat.grad)
        tr.optimizer_G.step()
        return out, gen

    # ---- graphs --------------------------------------------------------------------------
    def _capture(self, fn, pool):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):          # one eager run on a side stream (allocator warm-up)
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            fn()
        return g

    def capture(self):
        """Capture the phase graphs.  Runs every phase once eagerly first (the graphs' warm-up):
        parameters and optimizer state move on; callers that need a fixed starting point restore
        it afterwards (``snapshot`` / ``restore``)."""
        tr, B = self.tr, self.B
        # All serial phase graphs share ONE memory pool: they replay one after another, so a later
        # graph may reuse what an earlier one freed (per-graph pools would hold every phase's
        # peak at once).  Graphs that replay concurrently with them get pools of their own.
        pool = torch.cuda.graph_pool_handle()
        torch.cuda.empty_cache()
        if self.batch_fakes:
            # one generator forward makes all n_critic fake batches; each critic step copies its
            # batch into the critic graph's fixed input (3 MB, a few microseconds)
            bufs = {}

            def fakes():
                bufs["x"] = tr.generate_fakes(self.n_critic, B)

            self.graphs["fake"] = self._capture(fakes, pool)
            self.graphs["fake"].replay()
            self.xin = bufs["x"][0].clone()
            self.bufs = bufs
            self.graphs["critic"] = self._capture(lambda: tr.discriminator_backward(self.real(), B, gen_imgs=self.xin),
                                                  pool)
            if self.world == 1:
                self.graphs["dstep"] = self._capture(tr.optimizer_D.step, pool)
                self.graphs["gen"] = self._capture(lambda: (tr.generator_backward(B), tr.optimizer_G.step()), pool)
            else:
                self.graphs.update(dstep=self._capture(tr.optimizer_D.step, pool),
                                   gen=self._capture(lambda: tr.generator_backward(B), pool),
                                   gstep=self._capture(tr.optimizer_G.step, pool))
        elif self.overlap:
            bufs = [{}, {}]

            def fwd(k):
                def f():
                    bufs[k]["x"] = tr.generate_fake(B)
                return f

            def crit(k):
                return lambda: tr.discriminator_backward(self.real(), B, gen_imgs=bufs[k]["x"])

            g_fwd = [None, None]
            g_crit = [None, None]
            for k in range(2):
                g_fwd[k] = self._capture(fwd(k), torch.cuda.graph_pool_handle())
                g_fwd[k].replay()                # a valid fake batch for the critic capture
                g_crit[k] = self._capture(crit(k), pool)
            self.graphs = {"fake": g_fwd, "critic": g_crit,
                           "dstep": self._capture(tr.optimizer_D.step, pool),
                           "gen": self._capture(lambda: tr.generator_backward(B), pool),
                           "gstep": self._capture(tr.optimizer_G.step, pool)}
            self.side = torch.cuda.Stream()
            self.bufs = bufs
        else:
            crit = lambda: tr.discriminator_backward(self.real(), B)     # noqa: E731
            gen = lambda: tr.generator_backward(B)                      # noqa: E731
            if self.world == 1:
                self.graphs = {"critic": self._capture(lambda: (crit(), tr.optimizer_D.step()), pool),
                               "gen": self._capture(lambda: (gen(), tr.optimizer_G.step()), pool)}
            else:
                self.graphs = {"critic": self._capture(crit, pool), "dstep": self._capture(tr.optimizer_D.step, pool),
                               "gen": self._capture(gen, pool), "gstep": self._capture(tr.optimizer_G.step, pool)}
        torch.cuda.synchronize()
        self._captured = True

    def step(self):
        """Replay one iteration."""
        assert self._captured, "capture() first"
        g, tr = self.graphs, self.tr
        if self.batch_fakes:
            g["fake"].replay()
            for i in range(self.n_critic):
                self.xin.copy_(self.bufs["x"][i])
                g["critic"].replay()
                self.allreduce(tr.optimizer_D.flat.grad)
                g["dstep"].replay()
            g["gen"].replay()
            if self.world > 1:
                self.allreduce(tr.optimizer_G.flat.grad)
                g["gstep"].replay()
        elif self.overlap:
            cur = torch.cuda.current_stream()
            g["fake"][0].replay()                # G changed in the previous generator step
            for i in range(self.n_critic):
                if i + 1 < self.n_critic:        # the next step's fake batch, concurrently
                    self.side.wait_stream(cur)   # (its buffer was last read two steps ago)
                    with torch.cuda.stream(self.side):
                        g["fake"][(i + 1) % 2].replay()
                g["critic"][i % 2].replay()
                self.allreduce(tr.optimizer_D.flat.grad)
                g["dstep"].replay()
                cur.wait_stream(self.side)
            g["gen"].replay()
            self.allreduce(tr.optimizer_G.flat.grad)
            g["gstep"].replay()
        elif self.world == 1:
            for _ in range(self.n_critic):
                g["critic"].replay()
            g["gen"].replay()
        else:
            for _ in range(self.n_critic):
                g["critic"].replay()
                self.allreduce(tr.optimizer_D.flat.grad)
                g["dstep"].replay()
            g["gen"].replay()
            self.allreduce(tr.optimizer_G.flat.grad)
            g["gstep"].replay()

    def phase_ms(self):
        """One replay per phase graph, each timed alone (outside the timed region; N = 1)."""
        out = {}
        if self.batch_fakes:
            items = [(k, self.graphs[k]) for k in ("fake", "critic", "gen")]
        elif self.overlap:
            items = [("fake", self.graphs["fake"][0]), ("critic", self.graphs["critic"][0]), ("gen", self.graphs["gen"])]
        else:
            items = list(self.graphs.items())
        for key, g in items:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            out[key] = round(e0.elapsed_time(e1), 1)
        return out


def training_state(tr):
    """Every tensor one iteration reads and writes that persists across iterations: the flat
    parameters, gradients and AdamW state of both models, the generator's BatchNorm running
    statistics, and the device RNG offsets."""
    ts = []
    for opt in (tr.optimizer_G, tr.optimizer_D):
        ts += [opt.flat.data, opt.flat.grad, opt.exp_avg, opt.exp_avg_sq, opt.step_count]
    for m in (tr.generator, tr.discriminator):
        ts += [b for b in m.buffers()]
    return ts


def snapshot(tr):
    st = [t.detach().clone() for t in training_state(tr)]
    rng = tr.rng.state() if hasattr(tr.rng, "state") else None
    return st, rng


def restore(tr, snap):
    """Put the training state back (in place: captured graphs keep their pointers) and refresh
    the packed conv weights derived from the parameters."""
    st, rng = snap
    with torch.no_grad():
        for t, v in zip(training_state(tr), st):
            t.copy_(v)
    if rng is not None:
        tr.rng.set_state(rng)
    for opt in (tr.optimizer_G, tr.optimizer_D):
        opt.flat.epoch += 1
        opt.flat.packs.repack()
