"""The measured WGAN-GP iteration (train/wgangp.py:20-71 with n_critic critic steps per generator
step) as replayed HIP graphs, and its eager twin in the same stream order.

bench.py times ``Iteration.step`` and tests/test_pipeline_gpu.py checks that one replay equals one
``Iteration.eager`` call bit for bit, so the number the bench reports comes from a tested path.

Fake batches (no-grad generator forward, 41 % of a critic step's FLOPs) depend on G's weights only,
and G does not change during the n_critic critic steps, so they need not be made inside each step:

* ``fake_groups`` splits the n_critic fake batches into groups; a group of k is ONE generator
  forward over k * B samples with segmented BatchNorm (wgangp.Train.generate_fakes: per-B
  statistics, running statistics updated k times in order) -- wider launches that fill the chip
  better than k B-sample forwards.  k * B is bounded by the convs' 2^31-byte operand limit
  (B = 64: k <= 4).
* ``overlap=True``: group j + 1 is replayed on a second HIP stream while the
  critic steps of group j (critic passes, gradient penalty, N > 1: the RCCL all-reduce, AdamW) run
  on the main stream.  Every group has its own graph and output buffers; the groups share one
  memory pool, apart from the critic and generator graphs' pool.

Each critic step copies its fake batch into the critic graph's fixed input (3 MB).  ``overlap=False``
with groups of 1 is the reference's order: one graph per phase, the fake batch made inside the
critic step's graph (N = 1: backward + optimizer step in one graph).

Randomness: every consumer that can run concurrently with another owns its Philox stream
(rng.py DeviceRNG.fork): the generator's z and noise come from ``tr.rng_g`` (stream 1), the
critic's eps from ``tr.rng`` (stream 0), the synthetic real batches from stream 2.  The per-stream
draw order is the same in the replay and in ``eager``, so both draw identical numbers.

N > 1: the flat gradient of each optimizer step is all-reduced between the backward graph and the
optimizer graph (collectives stay outside capture).
"""
from __future__ import annotations

import os

import torch

from .dist import allreduce_mean_


def _sync_none(flat):
    return flat


class Iteration:
    """``Iteration(tr, B, n_critic, world)``; ``capture()`` once after an eager warm-up, then
    ``step()`` replays one iteration.  ``eager()`` runs the same iteration without graphs.
    ``fake_groups``: sizes of the fake-batch groups (default n_critic groups of 1).
    ``real_source``: callable returning a synthetic real batch (default: device Philox stream 2 of
    ``tr.rng``, N(0,1) [B,3,64,64], the reference's ImageNet-normalised scale)."""

    def __init__(self, tr, B, n_critic=5, world=1, overlap=True, real_source=None, allreduce=None,
                 fake_groups=None):
        self.tr, self.B, self.n_critic, self.world, self.overlap = tr, B, n_critic, world, overlap
        self.groups = [int(k) for k in fake_groups] if fake_groups else [1] * n_critic
        if sum(self.groups) != n_critic or min(self.groups) < 1:
            raise ValueError(f"fake_groups {self.groups} do not split {n_critic} critic steps")
        self.grouped = overlap or max(self.groups) > 1       # fake batches in graphs of their own
        self.dev = tr.device
        tr.rng_g                             # create the generator's RNG stream now (snapshot sees it)
        if real_source is None:
            data = tr.rng.fork(2)
            real_source = lambda: data.randn((B, 3, 64, 64))       # noqa: E731
        self.real = real_source
        self.allreduce = allreduce if allreduce is not None else (allreduce_mean_ if world > 1 else _sync_none)
        self.graphs = {}
        self._captured = False
        self.count_nodes = False        # set before capture(): count each graph's nodes (dispatches)
        self.nodes = {}

    def _fakes(self, k):
        tr = self.tr
        return tr.generate_fakes(k, self.B) if hasattr(tr, "generate_fakes") else [tr.generate_fake(self.B)]

    # ---- eager ---------------------------------------------------------------------------
    def eager(self):
        """One iteration without graphs, in the stream order of ``step`` (fake batches group by
        group, each critic step on a real batch; n_critic times; then the generator step)."""
        tr, B = self.tr, self.B
        out = []
        fakes, groups = [], list(self.groups)
        for _ in range(self.n_critic):
            if not fakes:
                fakes = list(self._fakes(groups.pop(0)))
            fake = fakes.pop(0)
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
        # the warm-up's blocks are cached against the throw-away stream s, where nothing can reuse
        # them: hand them back before the capture fills its pool (without this every phase graph
        # left its eager peak behind)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        g = torch.cuda.CUDAGraph(keep_graph=self.count_nodes)
        with torch.cuda.graph(g, pool=pool):
            fn()
        if self.count_nodes:            # dispatches per replay (bench.py reports them per iteration)
            from ._lib import graph_node_counts
            self.nodes[id(g)] = graph_node_counts(g.raw_cuda_graph())
            g.instantiate()
        if os.environ.get("DP_MEMLOG") == "1":
            torch.cuda.synchronize()
            print(f"[mem] captured {getattr(fn, '__name__', fn)}: allocated {torch.cuda.memory_allocated() / 2**30:.1f} "
                  f"GiB, reserved {torch.cuda.memory_reserved() / 2**30:.1f} GiB", flush=True)
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
        g = {}
        if self.grouped:
            bufs = [{} for _ in self.groups]

            def fakes(j):
                def f():
                    bufs[j]["x"] = self._fakes(self.groups[j])
                return f

            # with overlap the fake groups replay beside the critic graphs, so not in their pool; but
            # never beside each other (group j + 1 is issued after group j on the stream that ran it,
            # or on the side stream after it waited for the main one), in capture order: one pool for
            # all of them (one per group held ~13 GB more at B = 64)
            fpool = torch.cuda.graph_pool_handle() if self.overlap else pool
            g["fake"] = [self._capture(fakes(j), fpool) for j in range(len(self.groups))]
            g["fake"][0].replay()                # a valid fake batch for the critic capture
            self.xin = bufs[0]["x"][0].clone()
            self.bufs = bufs
            g["critic"] = self._capture(lambda: tr.discriminator_backward(self.real(), B, gen_imgs=self.xin), pool)
            g["dstep"] = self._capture(tr.optimizer_D.step, pool)
            self.side = torch.cuda.Stream()
        else:
            crit = lambda: tr.discriminator_backward(self.real(), B)     # noqa: E731
            if self.world == 1:
                g["critic"] = self._capture(lambda: (crit(), tr.optimizer_D.step()), pool)
            else:
                g["critic"] = self._capture(crit, pool)
                g["dstep"] = self._capture(tr.optimizer_D.step, pool)
        gen = lambda: tr.generator_backward(B)                          # noqa: E731
        if self.world == 1:
            g["gen"] = self._capture(lambda: (gen(), tr.optimizer_G.step()), pool)
        else:
            g["gen"] = self._capture(gen, pool)
            g["gstep"] = self._capture(tr.optimizer_G.step, pool)
        self.graphs = g
        torch.cuda.synchronize()
        self._captured = True

    def _critic_step(self):
        g = self.graphs
        g["critic"].replay()
        if "dstep" in g:
            self.allreduce(self.tr.optimizer_D.flat.grad)
            g["dstep"].replay()

    def step(self):
        """Replay one iteration."""
        assert self._captured, "capture() first"
        g = self.graphs
        if self.grouped:
            cur = torch.cuda.current_stream()
            g["fake"][0].replay()                # G changed in the previous generator step
            n = len(self.groups)
            for j, k in enumerate(self.groups):
                ahead = j + 1 < n
                if ahead and self.overlap:       # the next group's fake batches, concurrently
                    self.side.wait_stream(cur)
                    with torch.cuda.stream(self.side):
                        g["fake"][j + 1].replay()
                for q in range(k):
                    with torch.no_grad():        # (the critic step marks its fake batch requires_grad)
                        self.xin.copy_(self.bufs[j]["x"][q])
                    self._critic_step()
                if ahead:
                    if self.overlap:
                        cur.wait_stream(self.side)
                    else:
                        g["fake"][j + 1].replay()
        else:
            for _ in range(self.n_critic):
                self._critic_step()
        g["gen"].replay()
        if "gstep" in g:
            self.allreduce(self.tr.optimizer_G.flat.grad)
            g["gstep"].replay()

    def dispatches(self):
        """Graph nodes one ``step()`` replays, by type (``count_nodes`` set before ``capture``):
        the fake groups once each, the critic (and AdamW) graphs n_critic times, the generator
        step once."""
        g = self.graphs
        reps = [(x, 1) for x in g.get("fake", [])] + [(g["critic"], self.n_critic)]
        reps += [(g["dstep"], self.n_critic)] if "dstep" in g else []
        reps += [(g["gen"], 1)] + ([(g["gstep"], 1)] if "gstep" in g else [])
        out = {}
        for x, k in reps:
            for key, v in self.nodes.get(id(x), {}).items():
                out[key] = out.get(key, 0) + k * v
        return out

    def phase_ms(self):
        """One replay per phase graph, each timed alone (outside the timed region; N = 1).  The
        fake phase is the first group's graph (``groups[0]`` batches)."""
        out = {}
        items = [(k, v[0] if isinstance(v, list) else v) for k, v in self.graphs.items()]
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


def snapshot(tr, device=None):
    """The training state (``device``: where the copies live, default alongside the originals)."""
    st = [t.detach().to(device, copy=True) if device is not None else t.detach().clone() for t in training_state(tr)]
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
