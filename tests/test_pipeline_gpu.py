"""The timed path is the tested path: bench.py's pipelined HIP-graph iteration (gan_amd.pipeline)
against the same iteration run eagerly, and the device RNG's counter discipline under the
concurrency that pipeline creates.

test_pipelined_iteration_matches_eager  one replay of the captured iteration (fake batch of the
    next critic step on a side stream, double-buffered; critic graphs; AdamW graphs; generator
    step) and one eager iteration from the same state leave bit-identical parameters, gradients,
    AdamW moments, BatchNorm statistics and RNG offsets; the eager run's draws never share a
    Philox counter.  Case "bench" is bench.py's own timed schedule at its own batch: B = 64, fake
    groups [4, 1] (one 256-sample segmented-BatchNorm generator forward + one 64-sample one), no
    side stream at N = 1 -- the exact launch plans (B = 256 patch-conv grids, B = 64 split-K tails)
    whose replay the headline number times.  The eager steps it is compared with are the trainer's
    discriminator_backward / generator_backward, which test_critic_gpu.py::test_d_step_b64 and
    test_headline_gpu.py::test_g_step_b64_vs_oracle hold to the B = 64 oracle.
test_segmented_batchnorm_op / test_generate_fakes_matches_separate_batches  the batched fake
    generation (all n_critic fake batches from one generator forward with per-segment BatchNorm
    statistics) reproduces n separate generator calls.
test_branch_noise_draws                the first generator forward at a batch size draws its noise
    per StyleConv inside ResnetInit's parallel branch streams: every draw reads the same offset
    with its own draw index (checked against the numpy Philox oracle), and the offset advances
    exactly once per forward.
test_forks_concurrent                  two Philox streams drawing concurrently on two HIP streams
    produce exactly their sequential oracle values.
"""
import numpy as np
import pytest
import torch

from oracle import philox
from tests import dp_worker

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
B = 8


@pytest.fixture(scope="module")
def gan():
    import gan_amd
    return gan_amd


def _state(tr):
    from gan_amd.pipeline import training_state
    return [t.detach().clone() for t in training_state(tr)] + [o.clone() for o in tr.rng.state().values()]


# mode -> (batch, fake groups, side stream)
MODES = {"overlap": (B, None, True), "phases": (B, None, False), "batched": (B, [1, 3, 1], True),
         "bench": (64, [4, 1], False)}


@pytest.mark.parametrize("mode", list(MODES))
def test_pipelined_iteration_matches_eager(gan, mode):
    from gan_amd.pipeline import Iteration, restore, snapshot
    bs, groups, overlap = MODES[mode]
    if mode == "bench":          # bench.py's N = 1 default schedule, as bench.fake_schedule builds it
        import bench
        assert (tuple(groups), overlap) == (bench.FAKE_GROUPS, bench.FAKE_OVERLAP)
    G, D = dp_worker.make_models(gan, DEV)
    tr = gan.Train([], DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.DeviceRNG(DEV, 2024))
    it = Iteration(tr, bs, n_critic=5, overlap=overlap, fake_groups=groups)
    it.eager()                      # warm-up: packed weights, noise shapes (bulk draws from here on)
    torch.cuda.synchronize()
    snap = snapshot(tr)
    it.capture()                    # runs every phase once more eagerly, then captures
    restore(tr, snap)
    it.step()
    torch.cuda.synchronize()
    graph = _state(tr)

    restore(tr, snap)
    logs = []
    for r in [tr.rng, tr.rng.fork(1), tr.rng.fork(2)]:
        r.log = []
        logs.append(r.log)
    it.eager()
    torch.cuda.synchronize()
    for r in [tr.rng, tr.rng.fork(1), tr.rng.fork(2)]:
        r.log = None
    eager = _state(tr)

    assert len(graph) == len(eager)
    names = ["G.data", "G.grad", "G.m", "G.v", "G.step", "D.data", "D.grad", "D.m", "D.v", "D.step"]
    for i, (a, b) in enumerate(zip(graph, eager)):
        what = names[i] if i < len(names) else f"buffer/offset {i}"
        assert torch.equal(a, b), f"{what}: pipelined replay differs from eager (max |d| {(a.double() - b.double()).abs().max()})"
    # the iteration really moved the weights, and every draw had its own counter
    assert not torch.equal(graph[0], snap[0][0]) and not torch.equal(graph[5], snap[0][5])
    draws = [d for log in logs for d in log]
    ctrs = [(s, off, sub) for s, off, sub, _ in draws]
    assert len(set(ctrs)) == len(ctrs), "two draws of one iteration share a Philox counter"
    kinds = {s for s, *_ in draws}
    assert kinds == {0, 1, 2}, kinds            # eps, generator z + noise, real batches
    # per iteration: 5 eps, one z + one bulk noise draw per generator forward (one per fake group
    # + the generator step: groups of 1 -> 6 + 6, groups 1, 3, 1 -> 4 + 4, groups 4, 1 -> 3 + 3), 5 real batches
    n_fwd = len(groups or [1] * 5) + 1
    assert [sum(1 for d in draws if d[0] == s) for s in (0, 1, 2)] == [5, 2 * n_fwd, 5]


class _FixedNoise:
    """A noise source for the generator whose draw i is a fixed [C, n*B, H, W] tensor; a forward
    over samples [lo, hi) gets that slice of it, so a batched forward and the per-segment forwards
    see the same noise per sample."""

    def __init__(self, nB):
        self.nB, self.draws, self.i, self.sl = nB, [], 0, slice(None)
        self.gen = torch.Generator(device=DEV)
        self.gen.manual_seed(77)

    def noise(self, shape):
        Bs, C, H, W = shape
        if self.i == len(self.draws):
            self.draws.append(torch.randn((C, self.nB, H, W), device=DEV, generator=self.gen))
        t = self.draws[self.i][:, self.sl].contiguous()
        self.i += 1
        assert t.shape == (C, Bs, H, W)
        return t


def test_segmented_batchnorm_op(gan):
    """ops.bn_fwd_raw under bn_segments(n) == n separate train-mode BatchNorm+PReLU calls on the
    segments, bit for bit (same per-row kernel), running statistics included."""
    from gan_amd import ops
    torch.manual_seed(3)
    n, C, Bs, HW = 5, 24, 8, 16 * 16
    x = torch.randn(C, n * Bs, HW, device=DEV) * 2 + 0.5
    g, b, a = (torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV), torch.rand(C, device=DEV) * 0.3)
    rm0, rv0 = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5
    with torch.no_grad():
        rm, rv = rm0.clone(), rv0.clone()
        with ops.bn_segments(n):
            y, mean, invstd = ops.bn_fwd_raw(x, C, n * Bs * HW, g, b, a, rm, rv, 0.1, 1e-5)
        rm1, rv1 = rm0.clone(), rv0.clone()
        for k in range(n):
            xs = x[:, k * Bs:(k + 1) * Bs].contiguous()
            ys, ms, iv = ops.bn_fwd_raw(xs, C, Bs * HW, g, b, a, rm1, rv1, 0.1, 1e-5)
            assert torch.equal(y[:, k * Bs:(k + 1) * Bs], ys), k
            assert torch.equal(mean.view(C, n)[:, k], ms) and torch.equal(invstd.view(C, n)[:, k], iv)
    assert torch.equal(rm, rm1) and torch.equal(rv, rv1)
    with pytest.raises(gan._lib.GanAmdError):
        with ops.bn_segments(n):
            ops.bn_fwd_raw(x, C, n * Bs * HW + 1, g, b, a, rm, rv, 0.1, 1e-5)


def test_generate_fakes_matches_separate_batches(gan):
    """Train.generate_fakes(n, B) (one generator forward, segmented BatchNorm) makes the fake
    batches of n separate generator calls (wgangp.py:58-59 per critic step): same z and noise per
    sample -> same images (to fp32 summation-order differences of the wider GEMM tilings) and the
    same BatchNorm running statistics after n updates.  Without segmentation the images differ at
    O(1e-1) (batch statistics over n*B samples), so the bar has teeth."""
    from gan_amd import ops
    n, Bs = 5, 8
    G, D = dp_worker.make_models(gan, DEV)
    tr = gan.Train([], DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.DeviceRNG(DEV, 11))
    z = torch.randn(n * Bs, 256, 1, 1, device=DEV)
    src = _FixedNoise(n * Bs)
    G.noise_hub.attach(src)
    bufs0 = [t.clone() for t in G.buffers()]
    with torch.no_grad():
        with ops.bn_segments(n):
            src.i = 0
            big = G(z).chunk(n)
        bufs_big = [t.clone() for t in G.buffers()]
        for t, v in zip(G.buffers(), bufs0):
            t.copy_(v)
        sep = []
        for k in range(n):
            src.i, src.sl = 0, slice(k * Bs, (k + 1) * Bs)
            sep.append(G(z[k * Bs:(k + 1) * Bs]))
        bufs_sep = [t.clone() for t in G.buffers()]
        for t, v in zip(G.buffers(), bufs0):
            t.copy_(v)
        src.i, src.sl = 0, slice(None)
        joint = G(z).chunk(n)
    torch.cuda.synchronize()
    for k in range(n):
        d = (big[k] - sep[k]).abs().max().item()
        assert d < 2e-4, (k, d)
    worst_joint = max((joint[k] - sep[k]).abs().max().item() for k in range(n))
    assert worst_joint > 1e-2, worst_joint
    for a, b in zip(bufs_big, bufs_sep):
        if a.dtype.is_floating_point:
            torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
        else:
            assert torch.equal(a, b)
    # the trainer's entry: n views of one [n*B, 3, 64, 64] tensor
    G.noise_hub.attach(tr.rng_g)
    fakes = tr.generate_fakes(n, Bs)
    assert len(fakes) == n and all(f.shape == (Bs, 3, 64, 64) for f in fakes)


def test_branch_noise_draws(gan):
    G, _ = dp_worker.make_models(gan, DEV)
    rng = gan.DeviceRNG(DEV, 99).fork(1)
    got = []
    inner = rng.noise_at

    def rec(shape, idx):
        t = inner(shape, idx)
        got.append((idx, t))
        return t
    rng.noise_at = rec
    G.noise_hub.attach(rng)
    off0 = int(rng.offset.item())
    with torch.no_grad():
        G(torch.randn(4, 256, 1, 1, device=DEV))       # first forward at B = 4: per-draw noise
    torch.cuda.synchronize()
    assert int(rng.offset.item()) == off0 + 1
    assert len(got) == 253 and [i for i, _ in got] == list(range(1, 254))
    for idx, t in got[::23] + got[-1:]:
        want = philox.normal(t.numel(), rng.seed, off0, idx)
        np.testing.assert_allclose(t.reshape(-1).cpu().numpy(), want, rtol=1e-5, atol=1e-5)
    # the next forward draws all of its noise in one bulk draw at the next offset
    rng.noise_at = inner
    with torch.no_grad():
        G(torch.randn(4, 256, 1, 1, device=DEV))
    torch.cuda.synchronize()
    assert int(rng.offset.item()) == off0 + 2


def test_forks_concurrent(gan):
    base = gan.DeviceRNG(DEV, 5)
    a, b = base.fork(1), base.fork(2)
    assert a is base.fork(1) and a.stream == 1 and int(a.offset.item()) == 1 << 40
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    n, reps = 1 << 16, 20
    outs = {1: [], 2: []}
    for _ in range(reps):
        with torch.cuda.stream(s1):
            outs[1].append(a.randn((n,)))
        with torch.cuda.stream(s2):
            outs[2].append(b.rand((n,)))
    torch.cuda.synchronize()
    for k in range(0, reps, 7):
        np.testing.assert_allclose(outs[1][k].cpu().numpy(), philox.normal(n, 5, (1 << 40) + k), rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(outs[2][k].cpu().numpy(), philox.uniform(n, 5, (2 << 40) + k))
    assert int(a.offset.item()) == (1 << 40) + reps and int(b.offset.item()) == (2 << 40) + reps
