"""Data parallelism of the real GPU trainer (SURVEY.md §8(e) "Parity"), rehearsed with 2 ranks
over gloo on one MI355X (the 8-GPU RCCL run is the driver's).

test_dp_steps_match_shard_mean: tests/dp_worker.py runs a critic step (all-reduce, AdamW) and a
generator backward (all-reduce) on two ranks; here, in one process, the same two shards run
one after another on the same weights and replayed random streams, their gradients are averaged
by hand, and the critic update is applied from that mean.  The all-reduced gradients and the
updated critic must match at 1e-5 (gloo sums the fp32 buffers on the host: one rounding).

test_dp_graph_iteration_matches_shard_mean: the bench's N > 1 GRAPH-mode path (pipeline.Iteration
with the bench's fake-batch groups 4 + 1 from segmented-BatchNorm generator forwards, the second
group on the side stream during the first group's critic steps and all-reduces -- and the serial
order -- all-reduce between captured graphs) on two ranks equals, after
one full iteration (5 critic steps + generator step), the same iteration run here eagerly with the
two shards one after another and their gradients averaged by hand before every optimizer step.
At B = 8 per rank (both schedules) and at B = 64 per rank with the side stream on: config 3's
per-GPU batch and its N > 1 default schedule (the 64-sample fifth fake forward beside critic steps
1-4, their all-reduces and AdamW; two such ranks on one MI355X).  The first all-reduced critic
gradient (before any AdamW step) must equal the shard mean at 1e-6.

test_dp_progan_four_ranks_match_shard_mean: config 5's split (the progan pair on 4 ranks, 64 images
each, BASELINE.json) through the bench's progan schedule (fake batch of the next critic step on a
side stream) against the four shards run one after another with hand-averaged gradients.  The
FIRST all-reduced critic gradient -- before any AdamW step, where a DP bug shows unamplified --
must equal the shard mean at 1e-6 (four fp32 buffers summed in gloo's ring order: one rounding
per add).  After the whole iteration the bar is 3x of how far that shard mean moves when its four
shards are summed in the opposite order (the iteration amplifies last-bit differences: AdamW's
first update is ~lr * sign(g)); with GANAMD_TEST_PROGAN_WORLD=2 it is the 1e-5 of the two-rank tests.

test_bench_two_ranks: ``bench.py --gpus 2 --backend gloo`` starts its own ranks and reports
n_gpus 2 (it used to run one rank silently), in eager and in graph mode.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from tests import dp_worker

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _release_gpu_cache():
    """The ranks share this process's GPU: hand back what earlier tests in this process left cached
    (the in-process reference runs of B = 64 models hold tens of GB), before and after each test --
    eight ranks that started after the 2-rank B = 64 test's reference ran out of memory otherwise."""
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    yield
    gc.collect()
    torch.cuda.empty_cache()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = "4"
    return env


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def test_dp_steps_match_shard_mean(tmp_path):
    out = str(tmp_path / "rank0.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "tests", "dp_worker.py"), out]
    r = subprocess.run(cmd, cwd=REPO, env=_env(), timeout=600, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = torch.load(out, weights_only=True)
    assert got["world"] == 2

    import gan_amd
    dev = torch.device("cuda", 0)
    G, D = dp_worker.make_models(gan_amd, dev)
    tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4")
    shards = [dp_worker.shard_inputs(r) for r in range(2)]
    rngs = [gan_amd.ReplayRNG(seed, dev) for _, seed in shards]
    dg = []
    for (images, _), rng in zip(shards, rngs):
        tr.rng = rng
        tr.discriminator_backward(images.to(dev), dp_worker.B)
        dg.append(tr.optimizer_D.flat.grad.detach().clone())
    tr.optimizer_D.flat.grad.copy_((dg[0] + dg[1]) / 2)
    d_want = tr.optimizer_D.flat.grad.detach().cpu().clone()
    tr.optimizer_D.step()
    gg = []
    for rng in rngs:
        tr.rng = rng
        tr.generator_backward(dp_worker.B)
        gg.append(tr.optimizer_G.flat.grad.detach().clone())
    g_want = ((gg[0] + gg[1]) / 2).cpu()
    # the two shards really differ (a DP bug that used one shard's gradient would not pass)
    assert _rel(dg[0].cpu(), dg[1].cpu()) > 1e-2 and _rel(gg[0].cpu(), gg[1].cpu()) > 1e-2
    assert _rel(got["d_grad"], d_want) < 1e-5
    assert _rel(got["d_data"], tr.optimizer_D.flat.data.detach().cpu()) < 1e-6
    assert _rel(got["g_grad"], g_want) < 1e-5


@pytest.mark.parametrize("schedule,B", [("overlap", 8), ("serial", 8), ("overlap", 64)])
def test_dp_graph_iteration_matches_shard_mean(tmp_path, schedule, B):
    import gc
    gc.collect()
    torch.cuda.empty_cache()           # two B = 64 ranks share this GPU with this process's cache
    free, total = torch.cuda.mem_get_info()
    print(f"before the ranks: {free / 2**30:.1f} of {total / 2**30:.1f} GiB free, this process reserves "
          f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB ({torch.cuda.memory_allocated() / 2**30:.1f} allocated)")
    if os.environ.get("DP_MEMLOG") == "1":
        big = sorted(((o.numel() * o.element_size(), tuple(o.shape)) for o in gc.get_objects()
                      if torch.is_tensor(o) and o.is_cuda), reverse=True)[:15]
        print("largest live tensors:", [(round(n / 2**30, 2), s) for n, s in big])
        top = [o for o in gc.get_objects() if torch.is_tensor(o) and o.is_cuda and o.numel() == big[0][1][0]][:3]
        for t in top:
            for r in gc.get_referrers(t):
                desc = type(r).__name__
                if isinstance(r, dict):
                    desc += " keys " + str([k for k, v in r.items() if v is t][:3]) + " of " + str(list(r.keys())[:6])
                elif isinstance(r, (list, tuple)):
                    owners = [type(q).__name__ for q in gc.get_referrers(r)][:4]
                    desc += f" len {len(r)} held by {owners}"
                print("  referrer:", desc[:300])
    out = str(tmp_path / "rank0_graph.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "tests", "dp_worker.py"), out,
           "graph", schedule, str(B)]
    r = subprocess.run(cmd, cwd=REPO, env=_env(), timeout=900, capture_output=True, text=True)
    if r.returncode != 0 and os.path.isdir(os.path.join(REPO, "gpurun_out")):   # the whole log, for the record
        with open(os.path.join(REPO, "gpurun_out", f"dp_graph_{schedule}_{B}_fail.log"), "w") as f:
            f.write(r.stdout + "\n==== stderr\n" + r.stderr)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = torch.load(out, weights_only=True)
    assert got["world"] == 2 and got["batch"] == B and got["d_grad0"] is not None
    print(f"rank 0: peak {got['peak_reserved'] / 2**30:.1f} GiB reserved, {got['reserved'] / 2**30:.1f} GiB at the end")

    import gan_amd
    dev = torch.device("cuda", 0)
    G, D = dp_worker.make_models(gan_amd, dev)
    tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.DeviceRNG(dev, 1))
    g0, d0 = tr.optimizer_G.flat.data.detach().cpu().clone(), tr.optimizer_D.flat.data.detach().cpu().clone()
    for k in set(dp_worker.GRAPH_FAKE_GROUPS):
        tr.generate_fakes(k, B)    # the workers' warm-up recorded the noise shapes: bulk draws from here
    rngs = [gan_amd.DeviceRNG(dev, dp_worker.graph_seed(r)) for r in range(2)]
    fakes = []                     # each rank's fake batches, group by group (G is fixed until the G step)
    for rng in rngs:
        tr.rng = rng
        fakes.append([f for k in dp_worker.GRAPH_FAKE_GROUPS for f in tr.generate_fakes(k, B)])

    def mean_into(flat_grad, gs):
        flat_grad.copy_(gs[0] + gs[1]).mul_(0.5)          # gloo: SUM, then * 1/N (dist.allreduce_mean_)

    first = None
    for i in range(5):
        gs = []
        for r, rng in enumerate(rngs):
            tr.rng = rng
            tr.discriminator_backward(rng.fork(2).randn((B, 3, 64, 64)), B, gen_imgs=fakes[r][i])
            gs.append(tr.optimizer_D.flat.grad.detach().clone())
        assert _rel(gs[0].cpu(), gs[1].cpu()) > 1e-2       # the shards really differ
        mean_into(tr.optimizer_D.flat.grad, gs)
        if first is None:
            first = tr.optimizer_D.flat.grad.detach().cpu().clone()
        tr.optimizer_D.step()
    gs = []
    for rng in rngs:
        tr.rng = rng
        tr.generator_backward(B)
        gs.append(tr.optimizer_G.flat.grad.detach().clone())
    mean_into(tr.optimizer_G.flat.grad, gs)
    tr.optimizer_G.step()
    torch.cuda.synchronize()
    want = {"g_data": tr.optimizer_G.flat.data, "g_grad": tr.optimizer_G.flat.grad,
            "d_data": tr.optimizer_D.flat.data, "d_grad": tr.optimizer_D.flat.grad}
    errs = {k: _rel(got[k], v.detach().cpu()) for k, v in want.items()}
    errs["d_grad0"] = _rel(got["d_grad0"], first)
    # parameters relative to how far the iteration moved them
    errs["g_move"] = float((got["g_data"] - want["g_data"].cpu()).double().norm() / (want["g_data"].cpu() - g0).double().norm())
    errs["d_move"] = float((got["d_data"] - want["d_data"].cpu()).double().norm() / (want["d_data"].cpu() - d0).double().norm())
    print(f"graph-mode DP (B={B}/rank, {schedule}) vs shard mean:", errs)
    assert errs["d_grad0"] < 1e-6, errs
    assert errs["g_grad"] < 1e-5 and errs["d_grad"] < 1e-5, errs
    assert errs["g_move"] < 1e-4 and errs["d_move"] < 1e-4, errs


def _shard_mean_iteration(tr, rngs, B, groups, reverse=False):
    """One WGAN-GP iteration with the shards run one after another on the same weights and the
    gradients of every optimizer step averaged by hand (gloo: SUM, then * 1/N; ``reverse``: the
    shards summed in the opposite order -- another legitimate fp32 rounding of the same mean).
    Returns the first averaged critic gradient (before any optimizer step), on the host."""
    n = len(rngs)
    for k in set(groups):
        tr.generate_fakes(k, B)    # warm-up: the workers' warm-up recorded the noise shapes
    fakes = []                     # each rank's fake batches, group by group (G is fixed until the G step)
    for rng in rngs:
        tr.rng = rng
        fakes.append([f for k in groups for f in tr.generate_fakes(k, B)])

    def mean_into(flat_grad, gs):
        gs = gs[::-1] if reverse else gs
        acc = gs[0].clone()
        for g in gs[1:]:
            acc.add_(g)
        flat_grad.copy_(acc).mul_(1.0 / n)

    for i in range(5):
        gs = []
        for r, rng in enumerate(rngs):
            tr.rng = rng
            tr.discriminator_backward(rng.fork(2).randn((B, 3, 64, 64)), B, gen_imgs=fakes[r][i])
            gs.append(tr.optimizer_D.flat.grad.detach().clone())
        assert _rel(gs[0].cpu(), gs[1].cpu()) > 1e-2       # the shards really differ
        mean_into(tr.optimizer_D.flat.grad, gs)
        if i == 0:
            first = tr.optimizer_D.flat.grad.detach().cpu().clone()
        tr.optimizer_D.step()
    gs = []
    for rng in rngs:
        tr.rng = rng
        tr.generator_backward(B)
        gs.append(tr.optimizer_G.flat.grad.detach().clone())
    mean_into(tr.optimizer_G.flat.grad, gs)
    tr.optimizer_G.step()
    torch.cuda.synchronize()
    return first


def _dp_errors(got, tr, g0, d0):
    want = {"g_data": tr.optimizer_G.flat.data, "g_grad": tr.optimizer_G.flat.grad,
            "d_data": tr.optimizer_D.flat.data, "d_grad": tr.optimizer_D.flat.grad}
    errs = {k: _rel(got[k], v.detach().cpu()) for k, v in want.items()}
    errs["g_move"] = float((got["g_data"] - want["g_data"].cpu()).double().norm() / (want["g_data"].cpu() - g0).double().norm())
    errs["d_move"] = float((got["d_data"] - want["d_data"].cpu()).double().norm() / (want["d_data"].cpu() - d0).double().norm())
    return errs


def test_dp_graph_eight_ranks_match_shard_mean(tmp_path):
    """Config 3's world size: EIGHT ranks (gloo, all on this GPU) run the bench's
    N > 1 graph schedule for G13_5 / D9_4 -- pipeline.Iteration with fake groups (4, 1), the fifth
    fake batch on the side stream during critic steps 1-4, their all-reduces and AdamW -- at B = 8
    per rank, per-rank Philox seeds.  The first all-reduced critic gradient must equal the shard
    mean at 1e-6; after the whole iteration the bar is 3x the shard mean's own spread under the
    opposite summation order (gloo's ring adds eight buffers in another order than the hand-made
    mean, and the iteration amplifies last-bit differences -- the 4-rank progan test's bar)."""
    W, B = 8, 8
    out = str(tmp_path / "rank0_graph8.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={W}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "tests", "dp_worker.py"), out,
           "graph", "overlap", str(B)]
    env = _env()
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run(cmd, cwd=REPO, env=env, timeout=1500, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = torch.load(out, weights_only=True)
    assert got["world"] == W and got["batch"] == B and got["d_grad0"] is not None
    print(f"rank 0: peak {got['peak_reserved'] / 2**30:.1f} GiB reserved")

    import gan_amd
    dev = torch.device("cuda", 0)

    def shard_mean(reverse):
        G, D = dp_worker.make_models(gan_amd, dev)
        tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.DeviceRNG(dev, 1))
        g0, d0 = tr.optimizer_G.flat.data.detach().cpu().clone(), tr.optimizer_D.flat.data.detach().cpu().clone()
        rngs = [gan_amd.DeviceRNG(dev, dp_worker.graph_seed(q)) for q in range(W)]
        first = _shard_mean_iteration(tr, rngs, B, list(dp_worker.GRAPH_FAKE_GROUPS), reverse=reverse)
        return tr, g0, d0, first

    tr, g0, d0, first = shard_mean(False)
    errs = _dp_errors(got, tr, g0, d0)
    errs["d_grad0"] = _rel(got["d_grad0"], first)
    mid = {k: v.detach().cpu().clone() for k, v in (("g_data", tr.optimizer_G.flat.data),
                                                   ("g_grad", tr.optimizer_G.flat.grad),
                                                   ("d_data", tr.optimizer_D.flat.data),
                                                   ("d_grad", tr.optimizer_D.flat.grad))}
    del tr
    tr2, _, _, _ = shard_mean(True)
    spread = _dp_errors(mid, tr2, g0, d0)
    print(f"G13_5 {W}-rank graph DP vs shard mean: {errs}; shard-mean spread under reverse order: {spread}")
    assert errs["d_grad0"] < 1e-6, errs
    for k in ("g_grad", "d_grad", "g_data", "d_data", "g_move", "d_move"):
        assert errs[k] <= max(3 * spread[k], 1e-5), (k, errs, spread)


def test_dp_progan_four_ranks_match_shard_mean(tmp_path):
    out = str(tmp_path / "rank0_progan.pt")
    W = dp_worker.PROGAN_WORLD
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={W}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "tests", "dp_worker.py"), out,
           "progan"]
    r = subprocess.run(cmd, cwd=REPO, env=_env(), timeout=900, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = torch.load(out, weights_only=True)
    assert got["world"] == W

    import gan_amd
    if os.environ.get("GANAMD_TEST_PATCH_MASK"):      # diagnosis: kernel selection A/B (dp_worker too)
        gan_amd.ops.set_patch(int(os.environ["GANAMD_TEST_PATCH_MASK"]))
    dev = torch.device("cuda", 0)
    B = dp_worker.B_PROGAN

    def shard_mean(reverse):
        G, D = dp_worker.make_progan(gan_amd, dev)
        tr = gan_amd.Train([], dev, 1, 256, G, "G3_progan", D, "D3_progan", rng=gan_amd.DeviceRNG(dev, 1))
        g0, d0 = tr.optimizer_G.flat.data.detach().cpu().clone(), tr.optimizer_D.flat.data.detach().cpu().clone()
        rngs = [gan_amd.DeviceRNG(dev, dp_worker.progan_seed(r)) for r in range(W)]
        first = _shard_mean_iteration(tr, rngs, B, [1] * 5, reverse=reverse)
        return tr, g0, d0, first

    tr, g0, d0, first = shard_mean(False)
    errs = _dp_errors(got, tr, g0, d0)
    errs["d_grad0"] = _rel(got["d_grad0"], first)
    print(f"progan {W}-rank DP vs shard mean:", errs)
    # the first all-reduced critic gradient: the shard mean before any AdamW step, up to the order
    # in which the ranks' fp32 buffers are summed (a wrong shard, scale or bucket shows at O(1))
    assert errs["d_grad0"] < 1e-6, errs
    if W <= 2:
        # two shards sum the same way in any order (fp32 addition commutes): bit-level agreement
        assert errs["g_grad"] < 1e-5 and errs["d_grad"] < 1e-5, errs
        assert errs["g_move"] < 1e-4 and errs["d_move"] < 1e-4, errs
        return
    # With four shards gloo's ring sums them in another order than the hand-made mean, and this
    # iteration amplifies a last-bit difference of the critic gradients (one shared PReLU slope per
    # layer, five AdamW steps whose first update is ~lr * sign(g)) to ~1e-3 of the generator gradient.
    # The bar is that spread itself: the same shard mean with the shards summed in reverse order.
    mid = {k: v.detach().cpu().clone() for k, v in (("g_data", tr.optimizer_G.flat.data),
                                                   ("g_grad", tr.optimizer_G.flat.grad),
                                                   ("d_data", tr.optimizer_D.flat.data),
                                                   ("d_grad", tr.optimizer_D.flat.grad))}
    tr2, _, _, _ = shard_mean(True)
    spread = _dp_errors(mid, tr2, g0, d0)
    print(f"progan {W}-rank: shard mean vs the same with the shards summed in reverse:", spread)
    for k in ("g_grad", "d_grad", "g_data", "d_data", "g_move", "d_move"):
        assert errs[k] <= max(3 * spread[k], 1e-5), (k, errs, spread)


@pytest.mark.parametrize("mode,n", [("eager", 2), ("graph", 2), ("graph", 8)])
def test_bench_ranks(mode, n):
    """``bench.py --gpus N --backend gloo`` starts its own N ranks (the driver's N = 8 launch path:
    launch_ranks, per-rank seeds, the N > 1 side-stream schedule) and reports n_gpus N."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--backend", "gloo", "--batch", "8",
           "--steps", "1", "--warmup", "1", "--mode", mode, "--no-cpu-baseline", "--no-extras"]
    env = _env()
    if n > 2:
        env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run(cmd, cwd=REPO, env=env, timeout=1500, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == n and res["config"]["global_batch"] == 8 * n and res["value"] > 0, res
    assert res["config"]["parallelism"] == f"dp{n}" and res["config"]["fake_overlap"] is True, res
