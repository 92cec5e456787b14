"""Data parallelism of the real GPU trainer (SURVEY.md §8(e) "Parity"), rehearsed with 2 ranks
over gloo on one MI355X (the 8-GPU RCCL run is the driver's).

test_dp_steps_match_shard_mean: tests/dp_worker.py runs a critic step (all-reduce, AdamW) and a
generator backward (all-reduce) on two ranks; here, in one process, the same two shards run
one after another on the same weights and replayed random streams, their gradients are averaged
by hand, and the critic update is applied from that mean.  The all-reduced gradients and the
updated critic must match at 1e-5 (gloo sums the fp32 buffers on the host: one rounding).

test_bench_two_ranks: ``bench.py --gpus 2 --backend gloo`` starts its own ranks and reports
n_gpus 2 (it used to run one rank silently).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from tests import dp_worker

pytestmark = pytest.mark.gpu
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


def test_bench_two_ranks():
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo", "--batch", "8",
           "--steps", "1", "--warmup", "1", "--mode", "eager", "--no-cpu-baseline", "--no-extras"]
    r = subprocess.run(cmd, cwd=REPO, env=_env(), timeout=900, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 16 and res["value"] > 0, res
