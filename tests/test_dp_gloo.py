"""CPU, world_size 2 over gloo: the data-parallel contract of SURVEY.md §8(e).

Each rank computes the critic's gradient-penalty gradients on its own 4-image shard (the CPU
oracle stands in for the GPU step here); gan_amd.dist.allreduce_mean_ over the flat gradient
buffer must equal the mean of the per-shard gradients computed in one process.  Also checks
the max-over-ranks timing reduction bench.py uses."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import model as om

B = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grads(rank):
    torch.manual_seed(0)                       # identical weights on every rank
    DP = om.Params(lazy=True, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        om.discriminator(DP, torch.zeros(B, 3, 64, 64))
    g = torch.Generator().manual_seed(100 + rank)   # per-rank data
    xr = torch.randn(B, 3, 64, 64, generator=g)
    xf = torch.randn(B, 3, 64, 64, generator=g)
    eps = torch.rand(B, generator=g).view(B, 1, 1, 1)
    xi = ((1 - eps) * xr + eps * xf).requires_grad_()
    gx, = torch.autograd.grad(om.discriminator(DP, xi).sum(), xi, create_graph=True)
    (10 * ((gx.pow(2).view(B, -1).sum(1).sqrt() - 1) ** 2).mean()).backward()
    names = sorted(DP.t)
    # biases only shift PReLU kinks: the penalty has no gradient path to them (None)
    return torch.cat([(DP.t[n].grad if DP.t[n].grad is not None else torch.zeros_like(DP.t[n])).reshape(-1)
                      for n in names])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gan_amd.dist import allreduce_mean_
    flat = _shard_grads(rank)
    allreduce_mean_(flat)
    t = torch.tensor([1.0 + rank])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        torch.save({"flat": flat, "tmax": float(t)}, out)
    dist.destroy_process_group()


@pytest.mark.slow
def test_allreduce_mean_matches_single_process_mean(tmp_path):
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    torch.set_num_threads(4)
    want = (_shard_grads(0) + _shard_grads(1)) / 2
    assert got["tmax"] == 2.0
    assert float((got["flat"] - want).norm() / want.norm()) < 1e-5
