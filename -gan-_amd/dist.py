"""Data parallelism over RCCL (xGMI): one process per GPU, replicated G and D, gradients of every
optimizer step averaged across ranks before the fused AdamW update.

The reference has no multi-GPU path (``nn.DataParallel`` is commented out at
units/get_generators.py:19-20); SURVEY.md §8(e) defines the build's: batch-parallel replicas
(per-replica BatchNorm / MiniBatchStdDev statistics, exactly the reference's semantics at 64
images per shard) with one all-reduce of the flat fp32 gradient buffer per optimizer step
(D: 152.7 M elements after every critic step; G: 362.3 M after the generator step).

Because FusedAdamW keeps every gradient in ONE contiguous buffer, the all-reduce is a single
large collective -- the shape ring all-reduce over xGMI runs at its per-link bandwidth.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def allreduce_mean_(flat: torch.Tensor, group=None):
    """In-place mean of ``flat`` over the process group (SUM + scale: gloo has no AVG)."""
    world = dist.get_world_size(group)
    if world == 1:
        return flat
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.mul_(1.0 / world)
    return flat


def attach_grad_sync(optimizer, group=None):
    """Make ``optimizer.step()`` average the flat gradient over ranks first."""
    inner = optimizer.step

    def step():
        allreduce_mean_(optimizer.flat.grad, group)
        inner()

    optimizer.step = step
    return optimizer
