"""Flat-buffer parameters and the fused AdamW of the hot path.

``torch.optim.AdamW`` as configured at train/wgangp.py:17-18 runs a per-tensor loop over
10,653 generator tensors.  Here every trainable parameter of a model is re-homed into ONE
contiguous fp32 buffer (``param.data`` becomes a view), its gradient into a second one
(``param.grad`` is pre-bound to a view, so autograd accumulates in place), and the whole update
is one ``ganamd_adamw`` launch over the buffer.  The step counter lives on the device so a
captured HIP graph replays the bias corrections correctly.

Semantics kept from torch.optim.AdamW (weight_decay 0.01, eps 1e-8): parameters that never
receive a gradient are never touched (torch skips ``grad is None``): the frozen Smooth kernels
(requires_grad=False) and the no-op StyleConv biases (generator_13_5.py:258,263) are placed
outside the updated range.
"""
from __future__ import annotations

import torch

from ._lib import LIB, check, iptr, ptr, stream
from .ops import PackRegistry, invalidate_packed


def _never_gets_grad(owner_cls: str, pname: str) -> bool:
    return owner_cls == "StyleConv" and pname == "bias"


class FlatParams:
    def __init__(self, module: torch.nn.Module):
        owners = {}
        for mname, mod in module.named_modules():
            for pname, p in mod.named_parameters(recurse=False):
                owners[id(p)] = (type(mod).__name__, pname)
        layout = getattr(module, "flat_layout", None)
        params = list(layout()) if layout is not None else list(module.parameters())
        assert len({id(p) for p in params}) == len(list(module.parameters())), "flat_layout must permute parameters()"
        train = [p for p in params if p.requires_grad and not _never_gets_grad(*owners[id(p)])]
        tids = {id(p) for p in train}
        rest = [p for p in params if id(p) not in tids]
        self.trainable, self.frozen = train, rest
        dev = params[0].device
        n_train = sum(p.numel() for p in train)
        n_all = n_train + sum(p.numel() for p in rest)
        self.n_train = n_train
        self.data = torch.empty(n_all, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(n_train, device=dev, dtype=torch.float32)
        off = 0
        for p in train + rest:
            n = p.numel()
            view = self.data[off:off + n].view_as(p)
            view.copy_(p.detach())
            p.data = view
            if off < n_train:
                p.grad = self.grad[off:off + n].view_as(p)
            off += n
            p._gan_flat = self
        self.epoch = 0
        self.packs = PackRegistry(self)   # persistent packed conv weights (ops.PackCache)
        invalidate_packed()
        module.__dict__["_flat"] = self      # lets the module find its flat buffers (style bank)

    def zero_grad(self):
        self.grad.zero_()


class FusedAdamW:
    """Drop-in for ``torch.optim.AdamW(module.parameters(), lr, betas)`` over FlatParams."""

    def __init__(self, module: torch.nn.Module, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        self.flat = FlatParams(module)
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        dev = self.flat.data.device
        self.exp_avg = torch.zeros(self.flat.n_train, device=dev, dtype=torch.float32)
        self.exp_avg_sq = torch.zeros_like(self.exp_avg)
        self.step_count = torch.zeros(1, device=dev, dtype=torch.int32)

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def state_dict(self):
        """Moments over the trainable flat range + the step counter (checkpoint.py)."""
        return {"exp_avg": self.exp_avg.detach().cpu(), "exp_avg_sq": self.exp_avg_sq.detach().cpu(),
                "step": self.step_count.detach().cpu(), "n_train": self.flat.n_train,
                "lr": self.lr, "betas": list(self.betas), "eps": self.eps, "weight_decay": self.weight_decay}

    def load_state_dict(self, sd):
        if int(sd["n_train"]) != self.flat.n_train:
            raise ValueError(f"optimizer state for {sd['n_train']} parameters, this model trains {self.flat.n_train}")
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_count.copy_(sd["step"])
        self.flat.epoch += 1      # parameters may have been reloaded: packed conv weights are stale

    @torch.no_grad()
    def step(self):
        f = self.flat
        check(LIB.ganamd_adamw(ptr(f.data), ptr(f.grad), ptr(self.exp_avg), ptr(self.exp_avg_sq), f.n_train,
                               iptr(self.step_count), float(self.lr), float(self.betas[0]), float(self.betas[1]),
                               float(self.eps), float(self.weight_decay), stream()), "adamw")
        f.epoch += 1   # packed conv weights of these parameters (ops.PackCache) are stale now ...
        f.packs.repack()   # ... until this one launch refreshes every registered copy
