"""Drop-in vanilla MLP generator (reference: generators/generator_1.py ``Generator``).

Same module tree (``generator`` = Sequential of Linear / LeakyReLU(0.2) / Linear / LeakyReLU(0.2) /
Linear / Tanh, children named "0".."5"), so ``named_parameters()`` / ``state_dict`` keys and the
default nn.Linear initialisation are the reference's.  The forward runs on the build's kernels:
each Linear is one GEMM of libganamd (ops.linear: features x batch, the "channel rows" layout of
the rest of the hot path), LeakyReLU and Tanh are csrc/act.hip kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops


def mlp_forward(seq: nn.Sequential, x):
    """Run a Sequential of Linear / LeakyReLU / Tanh / Sigmoid on x[features][batch]."""
    for m in seq:
        if isinstance(m, nn.Linear):
            x = ops.linear(x, m.weight, m.bias, 1.0)
        elif isinstance(m, nn.LeakyReLU):
            x = ops.leaky_relu(x, m.negative_slope)
        elif isinstance(m, nn.Tanh):
            x = ops.tanh(x)
        elif isinstance(m, nn.Sigmoid):
            x = ops.sigmoid(x)
        else:
            raise TypeError(f"unsupported layer {type(m).__name__}")
    return x


def rows_to_batch_major(x):
    """[F, B] (features x batch) -> [B, F]."""
    F_, B = x.shape
    return ops.cnhw_to_nchw(x.reshape(F_, B, 1, 1)).reshape(B, F_)


def batch_major_to_rows(x):
    """[B, ...] -> [F, B]."""
    B = x.shape[0]
    return ops.nchw_to_cnhw(x.reshape(B, -1, 1, 1)).reshape(-1, B)


class Generator(nn.Module):
    def __init__(self, z_dim, target_image_size):
        """generator_1.py:7-23: z_dim latent size, target_image_size (3, h, w)."""
        super().__init__()
        self.view_image_size = target_image_size[0] * target_image_size[1] * target_image_size[2]
        self.out_image_size = target_image_size
        self.z_dim = z_dim
        self.generator = nn.Sequential()
        self.generator.add_module(name="0", module=nn.Linear(in_features=self.z_dim, out_features=256))
        self.generator.add_module(name="1", module=nn.LeakyReLU(0.2))
        self.generator.add_module(name="2", module=nn.Linear(in_features=256, out_features=512))
        self.generator.add_module(name="3", module=nn.LeakyReLU(0.2))
        self.generator.add_module(name="4", module=nn.Linear(in_features=512, out_features=self.view_image_size))
        self.generator.add_module(name="5", module=nn.Tanh())

    def forward(self, x):
        """generator_1.py:25-29: [B, z_dim(, 1, 1)] -> [B, *target_image_size]."""
        B = x.shape[0]
        h = mlp_forward(self.generator, batch_major_to_rows(x.contiguous()))
        return rows_to_batch_major(h).view(B, *self.out_image_size)
