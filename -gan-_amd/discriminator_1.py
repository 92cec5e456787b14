"""Drop-in vanilla MLP critic (reference: discriminators/discriminator_1.py ``Discriminator``).

Same module tree (``discriminator`` = Sequential of Linear / LeakyReLU(0.2) / Linear /
LeakyReLU(0.2) / Linear / Sigmoid, children "0".."5"); the forward runs on libganamd's GEMM and
activation kernels (see generator_1.py).
"""
from __future__ import annotations

import torch.nn as nn

from .generator_1 import batch_major_to_rows, mlp_forward, rows_to_batch_major


class Discriminator(nn.Module):
    def __init__(self, image_size):
        """discriminator_1.py:6-20: image_size (3, h, w)."""
        super().__init__()
        self.in_image_size = image_size[0] * image_size[1] * image_size[2]
        self.discriminator = nn.Sequential()
        self.discriminator.add_module(name="0", module=nn.Linear(in_features=self.in_image_size, out_features=256))
        self.discriminator.add_module(name="1", module=nn.LeakyReLU(0.2))
        self.discriminator.add_module(name="2", module=nn.Linear(in_features=256, out_features=64))
        self.discriminator.add_module(name="3", module=nn.LeakyReLU(0.2))
        self.discriminator.add_module(name="4", module=nn.Linear(in_features=64, out_features=1))
        self.discriminator.add_module(name="5", module=nn.Sigmoid())

    def forward(self, x):
        """discriminator_1.py:22-25: [B, 3, h, w] -> [B, 1] probabilities."""
        return rows_to_batch_major(mlp_forward(self.discriminator, batch_major_to_rows(x.contiguous())))
