"""CPU oracle of the real-data transform chain (units/dataloader.py:5-14).

TEST INFRASTRUCTURE ONLY (the checker): imported by tests/.  torchvision is absent here, so the
chain is restated with the torch ops torchvision 0.17 (the reference's torch 2.2.2 pairing)
calls on tensors: ToTensor = u8 HWC -> f32 CHW / 255; RandomHorizontalFlip = flip of the last
axis; Resize((S, S), BICUBIC) = F.interpolate(mode='bicubic', align_corners=False,
antialias=True); Normalize = (x - mean) / std.  Parity of the build's tap tables with
F.interpolate is exact (tests/test_data.py); the torchvision wrapper itself is unpinned.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def transform(u8_hwc: torch.Tensor, flip: bool, size=64, mean=MEAN, std=STD) -> torch.Tensor:
    x = u8_hwc.permute(2, 0, 1).to(torch.float32).div(255)            # ToTensor
    if flip:
        x = x.flip(-1)                                                 # RandomHorizontalFlip
    x = F.interpolate(x[None], size=(size, size), mode="bicubic", align_corners=False, antialias=True)[0]
    m = torch.tensor(mean).view(3, 1, 1)
    s = torch.tensor(std).view(3, 1, 1)
    return (x - m) / s                                                 # Normalize
