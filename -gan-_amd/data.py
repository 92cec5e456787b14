"""Real-data input pipeline (reference: units/dataloader.py:5-14 ``get_dataset`` and :29-31
``get_dataloader``).

The reference decodes each image with PIL (torchvision ImageFolder) and runs, per image on the
CPU: ToTensor -> RandomHorizontalFlip -> Resize((64, 64), BICUBIC) -> Normalize(ImageNet mean /
std), then batches with shuffle and drop_last.  Here decoding stays on the host (PIL), and the
whole transform chain runs on the GPU for a batch at once: one ``ganamd_image_batch`` call per
distinct source size in the batch (two separable passes over antialiased-bicubic tap tables,
tables.bicubic_aa_1d, equal to torch's ``F.interpolate(mode='bicubic', antialias=True)`` that
torchvision's tensor Resize calls).  Flips are drawn on the device (p = 0.5 per image).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import tables
from ._lib import LIB, check, ptr, stream, workspace
from ._lib import ws as wsarg

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # units/dataloader.py:12
IMAGENET_STD = (0.229, 0.224, 0.225)
IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


class ImagePipeline:
    """u8 [B, H, W, 3] (device) -> f32 [B, 3, size, size]: ToTensor, RandomHorizontalFlip,
    Resize(bicubic, antialias), Normalize."""

    def __init__(self, size=64, mean=IMAGENET_MEAN, std=IMAGENET_STD, flip_p=0.5, device="cuda"):
        self.size, self.flip_p = size, flip_p
        self.device = torch.device(device)
        self.mean = torch.tensor(mean, dtype=torch.float32, device=self.device)
        self.std = torch.tensor(std, dtype=torch.float32, device=self.device)
        self._tabs = {}

    def _table(self, n_in):
        t = self._tabs.get(n_in)
        if t is None:
            idx, w = tables.ell(tables.bicubic_aa_1d(n_in, self.size))
            t = self._tabs[n_in] = (torch.from_numpy(idx).to(self.device), torch.from_numpy(w).to(self.device),
                                    idx.shape[1])
        return t

    def __call__(self, images: torch.Tensor, flip: torch.Tensor | None = None) -> torch.Tensor:
        if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[3] != 3 or not images.is_cuda:
            raise ValueError(f"expected a uint8 [B,H,W,3] device tensor, got {images.dtype} {tuple(images.shape)}")
        images = images.contiguous()
        B, H, W, _ = images.shape
        if flip is None:
            flip = torch.rand(B, device=images.device) < self.flip_p
        flip = flip.to(device=images.device, dtype=torch.uint8).contiguous()
        if flip.numel() != B:
            raise ValueError("flip needs one entry per image")
        ix, wx, kx = self._table(W)
        iy, wy, ky = self._table(H)
        y = torch.empty(B, 3, self.size, self.size, device=images.device, dtype=torch.float32)
        ws = workspace(LIB.ganamd_image_batch_workspace(B, H, self.size), images.device)
        check(LIB.ganamd_image_batch(images.data_ptr(), B, H, W, flip.data_ptr(), ix.data_ptr(), ptr(wx), kx,
                                     self.size, iy.data_ptr(), ptr(wy), ky, self.size, ptr(self.mean), ptr(self.std),
                                     ptr(y), *wsarg(ws), stream()), "image_batch")
        return y


class ImageFolder:
    """Files under ``root/<class>/`` (sorted classes, as torchvision's ImageFolder) decoded by PIL
    into u8 [H, W, 3] arrays; ``[i] -> (array, class index)``."""

    def __init__(self, root):
        classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
        self.classes = classes
        self.samples = []
        for ci, c in enumerate(classes):
            for dirpath, _, files in sorted(os.walk(os.path.join(root, c))):
                for f in sorted(files):
                    if f.lower().endswith(IMG_EXTENSIONS):
                        self.samples.append((os.path.join(dirpath, f), ci))

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        from PIL import Image
        path, label = self.samples[i]
        with Image.open(path) as im:
            return np.asarray(im.convert("RGB"), dtype=np.uint8), label


class DataLoader:
    """``get_dataloader`` (units/dataloader.py:29-31): shuffled batches, drop_last, transformed on
    the GPU; yields (images f32 [B, 3, size, size] on the device, labels int64 [B])."""

    def __init__(self, dataset, batch_size, size=64, device="cuda", shuffle=True, drop_last=True, generator=None):
        self.dataset, self.batch_size = dataset, batch_size
        self.shuffle, self.drop_last, self.generator = shuffle, drop_last, generator
        self.pipeline = ImagePipeline(size=size, device=device)

    def __len__(self):
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        n = len(self.dataset)
        order = torch.randperm(n, generator=self.generator).tolist() if self.shuffle else list(range(n))
        for s in range(0, len(self) * self.batch_size, self.batch_size):
            items = [self.dataset[i] for i in order[s:s + self.batch_size]]
            yield self.transform([a for a, _ in items]), torch.tensor([l for _, l in items])

    def transform(self, arrays):
        """One kernel call per distinct source size; results in batch order."""
        dev = self.pipeline.device
        out = torch.empty(len(arrays), 3, self.pipeline.size, self.pipeline.size, device=dev)
        groups = {}
        for j, a in enumerate(arrays):
            groups.setdefault(a.shape, []).append(j)
        for shape, idx in groups.items():
            u8 = torch.from_numpy(np.stack([arrays[j] for j in idx])).to(dev, non_blocking=True)
            out[torch.tensor(idx, device=dev)] = self.pipeline(u8)
        return out
