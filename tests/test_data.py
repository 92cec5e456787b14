"""Real-data pipeline (units/dataloader.py:5-31): the antialiased-bicubic tap tables equal
torch's F.interpolate(antialias=True) operator (CPU), and the GPU batch transform equals the CPU
oracle (oracle/data.py) per image, with and without the flip, for down- and up-scaling and
non-square sources (GPU)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gan_amd import tables
from oracle import data as od
from tests._util import rel_err


@pytest.mark.parametrize("n_in,n_out", [(512, 64), (100, 64), (64, 64), (37, 64), (333, 64), (64, 32)])
def test_aa_bicubic_table_matches_torch(n_in, n_out):
    m = tables.bicubic_aa_1d(n_in, n_out)
    x = torch.eye(n_in, dtype=torch.float64).reshape(n_in, 1, n_in, 1).expand(n_in, 1, n_in, 3).contiguous()
    y = F.interpolate(x, size=(n_out, 3), mode="bicubic", antialias=True, align_corners=False)[:, 0, :, 1].T
    assert np.abs(m - y.numpy()).max() < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", [(512, 512), (100, 80), (64, 64), (37, 50)])
def test_image_batch_matches_oracle(h, w):
    from gan_amd.data import ImagePipeline
    g = torch.Generator().manual_seed(h * 1000 + w)
    u8 = torch.randint(0, 256, (4, h, w, 3), generator=g, dtype=torch.uint8)
    flip = torch.tensor([True, False, True, False])
    out = ImagePipeline(64, device="cuda")(u8.cuda(), flip.cuda()).cpu()
    want = torch.stack([od.transform(u8[i], bool(flip[i])) for i in range(4)])
    assert out.shape == (4, 3, 64, 64)
    assert rel_err(out.numpy(), want.numpy()) < 1e-5
    assert (out - want).abs().max() < 1e-4


@pytest.mark.gpu
def test_dataloader_folder(tmp_path):
    from PIL import Image
    from gan_amd.data import DataLoader, ImageFolder
    rng = np.random.default_rng(0)
    arrays = []
    for c, n in (("cats", 3), ("dogs", 4)):
        (tmp_path / c).mkdir()
        for i in range(n):
            a = rng.integers(0, 256, (96 if i % 2 else 128, 128, 3), dtype=np.uint8)
            Image.fromarray(a).save(tmp_path / c / f"{i}.png")
            arrays.append(a)
    ds = ImageFolder(str(tmp_path))
    assert len(ds) == 7 and ds.classes == ["cats", "dogs"]
    dl = DataLoader(ds, batch_size=3, device="cuda", shuffle=False)
    batches = list(dl)
    assert len(dl) == 2 and len(batches) == 2                  # drop_last
    imgs, labels = batches[0]
    assert imgs.shape == (3, 3, 64, 64) and labels.tolist() == [0, 0, 0]
    # mixed source sizes in one batch, results in batch order: match the oracle up to the flip
    for j in range(3):
        got = imgs[j].cpu()
        cand = [od.transform(torch.from_numpy(arrays[j]), f) for f in (False, True)]
        assert min(rel_err(got.numpy(), c.numpy()) for c in cand) < 1e-5
