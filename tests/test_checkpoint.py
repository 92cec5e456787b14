"""CPU: checkpoint save / resume (train/trainunits.py:58-130 naming and fields; state_dicts keyed
by the reference's names; in-place load keeps the optimizers bound; optimizer state round trip)."""
import json
import os

import torch

import gan_amd
from tests._util import GOLDEN


def _trainer(tmp_path):
    with open(os.path.join(GOLDEN, "plan_progan.json")) as f:
        pp = json.load(f)
    torch.manual_seed(0)
    G = gan_amd.generator_3_progan.Generator(1, 256, pp["ngf"], 3)
    D = gan_amd.discriminator_3_wgangp_progan.Discriminator(1, pp["ndf"], 3)
    tr = gan_amd.Train([0] * 7, "cpu", 1, 256, G, "G3", D, "D3")
    tr.ckpt_root = str(tmp_path / "checkpoint")
    return pp, tr


def test_checkpoint_round_trip(tmp_path):
    pp, tr = _trainer(tmp_path)
    tr.epoch, tr.i = 2, 5
    with torch.no_grad():
        tr.optimizer_D.exp_avg.normal_()
        tr.optimizer_D.step_count.fill_(3)
    path = tr.save_ckpt("WGANGP", 1, 4)
    # reference naming and epoch/i carry: epoch + self.epoch + (i + self.i) // len, (i + self.i) % len
    assert os.path.basename(path) == "G3 D3 WGANGP epoch_4 i_2_ckpt.pth"
    ck = torch.load(path, weights_only=True)
    assert (ck["generator_name"], ck["discriminator_name"], ck["method"], ck["epoch"], ck["i"]) == \
        ("G3", "D3", "WGANGP", 4, 2)
    # state_dict keys are the reference's parameter + buffer names
    assert list(ck["generator"]) == [n for n, _ in tr.generator.state_dict().items()]
    assert {n for n, _, _ in pp["g_params"]} | set(pp["g_buffers"]) == set(ck["generator"])
    assert {n for n, _, _ in pp["d_params"]} == set(ck["discriminator"])
    want_g = {k: v.clone() for k, v in tr.generator.state_dict().items()}
    want_m = tr.optimizer_D.exp_avg.clone()
    flat_ptr = tr.optimizer_G.flat.data.data_ptr()
    with torch.no_grad():
        for p in tr.generator.parameters():
            p.add_(1.0)
        tr.optimizer_D.exp_avg.zero_()
    os.replace(path, os.path.join(tr.ckpt_root, "resume.pth"))
    assert tr.load_generator_ckpt("resume") and tr.load_discriminator_ckpt("resume")
    got = tr.generator.state_dict()
    assert all(torch.equal(got[k], v) for k, v in want_g.items())
    assert torch.equal(tr.optimizer_D.exp_avg, want_m) and int(tr.optimizer_D.step_count) == 3
    # loaded in place: parameters are still views of the optimizer's flat buffer
    assert all(p.data_ptr() >= flat_ptr for p in tr.generator.parameters())
    assert tr.optimizer_G.flat.data.data_ptr() == flat_ptr
    assert (tr.epoch, tr.i) == (4, 2)
    assert not tr.load_generator_ckpt("missing")


def test_pickled_module_checkpoint_is_refused_clearly(tmp_path):
    """The reference saves pickled nn.Modules (trainunits.py:58-76); they are never unpickled here."""
    import pytest
    _pp, tr = _trainer(tmp_path)
    os.makedirs(tr.ckpt_root, exist_ok=True)
    torch.save({"generator": torch.nn.Linear(2, 2), "epoch": 1, "i": 0},
               os.path.join(tr.ckpt_root, "old.pth"))
    with pytest.raises(RuntimeError, match="not a state_dict checkpoint"):
        tr.load_generator_ckpt("old")


def test_checkpoint_restores_rng_streams(tmp_path):
    """The device RNG's stream offsets travel with the checkpoint: a resumed run continues the
    z / noise, eps and data sequences instead of redrawing the first run's numbers."""
    _pp, tr = _trainer(tmp_path)
    rng = tr.rng
    data = rng.fork(2)
    with torch.no_grad():
        rng.offset.fill_(7)
        data.offset.fill_((2 << rng.STREAM_SHIFT) + 11)
    tr.save_ckpt("WGANGP", 0, 0)
    name = os.path.splitext(os.path.basename(tr.save_ckpt("WGANGP", 0, 0)))[0]
    _pp2, tr2 = _trainer(tmp_path)
    assert int(tr2.rng.offset) == 0
    assert tr2.load_generator_ckpt(name)
    assert int(tr2.rng.offset) == 7
    assert int(tr2.rng.fork(2).offset) == (2 << rng.STREAM_SHIFT) + 11


def test_checkpoint_restores_rng_seed(tmp_path):
    """The offsets index the saved key's sequence: a trainer built with ANOTHER seed resumes the
    saved seed (and its forks follow), so its next draws are the ones the first run would make."""
    _pp, tr = _trainer(tmp_path)
    tr.rng = gan_amd.DeviceRNG("cpu", seed=1234)
    with torch.no_grad():
        tr.rng.offset.fill_(5)
    name = os.path.splitext(os.path.basename(tr.save_ckpt("WGANGP", 0, 0)))[0]
    _pp2, tr2 = _trainer(tmp_path)
    tr2.rng = gan_amd.DeviceRNG("cpu", seed=99)
    data = tr2.rng.fork(2)
    assert tr2.load_generator_ckpt(name)
    assert tr2.rng.seed == 1234 and data.seed == 1234 and int(tr2.rng.offset) == 5



def _dp_ckpt_worker(rank, world, port, root, out):
    """One rank of the DP checkpoint test: every rank draws with its own key (bench.py: 4321 + rank),
    saves (rank 0 writes), then a fresh trainer seeded otherwise resumes."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _pp, tr = _trainer(root)
    tr.rng = gan_amd.DeviceRNG("cpu", seed=4321 + rank)
    with torch.no_grad():
        tr.rng.offset.fill_(10 + rank)
        tr.rng.fork(2).offset.fill_((2 << tr.rng.STREAM_SHIFT) + 20 + rank)
    name = os.path.splitext(os.path.basename(tr.save_ckpt("WGANGP", 0, 0)))[0]
    _pp2, tr2 = _trainer(root)
    tr2.rng = gan_amd.DeviceRNG("cpu", seed=7)
    data = tr2.rng.fork(2)
    assert tr2.load_generator_ckpt(name)
    res = torch.tensor([tr2.rng.seed, int(tr2.rng.key), int(tr2.rng.offset), int(data.offset), data.seed],
                       dtype=torch.float64)
    got = [torch.zeros_like(res) for _ in range(world)]
    dist.all_gather(got, res)
    if rank == 0:
        torch.save(torch.stack(got), out)
    dist.destroy_process_group()


def test_dp_checkpoint_keeps_each_ranks_stream(tmp_path):
    """rank 0 writes the file, but every rank resumes ITS OWN Philox key and
    offsets, so the ranks keep drawing different z / noise / eps / data after a DP resume."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "ranks.pt")
    mp.spawn(_dp_ckpt_worker, args=(2, port, tmp_path, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    for r in range(2):
        seed, key, off, doff, dseed = (int(v) for v in got[r])
        assert seed == key == dseed == 4321 + r, (r, got)
        assert off == 10 + r and doff == (2 << 40) + 20 + r, (r, got)


def test_rekey_reaches_forks_in_place():
    """set_seed writes the device key in place (graphs captured before it see it) and forks share it."""
    rng = gan_amd.DeviceRNG("cpu", seed=(1 << 64) - 3)
    data = rng.fork(2)
    ptr = rng.key.data_ptr()
    assert int(rng.key) == -3 and data.key.data_ptr() == ptr
    rng.set_seed(99)
    assert rng.key.data_ptr() == ptr and int(data.key) == 99 and data.seed == 99
