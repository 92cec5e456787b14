"""Checkpoint resume under captured HIP graphs (train/trainunits.py:58-130).

A run of the bench's graph schedule (pipeline.Iteration, fake groups (4, 1), B = 8) takes one
replayed iteration, saves a checkpoint, and takes a second one.  A FRESH trainer -- other initial
weights, another Philox seed, its graphs captured BEFORE the load -- loads that checkpoint and
replays one iteration.  Its state must equal the uninterrupted run's bit for bit: both models'
parameters, gradients, AdamW moments and step counters, every BatchNorm statistic, and the RNG
key and stream offsets.  This holds only if the load refreshes what the graphs baked in: the
persistent packed conv-weight copies (checkpoint._refresh_packed) and the device-resident Philox
key (rng.DeviceRNG.key, ganamd_philox_draw_keyed).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
B = 8


def _trainer(gan, wseed, rseed):
    from gan_amd.pipeline import Iteration
    torch.manual_seed(wseed)
    G = gan.Generator(256).to(DEV)
    D = gan.Discriminator().to(DEV)
    tr = gan.Train([], DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.DeviceRNG(DEV, rseed))
    it = Iteration(tr, B, 5, 1, overlap=False, fake_groups=[4, 1])
    it.eager()                     # warm-up, then capture (the bench's order)
    it.capture()
    return tr, it


def _state(tr):
    from gan_amd.pipeline import training_state
    st = [t.detach().cpu().clone() for t in training_state(tr)]
    rng = {k: int(v) for k, v in tr.rng.state().items()}
    return st, rng, int(tr.rng.key)


def test_graph_resume_is_bit_identical(tmp_path):
    import gan_amd as gan
    trA, itA = _trainer(gan, 1, 11)
    itA.step()
    trA.ckpt_root = str(tmp_path)
    name = trA.save_ckpt("WGANGP", 0, 0).rsplit("/", 1)[1][:-4]
    itA.step()
    torch.cuda.synchronize()
    want_st, want_rng, want_key = _state(trA)
    del itA, trA
    torch.cuda.empty_cache()

    trB, itB = _trainer(gan, 2, 22)       # other weights, other key, captured before the load
    trB.ckpt_root = str(tmp_path)
    assert trB.load_generator_ckpt(name) and trB.load_discriminator_ckpt(name)
    itB.step()
    torch.cuda.synchronize()
    got_st, got_rng, got_key = _state(trB)
    assert got_key == want_key == 11 and got_rng == want_rng, (got_key, got_rng, want_rng)
    bad = [i for i, (a, b) in enumerate(zip(got_st, want_st)) if not torch.equal(a, b)]
    assert not bad, [(i, tuple(want_st[i].shape), float((got_st[i].double() - want_st[i].double()).abs().max()))
                     for i in bad[:8]]
