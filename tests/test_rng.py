"""Device random numbers (csrc/rng.hip) against the numpy Philox4x32-10 restatement (oracle/philox.py).

CPU: the oracle against the Random123 known-answer vectors, and the word->float maps' ranges
and moments.  GPU: uniform draws bit-exact with the oracle; normal draws within
atol 1e-5 + rtol 1e-5 (device logf / sincosf in fp32 against float64); offset advance per call,
also under graph replay; 64-bit seeds and group indices; ragged n.
"""
import numpy as np
import pytest
import torch

from oracle import philox

# Random123 kat_vectors, philox4x32 R=10: (counter, key) -> output
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize("ctr,key,out", KAT)
def test_oracle_known_answers(ctr, key, out):
    got = philox.philox4x32_10(np.array([ctr], dtype=np.uint32), key)[0]
    assert tuple(int(v) for v in got) == out


def test_oracle_maps():
    u = philox.uniform(1 << 16, 7, 0)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01
    z = philox.normal(1 << 16, 7, 0)
    assert np.isfinite(z).all()
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1.0) < 0.02
    assert not np.array_equal(philox.uniform(64, 7, 0), philox.uniform(64, 7, 1))
    assert not np.array_equal(philox.uniform(64, 7, 0), philox.uniform(64, 8, 0))


SEEDS = [0, 4321, 0xDEADBEEFCAFEF00D]
SIZES = [1, 5, 1023, (1 << 20) + 3]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("n", SIZES)
def test_device_draws_match_oracle(seed, n):
    from gan_amd import DeviceRNG
    r = DeviceRNG("cuda", seed)
    u0 = r.rand((n,)).cpu().numpy()
    z1 = r.randn((n,)).cpu().numpy()
    u2 = r.rand((n,)).cpu().numpy()
    assert int(r.offset.item()) == 3
    np.testing.assert_array_equal(u0, philox.uniform(n, seed, 0))
    np.testing.assert_allclose(z1, philox.normal(n, seed, 1), rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(u2, philox.uniform(n, seed, 2))


@pytest.mark.gpu
def test_device_group_index_high_word():
    """n > 2^34 elements is out of reach; check the offset's high word instead."""
    from gan_amd import DeviceRNG
    r = DeviceRNG("cuda", 99)
    r.offset.fill_((1 << 32) + 5)
    u = r.rand((4099,)).cpu().numpy()
    np.testing.assert_array_equal(u, philox.uniform(4099, 99, (1 << 32) + 5))


@pytest.mark.gpu
def test_device_draws_fresh_under_graph_replay():
    from gan_amd import DeviceRNG
    r = DeviceRNG("cuda", 11)
    n = 3 * 4096 + 1
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        r.randn((8,))                                  # warm-up draw at offset 0
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = r.randn((n,))
    # capture does not run the kernels: the offset is still 1
    outs = []
    for _ in range(3):
        g.replay()
        outs.append(out.cpu().numpy().copy())
    torch.cuda.synchronize()
    assert int(r.offset.item()) == 4
    for k, o in enumerate(outs):
        np.testing.assert_allclose(o, philox.normal(n, 11, 1 + k), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_device_normal_moments():
    from gan_amd import DeviceRNG
    z = DeviceRNG("cuda", 5).randn((1 << 22,)).double()
    assert abs(float(z.mean())) < 3e-3
    assert abs(float(z.std()) - 1.0) < 3e-3
    assert abs(float((z ** 3).mean())) < 1e-2
    assert abs(float((z ** 4).mean()) - 3.0) < 3e-2
