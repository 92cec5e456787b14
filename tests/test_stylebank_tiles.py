"""CPU: the style bank's grouped-GEMM tile lists compute, per modulated conv, exactly the products
the per-module path computes (generator_13_5.py:219-248).  The tiles are executed by a numpy
emulation of ``ganamd_grouped_gemm``'s contract (include/ganamd.h); the GPU kernel itself is
checked against torch in tests/test_ops_gpu.py and the whole bank in tests/test_models_gpu.py."""
import numpy as np
import pytest
import torch

EPI_STORE, EPI_BIAS, EPI_DEMOD, EPI_ACCUM, EPI_SCALE = 0, 1, 2, 3, 4


def emulate(A, Bm, C, tiles, a_trans=False, b_trans=False, b_square=False, bias=None):
    A, Bm = A.reshape(-1), Bm.reshape(-1)
    flatC = C.reshape(-1)
    for t in tiles:
        a_off, lda, b_off, ldb, c_off, ldc, rows, cols, K, epi, bias_off = (int(v) for v in t[:11])
        scale = float(np.int32(t[11]).view(np.float32))
        r = np.arange(rows)[:, None]
        k = np.arange(K)[None, :]
        Ablk = A[a_off + k * lda + r] if a_trans else A[a_off + r * lda + k]           # [rows, K]
        kk = np.arange(K)[:, None]
        n = np.arange(cols)[None, :]
        Bblk = Bm[b_off + n * ldb + kk] if b_trans else Bm[b_off + kk * ldb + n]       # [K, cols]
        if b_square:
            Bblk = Bblk * Bblk
        v = Ablk @ Bblk
        idx = c_off + np.arange(rows)[:, None] * ldc + np.arange(cols)[None, :]
        if epi == EPI_BIAS:
            flatC[idx] = scale * v + bias[bias_off:bias_off + rows, None]
        elif epi == EPI_DEMOD:
            flatC[idx] = 1.0 / np.sqrt(scale * scale * v + 1e-8)
        elif epi == EPI_ACCUM:
            flatC[idx] += scale * v
        elif epi == EPI_SCALE:
            flatC[idx] = scale * v
        else:
            flatC[idx] = v
    return C


@pytest.fixture(scope="module")
def bank():
    from gan_amd import Generator
    from gan_amd.optim import FlatParams
    from gan_amd.stylebank import StyleBank
    torch.manual_seed(0)
    G = Generator(256)
    flat = FlatParams(G)
    return StyleBank(G, flat)


@pytest.mark.parametrize("B", [4, 70])
def test_bank_tiles_match_per_module_products(bank, B):
    rng = np.random.default_rng(B)
    T = {k: v.cpu().numpy() for k, v in bank._make_tiles(B).items()}
    n, dl = bank.n, bank.dl
    W2 = rng.standard_normal(bank.regions["W2"][1])
    b2 = rng.standard_normal(bank.S_rows)
    Y1 = rng.standard_normal((n * dl, B))
    Wsq = rng.random(bank.wsq_numel)
    S = rng.standard_normal((bank.S_rows, B))
    gq = rng.standard_normal((bank.D_rows, B))
    gSp = rng.standard_normal((bank.S_rows, B))

    Sp = emulate(W2, Y1, np.zeros((bank.S_rows, B)), T["L2"], bias=b2)
    D = emulate(Wsq, S, np.zeros((bank.D_rows, B)), T["DEM"], b_square=True)
    Tm = emulate(Wsq, gq, np.zeros((bank.S_rows, B)), T["DEMT"], a_trans=True)
    gWsq = emulate(gq, S, np.zeros(bank.wsq_numel), T["GWSQ"], b_trans=True, b_square=True)
    gY1 = emulate(W2, gSp, np.zeros((n * dl, B)), T["L2T"], a_trans=True)
    gW2 = emulate(gSp, Y1, np.ones(W2.size), T["GW2"], b_trans=True)

    c2 = bank.c2
    w2o = 0
    for i in range(n):
        cin, cout = bank.cin[i], bank.cout[i]
        so, do, wo = int(bank.s_off[i]), int(bank.d_off_mod[i]), int(bank.wsq_off[i])
        W2i = W2[w2o:w2o + cin * dl].reshape(cin, dl)
        Y1i = Y1[i * dl:(i + 1) * dl]
        Wsqi = Wsq[wo:wo + cout * cin].reshape(cout, cin)
        Si, gqi, gSpi = S[so:so + cin], gq[do:do + cout], gSp[so:so + cin]
        np.testing.assert_allclose(Sp[so:so + cin], c2 * W2i @ Y1i + b2[so:so + cin, None], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(D[do:do + cout], 1 / np.sqrt(bank.cconv[i] ** 2 * Wsqi @ Si ** 2 + 1e-8),
                                   rtol=1e-6)
        np.testing.assert_allclose(Tm[so:so + cin], Wsqi.T @ gqi, rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(gWsq[wo:wo + cout * cin].reshape(cout, cin), gqi @ (Si ** 2).T, rtol=1e-10,
                                   atol=1e-7)
        np.testing.assert_allclose(gY1[i * dl:(i + 1) * dl], c2 * W2i.T @ gSpi, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(gW2[w2o:w2o + cin * dl].reshape(cin, dl), 1 + c2 * gSpi @ Y1i.T, rtol=1e-6,
                                   atol=1e-7)
        w2o += cin * dl
        if B > 64 and i >= 40:
            break


def test_bank_layout(bank):
    """Bank parameters are contiguous and first in the flat buffer; BN buffers are bank views."""
    flat = bank.flat
    assert bank.regions["W1"][0] == 0
    for m in bank.mods[:5]:
        assert m.to_style[2].running_mean.data_ptr() >= bank.rm2.data_ptr()
    o = 0
    for name in ("W1", "b1", "g1", "be1", "a1", "W2", "b2", "g2", "be2"):
        assert bank.regions[name][0] == o
        o += bank.regions[name][1]
    assert bank.regions["W1"][1] == bank.n * bank.dl * bank.dl
    assert o + sum(bank.regions[f"Wc{k}"][1] for k, _ in bank.kgroups) <= flat.n_train
    assert bank.wsq_numel == sum(c * i for c, i in zip(bank.cout, bank.cin))
