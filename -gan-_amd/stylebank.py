"""The style bank: all 519 style MLPs and demodulation products of G13_5 as a handful of launches.

Every ``Conv2dWeightModulate`` of the reference (generator_13_5.py:219-248) owns a style MLP
``to_style = [EqLinear(256,256), BN1d, PReLU] -> EqLinear(256, Cin) -> BN1d(Cin)`` applied to the
SAME latent ``w`` (the mapping network's output), and a demodulation product
``d = rsqrt(c^2 * (sum_k W^2) @ s^2 + eps)``.  Run module by module that is ~15 launches per conv
x 519 convs per forward, all on [<=384, 64]-sized matrices.  Since nothing in the bank depends
on the feature maps, the drop-in computes it up front, once per forward:

  H1 = c1 * W1bank @ w + b1          one linear over the 519 stacked first layers  [519*256, B]
  Y1 = PReLU(BN1d(H1))               one banked BatchNorm (rows are independent channels)
  S~ = c2 * W2_g @ Y1_g + b2_g       one grouped GEMM (519 groups, ganamd_grouped_gemm)
  S  = BN1d(S~)                      one banked BatchNorm
  Q  = Wsq_g @ S_g^2;  D = rsqrt(c_g^2 Q + eps)   segment_sumsq x3 + one grouped GEMM

The backward is the same handful of launches, and writes the bank's parameter gradients
straight into the flat gradient buffer (the parameters are contiguous there because
``Generator.flat_layout`` orders them bank-first).  BatchNorm running statistics live in two
bank buffers; each module's ``running_mean``/``running_var`` is a view into them.

Numerics are identical in form to the per-module path (same kernels, same reductions per row);
``tests/test_models_gpu.py::test_style_bank_matches_modules`` checks it.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from . import _lib
from ._lib import LIB, check, iptr, ptr, stream, workspace
from . import ops

TILE = 64


def _bank_modules(G):
    from .generator_13_5 import Conv2dWeightModulate
    return [m for m in G.modules() if isinstance(m, Conv2dWeightModulate)]


def _kgroups(mods):
    ks = sorted({m.k for m in mods})
    return [(k, [i for i, m in enumerate(mods) if m.k == k]) for k in ks]


def bank_param_order(G):
    """Parameters in bank order (the prefix of Generator.flat_layout)."""
    mods = _bank_modules(G)
    l1 = [m.to_style[0].net[0] for m in mods]
    bn1 = [m.to_style[0].net[1] for m in mods]
    act1 = [m.to_style[0].net[2] for m in mods]
    l2 = [m.to_style[1] for m in mods]
    bn2 = [m.to_style[2] for m in mods]
    order = [l.weight.weights for l in l1] + [l.bias for l in l1] + [b.weight for b in bn1] + \
        [b.bias for b in bn1] + [a.weight for a in act1] + [l.weight.weights for l in l2] + \
        [l.bias for l in l2] + [b.weight for b in bn2] + [b.bias for b in bn2]
    for _, idx in _kgroups(mods):
        order += [mods[i].weight.weights for i in idx]
    return order


def _tiles(rows: np.ndarray) -> np.ndarray:
    """Pack a list of int32 descriptor rows (last column = float scale) as ganamd_gtile[]."""
    a = np.asarray(rows, dtype=np.float64)
    out = a[:, :11].astype(np.int32)
    sc = a[:, 11].astype(np.float32).view(np.int32)
    return np.concatenate([out, sc[:, None]], axis=1)


def _check_tiles(t: np.ndarray, a_numel, b_numel, c_numel, a_trans=False, b_trans=False):
    """Host-side bounds check of a tile list before it ever reaches the kernel."""
    a_off, lda, b_off, ldb, c_off, ldc, rows, cols, K = (t[:, i].astype(np.int64) for i in range(9))
    if (rows < 1).any() or (rows > TILE).any() or (cols < 1).any() or (cols > TILE).any() or (K < 1).any():
        raise _lib.GanAmdError("grouped gemm: tile extents out of range")
    a_hi = a_off + ((K - 1) * lda + rows - 1 if a_trans else (rows - 1) * lda + K - 1)
    b_hi = b_off + ((cols - 1) * ldb + K - 1 if b_trans else (K - 1) * ldb + cols - 1)
    c_hi = c_off + (rows - 1) * ldc + cols - 1
    if min(a_off.min(), b_off.min(), c_off.min()) < 0 or a_hi.max() >= a_numel or b_hi.max() >= b_numel \
            or c_hi.max() >= c_numel:
        raise _lib.GanAmdError("grouped gemm: tile reaches outside its operands")


class StyleBank:
    def __init__(self, G, flat):
        mods = _bank_modules(G)
        self.mods, self.n = mods, len(mods)
        self.flat = flat
        dev = flat.data.device
        self.device = dev
        d_latent = mods[0].to_style[1].weight.weights.shape[1]
        self.dl = d_latent
        for m in mods:
            assert m.to_style[0].net[0].weight.weights.shape == (d_latent, d_latent)
            for bn in (m.to_style[0].net[1], m.to_style[2]):
                assert bn.momentum == 0.1 and bn.eps == 1e-5 and bn.affine and bn.track_running_stats
        self.cin = [m.to_style[1].weight.weights.shape[0] for m in mods]
        self.cout = [m.out_planes for m in mods]
        self.k = [m.k for m in mods]
        self.c1 = mods[0].to_style[0].net[0].weight.scale
        self.c2 = mods[0].to_style[1].weight.scale
        assert all(m.to_style[1].weight.scale == self.c2 for m in mods)
        self.cconv = [m.weight.scale for m in mods]

        # ---- regions of the flat buffers ------------------------------------------------
        base = flat.data.data_ptr()
        order = bank_param_order(G)
        off = None
        self.regions = {}
        cursor = 0
        for p in order:
            o = (p.data_ptr() - base) // 4
            if off is None:
                off = o
                cursor = o
            if o != cursor or not (0 <= o < flat.n_train):
                raise RuntimeError("style bank: parameters are not laid out bank-first in the flat buffer")
            cursor += p.numel()
        self.first_param = order[0]
        self.first_ptr = order[0].data_ptr()

        def seg(name, params):
            nonlocal off
            n = sum(p.numel() for p in params)
            self.regions[name] = (off, n)
            off += n

        n = self.n
        seg("W1", order[0:n]); seg("b1", order[n:2 * n]); seg("g1", order[2 * n:3 * n])
        seg("be1", order[3 * n:4 * n]); seg("a1", order[4 * n:5 * n]); seg("W2", order[5 * n:6 * n])
        seg("b2", order[6 * n:7 * n]); seg("g2", order[7 * n:8 * n]); seg("be2", order[8 * n:9 * n])
        self.kgroups = _kgroups(mods)
        pos = 9 * n
        for k, idx in self.kgroups:
            seg(f"Wc{k}", order[pos:pos + len(idx)])
            pos += len(idx)

        # row offsets of each group in the stacked matrices
        self.s_off = np.concatenate([[0], np.cumsum(self.cin)]).astype(np.int64)      # S rows
        self.d_off_mod = np.zeros(n, np.int64)                                          # D rows (module order)
        self.d_off_mod[:] = np.concatenate([[0], np.cumsum(self.cout)])[:-1]
        self.S_rows, self.D_rows = int(self.s_off[-1]), int(sum(self.cout))
        # Wsq layout: k-groups in flat order, modules in group order
        self.wsq_off = np.zeros(n, np.int64)
        o = 0
        self.wsq_group = []
        for k, idx in self.kgroups:
            g0 = o
            for i in idx:
                self.wsq_off[i] = o
                o += self.cout[i] * self.cin[i]
            self.wsq_group.append((k, g0, o - g0))
        self.wsq_numel = o
        self.w2_row = self.s_off[:-1]      # W2 bank rows coincide with S rows

        # ---- BN running statistics re-homed into bank buffers ------------------------------
        self.rm1 = torch.empty(n * d_latent, device=dev)
        self.rv1 = torch.empty_like(self.rm1)
        self.rm2 = torch.empty(self.S_rows, device=dev)
        self.rv2 = torch.empty_like(self.rm2)
        for i, m in enumerate(mods):
            for bn, rm, rv, o0, c in ((m.to_style[0].net[1], self.rm1, self.rv1, i * d_latent, d_latent),
                                      (m.to_style[2], self.rm2, self.rv2, int(self.s_off[i]), self.cin[i])):
                rm[o0:o0 + c].copy_(bn.running_mean)
                rv[o0:o0 + c].copy_(bn.running_var)
                bn.running_mean = rm[o0:o0 + c]
                bn.running_var = rv[o0:o0 + c]

        # per-row -0.5 * c^2 for the demodulation backward (rows of D, module order)
        c2rows = np.concatenate([np.full(self.cout[i], -0.5 * self.cconv[i] ** 2) for i in range(n)])
        self.neg_half_c2 = torch.tensor(c2rows, dtype=torch.float32, device=dev)[:, None]
        self._tile_cache = {}

    # ---- views ---------------------------------------------------------------------------
    def pdata(self, name):
        o, n = self.regions[name]
        return self.flat.data[o:o + n]

    def pgrad(self, name):
        o, n = self.regions[name]
        return self.flat.grad[o:o + n]

    def valid(self):
        return self.first_param.data_ptr() == self.first_ptr

    # ---- tile lists ------------------------------------------------------------------------
    def tiles(self, B):
        t = self._tile_cache.get(B)
        if t is None:
            t = self._tile_cache[B] = self._make_tiles(B)
        return t

    def _make_tiles(self, B):
        E = _lib
        dl = self.dl
        L2, DEM, DEMT, GWSQ, L2T, GW2 = [], [], [], [], [], []
        for i in range(self.n):
            cin, cout = self.cin[i], self.cout[i]
            so, do, wo, w2 = int(self.s_off[i]), int(self.d_off_mod[i]), int(self.wsq_off[i]), int(self.w2_row[i])
            for n0 in range(0, B, TILE):
                nc = min(TILE, B - n0)
                for r0 in range(0, cin, TILE):
                    rr = min(TILE, cin - r0)
                    # S~[so+r, n] = c2 * sum_k W2[w2+r, k] Y1[i*dl+k, n] + b2[so+r]
                    L2.append([(w2 + r0) * dl, dl, i * dl * B + n0, B, (so + r0) * B + n0, B, rr, nc, dl,
                               E.EPI_BIAS, so + r0, self.c2])
                    # T[so+r, n] = sum_co Wsq[co, r] gq[do+co, n]              (A transposed)
                    DEMT.append([wo + r0, cin, do * B + n0, B, (so + r0) * B + n0, B, rr, nc, cout,
                                 E.EPI_STORE, 0, 1.0])
                for r0 in range(0, cout, TILE):
                    rr = min(TILE, cout - r0)
                    # D[do+r, n] = rsqrt(c^2 * sum_ci Wsq[r, ci] S[so+ci, n]^2 + eps)
                    DEM.append([wo + r0 * cin, cin, so * B + n0, B, (do + r0) * B + n0, B, rr, nc, cin,
                                E.EPI_DEMOD, 0, self.cconv[i]])
                for m0 in range(0, dl, TILE):
                    # gY1[i*dl+m, n] = c2 * sum_r W2[w2+r, m] gS~[so+r, n]      (A transposed)
                    L2T.append([w2 * dl + m0, dl, so * B + n0, B, (i * dl + m0) * B + n0, B, min(TILE, dl - m0), nc,
                                cin, E.EPI_SCALE, 0, self.c2])
            for r0 in range(0, cout, TILE):
                for j0 in range(0, cin, TILE):
                    # gWsq[r, ci] = sum_n gq[do+r, n] S[so+ci, n]^2           (B transposed, squared)
                    GWSQ.append([(do + r0) * B, B, (so + j0) * B, B, wo + r0 * cin + j0, cin, min(TILE, cout - r0),
                                 min(TILE, cin - j0), B, E.EPI_STORE, 0, 1.0])
            for r0 in range(0, cin, TILE):
                for j0 in range(0, dl, TILE):
                    # gW2[w2+r, k] += c2 * sum_n gS~[so+r, n] Y1[i*dl+k, n]    (B transposed)
                    GW2.append([(so + r0) * B, B, (i * dl + j0) * B, B, (w2 + r0) * dl + j0, dl, min(TILE, cin - r0),
                                min(TILE, dl - j0), B, E.EPI_ACCUM, 0, self.c2])
        nW2, nY1, nS, nD = self.regions["W2"][1], self.n * dl * B, self.S_rows * B, self.D_rows * B
        nQ = self.wsq_numel
        spec = {"L2": (L2, nW2, nY1, nS, False, False), "DEM": (DEM, nQ, nS, nD, False, False),
                "DEMT": (DEMT, nQ, nD, nS, True, False), "GWSQ": (GWSQ, nD, nS, nQ, False, True),
                "L2T": (L2T, nW2, nS, nY1, True, False), "GW2": (GW2, nS, nY1, nW2, False, True)}
        out = {}
        for name, (rows, na, nb, nc, at, bt) in spec.items():
            t = _tiles(rows)
            _check_tiles(t, na, nb, nc, at, bt)
            out[name] = torch.from_numpy(t).to(self.device)
        return out

    # ---- forward entry -------------------------------------------------------------------
    def __call__(self, w):
        outs = _BankFn.apply(w, self)
        n = self.n
        return outs[:n], outs[n:]


def grouped_gemm(A, Bm, C, tiles, a_trans=False, b_trans=False, b_square=False, bias=None):
    check(LIB.ganamd_grouped_gemm(ptr(A), ptr(Bm), ptr(C), ptr(bias), iptr(tiles), tiles.shape[0], int(a_trans),
                                  int(b_trans), int(b_square), stream()), "grouped_gemm")
    return C


def _bn_fwd(x, C, L, gamma, beta, alpha, rm, rv):
    from .ops import bn_fwd_raw       # segmented statistics when ops.BN_SEGMENTS says so
    return bn_fwd_raw(x, C, L, gamma, beta, alpha, rm, rv, 0.1, 1e-5)


def _bn_bwd(gy, x, C, L, gamma, beta, alpha, mean, invstd, gg, gb, ga):
    """gx; the parameter gradients are ACCUMULATED into gg/gb/ga (flat-buffer regions)."""
    gx = torch.empty_like(x)
    ws = workspace(LIB.ganamd_rowreduce_workspace(C, L), x.device)
    check(LIB.ganamd_bn_act_bwd(ptr(gy), ptr(x), C, L, ptr(gamma), ptr(beta), ptr(alpha), ptr(mean), ptr(invstd),
                                ptr(gx), ptr(gg), ptr(gb), ptr(ga), 1, *_lib.ws(ws), stream()), "bn_act_bwd")
    return gx


class _BankFn(Function):
    @staticmethod
    def forward(ctx, w, bank: StyleBank):
        w = w.contiguous()
        dl, B = w.shape
        n = bank.n
        T = bank.tiles(B)
        geo1 = ops.linear_geo(B, dl, n * dl)
        H1 = ops._conv_fwd(geo1, w, bank.pdata("W1"), bank.pdata("b1"), alpha=bank.c1).view(n * dl, B)
        Y1, m1, i1 = _bn_fwd(H1, n * dl, B, bank.pdata("g1"), bank.pdata("be1"), bank.pdata("a1"), bank.rm1, bank.rv1)
        Sp = torch.empty((bank.S_rows, B), device=w.device)
        grouped_gemm(bank.pdata("W2"), Y1, Sp, T["L2"], bias=bank.pdata("b2"))
        S, m2, i2 = _bn_fwd(Sp, bank.S_rows, B, bank.pdata("g2"), bank.pdata("be2"), None, bank.rm2, bank.rv2)
        Wsq = torch.empty(bank.wsq_numel, device=w.device)
        for k, g0, gn in bank.wsq_group:
            check(LIB.ganamd_segment_sumsq(ptr(bank.pdata(f"Wc{k}")), gn, k * k, ptr(Wsq[g0:]), stream()),
                  "segment_sumsq")
        D = torch.empty((bank.D_rows, B), device=w.device)
        grouped_gemm(Wsq, S, D, T["DEM"], b_square=True)
        ctx.bank = bank
        ctx.save_for_backward(w, H1, Y1, Sp, S, D, Wsq, m1, i1, m2, i2)
        s_list = torch.split(S, bank.cin)
        d_list = torch.split(D, bank.cout)
        return tuple(s_list) + tuple(d_list)

    @staticmethod
    @once_differentiable
    def backward(ctx, *grads):
        bank: StyleBank = ctx.bank
        w, H1, Y1, Sp, S, D, Wsq, m1, i1, m2, i2 = ctx.saved_tensors
        n = bank.n
        dl, B = w.shape
        T = bank.tiles(B)
        gS = torch.cat(grads[:n])
        gD = torch.cat(grads[n:])
        # demodulation: D = (c^2 q + eps)^(-1/2)  =>  dD/dq = -c^2/2 * D^3
        gq = gD * D.pow(3) * bank.neg_half_c2
        Tm = torch.empty_like(S)
        grouped_gemm(Wsq, gq, Tm, T["DEMT"], a_trans=True)
        gS.addcmul_(S, Tm, value=2.0)
        gWsq = torch.empty_like(Wsq)
        grouped_gemm(gq, S, gWsq, T["GWSQ"], b_trans=True, b_square=True)
        for k, g0, gn in bank.wsq_group:
            kk = k * k
            bank.pgrad(f"Wc{k}").view(gn, kk).addcmul_(bank.pdata(f"Wc{k}").view(gn, kk), gWsq[g0:g0 + gn, None],
                                                     value=2.0)
        # second BatchNorm (no activation)
        gSp = _bn_bwd(gS, Sp, bank.S_rows, B, bank.pdata("g2"), bank.pdata("be2"), None, m2, i2, bank.pgrad("g2"),
                      bank.pgrad("be2"), None)
        # second linear (grouped)
        ops.row_sum_acc(gSp, bank.pgrad("b2"))
        gY1 = torch.empty_like(Y1)
        grouped_gemm(bank.pdata("W2"), gSp, gY1, T["L2T"], a_trans=True)
        grouped_gemm(gSp, Y1, bank.pgrad("W2"), T["GW2"], b_trans=True)
        # first BatchNorm + PReLU
        gH1 = _bn_bwd(gY1, H1, n * dl, B, bank.pdata("g1"), bank.pdata("be1"), bank.pdata("a1"), m1, i1,
                      bank.pgrad("g1"), bank.pgrad("be1"), bank.pgrad("a1"))
        # first linear (one stacked GEMM)
        ops.row_sum_acc(gH1, bank.pgrad("b1"))
        geo1 = ops.linear_geo(B, dl, n * dl)
        ops._conv_wgrad(geo1, w, gH1, alpha=bank.c1, out=bank.pgrad("W1"), accumulate=True)
        gw = ops._conv_dgrad(geo1, gH1, bank.pdata("W1"), alpha=bank.c1).view(dl, B)
        return gw, None
