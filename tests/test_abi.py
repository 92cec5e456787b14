"""CPU: libganamd.so loads and exports every entry point include/ganamd.h declares, with the
signatures the ctypes binding uses; invalid arguments are rejected without touching a GPU."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ganamd.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ganamd_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_abi():
    names = declared()
    assert "ganamd_conv_fwd" in names and "ganamd_adamw" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    from gan_amd import _lib
    lib = ctypes.CDLL(_lib.SO_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding covers exactly the declared ABI
    assert sorted(_lib.EXPORTS) == declared()


def test_library_is_gfx950():
    from gan_amd import _lib
    blob = open(_lib.SO_PATH, "rb").read()
    assert b"gfx950" in blob
    import __graft_entry__
    assert "gfx950" in _lib.version() and _lib.version().endswith("src:" + __graft_entry__.source_hash())


def test_invalid_arguments_rejected():
    from gan_amd import _lib
    L = _lib.LIB
    d = _lib.ConvDesc(0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)   # B = 0: invalid geometry
    n = _lib.c_size_t(0)
    assert L.ganamd_conv_workspace(d, 0, n) == -1
    assert L.ganamd_conv_fwd(d, None, None, None, None, None, 1.0, None, None, 0, None) == -1
    assert L.ganamd_prelu_fwd(None, None, 0, 0, None, None) == -1
    assert L.ganamd_adamw(None, None, None, None, 0, None, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -1


def test_workspace_sizes():
    from gan_amd import _lib
    L = _lib.LIB
    d = _lib.ConvDesc(4, 8, 16, 16, 8, 16, 16, 3, 3, 1, 1, 1, 0, 0, 0, 0)
    n = _lib.c_size_t(0)
    assert L.ganamd_conv_workspace(d, _lib.CONV_DGRAD, n) == 0
    assert n.value >= 4 * 8 * 4 * (18 * 18 - 16 * 16)   # the frame-split dgrad's ring buffer (replication pad)
    assert L.ganamd_rowreduce_workspace(8, 4096) >= 8 * 3 * 4
    bad = _lib.ConvDesc(4, 8, 16, 16, 8, 16, 16, 3, 3, 1, 1, 1, 0, 0, 7, 0)   # unknown math mode
    assert L.ganamd_conv_workspace(bad, _lib.CONV_FWD, n) == -1
    bad = _lib.ConvDesc(4, 8, 16, 16, 8, 16, 16, 3, 3, 1, 1, 1, 0, 0, 0, 16)  # unknown kernel_off bit
    assert L.ganamd_conv_workspace(bad, _lib.CONV_FWD, n) == -1
    # the direct conv of Cout <= 4 forwards (raw weights) needs none; packed weights take the GEMM
    rgb = _lib.ConvDesc(4, 108, 64, 64, 3, 64, 64, 5, 5, 1, 2, 1, 0, 0, 0, 0)
    assert L.ganamd_conv_workspace(rgb, _lib.CONV_FWD, n) == 0 and n.value == 0
    rgb = _lib.ConvDesc(4, 108, 64, 64, 3, 64, 64, 5, 5, 1, 2, 1, 0, 0, 0, _lib.KERNEL_SMALL)
    assert L.ganamd_conv_workspace(rgb, _lib.CONV_FWD, n) == 0 and n.value > 0


@pytest.mark.parametrize("bad", ["x", "w"])
def test_python_wrappers_check_shapes(bad):
    """A wrong operand size raises on the host (never reaches a kernel)."""
    import torch
    from gan_amd import ops
    geo = ops.conv_geo(2, 3, 8, 8, 4, 3, 1, 1)
    x = torch.empty(3 * 2 * 8 * 8 + (1 if bad == "x" else 0))
    w = torch.empty(4 * 3 * 9 + (1 if bad == "w" else 0))
    with pytest.raises(Exception):
        ops._conv_fwd(geo, x, w)


@pytest.mark.parametrize("shape", [
    # B, Cin, H, Cout, k, stride, pad: the census' large and small GEMMs
    (128, 128, 32, 128, 3, 1, 1), (64, 96, 64, 96, 5, 1, 2), (64, 1025, 4, 1025, 3, 1, 1),
    (64, 192, 5, 192, 3, 1, 1), (64, 1024, 16, 1024, 1, 1, 0), (64, 4100, 1, 4100, 1, 1, 0),
    (128, 1024, 8, 1024, 3, 2, 1), (4, 5, 8, 7, 3, 1, 1), (128, 64, 64, 64, 3, 2, 1), (64, 128, 32, 128, 3, 2, 1)])
@pytest.mark.parametrize("op", [0, 1])
def test_conv_block_schedule(shape, op):
    """Host-side invariants of the conv GEMM block schedule (whole tiles + K-split tail)."""
    from gan_amd import _lib, ops
    B, cin, h, cout, k, s, p = shape
    geo = ops.conv_geo(B, cin, h, h, cout, k, s, p)
    for scaled in (False, True):
        pl = ops.plan_info(geo, op, scaled)
        assert 0 <= pl["nfull_t"] <= pl["gx"] and pl["S"] >= 1
        assert pl["blocks"] == pl["nfull_t"] * pl["gy"] + (pl["gx"] - pl["nfull_t"]) * pl["gy"] * pl["S"]
        if pl["nfull_t"] == pl["gx"]:
            assert pl["S"] == 1
        # every split of a tail tile owns at least one K-step (no block leaves its slab unwritten)
        nct = -(-(geo.Cout if op == 1 else geo.Cin) // 16)
        # dgrad: the scatter form (one tap) on small maps, the phased form (phase 0's taps) for strided
        # convs on larger maps (conv_gemm.hip dgrad_scatter / dgrad_phased)
        phased = op == 1 and s > 1 and k > 1 and h * h > 100 and (h + 2 * p) % s == 0
        taps = 1 if (op == 1 and (s > 1 or h * h <= 100) and k > 1 and not phased) else \
            (-(-k // s)) ** 2 if phased else k * k
        kt_total = nct * taps
        assert (pl["S"] - 1) * pl["kt_per_split"] < kt_total <= pl["S"] * pl["kt_per_split"]
        n = _lib.c_size_t(0)
        assert _lib.LIB.ganamd_conv_workspace(geo.desc(), op, n) == 0
        # the unpacked call packs the weights into the workspace first: the whole packed copy must
        # fit (the phased dgrad packs all s*s phases -- a round-4 bug sized it for phase 0 alone)
        pb, nraw, npre = _lib.c_size_t(0), _lib.c_size_t(0), _lib.c_size_t(0)
        raw, pre = geo.desc(packed=False), geo.desc(packed=True)
        assert _lib.LIB.ganamd_conv_pack_bytes(raw, op, pb) == 0
        assert _lib.LIB.ganamd_conv_workspace(raw, op, nraw) == 0
        assert _lib.LIB.ganamd_conv_workspace(pre, op, npre) == 0
        assert nraw.value - npre.value >= pb.value, (nraw.value, npre.value, pb.value)
        if pl["S"] > 1:
            tail_cols = (geo.B * (geo.OH * geo.OW if op == 0 else 1)) - pl["nfull_t"] * pl["bn"]
            if op == 0:
                assert n.value >= 4 * pl["S"] * geo.Cout * tail_cols


def _critic_op(kind, ins, **kw):
    from gan_amd import _lib
    e = _lib.CriticOp()
    e.kind = _lib.COP[kind]
    for j, v in enumerate(list(ins) + [-1] * (3 - len(ins))):
        e.ins[j] = v
    for k, v in kw.items():
        setattr(e, k, v)
    return e


def _critic_plan(ops, B=4, C0=3, H0=8, W0=8, S=1):
    from gan_amd import _lib
    t = (_lib.CriticOp * len(ops))(*ops)
    return _lib.LIB.ganamd_critic_create(t, len(ops), B, C0, H0, W0, S, 0, 0)


def test_critic_engine_plan():
    """The C-ABI critic engine (ganamd_critic_*) validates a program and sizes its workspace on
    the host: a tiny critic swap -> conv 3x3 -> PReLU -> SE gate (pmean, linear, sigmoid, x*s + r)
    -> MiniBatchStdDev -> pmean -> linear to [1][B]; malformed programs give NULL."""
    from gan_amd import _lib
    L = _lib.LIB
    fake = 0x1000                   # never dereferenced by create / workspace
    good = [_critic_op("swap", [0]),
            _critic_op("conv", [1], cout=4, k=3, stride=1, pad=1, pad_mode=1, alpha=1.0, w=fake),    # v2 [4,B,8,8]
            _critic_op("prelu", [2], w=fake),                                                        # v3
            _critic_op("pmean", [3]),                                                                # v4 [4,B]
            _critic_op("conv", [4], cout=4, k=1, stride=1, pad=0, pad_mode=0, alpha=1.0, w=fake),    # v5 linear
            _critic_op("sigmoid", [5]),                                                              # v6
            _critic_op("scale_add", [3, 6, 2]),                                                      # v7
            _critic_op("mbstd", [7], group=4),                                                       # v8 [5,B,8,8]
            _critic_op("pmean", [8]),                                                                # v9 [5,B]
            _critic_op("conv", [9], cout=1, k=1, stride=1, pad=0, pad_mode=0, alpha=1.0, w=fake)]    # v10 [1,B]
    p = _critic_plan(good)
    assert p
    n = _lib.c_size_t(0)
    assert L.ganamd_critic_workspace(p, ctypes.byref(n)) == 0
    # X, G, XD, A of every value at least
    vals = [4 * 4 * 64, 4 * 4 * 64, 4 * 4, 4 * 4, 4 * 4, 4 * 4 * 64, 5 * 4 * 64, 5 * 4, 4] + [3 * 4 * 64]
    assert n.value >= 4 * 4 * sum(vals)
    regions = []
    for r in range(4):
        b = _lib.c_size_t(0)
        assert L.ganamd_critic_region_bytes(p, r, ctypes.byref(b)) == 0
        regions.append(b.value)
    assert sum(regions) == n.value and regions[1] == regions[2] == regions[3] >= 4 * sum(vals[:-1])
    assert L.ganamd_critic_bind(p, 1, ctypes.c_void_p(fake), regions[1] - 4) == -1      # region too small
    assert L.ganamd_critic_bind(p, 1, ctypes.c_void_p(fake), regions[1]) == 0
    # a sweep whose regions are not all bound is refused before any launch
    assert L.ganamd_critic_forward(p, ctypes.c_void_p(fake), None, None, 0, None) == -1
    # a contiguous workspace smaller than the query is refused before any launch
    assert L.ganamd_critic_forward(p, ctypes.c_void_p(fake), None, ctypes.c_void_p(fake), n.value - 4, None) == -1
    ptr = ctypes.c_void_p()
    assert L.ganamd_critic_value(p, 0, 3, ctypes.byref(ptr)) == 0 and not ptr.value   # nothing run yet
    assert L.ganamd_critic_value(p, 4, 3, ctypes.byref(ptr)) == -1
    # sweeps out of order are refused before any launch
    assert L.ganamd_critic_backward(p, None, None, None, ctypes.c_void_p(fake), n.value, None) == -1
    assert L.ganamd_critic_tangent(p, ctypes.c_void_p(fake), None, ctypes.c_void_p(fake), n.value, None) == -1
    L.ganamd_critic_destroy(p)
    bad = [
        good[:-1] + [_critic_op("conv", [9], cout=2, k=1, pad_mode=0, alpha=1.0, stride=1, w=fake)],  # output not [1][B]
        [_critic_op("conv", [0], cout=1, k=1, stride=1, alpha=1.0, w=fake)],                         # conv on NCHW input
        good[:6] + [_critic_op("scale_add", [3, 2, 2])] + good[7:],                                    # gate not [C][B]
        good[:3] + [_critic_op("pmean", [7])] + good[4:],                                              # used before defined
        good[:1] + [_critic_op("conv", [1], cout=4, k=9, stride=1, pad=0, alpha=1.0, w=fake)] + good[2:],  # kernel > map
    ]
    for ops in bad:
        assert not _critic_plan(ops)
    assert not _critic_plan(good, B=6, S=4)          # segments must divide the batch


def test_undersized_workspace_rejected():
    """Every entry point that takes a workspace also takes its size and refuses (GANAMD_EINVAL, -1)
    a workspace smaller than its own query -- before launching anything, so these calls with
    never-dereferenced pointers are safe without a GPU.  (tests/test_ops_gpu.py::
    test_workspace_bytes_enforced runs the same calls on real buffers: one byte short -> -1, the
    queried size -> 0.)"""
    from gan_amd import _lib, ops
    L = _lib.LIB
    f = ctypes.c_void_p(0x1000)               # never dereferenced: the size check comes first
    st = None
    # convs: a replicate-padded 3x3 (packs the weight into the workspace), a strided one (phased
    # dgrad), a 1x1 linear (the BN-fused skinny GEMM)
    for geo in (ops.conv_geo(4, 8, 16, 16, 8, 3, 1, 1), ops.conv_geo(4, 16, 32, 32, 16, 3, 2, 1),
                ops.conv_geo(8, 64, 64, 64, 64, 3, 1, 1)):
        d = geo.desc()
        for op in (_lib.CONV_FWD, _lib.CONV_DGRAD, _lib.CONV_WGRAD):
            need = geo.ws_bytes(op)
            if need == 0:
                continue
            short = need - 1
            if op == _lib.CONV_FWD:
                assert L.ganamd_conv_fwd(d, f, f, None, None, None, 1.0, f, f, short, st) == -1
                assert L.ganamd_conv_fwd(d, f, f, None, None, None, 1.0, f, None, 0, st) == -1
                assert L.ganamd_conv_fwd_ex(d, f, f, None, None, None, 1.0, None, None, None, f, f, short, st) == -1
            elif op == _lib.CONV_DGRAD:
                assert L.ganamd_conv_dgrad(d, f, f, None, 1.0, f, f, short, st) == -1
            else:
                assert L.ganamd_conv_wgrad(d, f, f, None, None, 1.0, f, 0, f, short, st) == -1
                assert L.ganamd_conv_wgrad2(d, f, f, f, f, 1.0, f, 0, f, short, st) == -1
    lin = ops.linear_geo(16, 256, 256)
    need = lin.ws_bytes(_lib.CONV_FWD)
    assert need > 0
    assert L.ganamd_linear_bn_act(lin.desc(), f, f, None, 1.0, f, f, None, f, f, 0.1, 1e-5, f, f, need - 1, st) == -1
    # row reductions (BatchNorm, PReLU slope, bias gradients): ganamd_rowreduce_workspace
    C, Ln = 8, 1 << 16
    short = L.ganamd_rowreduce_workspace(C, Ln) - 1
    assert L.ganamd_bn_act_fwd(f, C, Ln, f, f, None, None, None, 0.1, 1e-5, f, f, f, f, short, st) == -1
    assert L.ganamd_bn_act_fwd_seg(f, C, Ln, 2, f, f, None, None, None, 0.1, 1e-5, f, f, f, f, f,
                                   L.ganamd_rowreduce_workspace(2 * C, Ln // 2) - 1, st) == -1
    assert L.ganamd_bn_act_bwd(f, f, C, Ln, f, f, None, f, f, f, f, f, None, 0, f, short, st) == -1
    assert L.ganamd_prelu_bwd(f, f, f, C, Ln, f, f, 0, f, short, st) == -1
    assert L.ganamd_prelu_bwd_bwd(f, None, f, f, f, C, Ln, f, None, f, f, short, st) == -1
    assert L.ganamd_prelu_tangent(f, f, f, f, C, Ln, f, f, 0, f, short, st) == -1
    assert L.ganamd_row_dot(f, None, C, Ln, f, 0, f, short, st) == -1
    # penalty, MiniBatchStdDev, image batch
    assert L.ganamd_gp_fwd(f, 8, 3 * 64 * 64, 1.0, 10.0, 0, f, f, f, L.ganamd_gp_workspace(8, 3 * 64 * 64) - 1, st) == -1
    mb = L.ganamd_mbstd_workspace(2) - 1
    assert L.ganamd_mbstd_fwd(f, 64, 4, 8, 16, 2, 4, f, 64, None, f, mb, st) == -1
    assert L.ganamd_mbstd_bwd(f, 64, f, 64, 4, 8, 16, 2, 4, f, f, mb, st) == -1
    assert L.ganamd_mbstd_tangent(f, f, 64, 4, 8, 16, 2, 4, f, 64, f, mb, st) == -1
    assert L.ganamd_mbstd_adjoint(f, f, 64, f, f, 64, 4, 8, 16, 2, 4, f, f, mb, st) == -1
    assert L.ganamd_image_batch(f, 2, 80, 80, None, f, f, 4, 64, f, f, 4, 64, f, f, f, f,
                                L.ganamd_image_batch_workspace(2, 80, 64) - 1, st) == -1


def test_python_call_sites_match_signatures():
    """Every ``LIB.ganamd_*(...)`` call in the package passes as many arguments as its ctypes
    signature declares (a ``*ws(...)`` / ``*wsarg(...)`` expansion counts as the two workspace
    arguments, pointer and bytes) -- ctypes would only notice on the GPU, at call time."""
    import ast
    from gan_amd import _lib
    files = [os.path.join(d, f) for d in (os.path.join(REPO, "-gan-_amd"), os.path.join(REPO, "tests"))
             for f in sorted(os.listdir(d)) if f.endswith(".py")] + [os.path.join(REPO, "bench.py")]
    bad = []
    for path in files:
        fn = os.path.relpath(path, REPO)
        tree = ast.parse(open(path).read())
        for node in ast.walk(tree):
            if not (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)
                    and node.func.attr.startswith("ganamd_")):
                continue
            name = node.func.attr
            if name not in _lib._SIGS:
                bad.append(f"{fn}:{node.lineno} {name}: not in the binding")
                continue
            n = 0
            for a in node.args:
                if isinstance(a, ast.Starred):
                    f = a.value.func if isinstance(a.value, ast.Call) else None
                    fname = f.attr if isinstance(f, ast.Attribute) else getattr(f, "id", None)
                    if fname not in ("ws", "wsarg"):      # another expansion (e.g. a padded pointer list)
                        n = None
                        break
                    n += 2
                else:
                    n += 1
            want = len(_lib._SIGS[name][1])
            if n is not None and n != want:
                bad.append(f"{fn}:{node.lineno} {name}: {n} arguments, signature has {want}")
    assert not bad, bad
