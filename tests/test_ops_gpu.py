"""GPU: every libganamd kernel against a float64 PyTorch-CPU restatement of the same op.

Layout: our ops take CNHW; the references are written NCHW and permuted.  Tolerance: 1e-4
norm-relative (fp32 MFMA / fp32 reductions against float64)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def cn(x):  # NCHW cpu -> CNHW gpu fp32
    return x.detach().permute(1, 0, 2, 3).contiguous().float().to(DEV)


def nc(x):  # CNHW gpu -> NCHW cpu double
    return x.permute(1, 0, 2, 3).double().cpu()


@pytest.fixture(scope="module")
def ops():
    import gan_amd.ops as o
    return o


def ref_conv(x, w, b, k, stride, pad, mode):
    if pad:
        x = F.pad(x, (pad,) * 4, mode="replicate" if mode == 1 else "constant")
    return F.conv2d(x, w, b, stride=stride)


CONV_CASES = [
    # B, Cin, H, Cout, k, stride, pad, mode
    (4, 5, 8, 7, 3, 1, 1, 1),
    (2, 48, 16, 48, 5, 1, 2, 1),
    # 33..48 output rows take the 48-row tile (16x16x4 MFMA blocks); ragged rows, split tails
    (4, 40, 16, 45, 3, 1, 1, 1),
    (8, 48, 32, 48, 3, 1, 1, 0),
    (4, 16, 8, 33, 3, 2, 1, 1),
    (3, 20, 5, 20, 3, 1, 0, 0),
    (4, 17, 6, 9, 1, 1, 0, 0),
    (4, 64, 8, 200, 3, 1, 1, 1),
    (2, 130, 4, 260, 3, 1, 1, 1),
    (8, 3, 64, 64, 3, 1, 1, 1),
    (4, 96, 32, 96, 5, 1, 2, 1),
    (4, 1025, 4, 1025, 3, 1, 1, 1),
    # small maps take the scatter-form dgrad (GEMM over output pixels + fold): edges on both sides
    (4, 20, 2, 24, 3, 1, 1, 1),
    (4, 8, 1, 8, 3, 1, 1, 1),
    (4, 12, 4, 12, 3, 1, 1, 0),
    (2, 6, 7, 5, 5, 1, 2, 1),
    # stride 2: the phased dgrad (s*s phase GEMMs over the padded frame) on maps > 10x10 with an
    # even frame, the scatter form otherwise (D9_4's 3x3 s2 downsampling convs)
    (4, 24, 16, 20, 3, 2, 1, 1),
    (2, 16, 64, 16, 3, 2, 1, 1),
    (2, 8, 32, 12, 3, 2, 1, 0),
    (2, 6, 12, 5, 5, 2, 2, 1),
    (2, 5, 14, 4, 4, 2, 1, 1),
    (3, 10, 9, 7, 3, 2, 1, 0),
    (2, 8, 5, 6, 3, 2, 1, 1),
    (2, 4, 2, 4, 3, 2, 1, 1),
    (2, 6, 11, 5, 5, 2, 2, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(ops, case):
    B, Cin, H, Cout, k, s, p, mode = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(Cout, generator=g, dtype=torch.float64, requires_grad=True)
    alpha = 0.37
    y = ref_conv(x, w * alpha, b, k, s, p, mode)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), gy)

    geo = ops.conv_geo(B, Cin, H, H, Cout, k, s, p, mode)
    assert (geo.OH, geo.OW) == tuple(y.shape[2:])
    xg, wg, bg = cn(x), w.detach().float().to(DEV), b.detach().float().to(DEV)
    yg = ops._conv_fwd(geo, xg, wg, bg, alpha=alpha)
    assert rel(nc(yg), y) < 1e-4
    gyg = cn(gy)
    assert rel(nc(ops._conv_dgrad(geo, gyg, wg, alpha=alpha)), gx) < 1e-4
    assert rel(ops._conv_wgrad(geo, xg, gyg, alpha=alpha), gw) < 1e-4
    # through autograd (bias grad included)
    xa = xg.clone().requires_grad_()
    wa = wg.clone().requires_grad_()
    ba = bg.clone().requires_grad_()
    ya = ops.conv2d(xa, wa, ba, geo, alpha)
    ya.backward(gyg)
    assert rel(nc(xa.grad), gx) < 1e-4 and rel(wa.grad, gw) < 1e-4 and rel(ba.grad, gb) < 1e-4


CONVT_CASES = [
    # B, Cin, H, Cout, k, stride, pad
    (4, 7, 4, 5, 4, 2, 1),
    (4, 256, 1, 384, 4, 1, 0),
    (2, 108, 32, 108, 4, 2, 1),
    (4, 3, 8, 3, 4, 2, 1),
]


@pytest.mark.parametrize("case", CONVT_CASES)
def test_conv_transpose(ops, case):
    B, Cin, H, Cout, k, s, p = case
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(Cin, Cout, k, k, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(Cout, generator=g, dtype=torch.float64, requires_grad=True)
    y = F.conv_transpose2d(x, w, b, stride=s, padding=p)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), gy)
    geo = ops.convT_geo(B, Cin, H, H, Cout, k, s, p)
    xa = cn(x).requires_grad_()
    wa = w.detach().float().to(DEV).requires_grad_()
    ba = b.detach().float().to(DEV).requires_grad_()
    ya = ops.conv2d(xa, wa, ba, geo, 1.0)
    assert rel(nc(ya), y) < 1e-4
    ya.backward(cn(gy))
    assert rel(nc(xa.grad), gx) < 1e-4 and rel(wa.grad, gw) < 1e-4 and rel(ba.grad, gb) < 1e-4


@pytest.mark.parametrize("B,cin,cout", [(4, 256, 256), (64, 4100, 4100), (8, 4100, 1), (64, 256, 3072), (128, 192, 192),
                                        (384, 96, 48), (64, 1025, 1025), (192, 3, 70)])
def test_linear(ops, B, cin, cout):
    g = torch.Generator().manual_seed(B + cin)
    x = torch.randn(B, cin, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(cout, cin, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(cout, generator=g, dtype=torch.float64, requires_grad=True)
    c = cin ** -0.5
    y = F.linear(x, w * c, b)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), gy)
    xa = x.detach().t().contiguous().float().to(DEV).requires_grad_()
    wa = w.detach().float().to(DEV).requires_grad_()
    ba = b.detach().float().to(DEV).requires_grad_()
    ya = ops.linear(xa, wa, ba, c)
    assert rel(ya.t(), y) < 1e-4
    ya.backward(gy.t().contiguous().float().to(DEV))
    assert rel(xa.grad.t(), gx) < 1e-4 and rel(wa.grad, gw) < 1e-4 and rel(ba.grad, gb) < 1e-4


@pytest.mark.parametrize("B,cin,cout,H,k", [(4, 48, 54, 16, 3), (4, 54, 48, 16, 5), (4, 96, 96, 8, 5), (2, 192, 192, 8, 3), (8, 390, 192, 4, 1)])
def test_modconv(ops, B, cin, cout, H, k):
    """Batch-shared modulated conv vs the reference's per-sample grouped conv (generator_13_5.py:234-248)."""
    g = torch.Generator().manual_seed(cin + cout)
    x = torch.randn(B, cin, H, H, generator=g, dtype=torch.float64, requires_grad=True)
    s = torch.randn(B, cin, generator=g, dtype=torch.float64, requires_grad=True)
    W = torch.randn(cout, cin, k, k, generator=g, dtype=torch.float64, requires_grad=True)
    c = (cin * k * k) ** -0.5
    wts = (W * c)[None] * s[:, None, :, None, None]
    wts = wts * torch.rsqrt(wts.pow(2).sum(dim=(2, 3, 4), keepdim=True) + 1e-8)
    xp = F.pad(x.reshape(1, -1, H, H), ((k - 1) // 2,) * 4, mode="replicate")
    y = F.conv2d(xp, wts.reshape(B * cout, cin, k, k), groups=B).reshape(B, cout, H, H)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    gx, gs, gW = torch.autograd.grad(y, (x, s, W), gy)
    geo = ops.conv_geo(B, cin, H, H, cout, k, 1, (k - 1) // 2)
    xa = cn(x).requires_grad_()
    sa = s.detach().t().contiguous().float().to(DEV).requires_grad_()
    Wa = W.detach().float().to(DEV).requires_grad_()
    ya = ops.modconv(xa, sa, Wa, geo, c)
    assert rel(nc(ya), y) < 1e-4
    ya.backward(cn(gy))
    assert rel(nc(xa.grad), gx) < 1e-4
    assert rel(sa.grad.t(), gs) < 1e-4
    assert rel(Wa.grad, gW) < 1e-4


@pytest.mark.parametrize("shape,act", [((5, 4, 8, 8), True), ((300, 64), True), ((3, 64, 64, 64), False),
                                       ((48, 8, 64, 64), True),
                                       # one block per row (512 < L <= 8192): 5x5 pools, the boundary, ragged
                                       ((48, 64, 5, 5), True), ((7, 128, 8, 8), False), ((6, 3, 17, 11), True)])
def test_bn_act(ops, shape, act):
    g = torch.Generator().manual_seed(len(shape) + shape[0])
    C = shape[0]
    x = (torch.randn(shape, generator=g, dtype=torch.float64) * 3 + 1).requires_grad_()
    gam = (1 + 0.1 * torch.randn(C, generator=g, dtype=torch.float64)).requires_grad_()
    bet = (0.1 * torch.randn(C, generator=g, dtype=torch.float64)).requires_grad_()
    al = (0.25 + 0.05 * torch.randn(C, generator=g, dtype=torch.float64)).requires_grad_()
    xn = x.transpose(0, 1) if len(shape) == 2 else x.permute(1, 0, 2, 3)   # to reference NC(HW)
    rm = torch.zeros(C, dtype=torch.float64)
    rv = torch.ones(C, dtype=torch.float64)
    y = F.batch_norm(xn, rm, rv, gam, bet, training=True, momentum=0.1, eps=1e-5)
    if act:
        y = F.prelu(y, al)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    grads = torch.autograd.grad(y, (x, gam, bet, al) if act else (x, gam, bet), gy)
    bn = torch.nn.BatchNorm1d(C).to(DEV) if len(shape) == 2 else torch.nn.BatchNorm2d(C).to(DEV)
    pr = torch.nn.PReLU(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(gam)
        bn.bias.copy_(bet)
        pr.weight.copy_(al)
    xa = x.detach().float().to(DEV).requires_grad_()
    ya = ops.bn_act(xa, bn, pr if act else None)
    yref = y.transpose(0, 1) if len(shape) == 2 else y.permute(1, 0, 2, 3)
    assert rel(ya, yref) < 1e-4
    assert rel(bn.running_mean, rm) < 1e-5 and rel(bn.running_var, rv) < 1e-5
    gya = (gy.transpose(0, 1) if len(shape) == 2 else gy.permute(1, 0, 2, 3)).contiguous().float().to(DEV)
    ya.backward(gya)
    assert rel(xa.grad, grads[0]) < 1e-4
    assert rel(bn.weight.grad, grads[1]) < 1e-4 and rel(bn.bias.grad, grads[2]) < 1e-4
    if act:
        assert rel(pr.weight.grad, grads[3]) < 1e-4


def test_prelu_double_backward(ops):
    """grad of ||d(sum r*prelu(x))/dx||^2 w.r.t. x, alpha and r -- the GP pattern."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(6, 4, 5, 5, generator=g, dtype=torch.float64, requires_grad=True)
    a = (0.25 + 0.1 * torch.randn(6, generator=g, dtype=torch.float64)).requires_grad_()
    r = torch.randn(6, 4, 5, 5, generator=g, dtype=torch.float64, requires_grad=True)

    def run(xx, aa, rr, f):
        y = f(xx, aa)
        gxx, = torch.autograd.grad((y * rr).sum(), xx, create_graph=True)
        ((gxx * gxx).sum() + (gxx * xx).sum()).backward()
        return xx.grad, aa.grad, rr.grad

    want = run(x, a, r, lambda t, s: F.prelu(t.transpose(0, 1), s).transpose(0, 1))
    xa = x.detach().float().to(DEV).requires_grad_()
    aa = a.detach().float().to(DEV).requires_grad_()
    ra = r.detach().float().to(DEV).requires_grad_()
    got = run(xa, aa, ra, ops.prelu)
    for gg, ww in zip(got, want):
        assert rel(gg, ww) < 1e-5


def test_conv_prelu_double_backward(ops):
    """Double backward through conv -> prelu -> conv (weights and input), as in the critic."""
    g = torch.Generator().manual_seed(5)
    B, C, H = 4, 6, 8
    x = torch.randn(B, 3, H, H, generator=g, dtype=torch.float64, requires_grad=True)
    w1 = torch.randn(C, 3, 3, 3, generator=g, dtype=torch.float64, requires_grad=True)
    w2 = torch.randn(C, C, 3, 3, generator=g, dtype=torch.float64, requires_grad=True)
    b1 = torch.randn(C, generator=g, dtype=torch.float64, requires_grad=True)
    a = (0.25 + 0.1 * torch.randn(C, generator=g, dtype=torch.float64)).requires_grad_()

    def ref(xx, w1, w2, b1, a):
        y = ref_conv(xx, w1, b1, 3, 1, 1, 1)
        y = F.prelu(y, a)
        y = ref_conv(y, w2, None, 3, 2, 1, 1)
        return y.sum(dim=(1, 2, 3))

    def mine(xx, w1, w2, b1, a):
        x_c = xx.permute(1, 0, 2, 3).contiguous()
        y = ops.conv2d(x_c, w1, b1, ops.conv_geo(B, 3, H, H, C, 3, 1, 1), 1.0)
        y = ops.prelu(y, a)
        y = ops.conv2d(y, w2, None, ops.conv_geo(B, C, H, H, C, 3, 2, 1), 1.0)
        return y.sum(dim=(0, 2, 3))

    def gp(f, leaves):
        out = f(*leaves)
        gx, = torch.autograd.grad(out.sum(), leaves[0], create_graph=True)
        loss = ((gx.pow(2).flatten(1).sum(1).sqrt() - 1) ** 2).mean()
        loss.backward()
        return [t.grad for t in leaves]

    want = gp(ref, [x, w1, w2, b1, a])
    got = gp(mine, [t.detach().float().to(DEV).requires_grad_() for t in (x, w1, w2, b1, a)])
    for gg, ww in zip(got[1:], want[1:]):
        assert rel(gg, ww) < 1e-4
    assert rel(got[0], want[0]) < 1e-4


@pytest.mark.parametrize("kind,n,planes", [("smooth", 64, 15), ("up2_smooth", 8, 15), ("smooth_down2", 32, 15),
                                           ("pool5", 16, 15), ("pool5", 64, 101), ("up2_smooth", 32, 67),
                                           ("smooth_down2", 64, 33), ("smooth", 5, 250), ("smooth", 6, 9)])
def test_resample_and_adjoint(ops, kind, n, planes):
    """Both directions (forward table and adjoint) against the dense float64 operator; plane
    counts that leave a ragged last workgroup, 5- and 6-wide maps (the one-column path)."""
    from gan_amd import tables
    g = torch.Generator().manual_seed(n)
    x = torch.randn(planes, 1, n, n, generator=g, dtype=torch.float64, requires_grad=True)
    m = torch.from_numpy(tables.operator_1d(kind, n))
    y = torch.einsum("oh,pw,bchw->bcop", m, m, x)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    gx, = torch.autograd.grad(y, x, gy)
    xa = x.detach().float().to(DEV).requires_grad_()
    ya = ops.resample(xa, kind)
    assert rel(ya, y) < 1e-5
    ya.backward(gy.float().to(DEV))
    assert rel(xa.grad, gx) < 1e-5


@pytest.mark.parametrize("H", [8, 64])
def test_plane_mean_and_dot(ops, H):
    x = torch.randn(7, 4, H, H, dtype=torch.float64)
    y = torch.randn(7, 4, H, H, dtype=torch.float64)
    xa = x.float().to(DEV)
    assert rel(ops.plane_mean(xa), x.mean(dim=(2, 3))) < 1e-6
    assert rel(ops.plane_dot(xa, y.float().to(DEV)), (x * y).sum(dim=(2, 3))) < 1e-5


def test_adamw_matches_torch():
    from gan_amd.optim import FusedAdamW
    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5)).to(DEV)
    m2 = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5)).to(DEV)
    m2.load_state_dict(m1.state_dict())
    o1 = torch.optim.AdamW(m1.parameters(), lr=4e-4, betas=(0.5, 0.999))
    o2 = FusedAdamW(m2, lr=4e-4, betas=(0.5, 0.999))
    for it in range(5):
        x = torch.randn(8, 33, device=DEV)
        o1.zero_grad()
        o2.zero_grad()
        m1(x).pow(2).sum().backward()
        m2(x).pow(2).sum().backward()
        o1.step()
        o2.step()
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(p1, p2, rtol=1e-5, atol=1e-6)
    assert int(o2.step_count.item()) == 5


@pytest.mark.parametrize("a_t,b_t,sq", [(0, 0, 0), (1, 0, 0), (0, 1, 1), (1, 1, 0), (0, 0, 1)])
def test_grouped_gemm(a_t, b_t, sq):
    """ganamd_grouped_gemm vs float64 torch over ragged groups, every epilogue, multi-tile groups."""
    from gan_amd import _lib
    from gan_amd.stylebank import _tiles, grouped_gemm
    g = torch.Generator().manual_seed(11 + 2 * a_t + b_t)
    shapes = [(70, 33, 5), (64, 64, 64), (1, 17, 130), (130, 1, 3), (96, 80, 257)]   # rows, cols, K
    epis = [_lib.EPI_STORE, _lib.EPI_BIAS, _lib.EPI_SCALE, _lib.EPI_ACCUM, _lib.EPI_DEMOD]
    A, Bm, Cinit, want, tiles = [], [], [], [], []
    ao = bo = co = 0
    bias = torch.randn(512, generator=g, dtype=torch.float64)
    for gi, ((R, N, K), epi) in enumerate(zip(shapes, epis)):
        a = torch.randn(R, K, generator=g, dtype=torch.float64)
        b = torch.randn(K, N, generator=g, dtype=torch.float64)
        if epi == _lib.EPI_DEMOD:
            a = a.abs()
        c0 = torch.randn(R, N, generator=g, dtype=torch.float64)
        scale = 0.37 + gi
        acc = a @ (b * b if sq else b)
        if epi == _lib.EPI_STORE:
            w = acc
        elif epi == _lib.EPI_BIAS:
            w = scale * acc + bias[gi:gi + R, None]
        elif epi == _lib.EPI_SCALE:
            w = scale * acc
        elif epi == _lib.EPI_ACCUM:
            w = c0 + scale * acc
        else:
            w = 1 / torch.sqrt(scale * scale * (a @ (b * b)) + 1e-8) if sq else None
        if w is None:   # DEMOD needs a non-negative accumulator: use |a| @ b^2 via squared B
            continue
        A.append((a.t() if a_t else a).contiguous().reshape(-1))
        Bm.append((b.t() if b_t else b).contiguous().reshape(-1))
        Cinit.append(c0.reshape(-1))
        want.append(w.reshape(-1))
        lda = R if a_t else K
        ldb = K if b_t else N
        for r0 in range(0, R, 64):
            for n0 in range(0, N, 64):
                a_off = ao + (r0 if a_t else r0 * K)
                b_off = bo + (n0 * K if b_t else n0)
                tiles.append([a_off, lda, b_off, ldb, co + r0 * N + n0, N, min(64, R - r0), min(64, N - n0), K, epi,
                              gi + r0, scale])
        ao += R * K
        bo += K * N
        co += R * N
    dev = "cuda"
    T = torch.from_numpy(_tiles(tiles)).to(dev)
    C = torch.cat(Cinit).float().to(dev)
    grouped_gemm(torch.cat(A).float().to(dev), torch.cat(Bm).float().to(dev), C, T, a_trans=bool(a_t),
                 b_trans=bool(b_t), b_square=bool(sq), bias=bias.float().to(dev))
    got = C.double().cpu()
    ref = torch.cat(want)
    assert rel(got, ref) < 1e-5


def test_packed_weight_cache_tracks_updates(ops):
    """The packed-weight cache (ops.PackCache) never serves a stale weight: after a torch in-place
    update of the Parameter and after a fused AdamW step the conv sees the new values."""
    from gan_amd.optim import FusedAdamW
    torch.manual_seed(0)
    geo = ops.conv_geo(4, 8, 16, 16, 12, 3, 1, 1)
    lin = torch.nn.Module()
    lin.w = torch.nn.Parameter(torch.randn(12, 8, 3, 3, device="cuda"))
    x = torch.randn(8, 4, 16, 16, device="cuda")

    def run():
        return ops.conv2d(x, lin.w, None, geo, 0.5)

    def fresh():   # a plain tensor is never cached
        return ops.conv2d(x, lin.w.detach().clone(), None, geo, 0.5)

    y0 = run()
    assert rel(run(), y0) == 0
    with torch.no_grad():
        lin.w.mul_(2)
    assert rel(run(), 2 * y0) < 1e-6
    opt = FusedAdamW(lin, lr=0.1)
    y1 = run()
    (y1 * torch.randn_like(y1)).sum().backward()
    opt.step()
    assert rel(run(), fresh()) == 0
    assert rel(run(), y1) > 1e-3
    # the weight has a persistent copy, refreshed by the optimizer's batched repack -- also when
    # the update is a captured graph replayed later
    assert len(opt.flat.packs.entries) >= 1

    def train_step():
        y = run()
        (y * 0.01).sum().backward()
        opt.step()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        train_step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        train_step()
    y2 = run()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    assert rel(run(), fresh()) == 0
    assert rel(run(), y2) > 1e-4


@pytest.mark.parametrize("M,H", [(2, 8), (2, 5), (3, 4), (1, 16), (2, 32), (1, 64)])
def test_mix_fwd_bwd(ops, M, H):
    g = torch.Generator().manual_seed(M * 10 + H)
    C, B = 6, 4
    feas = [torch.randn(C, B, H, H, generator=g, dtype=torch.float64, requires_grad=True) for _ in range(M)]
    att = torch.rand(M, C, B, generator=g, dtype=torch.float64, requires_grad=True)
    ref = sum(f * att[m][:, :, None, None] for m, f in enumerate(feas))
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    want = torch.autograd.grad(ref, feas + [att], gy)
    fg = [f.detach().float().cuda().requires_grad_() for f in feas]
    ag = att.detach().float().cuda().requires_grad_()
    y = ops.mix(fg, ag)
    got = torch.autograd.grad(y, fg + [ag], gy.float().cuda())
    assert rel(y, ref) < 1e-6
    for a, b in zip(got, want):
        assert rel(a, b) < 1e-5


def test_add_prelu_fwd_bwd(ops):
    g = torch.Generator().manual_seed(3)
    a = torch.randn(5, 4, 6, 6, generator=g, dtype=torch.float64, requires_grad=True)
    b = torch.randn(5, 4, 6, 6, generator=g, dtype=torch.float64, requires_grad=True)
    al = torch.rand(5, generator=g, dtype=torch.float64, requires_grad=True)
    z = a + b
    ref = torch.where(z > 0, z, al[:, None, None, None] * z)
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    want = torch.autograd.grad(ref, (a, b, al), gy)
    ins = [t.detach().float().cuda().requires_grad_() for t in (a, b, al)]
    y = ops.add_prelu(*ins)
    got = torch.autograd.grad(y, ins, gy.float().cuda())
    assert rel(y, ref) < 1e-6
    for x, w in zip(got, want):
        assert rel(x, w) < 1e-5


def test_scale_add_double_backward(ops):
    """ScaleAdd / ScaleRows / PlaneDot are closed under differentiation (the critic's GP)."""
    g = torch.Generator().manual_seed(4)
    x = torch.randn(3, 4, 5, 5, generator=g, dtype=torch.float64, requires_grad=True)
    s = torch.rand(3, 4, generator=g, dtype=torch.float64, requires_grad=True)
    r = torch.randn(3, 4, 5, 5, generator=g, dtype=torch.float64, requires_grad=True)
    v = torch.randn(3, 4, 5, 5, generator=g, dtype=torch.float64)

    def loss(f, xx, ss, rr):
        y = f(xx, ss, rr)
        gx, gs = torch.autograd.grad((y * y * v.to(y)).sum(), (xx, ss), create_graph=True)
        return (gx.pow(2).sum() + gs.pow(3).sum())

    ref = loss(lambda a, b, c: c + a * b[:, :, None, None], x, s, r)
    want = torch.autograd.grad(ref, (x, s, r))
    ins = [t.detach().float().cuda().requires_grad_() for t in (x, s, r)]
    out = loss(ops.scale_add, *ins)
    got = torch.autograd.grad(out, ins)
    assert abs(float(out.detach()) - float(ref.detach())) / abs(float(ref.detach())) < 1e-5
    for a, b in zip(got, want):
        assert rel(a, b) < 1e-4


def test_conv_fwd_ex_noise_act(ops):
    g = torch.Generator().manual_seed(5)
    B, Cin, Cout, H, k = 4, 12, 10, 8, 3
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64)
    sx = torch.rand(Cin, B, generator=g, dtype=torch.float64) + 0.5
    sy = torch.rand(Cout, B, generator=g, dtype=torch.float64) + 0.5
    nz = torch.randn(Cout, B, H, H, generator=g, dtype=torch.float64)
    ns = torch.rand(Cout, generator=g, dtype=torch.float64)
    al = torch.rand(Cout, generator=g, dtype=torch.float64)
    xm = x * sx.t()[:, :, None, None]
    y = ref_conv(xm, w * 0.3, None, k, 1, 1, 1) * sy.t()[:, :, None, None]
    y = y + ns[None, :, None, None] * nz.permute(1, 0, 2, 3)
    y = torch.where(y > 0, y, al[None, :, None, None] * y)
    geo = ops.conv_geo(B, Cin, H, H, Cout, k, 1, 1)
    got = ops.modconv_fused(cn(x), sx.float().cuda(), sy.float().cuda(), w.float().cuda(), geo, 0.3,
                            nz.float().cuda(), ns.float().cuda(), al.float().cuda())
    assert rel(nc(got), y) < 1e-5


PATCH_CASES = [
    # B, Cin, H, Cout, k, pad mode, scaled, noise+act: shapes the split6 LDS-patch conv takes
    # (conv_patch.hip: stride 1, "same" padding, 32/64-wide maps, rows M <= 48 or 72 < M <= 96,
    # >= one full round of one block per CU)
    (32, 96, 64, 96, 5, 1, True, True),      # G13_5 modulated 5x5 (96 rows: 32x32x16 blocks)
    (32, 48, 64, 48, 3, 1, True, False),     # 48 rows: paired 16x16x32 blocks
    (32, 40, 64, 45, 5, 1, False, False),    # ragged rows, channels not a multiple of 16
    (64, 128, 32, 96, 3, 1, False, False),   # 32-wide map (256-pixel blocks, 4 waves)
    (32, 108, 64, 80, 5, 1, False, True),    # ragged 96-row tile
    (128, 64, 32, 96, 5, 1, True, False),    # 32-wide map, two rounds
]


@pytest.mark.parametrize("case", PATCH_CASES)
def test_conv_patch_kernel(ops, case):
    """The split6 LDS-patch conv (the default for these shapes) against float64, and the gather
    GEMM on the same shape (ganamd_conv_set_patch(0)) too."""
    B, Cin, H, Cout, k, mode, scaled, extra = case
    p = (k - 1) // 2
    geo = ops.conv_geo(B, Cin, H, H, Cout, k, 1, p, mode)
    pl = ops.plan_info(geo, 0, scaled)
    assert pl["kernel"] == 1 and pl["occupancy"] >= 1, pl
    g = torch.Generator().manual_seed(sum(case[:6]))
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64)
    sx = torch.rand(Cin, B, generator=g, dtype=torch.float64) + 0.5 if scaled else None
    sy = torch.rand(Cout, B, generator=g, dtype=torch.float64) + 0.5 if scaled else None
    xm = x * sx.t()[:, :, None, None] if scaled else x
    y = ref_conv(xm, w * 0.3, None, k, 1, p, mode)
    if scaled:
        y = y * sy.t()[:, :, None, None]
    f = (lambda t: None if t is None else t.float().to(DEV))
    nz = ns = al = None
    if extra:
        nz = torch.randn(Cout, B, H, H, generator=g, dtype=torch.float64)
        ns = torch.rand(Cout, generator=g, dtype=torch.float64)
        al = torch.rand(Cout, generator=g, dtype=torch.float64)
        y = y + ns[None, :, None, None] * nz.permute(1, 0, 2, 3)
        y = torch.where(y > 0, y, al[None, :, None, None] * y)
    got = ops._conv_fwd_ex(geo, cn(x), f(w), f(sx), f(sy), 0.3, f(nz), f(ns), f(al))
    assert rel(nc(got), y) < 1e-5
    # persistent packed weights (Parameter): the same kernel on the packed copy's bf16 planes
    wp = torch.nn.Parameter(f(w))
    if not extra:
        assert rel(nc(ops._conv_fwd(geo, cn(x), wp, None, f(sx), f(sy), 0.3)), y) < 1e-5
    with ops.patch_conv(0):                      # the gather GEMM on the same (x3-packed) operand
        assert ops.plan_info(geo, 0, scaled)["kernel"] == 0
        assert rel(nc(ops._conv_fwd_ex(geo, cn(x), wp, f(sx), f(sy), 0.3, f(nz), f(ns), f(al))), y) < 1e-5


DGRAD_PATCH_CASES = [
    # B, Cin, H, Cout, k, pad mode, scaled: stride-1 dgrads whose interior takes the split6 patch
    # conv (zero-padded, taps reversed) and -- replication padding -- the ring the gather GEMM (s = -2)
    (32, 96, 64, 96, 5, 1, True),            # G13_5 modulated 5x5 (gy scaled by the demodulation)
    (32, 48, 64, 40, 3, 1, False),           # 48 rows (paired 16x16x32), K channels not a multiple of 16
    (64, 96, 32, 128, 3, 1, False),          # 32-wide map
    (32, 96, 64, 80, 3, 0, False),           # zero padding: no ring
]


@pytest.mark.parametrize("case", DGRAD_PATCH_CASES)
def test_conv_patch_dgrad(ops, case):
    B, Cin, H, Cout, k, mode, scaled = case
    p = (k - 1) // 2
    geo = ops.conv_geo(B, Cin, H, H, Cout, k, 1, p, mode)
    assert ops.plan_info(geo, 1, scaled)["kernel"] == 1
    g = torch.Generator().manual_seed(sum(case[:6]) + 7)
    xm = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64)
    sy = torch.rand(Cout, B, generator=g, dtype=torch.float64) + 0.5 if scaled else None
    y = ref_conv(xm, w * 0.3, None, k, 1, p, mode)
    if scaled:
        y = y * sy.t()[:, :, None, None]
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    want, = torch.autograd.grad(y, xm, gy)
    f = (lambda t: None if t is None else t.float().to(DEV))
    got = ops._conv_dgrad(geo, cn(gy), f(w), f(sy), 0.3)
    assert rel(nc(got), want) < 1e-5
    wp = torch.nn.Parameter(f(w))
    got2 = ops._conv_dgrad(geo, cn(gy), wp, f(sy), 0.3)   # persistent packed copy
    assert rel(nc(got2), want) < 1e-5
    with ops.patch_conv(0):                      # the frame-split gather GEMM on the same copy
        assert rel(nc(ops._conv_dgrad(geo, cn(gy), wp, f(sy), 0.3)), want) < 1e-5


TAIL_CASES = [
    # B, Cin, H, Cout, k, pad: more output tiles than resident blocks, not a whole number of rounds
    (104, 128, 32, 128, 3, 1),
    (48, 32, 64, 64, 3, 1),
    (40, 96, 64, 96, 5, 2),
]


@pytest.mark.parametrize("case", TAIL_CASES)
def test_conv_tail_split_schedule(ops, case):
    """Large GEMMs run whole tiles plus K-split tail tiles (slabs + reduce with the epilogue):
    fwd with scales / bias-free noise / PReLU epilogue and dgrad against torch fp32 on the GPU."""
    B0, Cin, H, Cout, k, p = case
    torch.backends.cudnn.allow_tf32 = False

    def mixed(B):   # the fwd or dgrad plan runs whole tiles plus K-split tail tiles
        geo = ops.conv_geo(B, Cin, H, H, Cout, k, 1, p)
        pf, pd = ops.plan_info(geo, 0, True), ops.plan_info(geo, 1, False)
        return geo, pf, pd, any(0 < q["nfull_t"] < q["gx"] and q["S"] > 1 for q in (pf, pd))
    # the planner's choice moves with the kernels' occupancy: the nearest batch with a mixed plan
    B = next((b for b in sorted(range(8, 2 * B0 + 1, 8), key=lambda b: abs(b - B0)) if mixed(b)[3]), B0)
    geo, pf, pd, _ = mixed(B)
    print("plans", B, pf, pd)
    g = torch.Generator(device=DEV).manual_seed(sum(case))
    x = torch.randn(Cin, B, H, H, device=DEV, generator=g)
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g)
    sx = torch.rand(Cin, B, device=DEV, generator=g) + 0.5
    sy = torch.rand(Cout, B, device=DEV, generator=g) + 0.5
    nz = torch.randn(Cout, B, H, H, device=DEV, generator=g)
    ns = torch.rand(Cout, device=DEV, generator=g)
    al = torch.rand(Cout, device=DEV, generator=g)
    alpha = 1.0 / (Cin * k * k) ** 0.5
    xn = (x * sx[:, :, None, None]).permute(1, 0, 2, 3)
    y = F.conv2d(F.pad(xn, (p,) * 4, mode="replicate"), w * alpha).permute(1, 0, 2, 3) * sy[:, :, None, None]
    y = y + ns[:, None, None, None] * nz
    y = torch.where(y > 0, y, al[:, None, None, None] * y)
    got = ops.modconv_fused(x, sx, sy, w, geo, alpha, nz, ns, al)
    assert rel(got, y) < 2e-5
    # dgrad (transposed gather into the padded frame) through torch autograd as the reference
    xr = x.permute(1, 0, 2, 3).clone().requires_grad_()
    yr = F.conv2d(F.pad(xr, (p,) * 4, mode="replicate"), w * alpha)
    gy = torch.randn(yr.shape, device=DEV, generator=g)
    (gx,) = torch.autograd.grad(yr, xr, gy)
    got = ops._conv_dgrad(geo, gy.permute(1, 0, 2, 3).contiguous(), w, alpha=alpha)
    assert rel(got.permute(1, 0, 2, 3), gx) < 2e-5
    # at least the fwd or dgrad plan of each case exercises the mixed schedule on MI355X
    assert any(0 < q["nfull_t"] < q["gx"] and q["S"] > 1 for q in (pf, pd)), (pf, pd)


@pytest.mark.parametrize("case", [(4, 48, 16, 48, 5, 1, 2, 1), (4, 64, 8, 200, 3, 1, 1, 1), (4, 16, 8, 33, 3, 2, 1, 1),
                                  (4, 1025, 4, 1025, 3, 1, 1, 1)])
def test_conv_bf16_math(ops, case):
    """GANAMD_MATH_BF16: operands rounded to bf16, fp32 accumulation -- fwd / dgrad / wgrad within
    a bf16 bar (2^-8 relative per operand) of float64, and measurably different from fp32."""
    B, Cin, H, Cout, k, s, p, mode = case
    g = torch.Generator().manual_seed(sum(case) + 1)
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64, requires_grad=True)
    w = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64, requires_grad=True)
    y = ref_conv(x, w * 0.3, None, k, s, p, mode)
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    gx, gw = torch.autograd.grad(y, (x, w), gy)
    geo = ops.conv_geo(B, Cin, H, H, Cout, k, s, p, mode)
    xg, wg, gyg = cn(x), w.detach().float().to(DEV), cn(gy)
    got = {}
    for m in ("fp32", "bf16"):
        with ops.math_mode(m):
            got[m] = (nc(ops._conv_fwd(geo, xg, wg, alpha=0.3)), nc(ops._conv_dgrad(geo, gyg, wg, alpha=0.3)),
                      ops._conv_wgrad(geo, xg, gyg, alpha=0.3))
    for ref, a32, a16 in zip((y, gx, gw), got["fp32"], got["bf16"]):
        e32, e16 = rel(a32, ref), rel(a16, ref)
        assert e32 < 1e-5 and 3e-4 < e16 < 1e-2, (e32, e16)


@pytest.mark.parametrize("mode,center,lam", [(0, 1.0, 10.0), (1, 0.0, 5.0)])
def test_grad_penalty_fused(ops, mode, center, lam):
    """ganamd_gp_fwd/_bwd: the penalty of train/wgangp.py:34-54 (mode 0) and R1/R2 of
    wganlazygpR2.py:57-70 (mode 1) and its gradient w.r.t. the input gradient, vs float64."""
    g64 = (torch.randn(6, 3, 64, 64, generator=torch.Generator().manual_seed(7 + mode), dtype=torch.float64)
           * 0.02).requires_grad_()
    sq = g64.pow(2).view(6, -1).sum(1)
    ref = lam * ((sq.sqrt() - center).pow(2).mean() if mode == 0 else sq.mean())
    (want,) = torch.autograd.grad(ref * 0.7, g64)
    g = g64.detach().float().to(DEV).requires_grad_()
    out = ops.grad_penalty(g, center, lam, mode)
    assert abs(float(out) - float(ref)) / abs(float(ref)) < 1e-6
    (got,) = torch.autograd.grad(out * 0.7, g)
    assert rel(got, want) < 1e-6


@pytest.mark.parametrize("B,cin,cout,act", [(4, 48, 48, True), (64, 192, 192, True), (37, 384, 96, False),
                                            (64, 1025, 256, True), (2, 96, 40, True)])
def test_linear_bn_act_fused(ops, B, cin, cout, act):
    """ganamd_linear_bn_act (no-grad: linear + train-mode BatchNorm1d + PReLU in one launch) against
    the float64 torch composition; running statistics updated as torch's BatchNorm1d does."""
    g = torch.Generator().manual_seed(B + cin + cout)
    x = torch.randn(cin, B, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, generator=g, dtype=torch.float64)
    b = torch.randn(cout, generator=g, dtype=torch.float64)
    alpha = 1.0 / cin ** 0.5
    bn = torch.nn.BatchNorm1d(cout).double()
    with torch.no_grad():
        bn.weight.copy_(1 + 0.1 * torch.randn(cout, generator=g, dtype=torch.float64))
        bn.bias.copy_(0.1 * torch.randn(cout, generator=g, dtype=torch.float64))
        bn.running_mean.copy_(0.2 * torch.randn(cout, generator=g, dtype=torch.float64))
        bn.running_var.copy_(1 + 0.2 * torch.rand(cout, generator=g, dtype=torch.float64))
    pr = torch.nn.PReLU(cout).double() if act else None
    if pr is not None:
        with torch.no_grad():
            pr.weight.copy_(0.25 + 0.1 * torch.randn(cout, generator=g, dtype=torch.float64))
    bn_g = torch.nn.BatchNorm1d(cout).to(DEV)
    bn_g.load_state_dict({k: v.float() for k, v in bn.state_dict().items()})
    pr_g = None
    if pr is not None:
        pr_g = torch.nn.PReLU(cout).to(DEV)
        pr_g.load_state_dict({k: v.float() for k, v in pr.state_dict().items()})
    w_g = torch.nn.Parameter(w.float().to(DEV))
    with torch.no_grad():
        ref = bn((alpha * x.t() @ w.t() + b))          # [B, cout], updates bn's running stats
        if pr is not None:
            ref = pr(ref)
        assert ops.linear_bn_act_ok(x.float().to(DEV), w_g)
        y = ops.linear_bn_act(x.float().to(DEV), w_g, b.float().to(DEV), alpha, bn_g, pr_g)
    assert rel(y.t(), ref) < 1e-5
    assert rel(bn_g.running_mean, bn.running_mean) < 1e-5
    assert rel(bn_g.running_var, bn.running_var) < 1e-5


@pytest.mark.parametrize("kind,C,B,n", [("pool5", 48, 8, 64), ("pool5", 96, 3, 32), ("smooth", 7, 5, 32)])
def test_resample_sum(ops, kind, C, B, n):
    """ganamd_resample2d_sum (no-grad SK-attention pool of the branch sum) == resample of the
    materialised sum, bit for bit (the same fp32 sum, formed while staging)."""
    g = torch.Generator().manual_seed(C + B + n)
    a = torch.randn(C, B, n, n, generator=g).to(DEV)
    b = torch.randn(C, B, n, n, generator=g).to(DEV)
    with torch.no_grad():
        ref = ops.resample(a + b, kind)
        got = ops.resample_sum(a, b, kind)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("C,B,H", [(48, 8, 64), (96, 4, 16), (7, 3, 2)])
def test_plane_dot_pair(ops, C, B, H):
    """ganamd_plane_dot_pair: <a, b1> and <a, b2> per plane in one pass, against float64."""
    g = torch.Generator().manual_seed(C * B + H)
    a, b1, b2 = (torch.randn(C, B, H, H, generator=g, dtype=torch.float64) for _ in range(3))
    with torch.no_grad():
        out = ops.plane_dot_pair(a.float().to(DEV), b1.float().to(DEV), b2.float().to(DEV))
    assert out is not None
    assert rel(out[0], (a * b1).sum((2, 3))) < 1e-5
    assert rel(out[1], (a * b2).sum((2, 3))) < 1e-5


WGRAD2_CASES = [
    # B, Cin, H, Cout, k, stride, pad, mode: K = B*OH*OW a multiple of 32 -> one two-segment GEMM
    (8, 3, 64, 64, 3, 1, 1, 1),        # the critic's stem (tap-packed N)
    (4, 64, 16, 64, 3, 1, 1, 1),
    (4, 48, 32, 48, 5, 1, 2, 1),       # 48-row wgrad tile
    (8, 24, 16, 20, 3, 2, 1, 1),       # strided
    (64, 512, 1, 512, 1, 1, 0, 0),     # a linear at B = 64
    (32, 512, 4, 512, 3, 1, 1, 1),     # the 4x4 blocks, split K
    (4, 12, 3, 10, 3, 1, 1, 1),        # K = 36: not a whole K-step -> two launches
]


@pytest.mark.parametrize("case", WGRAD2_CASES)
def test_conv_wgrad2_two_segments(ops, case):
    """ganamd_conv_wgrad2 (the critic adjoint's x*a + xd*g, csrc/critic.hip): one GEMM over both
    pixel ranges == the sum of the two weight gradients (float64 reference), accumulating."""
    from gan_amd import _lib
    B, Cin, H, Cout, k, s, p, mode = case
    g = torch.Generator().manual_seed(7 * sum(case))
    geo = ops.conv_geo(B, Cin, H, H, Cout, k, s, p, mode)
    xs = [torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64) for _ in range(2)]
    gys = [torch.randn(B, Cout, geo.OH, geo.OW, generator=g, dtype=torch.float64) for _ in range(2)]
    w = torch.zeros(Cout, Cin, k, k, dtype=torch.float64, requires_grad=True)
    alpha = 0.7
    ref = sum(torch.autograd.grad(ref_conv(x, w * alpha, None, k, s, p, mode), w, gy)[0] for x, gy in zip(xs, gys))
    gw0 = torch.randn(Cout, Cin, k, k, generator=g, dtype=torch.float64)
    out = gw0.float().to(DEV)
    ws = _lib.workspace(geo.ws_bytes(_lib.CONV_WGRAD), DEV)
    xg, gyg = [cn(x) for x in xs], [cn(t) for t in gys]
    rc = _lib.LIB.ganamd_conv_wgrad2(geo.desc(), _lib.ptr(xg[0]), _lib.ptr(gyg[0]), _lib.ptr(xg[1]), _lib.ptr(gyg[1]),
                                     alpha, _lib.ptr(out), 1, *_lib.ws(ws), _lib.stream())
    assert rc == 0
    assert rel(out, gw0 + ref) < 1e-5


# ---- split6: fp32 products on the bf16 matrix cores are fp32-class ---------------------------
# (op, B, cin, H, cout, k, stride, pad, scaled, tile kind).  Every fp32 GEMM runs as six bf16
# products per 16 k (csrc/conv_gemm.hip split3 / mfma6_*); dropping any of the kept terms (h*l,
# l*h, m*m: ~2^-16 relative each) would show here as ~1e-5, fp32's own rounding is ~1e-7.
SPLIT6_CASES = [
    ("fwd", 2, 96, 64, 96, 5, 1, 2, True, "32x32 x3 LDS body (96-row tile), x*s gather, *d epilogue"),
    ("fwd", 2, 128, 32, 128, 3, 1, 1, False, "32x32 x3 LDS body (128-row tile)"),
    ("fwd", 2, 48, 64, 48, 5, 1, 2, True, "48-row tile: paired 16x16x32 products"),
    ("fwd", 2, 48, 64, 3, 5, 1, 2, False, "16-row tile (ToRGB): paired 16x16x32 products"),
    ("dgrad", 2, 64, 64, 64, 3, 1, 1, False, "32x32 x3 body, transposed gather over the padded frame"),
    ("dgrad", 4, 256, 16, 256, 3, 2, 1, False, "phased stride-2 dgrad (kPhase gather, frame split)"),
    ("dgrad", 8, 256, 8, 256, 3, 2, 1, False, "scatter-form dgrad GEMM (stride 2, 8x8)"),
    ("wgrad", 2, 48, 64, 48, 5, 1, 2, True, "gather wgrad, 48x64 tile: 16x16x16 split products"),
    ("wgrad", 2, 96, 32, 96, 5, 1, 2, True, "gather wgrad, 96-wide tile: 16x16x16 split products"),
    ("wgrad", 2, 128, 32, 128, 3, 1, 1, False, "gather wgrad, 32x32 tile"),
    ("wgrad", 2, 48, 64, 48, 5, 1, 2, True, "row-blocked wgrad, 48 rows (paired 16x16x32)"),
    ("wgrad", 2, 96, 32, 96, 5, 1, 2, True, "row-blocked wgrad, 96 rows (32x32x16)"),
    ("wgrad", 4, 128, 32, 128, 3, 1, 1, False, "row-blocked wgrad, 128 rows, split K"),
    ("wgrad", 8, 1025, 4, 1025, 3, 1, 1, False, "96x96 wgrad tiles, the 1025-channel 4x4 block"),
    ("fwd", 32, 96, 64, 96, 5, 1, 2, True, "split6 LDS-patch conv, 96 rows (32x32x16)"),
    ("fwd", 32, 48, 64, 48, 5, 1, 2, True, "split6 LDS-patch conv, 48 rows (paired 16x16x32)"),
    ("dgrad", 32, 96, 64, 96, 5, 1, 2, True, "split6 LDS-patch dgrad interior + ring GEMM"),
    # the 64-row patch tile (Cout in (48, 64]) at W = 64 and W = 32, forward and dgrad
    ("fwd", 32, 56, 64, 56, 3, 1, 1, False, "split6 LDS-patch conv, 64-row tile, W=64"),
    ("dgrad", 32, 56, 64, 56, 3, 1, 1, False, "split6 LDS-patch dgrad, 64-row tile, W=64"),
    ("fwd", 32, 64, 32, 60, 3, 1, 1, True, "64-row tile at W=32 (scaled, Cout 60)"),
    ("dgrad", 32, 60, 32, 64, 3, 1, 1, True, "64-row dgrad at W=32 (scaled, Cin 60)"),
]


@pytest.mark.parametrize("case", SPLIT6_CASES, ids=[c[-1] for c in SPLIT6_CASES])
def test_split6_fp32_class(ops, case):
    """Each tile kind of the fp32 GEMMs against float64 at <= 1e-6 (max |err| / max |ref|) on
    full-mantissa random operands -- or, on launches of millions of outputs whose error tail fp32
    accumulation alone takes past 1e-6, within 2x of the same convolution evaluated in float32 on
    the host: the split products are fp32-class."""
    _split6_check(ops, case, 600 + SPLIT6_CASES.index(case))


def test_split6_wide_gather_tile(ops):
    """the 128x256 gather tile the planner picks by cost (unscaled 128->128 3x3 at
    32x32) against float64 -- at the first batch whose plan on this GPU is that tile."""
    for B in (128, 256, 160, 192, 64, 96):
        g = ops.conv_geo(B, 128, 32, 32, 128, 3, 1, 1)
        info = ops.plan_info(g, 0, False)
        if info["kernel"] == 0 and info["bn"] == 256:
            break
    else:
        pytest.fail("no batch plans the 128x256 tile")
    _split6_check(ops, ("fwd", B, 128, 32, 128, 3, 1, 1, False, "128x256 gather tile (costed)"), 650, want_bn=256)


def _split6_check(ops, case, seed, want_bn=None):
    from tests._emu import emulate, max_rel
    op, B, cin, H, cout, k, s, p, scaled, _kind = case
    g = ops.conv_geo(B, cin, H, H, cout, k, s, p)
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(cin, B, H, H, generator=gen).to(DEV)
    w = torch.nn.Parameter(torch.randn(cout, cin, k, k, generator=gen).to(DEV))
    gy = torch.randn(cout, B, g.OH, g.OW, generator=gen).to(DEV)
    xs = (torch.rand(cin, B, generator=gen) + 0.5).to(DEV) if scaled else None
    ys = (torch.rand(cout, B, generator=gen) + 0.5).to(DEV) if scaled else None
    # the gather wgrad's tile kinds on shapes the row-blocked kernel would take: mask it off (bit 2)
    with torch.no_grad(), ops.patch_conv(3 if "gather wgrad" in case[-1] else 7):
        if op == "fwd":
            got = ops._conv_fwd(g, x, w, None, xs, ys, 0.7)
        elif op == "dgrad":
            got = ops._conv_dgrad(g, gy, w, ys, 0.7)
        else:
            got = ops._conv_wgrad(g, x, gy, xs, ys, 0.7)
    torch.cuda.synchronize()
    ref = emulate(op, g, x=x, w=w, gy=gy, xs=xs, ys=ys, alpha=0.7)
    e = max_rel(got, ref)
    e_bf = max_rel(got, emulate(op, g, x=x, w=w, gy=gy, xs=xs, ys=ys, alpha=0.7, bf16=True))
    info = ops.plan_info(g, {"fwd": 0, "dgrad": 1}[op], scaled) if op != "wgrad" else {}
    if "patch" in case[-1]:
        assert info["kernel"] == 1, info
    if "64-row" in case[-1] and info.get("kernel") == 1:
        assert info["bm"] == 64, info
    if want_bn is not None:
        assert info["bn"] == want_bn, info
    print(f"{case[-1]}: max rel err vs float64 {e:.2e} (vs a bf16-operand GEMM {e_bf:.2e}); plan {info}")
    if e > 1e-6:
        # millions of outputs: compare with fp32's own error tail -- a host float32 evaluation and
        # a plain fp32 FMA convolution on the device (one accumulator, K multiply-adds in order)
        e32 = max_rel(emulate(op, g, x=x, w=w, gy=gy, xs=xs, ys=ys, alpha=0.7, dtype=torch.float32), ref)
        from tests._emu import seq_fp32
        eseq = max_rel(seq_fp32(op, g, x=x, w=w, gy=gy, xs=xs, ys=ys, alpha=0.7), ref) if op != "wgrad" else 0.0
        print(f"   fp32 yardsticks: host float32 {e32:.2e}, sequential fp32 FMA {eseq:.2e}")
        # (the split adds up to six rounded partial products per k into the accumulator where the
        # FMA convolution rounds once, so its worst output over millions may sit a little above the
        # FMA's: the 128x256 tile at B = 128 measured 1.52e-6 against 1.43e-6)
        assert e <= max(2 * e32, 1.5 * eseq), (e, e32, eseq)
    assert e_bf > 1e-4                   # the operands really keep more than bf16


WGRAD_ROW_CASES = [
    # B, Cin, H, Cout, k, pad mode, scaled: the row-blocked split6 wgrad (conv_wgrad_row.hip)
    (16, 48, 64, 48, 5, 1, True),      # G13_5 48-channel modulated 5x5 (3 waves x 16-row blocks)
    (8, 96, 64, 96, 5, 1, True),       # 96-channel (3 waves x 32 rows)
    (16, 64, 64, 64, 3, 1, False),     # D9_4 64-channel block conv (2 waves)
    (8, 128, 32, 128, 3, 1, False),    # D9_4 128-channel (4 waves)
    (8, 40, 32, 45, 3, 0, False),      # zero padding, ragged rows / columns
    (4, 54, 64, 102, 5, 1, True),      # 102 rows: 4 waves, ragged 32-row block
]


@pytest.mark.parametrize("case", WGRAD_ROW_CASES)
def test_conv_wgrad_row(ops, case):
    """Row-blocked weight gradient (a block owns one kernel row and all its taps) against float64:
    overwrite and accumulate, and equal to the gather wgrad (mask bit 2 off) at the fp32 bar."""
    B, Cin, H, Cout, k, mode, scaled = case
    p = (k - 1) // 2
    geo = ops.conv_geo(B, Cin, H, H, Cout, k, 1, p, mode)
    g = torch.Generator().manual_seed(sum(case[:6]) + 11)
    x = torch.randn(B, Cin, H, H, generator=g, dtype=torch.float64)
    w = torch.zeros(Cout, Cin, k, k, dtype=torch.float64, requires_grad=True)
    sx = torch.rand(Cin, B, generator=g, dtype=torch.float64) + 0.5 if scaled else None
    sy = torch.rand(Cout, B, generator=g, dtype=torch.float64) + 0.5 if scaled else None
    xm = x * sx.t()[:, :, None, None] if scaled else x
    y = ref_conv(xm, w * 0.3, None, k, 1, p, mode)
    if scaled:
        y = y * sy.t()[:, :, None, None]
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    want, = torch.autograd.grad(y, w, gy)
    f = (lambda t: None if t is None else t.float().to(DEV))
    got = ops._conv_wgrad(geo, cn(x), cn(gy), f(sx), f(sy), 0.3)
    assert rel(got, want) < 1e-5
    base = torch.randn(want.shape, generator=g, dtype=torch.float64)
    acc = base.float().to(DEV)
    ops._conv_wgrad(geo, cn(x), cn(gy), f(sx), f(sy), 0.3, out=acc, accumulate=True)
    assert rel(acc, base + want) < 1e-5
    with ops.patch_conv(3):
        assert rel(ops._conv_wgrad(geo, cn(x), cn(gy), f(sx), f(sy), 0.3), want) < 1e-5


WGRAD_DET_CASES = WGRAD_ROW_CASES + [
    # the generator's 96-channel 3x3 stage (SK conv_0, 32x32 and 64x64 maps) and its 96 -> 54 conv3
    (8, 96, 32, 96, 3, 1, True), (8, 96, 64, 96, 3, 1, True), (8, 96, 64, 54, 3, 1, True),
    (8, 96, 32, 96, 5, 1, True), (32, 64, 64, 64, 3, 1, False),
]


@pytest.mark.parametrize("case", WGRAD_DET_CASES)
def test_conv_wgrad_deterministic(ops, case):
    """The weight gradient is a function of its inputs alone: eight calls on the same operands, each
    into a workspace the caching allocator hands back full of NaN, give the same bits (a partial sum
    read before it is written, or a slab entry no block writes, shows up here as a changed result)."""
    B, Cin, H, Cout, k, mode, scaled = case
    p = (k - 1) // 2
    geo = ops.conv_geo(B, Cin, H, H, Cout, k, 1, p, mode)
    g = torch.Generator(device=DEV).manual_seed(sum(case[:6]))
    x = torch.randn(Cin, B, H, H, generator=g, device=DEV)
    gy = torch.randn(Cout, B, H, H, generator=g, device=DEV)
    sx = torch.rand(Cin, B, generator=g, device=DEV) + 0.5 if scaled else None
    sy = torch.rand(Cout, B, generator=g, device=DEV) + 0.5 if scaled else None
    nb = geo.ws_bytes(ops._lib.CONV_WGRAD)
    outs = []
    for _ in range(8):
        junk = torch.full((max(nb, 4) // 4 + 1,), float("nan"), device=DEV)
        del junk
        outs.append(ops._conv_wgrad(geo, x, gy, sx, sy, 0.3))
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), float((o - outs[0]).abs().max())


@pytest.mark.parametrize("case", WGRAD_DET_CASES)
def test_conv_fwd_dgrad_deterministic(ops, case):
    """The same for the forward (LDS-patch conv or gather GEMM with split-K tails) and the input
    gradient (patch interior + ring fold, or the padded-frame GEMM): eight calls, NaN-poisoned
    workspaces, equal bits."""
    B, Cin, H, Cout, k, mode, scaled = case
    p = (k - 1) // 2
    geo = ops.conv_geo(B, Cin, H, H, Cout, k, 1, p, mode)
    g = torch.Generator(device=DEV).manual_seed(sum(case[:6]) + 1)
    x = torch.randn(Cin, B, H, H, generator=g, device=DEV)
    gy = torch.randn(Cout, B, H, H, generator=g, device=DEV)
    w = torch.nn.Parameter(torch.randn(Cout, Cin, k, k, generator=g, device=DEV) * 0.1)
    sx = torch.rand(Cin, B, generator=g, device=DEV) + 0.5 if scaled else None
    sy = torch.rand(Cout, B, generator=g, device=DEV) + 0.5 if scaled else None
    for op, fn in ((ops._lib.CONV_FWD, lambda: ops._conv_fwd(geo, x, w, None, sx, sy, 1.0)),
                   (ops._lib.CONV_DGRAD, lambda: ops._conv_dgrad(geo, gy, w, sy, 1.0))):
        nb = max(geo.ws_bytes(op, True), geo.ws_bytes(op, False))
        outs = []
        with torch.no_grad():
            for _ in range(8):
                junk = torch.full((max(nb, 4) // 4 + 1,), float("nan"), device=DEV)
                del junk
                outs.append(fn())
        torch.cuda.synchronize()
        assert torch.isfinite(outs[0]).all(), op
        for o in outs[1:]:
            assert torch.equal(o, outs[0]), (op, float((o - outs[0]).abs().max()))


@pytest.mark.parametrize("B,cin,cout,H,k,aligned", [(4, 48, 54, 16, 3, True), (3, 20, 12, 8, 5, True),
                                                    (2, 6, 5, 5, 3, False)])
def test_modconv_noise_grads(ops, B, cin, cout, H, k, aligned):
    """ModConv with the StyleConv noise (generator_13_5.py:234-248, 263-265) as the generator step runs
    it: d an input, noise_scale a parameter.  dL/dd and dL/dns come from ganamd_modconv_sd_bwd (one
    pass, double dots) on 16-byte planes, from plane dots otherwise; float64 reference."""
    g = torch.Generator().manual_seed(7 * cin + k)
    x = torch.randn(B, cin, H, H, generator=g, dtype=torch.float64, requires_grad=True)
    s = torch.randn(B, cin, generator=g, dtype=torch.float64, requires_grad=True)
    d = (torch.rand(B, cout, generator=g, dtype=torch.float64) + 0.5).requires_grad_()
    W = torch.randn(cout, cin, k, k, generator=g, dtype=torch.float64, requires_grad=True)
    ns = (torch.rand(cout, generator=g, dtype=torch.float64) * 0.1 + 0.2).requires_grad_()
    noise = torch.randn(B, cout, H, H, generator=g, dtype=torch.float64)
    c = (cin * k * k) ** -0.5
    xp = F.pad(x * s[:, :, None, None], ((k - 1) // 2,) * 4, mode="replicate")
    y = F.conv2d(xp, W * c) * d[:, :, None, None] + ns[None, :, None, None] * noise
    gy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    want = torch.autograd.grad(y, (x, s, d, W, ns), gy)
    geo = ops.conv_geo(B, cin, H, H, cout, k, 1, (k - 1) // 2)
    xa = cn(x).requires_grad_()
    sa = s.detach().t().contiguous().float().to(DEV).requires_grad_()
    da = d.detach().t().contiguous().float().to(DEV).requires_grad_()
    Wa = W.detach().float().to(DEV).requires_grad_()
    nsa = ns.detach().float().to(DEV).requires_grad_()
    ya = ops.ModConv.apply(xa, sa, da, Wa, geo, c, nsa, cn(noise))
    assert rel(nc(ya), y) < 1e-5
    ya.backward(cn(gy))
    got = (nc(xa.grad), sa.grad.t(), da.grad.t(), Wa.grad, nsa.grad)
    for name, a, b in zip(("x", "s", "d", "W", "ns"), got, want):
        assert rel(a, b) < 1e-5, (name, rel(a, b))
    if aligned:       # the fused kernel ran: plane dots in double
        r = ops.modconv_sd_bwd(cn(gy), ya.detach(), cn(noise), da.detach(), nsa.detach())
        assert r is not None and rel(r[0].t(), want[2]) < 1e-6


def test_route_backward(ops):
    """ops.route views (the dual-path splits of generator_13_5.py:448-467): one-pass backward
    (ganamd_route_bwd) == autograd's slice backward; overlapping, repeated, unused and empty views;
    rows of L % 4 != 0 take the scalar path."""
    for shape in ((10, 4, 8, 8), (7, 3, 3, 1)):
        g = torch.Generator().manual_seed(shape[0])
        x = torch.randn(shape, generator=g, dtype=torch.float64, requires_grad=True)
        C = shape[0]
        bounds = [(0, 3), (6, C), (3, C), (0, 3), (0, C), (C, C), (2, 5)]
        ws = [torch.randn((hi - lo,) + shape[1:], generator=g, dtype=torch.float64) for lo, hi in bounds]
        used = [True, True, True, True, True, False, False]
        loss = sum((x[lo:hi] * w).sum() for (lo, hi), w, u in zip(bounds, ws, used) if u)
        (want,) = torch.autograd.grad(loss, x)
        xa = x.detach().float().to(DEV).requires_grad_()
        views = ops.route(xa * 1.0, bounds)
        assert all(v.shape[0] == hi - lo for v, (lo, hi) in zip(views, bounds))
        la = sum((v * w.float().to(DEV)).sum() for v, w, u in zip(views, ws, used) if u)
        la.backward()
        assert rel(xa.grad, want) < 1e-6


@pytest.mark.parametrize("C,B,n", [(6, 4, 16), (3, 2, 8), (5, 3, 64)])
def test_pool_sum_fanout(ops, C, B, n):
    """SK attention's pool of the branch sum with the branches passed on to the mix
    (generator_13_5.py:82-89): t = pool5(f0 + f1) and each branch's gradient = pool5^T(g_t) + its own
    (ganamd_resample2d_sum / ganamd_resample2d_add) == autograd through the float64 reference;
    also with one branch's pass-through unused."""
    g = torch.Generator().manual_seed(C * n)
    f0 = torch.randn(B, C, n, n, generator=g, dtype=torch.float64, requires_grad=True)
    f1 = torch.randn(B, C, n, n, generator=g, dtype=torch.float64, requires_grad=True)
    wt = torch.randn(B, C, 5, 5, generator=g, dtype=torch.float64)
    w0 = torch.randn(B, C, n, n, generator=g, dtype=torch.float64)
    w1 = torch.randn(B, C, n, n, generator=g, dtype=torch.float64)
    for use1 in (True, False):
        t = F.adaptive_avg_pool2d(f0 + f1, 5)
        loss = (t * wt).sum() + (f0 * w0).sum() + ((f1 * w1).sum() if use1 else 0)
        g0, g1 = torch.autograd.grad(loss, (f0, f1))
        a0, a1 = cn(f0).requires_grad_(), cn(f1).requires_grad_()
        ta, b0, b1 = ops.pool_sum_fanout(a0, a1, "pool5")
        assert rel(nc(ta), t) < 1e-5
        la = (ta * cn(wt)).sum() + (b0 * cn(w0)).sum() + ((b1 * cn(w1)).sum() if use1 else 0)
        la.backward()
        assert rel(nc(a0.grad), g0) < 1e-5 and rel(nc(a1.grad), g1) < 1e-5


# ---- the C ABI's workspace sizes and per-call kernel selection (VERDICT r04 weak #9a, #10) -----

def test_workspace_bytes_enforced(ops):
    """Every conv entry point refuses a workspace one byte short of its query (GANAMD_EINVAL, nothing
    launched: the output keeps its sentinel) and runs with exactly the queried size."""
    from gan_amd import _lib
    L = _lib.LIB
    st = _lib.stream()
    for geo in (ops.conv_geo(4, 8, 16, 16, 8, 3, 1, 1), ops.conv_geo(4, 16, 32, 32, 16, 3, 2, 1)):
        d = geo.desc()
        x = torch.randn(geo.Cin, geo.B, geo.H, geo.W, device=DEV)
        gy = torch.randn(geo.Cout, geo.B, geo.OH, geo.OW, device=DEV)
        w = torch.randn(geo.Cout, geo.Cin, geo.K, geo.K, device=DEV)
        calls = {
            _lib.CONV_FWD: lambda out, ws, n: L.ganamd_conv_fwd(d, _lib.ptr(x), _lib.ptr(w), None, None, None, 1.0,
                                                                _lib.ptr(out), ws, n, st),
            _lib.CONV_DGRAD: lambda out, ws, n: L.ganamd_conv_dgrad(d, _lib.ptr(gy), _lib.ptr(w), None, 1.0,
                                                                    _lib.ptr(out), ws, n, st),
            _lib.CONV_WGRAD: lambda out, ws, n: L.ganamd_conv_wgrad(d, _lib.ptr(x), _lib.ptr(gy), None, None, 1.0,
                                                                    _lib.ptr(out), 0, ws, n, st),
        }
        shapes = {_lib.CONV_FWD: gy.shape, _lib.CONV_DGRAD: x.shape, _lib.CONV_WGRAD: w.shape}
        for op, call in calls.items():
            need = geo.ws_bytes(op)
            if need == 0:
                continue
            buf = torch.empty(need // 4 + 1, device=DEV)
            out = torch.full(shapes[op], 7.0, device=DEV)
            assert call(out, buf.data_ptr(), need - 1) == -1, (geo, op)
            torch.cuda.synchronize()
            assert bool((out == 7.0).all()), "a refused call launched"
            assert call(out, buf.data_ptr(), need) == 0, (geo, op)
            torch.cuda.synchronize()
            assert not bool((out == 7.0).any())


def test_kernel_selection_per_call_threads(ops):
    """The kernel choice is part of each call's descriptor (kernel_off), not library state: two host
    threads, each on its own HIP stream, one sending a patch-eligible conv to the split6 LDS-patch
    kernel (kernel_off 0) and the other to the gather GEMM (kernel_off = all off), interleaved, each
    get bit for bit what the same call gives single-threaded -- and the two kernels' results differ
    in the last bits (the selection has teeth)."""
    import threading
    from gan_amd import _lib
    L = _lib.LIB
    geo = ops.conv_geo(32, 96, 64, 64, 96, 5, 1, 2)     # 256 patch blocks: one per CU
    torch.manual_seed(5)
    x = torch.randn(geo.Cin, geo.B, geo.H, geo.W, device=DEV)
    w = torch.randn(geo.Cout, geo.Cin, geo.K, geo.K, device=DEV)
    sx = torch.rand(geo.Cin, geo.B, device=DEV) + 0.5
    sy = torch.rand(geo.Cout, geo.B, device=DEV) + 0.5
    offs = (0, _lib.KERNEL_PATCH_FWD | _lib.KERNEL_PATCH_DGRAD | _lib.KERNEL_WGRAD_ROW)

    def desc(off):
        d = geo.desc()
        return _lib.ConvDesc(*[getattr(d, n) for n, _ in _lib.ConvDesc._fields_[:-1]], off)

    for off, kernel in zip(offs, (1, 0)):          # the plan each descriptor selects
        info = (_lib.c_int * 11)()
        assert L.ganamd_conv_plan_info(desc(off), _lib.CONV_FWD, 1, info) == 0 and info[10] == kernel

    def run(off, out, s):
        d = desc(off)
        n = _lib.c_size_t(0)
        assert L.ganamd_conv_workspace(d, _lib.CONV_FWD, n) == 0
        buf = torch.empty(n.value // 4 + 1, device=DEV)
        rc = L.ganamd_conv_fwd(d, _lib.ptr(x), _lib.ptr(w), None, _lib.ptr(sx), _lib.ptr(sy), 0.1, _lib.ptr(out),
                               buf.data_ptr(), n.value, s.cuda_stream)
        assert rc == 0
        return buf

    single = []
    for off in offs:
        y = torch.empty(geo.Cout, geo.B, geo.OH, geo.OW, device=DEV)
        keep = run(off, y, torch.cuda.current_stream())
        torch.cuda.synchronize()
        single.append(y)
        del keep
    assert not torch.equal(single[0], single[1])
    assert rel(single[0], single[1]) < 1e-6
    outs = [[torch.empty_like(single[0]) for _ in range(6)] for _ in offs]
    errs = []

    def worker(k):
        try:
            s = torch.cuda.Stream()
            keep = []
            with torch.cuda.stream(s):
                for y in outs[k]:
                    keep.append(run(offs[k], y, s))
            s.synchronize()
        except Exception as e:          # noqa: BLE001 (reported below)
            errs.append(e)
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    torch.cuda.synchronize()
    for k in range(2):
        for y in outs[k]:
            assert torch.equal(y, single[k]), k


SMALL_CASES = [
    # B, Cin, H, Cout, k, pad mode, scaled: the direct conv of Cout <= 4 forwards (conv_small.hip)
    (4, 108, 64, 3, 5, 1, False),    # ToRGB at 64x64 (pad mode 1: replicate)
    (4, 108, 64, 3, 5, 1, True),     # modulated-style scales
    (3, 20, 64, 4, 3, 0, False),     # zero padding, 3x3, four outputs, a channel tail
    (2, 9, 64, 1, 1, 0, True),       # 1x1, one output, a channel tail
]


@pytest.mark.parametrize("case", SMALL_CASES)
def test_small_cout_conv(ops, case):
    """The direct vector-ALU conv (Cout <= 4: ToRGB, generator_13_5.py:470-493) against float64:
    plan_info reports it (kernel 2), it needs no workspace, and its error is at most that of a
    sequential fp32 FMA convolution (it IS one: channel, kernel row, kernel column order) or 1e-6."""
    from gan_amd import _lib
    from tests._emu import emulate, max_rel, seq_fp32
    B, cin, H, cout, k, mode, scaled = case
    g = ops.conv_geo(B, cin, H, H, cout, k, 1, (k - 1) // 2, mode)
    info = ops.plan_info(g, 0, scaled)
    assert info["kernel"] == 2 and g.ws_bytes(_lib.CONV_FWD) == 0, info
    assert ops.plan_info(ops.conv_geo(B, cin, 32, 32, cout, k, 1, (k - 1) // 2, mode), 0, scaled)["kernel"] != 2
    gen = torch.Generator().manual_seed(700 + SMALL_CASES.index(case))
    x = torch.randn(cin, B, H, H, generator=gen).to(DEV)
    w = torch.nn.Parameter(torch.randn(cout, cin, k, k, generator=gen).to(DEV))
    bias = torch.randn(cout, generator=gen).to(DEV)
    xs = (torch.rand(cin, B, generator=gen) + 0.5).to(DEV) if scaled else None
    ys = (torch.rand(cout, B, generator=gen) + 0.5).to(DEV) if scaled else None
    with torch.no_grad():
        got = ops._conv_fwd(g, x, w, bias, xs, ys, 0.7)
    torch.cuda.synchronize()
    ref = emulate("fwd", g, x=x, w=w, xs=xs, ys=ys, alpha=0.7, bias=bias)
    e = max_rel(got, ref)
    eseq = max_rel(seq_fp32("fwd", g, x=x, w=w, xs=xs, ys=ys, alpha=0.7) + bias[:, None, None, None], ref)
    print(f"{case}: max rel err vs float64 {e:.2e} (sequential fp32 FMA {eseq:.2e})")
    assert e <= max(1e-6, 2 * eseq), (e, eseq)
    with torch.no_grad(), ops.patch_conv(7):        # the same conv on the gather GEMM (bit 3 off)
        other = ops._conv_fwd(g, x, w, bias, xs, ys, 0.7)
    assert ops.plan_info(g, 0, scaled)["kernel"] == 2
    assert max_rel(other, ref) < 1e-5
