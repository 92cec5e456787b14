"""A/B timing of the iteration's dominant GEMM shapes across library builds.

    python tools/ab_shapes.py LIB1.so[:VAR=V,VAR2=V] [LIB2.so ...]   (each in its own child process,
                                                                     with those environment variables)

Shapes: the largest GEMMs of one WGAN-GP iteration at B=64 (profiles/*census*): generator
modulated convs (scaled), critic block convs on the 2B = 128 real+fake batch, their dgrad / wgrad,
the strided scatter dgrad and the 4x4 1025-channel block.  Prints us and TF/s per shape and the
count-weighted total."""
import os
import subprocess
import sys

import os as _os
SHAPES_WGRAD = [
    ("wgrad", 64, 96, 64, 96, 5, 1, 2, True, 10),
    ("wgrad", 64, 48, 64, 48, 5, 1, 2, True, 20),
    ("wgrad", 64, 48, 64, 48, 3, 1, 1, True, 30),
    ("wgrad", 64, 192, 16, 192, 5, 1, 2, True, 10),
    ("wgrad", 128, 3, 64, 64, 3, 1, 1, False, 5),
    ("wgrad", 64, 96, 32, 96, 3, 1, 1, True, 30),
    ("wgrad", 64, 1025, 4, 1025, 3, 1, 1, False, 60),
    ("wgrad", 128, 1025, 4, 1025, 3, 1, 1, False, 30),
    ("fwd", 64, 108, 64, 3, 5, 1, 2, False, 12),
    ("dgrad", 64, 48, 64, 48, 5, 1, 2, True, 20),
    ("wgrad", 128, 64, 64, 64, 3, 1, 1, False, 25),
    ("wgrad", 64, 64, 64, 64, 3, 1, 1, False, 50),
    ("wgrad", 128, 128, 32, 128, 3, 1, 1, False, 25),
    ("wgrad", 64, 128, 32, 128, 3, 1, 1, False, 50),
    ("wgrad", 64, 96, 64, 96, 3, 1, 1, True, 10),
    ("wgrad", 64, 96, 64, 48, 3, 1, 1, True, 20),
]
SHAPES_DG = [   # fwd vs dgrad vs wgrad of the same critic convs (AB_SET=dg)
    ("fwd", 128, 64, 64, 64, 3, 1, 1, False, 25),
    ("dgrad", 128, 64, 64, 64, 3, 1, 1, False, 25),
    ("wgrad", 128, 64, 64, 64, 3, 1, 1, False, 25),
    ("fwd", 128, 128, 32, 128, 3, 1, 1, False, 25),
    ("dgrad", 128, 128, 32, 128, 3, 1, 1, False, 25),
    ("fwd", 64, 256, 16, 256, 3, 1, 1, False, 55),
    ("dgrad", 64, 256, 16, 256, 3, 1, 1, False, 55),
]
SHAPES_WIDE = [    # unscaled critic GEMMs across the batches the step runs them at (AB_SET=wide)
    *[(op, b, c, h, c, 3, 1, 1, False, 1) for op in ("fwd", "dgrad")
      for c, h in ((64, 64), (128, 32), (256, 16), (512, 8)) for b in (32, 64, 96, 128)],
]
SHAPES_PATCH = [   # the LDS-patch conv's instances (AB_SET=patch)
    ("fwd", 64, 96, 64, 96, 5, 1, 2, True, 30),
    ("fwd", 256, 96, 64, 96, 5, 1, 2, True, 10),
    ("fwd", 256, 96, 64, 96, 3, 1, 1, True, 24),
    ("fwd", 256, 48, 64, 48, 5, 1, 2, True, 20),
    ("fwd", 256, 48, 64, 48, 3, 1, 1, True, 36),
    ("fwd", 256, 96, 32, 96, 5, 1, 2, True, 10),
    ("fwd", 256, 96, 32, 96, 3, 1, 1, True, 24),
    ("fwd", 128, 64, 64, 64, 3, 1, 1, False, 25),
    ("dgrad", 64, 96, 64, 96, 5, 1, 2, False, 10),
    ("dgrad", 128, 64, 64, 64, 3, 1, 1, False, 25),
]
SHAPES_P32 = [   # the patch conv at W = 32 on the fake batches' 256-sample grid (AB_SET=p32)
    ("fwd", 256, 96, 32, 96, 5, 1, 2, True, 10),
    ("fwd", 256, 96, 32, 96, 3, 1, 1, True, 10),
    ("fwd", 256, 48, 32, 48, 5, 1, 2, True, 20),
    ("fwd", 256, 48, 32, 48, 3, 1, 1, True, 30),
    ("fwd", 256, 48, 32, 54, 3, 1, 1, True, 10),
    ("fwd", 64, 96, 32, 96, 5, 1, 2, True, 20),
]
SHAPES = [  # (op, B, cin, H, cout, k, stride, pad, scaled, weight = launches per iteration)
    ("fwd", 64, 96, 64, 96, 5, 1, 2, True, 60),
    ("fwd", 64, 48, 64, 48, 5, 1, 2, True, 120),
    ("fwd", 64, 48, 64, 48, 3, 1, 1, True, 180),
    ("fwd", 128, 128, 32, 128, 3, 1, 1, False, 25),
    ("fwd", 64, 192, 16, 192, 5, 1, 2, True, 60),
    ("wgrad", 128, 128, 32, 128, 3, 1, 1, False, 25),
    ("wgrad", 64, 96, 64, 96, 5, 1, 2, True, 10),
    ("wgrad", 64, 1025, 4, 1025, 3, 1, 1, False, 90),
    ("wgrad", 128, 64, 64, 64, 3, 1, 1, False, 25),
    ("dgrad", 128, 64, 64, 64, 3, 1, 1, False, 25),
    ("dgrad", 64, 96, 64, 96, 5, 1, 2, True, 10),
    ("dgrad", 64, 1024, 8, 1024, 3, 2, 1, False, 11),
    ("dgrad", 64, 1025, 4, 1025, 3, 1, 1, False, 66),
]


def accuracy():
    """AB_ACC=1: every shape's op at B = 2 against float64 on the host (torch autograd of the
    replicate-padded conv): max |err| / max |ref| per shape."""
    import torch
    import torch.nn.functional as F
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gan_amd import ops
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(0)
    worst = 0.0
    for op, B, cin, H, cout, k, s, p, scaled, n in {"patch": SHAPES_PATCH, "p32": SHAPES_P32}.get(_os.environ.get("AB_SET"), SHAPES):
        B = 2
        g = ops.conv_geo(B, cin, H, H, cout, k, s, p)
        x = torch.randn(B, cin, H, H, generator=gen, dtype=torch.float64, requires_grad=True)
        w = torch.randn(cout, cin, k, k, generator=gen, dtype=torch.float64, requires_grad=True)
        sx = torch.rand(cin, B, generator=gen, dtype=torch.float64) + 0.5 if scaled else None
        sy = torch.rand(cout, B, generator=gen, dtype=torch.float64) + 0.5 if scaled else None
        xm = x * sx.t()[:, :, None, None] if scaled else x
        y = F.conv2d(F.pad(xm, (p, p, p, p), mode="replicate"), w, stride=s)
        if scaled:
            y = y * sy.t()[:, :, None, None]
        gy = torch.randn(y.shape, generator=gen, dtype=torch.float64)
        gx, gw = torch.autograd.grad(y, (x, w), gy)
        cn = (lambda t: t.permute(1, 0, 2, 3).contiguous().float().to(dev))
        f = (lambda t: None if t is None else t.float().to(dev))
        with torch.no_grad():
            if op == "fwd":
                got, ref = ops._conv_fwd(g, cn(x.detach()), torch.nn.Parameter(f(w.detach())), None, f(sx), f(sy), 1.0), y
                ref = ref.permute(1, 0, 2, 3)
            elif op == "dgrad":
                if scaled:
                    continue
                got, ref = ops._conv_dgrad(g, cn(gy), torch.nn.Parameter(f(w.detach())), None, 1.0), gx.permute(1, 0, 2, 3)
            else:
                if scaled:
                    continue
                got, ref = ops._conv_wgrad(g, cn(x.detach()), cn(gy), None, None, 1.0), gw
        err = float((got.double().cpu() - ref.detach()).abs().max() / ref.detach().abs().max())
        worst = max(worst, err)
        print(f"  {op:5s} {cin:5d}->{cout:5d} {H:3d}^2 k{k} s{s} {'S' if scaled else ' '}  rel err {err:.2e}", flush=True)
    print(f"  worst rel err {worst:.2e}", flush=True)


def child():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gan_amd import ops
    dev = torch.device("cuda")
    tot_t = tot_f = 0.0
    for op, B, cin, H, cout, k, s, p, scaled, n in {"wgrad": SHAPES_WGRAD, "dg": SHAPES_DG, "patch": SHAPES_PATCH, "wide": SHAPES_WIDE, "p32": SHAPES_P32}.get(_os.environ.get("AB_SET"), SHAPES):
        g = ops.conv_geo(B, cin, H, H, cout, k, s, p)
        x = torch.randn(g.Cin, g.B, g.H, g.W, device=dev)
        y = torch.randn(g.Cout, g.B, g.OH, g.OW, device=dev)
        w = torch.nn.Parameter(torch.randn(g.Cout, g.Cin, g.K, g.K, device=dev))
        sx = torch.rand(g.Cin, g.B, device=dev) if scaled else None
        sy = torch.rand(g.Cout, g.B, device=dev) if scaled else None
        f = {"fwd": lambda: ops._conv_fwd(g, x, w, None, sx, sy, 1.0),
             "dgrad": lambda: ops._conv_dgrad(g, y, w, sy, 1.0),
             "wgrad": lambda: ops._conv_wgrad(g, x, y, sx, sy, 1.0)}[op]
        with torch.no_grad():
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                f()
            e1.record()
            torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / reps
        flop = 2.0 * B * g.OH * g.OW * cin * cout * k * k
        tot_t += n * t
        tot_f += n * flop
        print(f"  {op:5s} B{B:4d} {cin:5d}->{cout:5d} {H:3d}^2 k{k} s{s} {'S' if scaled else ' '}  {t * 1e6:9.1f} us "
              f"{flop / t / 1e12:7.1f} TF/s", flush=True)
    print(f"  weighted: {tot_t * 1e3:.1f} ms  {tot_f / tot_t / 1e12:.1f} TF/s", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        (accuracy if _os.environ.get("AB_ACC") else child)()
        sys.exit(0)
    rc = 0
    for arg in sys.argv[1:]:
        so, _, kv = arg.partition(":")
        print(f"[{os.path.basename(so)} {kv}]", flush=True)
        env = dict(os.environ, GANAMD_SO=os.path.abspath(so))
        env.update(dict(x.split("=", 1) for x in kv.split(",") if x))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env, timeout=300)
        rc = rc or r.returncode
        if r.returncode != 0:
            break
    sys.exit(rc)
