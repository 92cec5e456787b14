"""Time a fixed set of representative conv GEMMs (HIP events, packed weights cached) under the
current GANAMD_CONV_TILE / GANAMD_* knobs.  One process per knob setting (knobs are read once):

    for t in 0 128x128 128x256 256x128; do GANAMD_CONV_TILE=$t python tools/tile_sweep.py; done
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (op, B, cin, H, cout, k, stride, pad, scaled) -- the largest shares of the census
SHAPES = [
    ("fwd", 64, 96, 64, 96, 5, 1, 2, True),
    ("fwd", 64, 48, 64, 48, 5, 1, 2, True),
    ("fwd", 128, 128, 32, 128, 3, 1, 1, False),
    ("fwd", 128, 64, 64, 64, 3, 1, 1, False),
    ("fwd", 64, 1025, 4, 1025, 3, 1, 1, False),
    ("fwd", 64, 192, 16, 192, 5, 1, 2, True),
    ("fwd", 64, 384, 8, 384, 5, 1, 2, True),
    ("fwd", 128, 512, 8, 512, 3, 1, 1, False),
    ("dgrad", 128, 128, 32, 128, 3, 1, 1, False),
    ("dgrad", 64, 96, 64, 96, 5, 1, 2, True),
    ("fwd", 64, 1024, 16, 1024, 1, 1, 0, False),
]


def main(reps=10):
    from gan_amd import ops
    dev = torch.device("cuda")
    tot_t = tot_f = 0.0
    for op, B, cin, H, cout, k, s, p, scaled in SHAPES:
        g = ops.conv_geo(B, cin, H, H, cout, k, s, p)
        x = torch.randn(g.Cin, g.B, g.H, g.W, device=dev)
        y = torch.randn(g.Cout, g.B, g.OH, g.OW, device=dev)
        w = torch.nn.Parameter(torch.randn(g.Cout, g.Cin, g.K, g.K, device=dev))
        sx = torch.rand(g.Cin, g.B, device=dev) if scaled else None
        sy = torch.rand(g.Cout, g.B, device=dev) if scaled else None
        with torch.no_grad():
            f = {"fwd": lambda: ops._conv_fwd(g, x, w, None, sx, sy, 1.0),
                 "dgrad": lambda: ops._conv_dgrad(g, y, w, sy, 1.0)}[op]
            for _ in range(2):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                f()
            e1.record()
            torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / reps
        flop = 2 * g.B * g.OH * g.OW * g.Cin * g.Cout * g.K * g.K
        tot_t += t
        tot_f += flop
        print(f"  {op:5s} B{B:4d} {cin:5d}->{cout:5d} {H:3d}^2 k{k} s{s} {'mod' if scaled else '   '}: "
              f"{t * 1e6:8.1f} us {flop / t / 1e12:6.1f} TF/s", flush=True)
    print(f"tile={os.environ.get('GANAMD_CONV_TILE', '0')} total {tot_t * 1e3:.2f} ms  {tot_f / tot_t / 1e12:.1f} TF/s",
          flush=True)


if __name__ == "__main__":
    main()
