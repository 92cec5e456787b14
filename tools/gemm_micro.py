"""Time one conv GEMM launch repeatedly (for A/B experiments and rocprofv3 counter runs).

    python tools/gemm_micro.py --op wgrad --B 64 --cin 128 --H 32 --cout 128 --k 3 --pad 1 [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="wgrad")
    for k, v in (("B", 64), ("cin", 128), ("H", 32), ("cout", 128), ("k", 3), ("stride", 1), ("pad", 1),
                 ("reps", 20)):
        ap.add_argument(f"--{k}", type=int, default=v)
    ap.add_argument("--scaled", action="store_true")
    ap.add_argument("--transposed", action="store_true")
    a = ap.parse_args()
    from gan_amd import ops
    dev = torch.device("cuda")
    if a.transposed:
        g = ops.convT_geo(a.B, a.cin, a.H, a.H, a.cout, a.k, a.stride, a.pad)
    else:
        g = ops.conv_geo(a.B, a.cin, a.H, a.H, a.cout, a.k, a.stride, a.pad)
    x = torch.randn(g.Cin, g.B, g.H, g.W, device=dev)
    y = torch.randn(g.Cout, g.B, g.OH, g.OW, device=dev)
    w = torch.randn((g.Cin, g.Cout, g.K, g.K) if g.transposed else (g.Cout, g.Cin, g.K, g.K), device=dev)
    sx = torch.rand(g.Cin, g.B, device=dev) if a.scaled else None
    sy = torch.rand(g.Cout, g.B, device=dev) if a.scaled else None
    f = {"fwd": lambda: ops._conv_fwd(g, x, w, None, sx, sy, 1.0),
         "dgrad": lambda: ops._conv_dgrad(g, y, w, sy, 1.0),
         "wgrad": lambda: ops._conv_wgrad(g, x, y, sx, sy, 1.0)}[a.op]
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / a.reps
    sp = g.H * g.W if g.transposed else g.OH * g.OW
    flop = 2 * g.B * sp * g.Cin * g.Cout * g.K * g.K
    print(f"{a.op} {g}: {t * 1e6:.1f} us  {flop / t / 1e12:.1f} TF/s  lib={os.path.basename(os.environ.get('GANAMD_SO', 'in-tree'))}")


if __name__ == "__main__":
    main()
