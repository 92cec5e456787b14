"""Time ganamd_resample2d per (kind, map size, direction) at the hot path's plane counts.

    python tools/resample_micro.py [--planes 6144] [--reps 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--planes", type=int, default=96 * 64)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from gan_amd import ops, tables
    dev = torch.device("cuda")
    for kind, n in (("pool5", 64), ("pool5", 32), ("smooth", 64), ("smooth", 32), ("up2_smooth", 32),
                    ("smooth_down2", 64), ("smooth_down2", 32)):
        t = tables.table(kind, n, dev)
        for adj in (False, True):
            n_in, n_out, tab = (t.n_out, t.n_in, t.adj) if adj else (t.n_in, t.n_out, t.fwd)
            x = torch.randn(a.planes, 1, n_in, n_in, device=dev)
            f = lambda: ops._resample(x, n_in, n_out, tab)
            f()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(a.reps):
                    f()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            mb = 4 * a.planes * (n_in * n_in + n_out * n_out) / 1e6
            print(f"{kind:13s} {'adj' if adj else 'fwd'} {n_in:3d}->{n_out:3d} planes {a.planes}: {us:8.1f} us "
                  f"{mb:7.1f} MB  {mb / us:5.2f} TB/s")


if __name__ == "__main__":
    main()
