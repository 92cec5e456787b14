"""Scatter-form dgrad (GEMM over output pixels + dgrad_fold_kernel) on the small-map / strided shapes
the critic and generator send there, for A/B of the fold kernel under rocprofv3 --kernel-trace --stats.

  GANAMD_SO=lib.so python3 tools/fold_micro.py OUT.pt [reps]

Writes every shape's input gradient to OUT.pt (compare two builds bit for bit with --compare A B).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (B, Cin, H, Cout, k, stride, pad): the critic's 4x4 / 8x8 blocks at B = 128 (real + fake), its
# strided DownSample-side convs, the generator's 4x4 / 8x8 StyleBlock convs and SK 5x5 maps at B = 64
SHAPES = [
    (128, 1025, 4, 1025, 3, 1, 1),
    (128, 512, 8, 512, 3, 1, 1),
    (128, 512, 8, 512, 3, 2, 1),
    (64, 396, 4, 396, 3, 1, 1),
    (64, 192, 8, 192, 3, 1, 1),
    (256, 96, 5, 96, 3, 1, 1),
]


def main():
    if sys.argv[1] == "--compare":
        a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
        bad = [k for k in a if not torch.equal(a[k], b[k])]
        print("fold A/B bit-identical" if not bad else f"fold A/B DIFFER: {bad}")
        sys.exit(1 if bad else 0)
    import gan_amd.ops as ops
    out, reps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    res = {}
    for (B, cin, H, cout, k, s, p) in SHAPES:
        g = ops.conv_geo(B, cin, H, H, cout, k, s, p)
        gen = torch.Generator().manual_seed(B + cin + H + s)
        w = torch.randn(cout, cin, k, k, generator=gen).to(dev)
        gy = torch.randn(cout, B, g.OH, g.OW, generator=gen).to(dev)
        with torch.no_grad():
            for _ in range(reps):
                gx = ops._conv_dgrad(g, gy, w, None, 0.7)
        torch.cuda.synchronize()
        res[f"{B}x{cin}x{H}s{s}"] = gx.cpu()
    torch.save(res, out)
    print("fold micro done", out)


if __name__ == "__main__":
    main()
