"""Census of the implicit-GEMM launches of one WGAN-GP iteration and their isolated speed.

    python tools/conv_census.py [--batch 64] [--top 40]

Records every conv/convT/linear GEMM (op, geometry) issued by one eager iteration, then times
each distinct launch in isolation (HIP events, median of 5) and prints the table sorted by
estimated total time per iteration = count x time.  Used to pick kernel work.
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import gan_amd
    from gan_amd import ops
    dev = torch.device("cuda")
    torch.manual_seed(0)
    G = gan_amd.Generator(256).to(dev)
    D = gan_amd.Discriminator().to(dev)
    tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4")
    B = a.batch
    rec = []
    ops.FlopCounter.record = rec
    for _ in range(5):
        tr.discriminator_trainstep(torch.randn(B, 3, 64, 64, device=dev), B)
    tr.generator_trainstep(B)
    ops.FlopCounter.record = None
    torch.cuda.synchronize()
    del tr, G, D
    torch.cuda.empty_cache()
    cnt = collections.Counter(rec)
    rows = []
    for (op, g, xs, ys, _math), n in cnt.items():
        xin = torch.randn(g.Cin, g.B, g.H, g.W, device=dev)
        yout = torch.randn(g.Cout, g.B, g.OH, g.OW, device=dev)
        wshape = (g.Cin, g.Cout, g.K, g.K) if g.transposed else (g.Cout, g.Cin, g.K, g.K)
        w = torch.randn(wshape, device=dev)
        sx = torch.rand(g.Cin, g.B, device=dev) if xs else None
        sy = torch.rand(g.Cout, g.B, device=dev) if ys else None
        if op == "fwd":
            f = lambda: ops._conv_fwd(g, xin, w, None, sx, sy, 1.0)
        elif op == "dgrad":  # the recorded flag is the gy (Cout-side) scale
            sgy = torch.rand(g.Cout, g.B, device=dev) if xs else None
            f = lambda: ops._conv_dgrad(g, yout, w, sgy, 1.0)
        else:
            f = lambda: ops._conv_wgrad(g, xin, yout, sx, sy, 1.0)
        f()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 1e3)
        t = sorted(ts)[2]
        sp = (g.H * g.W) if g.transposed else (g.OH * g.OW)
        flop = 2 * g.B * sp * g.Cin * g.Cout * g.K * g.K
        rows.append((n * t, n, t, flop / t / 1e12, op, g))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    totf = sum(r[1] * 2 * r[5].B * ((r[5].H * r[5].W) if r[5].transposed else (r[5].OH * r[5].OW)) * r[5].Cin *
               r[5].Cout * r[5].K ** 2 for r in rows)
    print(f"distinct launches {len(rows)}  total launches {sum(r[1] for r in rows)}  est GEMM time/iter {tot:.3f}s  "
          f"GEMM TFLOP/iter {totf / 1e12:.1f}  mean {totf / tot / 1e12:.1f} TF/s")
    print(f"{'share':>6} {'n':>5} {'us':>9} {'TF/s':>6}  op     B  Cin  H  Cout OH k s p T")
    for r in rows[:a.top]:
        g = r[5]
        print(f"{100 * r[0] / tot:6.2f} {r[1]:5d} {1e6 * r[2]:9.1f} {r[3]:6.1f}  {r[4]:5s} {g.B:3d} {g.Cin:4d} {g.H:3d} "
              f"{g.Cout:4d} {g.OH:3d} {g.K} {g.stride} {g.pad} {int(g.transposed)}")


if __name__ == "__main__":
    main()
