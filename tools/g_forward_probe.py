"""G13_5 forward (no_grad, B=64) in isolation: issued GEMM FLOPs, launches, graph-replay time,
and a kernel-family breakdown when run under rocprofv3 (tools/trace_summary.py)."""
import sys

import torch

sys.path.insert(0, ".")
import gan_amd  # noqa: E402
from gan_amd import ops  # noqa: E402
from gan_amd.optim import FlatParams  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda")
torch.manual_seed(0)
G = gan_amd.Generator(256).to(dev)
FlatParams(G)
z = torch.randn(B, 256, 1, 1, device=dev)


def fwd():
    with torch.no_grad():
        return G(z)


ops.FlopCounter.enabled = True
fwd()
ops.FlopCounter.enabled = False
torch.cuda.synchronize()
print(f"G forward B={B}: GEMM {ops.FlopCounter.flops / 1e12:.2f} TFLOP in {ops.FlopCounter.launches} launches")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    fwd()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    fwd()
g.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    g.replay()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(f"graph replay {ms:.1f} ms  -> GEMM-equivalent {ops.FlopCounter.flops / ms / 1e9:.1f} TF/s")

if len(sys.argv) > 2 and sys.argv[2] == "census":
    import collections
    rec = []
    ops.FlopCounter.record = rec
    fwd()
    ops.FlopCounter.record = None
    cnt = collections.Counter(rec)
    rows = []
    for (op, geo, xs, ys, _math), n in cnt.items():
        xin = torch.randn(geo.Cin, geo.B, geo.H, geo.W, device=dev)
        w = torch.randn((geo.Cin, geo.Cout, geo.K, geo.K) if geo.transposed else (geo.Cout, geo.Cin, geo.K, geo.K),
                        device=dev)
        sx = torch.rand(geo.Cin, geo.B, device=dev) if xs else None
        sy = torch.rand(geo.Cout, geo.B, device=dev) if ys else None
        f = lambda: ops._conv_fwd(geo, xin, w, None, sx, sy, 1.0)
        f()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(3):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 3 * 1e3
        fl = 2 * geo.B * geo.OH * geo.OW * geo.Cout * geo.Cin * geo.K * geo.K if not geo.transposed else \
            2 * geo.B * geo.H * geo.W * geo.Cout * geo.Cin * geo.K * geo.K
        rows.append((n * us, n, us, fl / us / 1e6, geo, xs))
    rows.sort(key=lambda r: -r[0])
    for t, n, us, tf, geo, xs in rows[:40]:
        print(f"{t / 1e3:8.2f}ms n={n:4d} {us:8.1f}us {tf:6.1f}TF/s Cin={geo.Cin} Cout={geo.Cout} H={geo.H} OH={geo.OH} "
              f"k={geo.K} s={geo.stride} T={int(geo.transposed)} mod={int(xs)}")
