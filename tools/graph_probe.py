"""Capture the hot-path pieces into HIP graphs one at a time (B=8) and replay them; prints the
stage reached.  Run with python -X faulthandler to get a Python stack on a crash."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def capture(name, fn):
    print(f"[probe] {name}: warm-up", flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    print(f"[probe] {name}: capture", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    print(f"[probe] {name}: replay", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"[probe] {name}: ok", flush=True)
    return g


def main():
    import gan_amd
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = 8
    D = gan_amd.Discriminator().to(dev)
    x = torch.randn(B, 3, 64, 64, device=dev)
    stage = sys.argv[1] if len(sys.argv) > 1 else "all"

    def d_fwd():
        with torch.no_grad():
            D(x)

    def d_fwd_bwd():
        D(x).mean().backward()

    def d_gp():
        xi = x.detach().requires_grad_()
        g, = torch.autograd.grad(D(xi).sum(), xi, create_graph=True)
        (g.pow(2).flatten(1).sum(1).sqrt() - 1).pow(2).mean().backward()

    for name, fn in (("d_fwd", d_fwd), ("d_fwd_bwd", d_fwd_bwd), ("d_gp", d_gp)):
        capture(name, fn)
        if stage == name:
            return
    G = gan_amd.Generator(256).to(dev)
    tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4")

    def g_fwd():
        with torch.no_grad():
            G(torch.randn(B, 256, 1, 1, device=dev))

    capture("g_fwd", g_fwd)
    capture("d_step", lambda: tr.discriminator_trainstep(torch.randn(B, 3, 64, 64, device=dev), B))
    capture("g_step", lambda: tr.generator_trainstep(B))
    print("[probe] all ok", flush=True)


if __name__ == "__main__":
    main()
