"""Timing probe: one no-grad G13_5 forward at 5*B versus five at B (graph replays, HIP events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import gan_amd
    dev = torch.device("cuda")
    torch.manual_seed(0)
    G = gan_amd.Generator(256).to(dev)
    D = gan_amd.Discriminator().to(dev)
    tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.DeviceRNG(dev, 1))
    for B in [int(b) for b in (sys.argv[1:] or [64, 128])]:
        out = {}
        fn = lambda: out.__setitem__("x", tr.generate_fake(B))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        for _ in range(3):
            g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 10
        print(f"B={B}: {t:.2f} ms per forward, {t / B * 64:.2f} ms per 64 images", flush=True)
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
