"""One training step in isolation as a HIP graph (B=64): 'critic' = discriminator_trainstep,
'generator' = generator_trainstep.  Prints the replay time; run under rocprofv3 and summarise the
last replay with tools/trace_summary.py --last."""
import sys

import torch

sys.path.insert(0, ".")
import gan_amd  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "critic"   # critic | generator | fake
B = 64
dev = torch.device("cuda")
torch.manual_seed(0)
G = gan_amd.Generator(256).to(dev)
D = gan_amd.Discriminator().to(dev)
tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.DeviceRNG(dev))
fn = {"critic": lambda: tr.discriminator_trainstep(torch.randn(B, 3, 64, 64, device=dev), B),
      "generator": lambda: tr.generator_trainstep(B),
      "fake": lambda: tr.generate_fake(B)}[which]
fn()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    fn()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    fn()
g.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    g.replay()
e1.record()
torch.cuda.synchronize()
print(f"{which} step graph replay {e0.elapsed_time(e1) / 3:.1f} ms")
