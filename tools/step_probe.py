"""One training step in isolation as a HIP graph (B=64): 'critic' = a critic step on a ready fake
batch, 'critic_fake' = discriminator_trainstep (its own fake batch), 'generator' =
generator_trainstep, 'fake' / 'fake4' = one / four fake batches (segmented BatchNorm).  Prints the replay time; run under rocprofv3 and summarise the
last replay with tools/trace_summary.py --last."""
import sys

import torch

sys.path.insert(0, ".")
import gan_amd  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "critic"
B = 64
dev = torch.device("cuda")
torch.manual_seed(0)
G = gan_amd.Generator(256).to(dev)
D = gan_amd.Discriminator().to(dev)
tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.DeviceRNG(dev))
fake = tr.generate_fake(B)
real = torch.randn(B, 3, 64, 64, device=dev)


def critic():   # a critic step on a ready fake batch (the bench schedule), optimizer step included
    out = tr.discriminator_backward(real, B, gen_imgs=fake)
    tr.optimizer_D.step()
    return out


fn = {"critic": critic,
      "critic_fake": lambda: tr.discriminator_trainstep(real, B),
      "generator": lambda: tr.generator_trainstep(B),
      "fake": lambda: tr.generate_fake(B),
      "fake4": lambda: tr.generate_fakes(4, B)}[which]
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
