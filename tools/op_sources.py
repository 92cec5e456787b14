"""Where the torch elementwise launches of one eager step come from: torch.profiler (CPU-side op
records with Python stacks), aggregated by (op, innermost gan_amd frame)."""
import collections
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
import gan_amd  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "generator"
B = 64
dev = torch.device("cuda")
torch.manual_seed(0)
G = gan_amd.Generator(256).to(dev)
D = gan_amd.Discriminator().to(dev)
tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.DeviceRNG(dev))
fn = (lambda: tr.discriminator_trainstep(torch.randn(B, 3, 64, 64, device=dev), B)) if which == "critic" else \
    (lambda: tr.generator_trainstep(B))
fn()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
    fn()
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    if not ev.name.startswith("aten::") or ev.name in ("aten::empty", "aten::empty_strided", "aten::view",
                                                        "aten::as_strided", "aten::reshape", "aten::t",
                                                        "aten::transpose", "aten::permute", "aten::slice",
                                                        "aten::select", "aten::detach", "aten::alias",
                                                        "aten::unbind", "aten::split", "aten::expand",
                                                        "aten::unsqueeze", "aten::squeeze", "aten::_reshape_alias",
                                                        "aten::result_type", "aten::is_nonzero", "aten::item",
                                                        "aten::_local_scalar_dense", "aten::lift_fresh",
                                                        "aten::contiguous", "aten::resolve_conj", "aten::resolve_neg"):
        continue
    frame = "?"
    for f in (ev.stack or []):
        if "gan_amd" in f or "-gan-_amd" in f:
            frame = f.split("/")[-1]
            break
    cnt[(ev.name, frame)] += 1
for (name, frame), n in cnt.most_common(45):
    print(f"{n:6d}  {name:32s} {frame}")
