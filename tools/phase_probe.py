"""Run one iteration of a bench config eagerly, phase by phase, with a device sync and a line of
output after each phase (localises a failing phase; run under AMD_SERIALIZE_KERNEL=3 to pin the
kernel).   usage: python tools/phase_probe.py --config lazy --batch 128
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

args = bench.parse()
if args.batch is None:
    args.batch = bench.CONFIGS[args.config][1]
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
G, D, tr, phases = bench.build(args, dev, 0)
print(f"[probe] built {args.config} B={args.batch}; {len(phases)} phases", flush=True)
for i, (key, bwd, opt, _) in enumerate(phases):
    t0 = time.perf_counter()
    bwd()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    opt.step()
    torch.cuda.synchronize()
    print(f"[probe] phase {i} {key}: backward {t1 - t0:.2f}s step {time.perf_counter() - t1:.2f}s "
          f"peak {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB", flush=True)
print("[probe] ok", flush=True)
