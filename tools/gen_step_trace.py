"""One generator step (train/wgangp.py:20-27 at the bench's batch) in isolation, for a rocprofv3
kernel trace of just that phase:
    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/gen_step_trace.py
    python3 tools/trace_summary.py DIR/.../run_kernel_trace.csv --last <printed seconds>
Warm-up: two eager generator steps; then, after a pause, the traced step (eager: the same kernels
the captured gen graph replays).  PHASE=critic traces one critic step (fake batch made before)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import gan_amd  # noqa: E402

B = int(os.environ.get("BATCH", "64"))
phase = os.environ.get("PHASE", "gen")
dev = torch.device("cuda", 0)
torch.manual_seed(1234)
G = gan_amd.Generator(256).to(dev)
D = gan_amd.Discriminator().to(dev)
tr = gan_amd.Train([], dev, 1, 256, G, "g", D, "d", rng=gan_amd.DeviceRNG(dev, 4321))
real = tr.rng.fork(2)


def step():
    if phase == "gen":
        tr.generator_backward(B)
        tr.optimizer_G.step()
    else:
        fake = tr.generate_fake(B)
        tr.discriminator_backward(real.randn((B, 3, 64, 64)), B, gen_imgs=fake)
        tr.optimizer_D.step()


for _ in range(2):
    step()
torch.cuda.synchronize()
time.sleep(0.5)
t0 = time.perf_counter()
step()
torch.cuda.synchronize()
print(f"[trace] {phase} step {time.perf_counter() - t0:.4f} s", flush=True)
