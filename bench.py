"""WGAN-GP throughput benchmark: G13_5 + D9_4, 64x64x3, n_critic = 5, fp32, on 1..8 MI355X.

One timed "step" is one WGAN-GP iteration = 5 critic steps (each: no-grad G forward, critic on a
fresh real batch and on the fake batch, gradient penalty with its double backward, AdamW) + 1
generator step (G forward, critic forward/backward into G, AdamW), exactly train/wgangp.py:20-71
with the iteration structure of the metric in BASELINE.json.  Per GPU the batch is 64 (config 2);
with N ranks (torchrun) every rank runs its own 64-image shard and the gradients of each optimizer
step are all-reduced over RCCL (config 3 at N = 8: 512 images).

value = images per second over all ranks = 64 * N * steps / max-over-ranks(timed seconds).
The real batches are synthetic N(0,1) [64,3,64,64] tensors drawn on the device inside the step
(the reference's ImageNet-normalised data has that scale); weights are the reference's init
distributions (random, seeded).

Also reported (rank 0):
  roofline      algorithmic conv FLOPs per iteration (1,559.5 GFLOP per image)
                over the measured iteration time, against the fp32 MFMA peak (157.3 TFLOP/s);
                plus the conv-GEMM FLOPs this build actually issues per iteration.
  cpu_baseline  the CPU oracle (oracle/model.py, fp32 PyTorch-CPU restatement pinned to the
                reference's golden fixtures) timed on the host: 1 D-step + 1 G-step at B=4.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "images/sec per WGAN-GP iter (G13_5+D9_4, 64x64, n_critic=5) at 1/2/4/8 MI355X"
ALGO_GFLOP_PER_IMAGE = 1559.5
FP32_MFMA_PEAK_TFLOPS = 157.3          # MI355X_MICROARCH.md, chip-level parameters
N_CRITIC = 5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=64, help="images per GPU")
    ap.add_argument("--mode", choices=["eager", "graph"], default="graph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the post-run breakdown and roofline probe (clean traces of the timed region)")
    ap.add_argument("--no-bank", action="store_true", help="per-module style MLPs (A/B against the style bank)")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) or gloo (functional test of N>1 on one GPU)")
    return ap.parse_args()


def setup_dist(n, backend):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":      # every rank on cuda:0 (rehearsal of the N>1 path on one GPU)
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    assert world == n or world == 1, f"--gpus {n} but WORLD_SIZE {world}"
    return world, rank, local


def cpu_baseline(threads):
    """Time the CPU oracle: 1 D-step + 1 G-step at B=4 -> images/sec of a full iteration."""
    from oracle import model as om
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    GP, DP = om.Params(lazy=True, generator=g), om.Params(lazy=True, generator=g)
    draw = om.Draw(1)
    with torch.no_grad():  # materialise every parameter once (lazy init) outside the timing
        om.generator(GP, torch.randn(4, 256, 1, 1), draw.randn)
        om.discriminator(DP, torch.randn(4, 3, 64, 64))
    tr = om.WGANGP(GP, DP)
    B = 4
    imgs = torch.randn(B, 3, 64, 64, generator=g)
    t0 = time.perf_counter()
    tr.discriminator_trainstep(imgs, B, draw)
    t1 = time.perf_counter()
    tr.generator_trainstep(B, draw)
    t2 = time.perf_counter()
    t_iter = N_CRITIC * (t1 - t0) + (t2 - t1)
    return {"value": B / t_iter, "unit": "images/sec", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"CPU oracle (fp32 PyTorch-CPU restatement), B=4: 1 D-step {t1 - t0:.2f}s + 1 G-step "
                      f"{t2 - t1:.2f}s, t_iter = 5*t_D + t_G = {t_iter:.1f}s; nproc={os.cpu_count()}"}


# Dominant kernel: the implicit-GEMM conv kernel (conv_gemm_kernel, all instances ~55 % of the
# iteration's GPU time; profiles/).  Representative launch: the critic's mid-level block conv in
# the real+fake pass -- D9_4 128->128 channels, 3x3 replication pad, 32x32, B = 128 -- one
# conv_gemm_kernel<128,128,2,2,1,false> launch per call (1024 tiles, no split-K).
PROBE = dict(B=128, cin=128, h=32, cout=128, k=3)


def roofline_probe(dev, reps=20):
    import gan_amd.ops as ops
    g = ops.conv_geo(PROBE["B"], PROBE["cin"], PROBE["h"], PROBE["h"], PROBE["cout"], PROBE["k"], 1, 1)
    x = torch.randn(g.Cin, g.B, g.H, g.W, device=dev)
    w = torch.nn.Parameter(torch.randn(g.Cout, g.Cin, g.K, g.K, device=dev))
    with torch.no_grad():
        for _ in range(3):
            ops._conv_fwd(g, x, w, None, None, None, 0.03)   # packs the weight once (ops.PackCache)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    with torch.no_grad():
        for _ in range(reps):
            ops._conv_fwd(g, x, w, None, None, None, 0.03)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    flop = 2.0 * g.B * g.OH * g.OW * g.Cout * g.Cin * g.K * g.K
    tf = flop / us / 1e6
    out = {"bound": "mfma", "kernel": "conv_gemm_kernel<128,128,2,2,1,false>",
           "shape": "conv fwd B=128 128->128 3x3 replicate-pad 32x32 (D9_4 block conv, critic real+fake pass)",
           "algorithmic_gflop_per_launch": flop / 1e9, "launch_us": us,
           "achieved": tf, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP32_MFMA_PEAK_TFLOPS,
           "traffic": None}
    # HBM bytes per launch from rocprofv3 PMC passes of this launch (tools/pmc_traffic.sh), if recorded
    tfile = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "roofline_traffic.json")
    if os.path.exists(tfile):
        t = json.load(open(tfile))
        out["traffic"] = t.get("bytes_per_launch")
        out["traffic_source"] = t.get("source")
    return out


def main():
    args = parse()
    world, rank, local = setup_dist(args.gpus, args.backend)
    dev = torch.device("cuda", torch.cuda.current_device())
    import gan_amd
    from gan_amd import ops
    from gan_amd.dist import allreduce_mean_, attach_grad_sync

    torch.manual_seed(1234)                         # identical initial weights on every rank
    G = gan_amd.Generator(256).to(dev)
    G.use_bank = not args.no_bank
    D = gan_amd.Discriminator().to(dev)
    torch.cuda.manual_seed(4321 + rank)             # per-rank data / z / noise / eps stream
    tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.DeviceRNG(dev))
    if world > 1 and args.mode == "eager":
        attach_grad_sync(tr.optimizer_G)
        attach_grad_sync(tr.optimizer_D)
    B = args.batch

    def iteration():
        for _ in range(N_CRITIC):
            images = torch.randn(B, 3, 64, 64, device=dev)
            tr.discriminator_trainstep(images, B)
        tr.generator_trainstep(B)

    def sync(opt):
        if world > 1:
            allreduce_mean_(opt.flat.grad)

    def iteration_split():
        # the same iteration with the gradient all-reduce outside the optimizer (graph mode)
        for _ in range(N_CRITIC):
            tr.discriminator_backward(torch.randn(B, 3, 64, 64, device=dev), B)
            sync(tr.optimizer_D)
            tr.optimizer_D.step()
        tr.generator_backward(B)
        sync(tr.optimizer_G)
        tr.optimizer_G.step()

    if args.mode == "graph" and world > 1:
        iteration = iteration_split

    # warm-up (eager); the first one also counts the conv FLOPs this build issues
    ops.FlopCounter.enabled = True
    iteration()
    ops.FlopCounter.enabled = False
    issued_flops = ops.FlopCounter.flops
    for _ in range(max(0, args.warmup - 1)):
        iteration()
    torch.cuda.synchronize()

    step = iteration
    if args.mode == "graph":
        # one HIP graph per critic step and one per generator step (the synthetic real batch,
        # z, noise and eps are drawn inside the graphs; torch advances the Philox offsets on
        # every replay), replayed 5 + 1 times per iteration
        # With N > 1 ranks the RCCL all-reduce of the flat gradient runs eagerly between a
        # forward/backward graph and an optimizer graph (collectives are kept out of capture).
        def capture(fn):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            return g

        if world == 1:
            gd = capture(lambda: tr.discriminator_trainstep(torch.randn(B, 3, 64, 64, device=dev), B))
            gg = capture(lambda: tr.generator_trainstep(B))
            torch.cuda.synchronize()

            def step():
                for _ in range(N_CRITIC):
                    gd.replay()
                gg.replay()
        else:
            gd = capture(lambda: tr.discriminator_backward(torch.randn(B, 3, 64, 64, device=dev), B))
            gdo = capture(tr.optimizer_D.step)
            gg = capture(lambda: tr.generator_backward(B))
            ggo = capture(tr.optimizer_G.step)
            torch.cuda.synchronize()

            def step():
                for _ in range(N_CRITIC):
                    gd.replay()
                    allreduce_mean_(tr.optimizer_D.flat.grad)
                    gdo.replay()
                gg.replay()
                allreduce_mean_(tr.optimizer_G.flat.grad)
                ggo.replay()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    wall0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - wall0
    if world > 1:
        dist.barrier()
    secs = ev0.elapsed_time(ev1) / 1e3
    t = torch.tensor([secs], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    secs = float(t)

    if rank == 0 and args.mode == "graph" and world == 1 and not args.no_extras:
        # breakdown (outside the timed region): one critic-step graph, one generator-step graph
        parts = {}
        for name, g in (("critic_step", gd), ("generator_step", gg)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            parts[name] = round(e0.elapsed_time(e1), 1)
        # eager pieces of the critic step (indicative; eager adds launch gaps)
        def timed(fn, n=2):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return round(e0.elapsed_time(e1) / n, 1)

        z = torch.randn(B, 256, 1, 1, device=dev)
        x2 = torch.randn(2 * B, 3, 64, 64, device=dev)

        def g_fwd():
            with torch.no_grad():
                G(z)

        def d_fwd_bwd():
            D(x2, segments=2).sum().backward()

        def gp():
            (10 * tr.gradient_penalty(x2[:B], x2[B:], B)).backward()

        parts.update(eager_g_forward=timed(g_fwd), eager_d_fwd_bwd_2B=timed(d_fwd_bwd), eager_gp=timed(gp))
        print(f"[bench] ms per graph / piece: {parts}", file=sys.stderr, flush=True)
    probe = None
    if rank == 0 and world == 1 and not args.no_extras:
        probe = roofline_probe(dev)
    if rank == 0:
        print(f"[bench] peak HBM allocated {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB, "
              f"issued GEMM launches/iter {ops.FlopCounter.launches}", file=sys.stderr, flush=True)
        n_img = B * world * args.steps
        t_iter = secs / args.steps
        achieved = ALGO_GFLOP_PER_IMAGE * 1e9 * B / t_iter / 1e12      # per GPU
        out = {
            "metric": METRIC,
            "value": n_img / secs,
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * t_iter,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic N(0,1) real batches drawn on device each critic step; random reference-init weights",
            "config": {"workload": "G13_5+D9_4 WGAN-GP iteration (5 critic steps with GP + 1 generator step), "
                                   "64x64x3", "global_batch": B * world, "per_gpu_batch": B, "n_critic": N_CRITIC,
                       "parallelism": f"dp{world}", "mode": args.mode},
            "roofline": dict(probe or {}, **{
                # whole iteration: algorithmic FLOPs / iteration time, per GPU
                "iteration_tflops": achieved, "iteration_frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                "algorithmic_gflop_per_iter": ALGO_GFLOP_PER_IMAGE * B,
                "issued_gemm_gflop_per_iter": issued_flops / 1e9}),
            "wall_s": wall,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
