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
                over the measured iteration time, against the ceiling of the pipe the fp32 GEMMs
                run on (split6: six bf16 MFMAs per fp32 product, 157.3 * 16 / 6 = 419.5 TFLOP/s;
                every `frac`), with the fraction of the fp32 MFMA peak (157.3) as `*_fp32`;
                plus the conv-GEMM FLOPs this build actually issues per iteration.
  cpu_baseline  the CPU oracle (oracle/model.py, fp32 PyTorch-CPU restatement pinned to the
                reference's golden fixtures) timed on the host at B=8: one
                warm-up D-step + G-step, then 2 timed D-steps + 1 timed G-step.
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
BF16_MFMA_PEAK_TFLOPS = 2500.0         # dense bf16 MFMA peak (MI355X_MICROARCH.md; no sparsity)
# The pipe the fp32 GEMMs actually run on ("split6", csrc/conv_gemm.hip): every fp32 product is six
# v_mfma_f32_32x32x16_bf16 per 16 k (x = h + m + l, exact to 24 bits), on the bf16 matrix cores at
# 16x the fp32 MFMA rate (MI355X_MICROARCH.md: fp32 MFMA = 1/16 of bf16) -> 157.3 * 16 / 6 TFLOP/s
# of fp32 work.  This, not 157.3, is the ceiling that bounds those kernels.
SPLIT6_PIPE_PEAK_TFLOPS = FP32_MFMA_PEAK_TFLOPS * 16 / 6
N_CRITIC = 5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default: the config's)")
    ap.add_argument("--config", choices=["wgangp", "lazy", "progan"], default="wgangp",
                    help="wgangp = the headline (configs 2/3); lazy = config 4 (bf16 GEMMs, fp32 R1/R2/GP); progan = config 5")
    ap.add_argument("--mode", choices=["eager", "graph"], default="graph")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default=None,
                    help="GEMM arithmetic (lazy config only; default bf16 there, as config 4 specifies)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the post-run breakdown and roofline probe (clean traces of the timed region)")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) or gloo (functional test of N>1 on one GPU)")
    ap.add_argument("--overlap", choices=["on", "off"], default=None,
                    help="make the next fake-batch group on a second stream during the current group's critic "
                         "steps (default: the headline schedule's FAKE_OVERLAP; groups of 1 without overlap = "
                         "one graph per phase, the reference's order)")
    ap.add_argument("--patch", choices=["on", "off"], default="on",
                    help="stride-1 convs on 32/64-wide maps through the split6 LDS-patch conv and the row-blocked "
                         "weight gradient, Cout <= 4 forwards through the direct conv (default) or everything "
                         "through the gather GEMMs (ops.set_patch 15 / 0: ganamd_conv_desc.kernel_off; A/B)")
    ap.add_argument("--fake-groups", default=None, metavar="K,K,...",
                    help="fake-batch groups of the n_critic steps, each one generator forward with segmented "
                         "BatchNorm (default: the headline schedule FAKE_GROUPS)")
    return ap.parse_args()


# Fake batches of the n_critic critic steps (pipeline.Iteration): groups made by one segmented-
# BatchNorm generator forward each, optionally the next group on a second stream during the current
# group's critic steps.  k * B must keep every conv operand under 2^31 bytes (B = 64: k <= 4).
# Measured at B = 64 (profiles/r03_ab_fake_groups.txt): (1,1,1,1,1) overlapped 41.3 img/s, (4,1)
# overlapped 42.7, (4,1) serial 42.8 -- the wide forward fills the chip on its own.
FAKE_GROUPS, FAKE_OVERLAP = (4, 1), False


def fake_schedule(args, B, world=1):
    """(overlap, real_source, allreduce, fake_groups) arguments of pipeline.Iteration.  With N > 1
    ranks the next fake-batch group is always made on the second stream while the current group's
    critic steps -- and their RCCL all-reduces -- run; FAKE_OVERLAP is the N = 1
    tuning, where there is no collective to hide."""
    if args.fake_groups:
        groups = [int(k) for k in args.fake_groups.split(",")]
    elif args.config == "wgangp" and B <= 64:
        groups = list(FAKE_GROUPS)
    else:
        groups = [1] * N_CRITIC
    default = (FAKE_OVERLAP or world > 1) if max(groups) > 1 else True
    overlap = default if args.overlap is None else args.overlap == "on"
    return overlap, None, None, groups


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """``bench.py --gpus N`` started without a launcher: run N ranks under torchrun as a CHILD
    process (this process has not touched the GPU: no exec, no HIP init) and exit with its code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print("[bench] launching:", " ".join(cmd), file=sys.stderr, flush=True)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def setup_dist(n, backend):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        raise SystemExit(f"bench.py --gpus {n} but WORLD_SIZE={world}: refusing to report a {world}-rank run as {n}")
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
    return world, rank, local


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(threads, B=8):
    """Time the CPU oracle: B=8, one warm-up D-step + G-step (untimed), then two
    timed D-steps and one timed G-step -> t_iter = 5 * mean(t_D) + t_G -> images/sec."""
    from oracle import model as om
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    GP, DP = om.Params(lazy=True, generator=g), om.Params(lazy=True, generator=g)
    draw = om.Draw(1)
    with torch.no_grad():  # materialise every parameter once (lazy init) outside the timing
        om.generator(GP, torch.randn(B, 256, 1, 1), draw.randn)
        om.discriminator(DP, torch.randn(B, 3, 64, 64))
    tr = om.WGANGP(GP, DP)
    tr.discriminator_trainstep(torch.randn(B, 3, 64, 64, generator=g), B, draw)     # warm-up
    tr.generator_trainstep(B, draw)
    t_d = []
    for _ in range(2):
        imgs = torch.randn(B, 3, 64, 64, generator=g)
        t0 = time.perf_counter()
        tr.discriminator_trainstep(imgs, B, draw)
        t_d.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    tr.generator_trainstep(B, draw)
    t_g = time.perf_counter() - t0
    t_iter = N_CRITIC * sum(t_d) / len(t_d) + t_g
    return {"value": B / t_iter, "unit": "images/sec", "cores": torch.get_num_threads(), "kind": "port",
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
            "note": "not 2 full iterations (BASELINE.md §4): 2 x (5 D-steps + 1 G-step) at B=8 is ~90 s of CPU per "
                    "bench run, past the bounded sample the bench contract allows (10-30 s); the per-step times "
                    "are timed and combined as 5 * mean(t_D) + t_G",
            "sample": f"CPU oracle (fp32 PyTorch-CPU restatement of the reference step), B={B}: 1 warm-up D-step + "
                      f"G-step, then D-steps {', '.join(f'{t:.2f}s' for t in t_d)} and G-step {t_g:.2f}s timed; "
                      f"t_iter = 5*mean(t_D) + t_G = {t_iter:.1f}s"}


# Kernel rooflines (MFMA-bound).  Two launches are timed live, each on the
# bench's current stream with its OWN pair of HIP events per launch (the per-dispatch duration a
# rocprofv3 kernel trace reports; back-to-back launches also give the sustained rate):
#   probe     D9_4's mid-level block conv, 128->128 channels, 3x3 replication pad, 32x32, at
#             B = 96: 768 output tiles = one round of the kernel's resident blocks, so it is ONE
#             launch of the critic's gather GEMM conv_gemm_kernel<128,128,2,2,1,false,false> (the
#             plan keeps the 128x128 tile at this batch: the 128x256 one would leave 1.5 rounds);
#   dominant  G13_5's 96-channel 5x5 modulated conv at 64x64 (x*s on the patch, *d in the
#             epilogue): launches of the split6 LDS-patch conv conv_patch_x3_kernel<96,...> at each
#             batch the iteration runs it at (round 6: B = 256 x 10 and B = 64 x 20 per iteration,
#             DOMINANT_MIX), averaged with those launch counts as weights
#             -- the top kernel FAMILY (the patch conv: 0.49 s of the iteration's 1.78 s busy), the
#             top single shape and, since round 5, the top kernel INSTANCE of the iteration trace
#             (profiles/r06_iteration_summary.txt: 0.112 s over 30 launches, the 8-wave paired
#             16x16x32 form since round 6; round 4's top instance was the critic GEMM).  `top_instance`
#             records which kernel leads the committed trace by instance.
PROBES = {
    "probe": dict(B=96, cin=128, h=32, cout=128, k=3, scaled=False,
                  shape="conv fwd B=96 128->128 3x3 replicate-pad 32x32 (D9_4 block conv; 768 whole tiles, one launch)"),
    "dominant": dict(B=64, cin=96, h=64, cout=96, k=5, scaled=True,
                     shape="modulated conv fwd B=64 96->96 5x5 replicate-pad 64x64 (G13_5 StyleConv; x*s gather, *d epilogue)"),
}


def _whole_tile_geo(ops, spec):
    """The probe's geometry at the spec's batch, or the nearest batch whose plan is ONE launch of
    whole tiles (no K-split tail + reduce launches), so a launch is the kernel's whole op."""
    for B in sorted(range(8, 4 * spec["B"] + 1, 8), key=lambda b: (abs(b - spec["B"]), b)):
        g = ops.conv_geo(B, spec["cin"], spec["h"], spec["h"], spec["cout"], spec["k"], 1, (spec["k"] - 1) // 2)
        pl = ops.plan_info(g, 0, spec["scaled"])
        if pl["nfull_t"] == pl["gx"] and pl["S"] == 1:
            return g, pl
    raise RuntimeError(f"no whole-tile batch for {spec['shape']}")


def probe_kernel(dev, spec, reps=20, batch=None):
    import gan_amd.ops as ops
    g, pl = _whole_tile_geo(ops, dict(spec, B=batch) if batch else spec)
    x = torch.randn(g.Cin, g.B, g.H, g.W, device=dev)
    w = torch.nn.Parameter(torch.randn(g.Cout, g.Cin, g.K, g.K, device=dev))
    xs = torch.rand(g.Cin, g.B, device=dev) if spec["scaled"] else None
    ys = torch.rand(g.Cout, g.B, device=dev) if spec["scaled"] else None
    if pl["kernel"] == 1:                                      # the split6 LDS-patch conv (conv_patch.hip)
        kernel = f"conv_patch_x3_kernel<{pl['bm']},...,{g.K},{g.W},{'true' if spec['scaled'] else 'false'},false>"
    else:
        kernel = f"conv_gemm_kernel<{pl['bm']},{pl['bn']},...,{'true' if spec['scaled'] else 'false'},false>"
    y = torch.empty(g.Cout, g.B, g.OH, g.OW, device=dev)

    def launch():
        ops._conv_fwd(g, x, w, None, xs, ys, 0.03, out=y)
    with torch.no_grad():
        for _ in range(3):
            launch()                                         # packs the weight once (ops.PackCache)
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in ev:                                    # one event pair per launch
            e0.record(s)
            launch()
            e1.record(s)
        torch.cuda.synchronize()
        per = [e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):                                # back to back
            launch()
        e1.record(s)
        torch.cuda.synchronize()
    b2b = e0.elapsed_time(e1) * 1e3 / reps
    us = sum(per) / len(per)
    flop = 2.0 * g.B * g.OH * g.OW * g.Cout * g.Cin * g.K * g.K
    tf = flop / us / 1e6
    shape = spec["shape"] if g.B == spec["B"] else spec["shape"].replace(f"B={spec['B']}", f"B={g.B}") + \
        f" (B={spec['B']} has a K-split tail; nearest whole-tile batch)"
    return {"bound": "mfma", "kernel": kernel, "shape": shape, "batch": g.B, "blocks": pl["blocks"],
            "resident_blocks_per_cu": pl["occupancy"],
            "algorithmic_gflop_per_launch": flop / 1e9, "launch_us": us, "launch_us_min": min(per),
            "launch_us_back_to_back": b2b, "achieved": tf, "peak": SPLIT6_PIPE_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": tf / SPLIT6_PIPE_PEAK_TFLOPS,
            "fp32_peak": FP32_MFMA_PEAK_TFLOPS, "frac_fp32": tf / FP32_MFMA_PEAK_TFLOPS,
            "peak_note": "peak = the split6 pipe (fp32 work as six bf16 MFMAs per 16 k: 157.3 * 16 / 6); "
                         "frac_fp32 = the same work against the fp32 MFMA peak 157.3",
            "traffic": None,
            "method": f"{reps} launches on the bench's stream, one HIP event pair each (mean); launch_us_back_to_back: "
                      f"{reps} launches between two events"}


# Which probed kernel leads the committed iteration trace by instance (kernel name with template
# arguments; tools/trace_summary.py), and by family -- from the profile of this round's build.
TOP_INSTANCE = {"kernel": "conv_patch_x3_kernel<96, 8, 512, 5, 64, true, false>", "probe": "dominant",
                "iteration_s": 0.112, "launches": 30, "family_top": "ganamd_patch::conv_patch_x3_kernel",
                "family_s": 0.488, "source": "profiles/r06_iteration_summary.txt"}


# The batches the iteration launches the dominant kernel at, and how often (the census of one
# iteration, profiles/r04_gemm_census.txt: 10 launches at B = 256 in the batched fake forward, 20 at
# B = 64 in the single-batch fake forward and the generator step) -- used when no live census is given.
DOMINANT_MIX = {256: 10, 64: 20}


def dominant_mix(rec):
    """{batch: launches per iteration} of the dominant shape, from the warm-up iteration's record."""
    spec, mix = PROBES["dominant"], {}
    for op, g, xs, ys, math in rec or ():
        if (op == "fwd" and math == "fp32" and bool(xs) == spec["scaled"] and not g.transposed and g.Cin == spec["cin"]
                and g.Cout == spec["cout"] and g.K == spec["k"] and g.H == spec["h"] and g.stride == 1):
            mix[g.B] = mix.get(g.B, 0) + 1
    return mix or dict(DOMINANT_MIX)


def roofline_probe(dev, rec=None):
    """The line's roofline object is the DOMINANT kernel's, over the batches the iteration launches
    it at: each batch is probed on its own (20 launches, one event pair each) and the launches are
    weighted by their count per iteration -- achieved = sum(n_B * FLOPs_B) / sum(n_B * us_B), i.e.
    the average launch's algorithmic FLOPs over the average launch's duration, as a kernel trace of
    the iteration would average them.  The critic probe rides along."""
    mix = dominant_mix(rec)
    per = [dict(probe_kernel(dev, PROBES["dominant"], batch=b), count=n) for b, n in sorted(mix.items(), reverse=True)]
    assert len({p["kernel"] for p in per}) == 1, [p["kernel"] for p in per]
    n = sum(p["count"] for p in per)
    flop = sum(p["count"] * p["algorithmic_gflop_per_launch"] for p in per) / n
    us = sum(p["count"] * p["launch_us"] for p in per) / n
    out = dict(per[0])
    out.update({"shape": PROBES["dominant"]["shape"].replace(f"B={PROBES['dominant']['B']}", "B=" + "/".join(
                    str(p["batch"]) for p in per)) + " at its launch mix",
                "batch": {str(p["batch"]): p["count"] for p in per}, "algorithmic_gflop_per_launch": flop,
                "launch_us": us, "achieved": flop / us * 1e3, "frac": flop / us * 1e3 / SPLIT6_PIPE_PEAK_TFLOPS,
                "frac_fp32": flop / us * 1e3 / FP32_MFMA_PEAK_TFLOPS,
                "per_batch": [{k: p[k] for k in ("batch", "count", "blocks", "algorithmic_gflop_per_launch", "launch_us",
                                                  "launch_us_min", "launch_us_back_to_back", "achieved", "frac")}
                              for p in per],
                "method": "each batch the iteration launches this kernel at (count per iteration from the warm-up "
                          "iteration's census): 20 launches on the bench's stream, one HIP event pair each; achieved = "
                          "launch-count-weighted FLOPs / launch-count-weighted mean duration"})
    for k in ("blocks", "count", "launch_us_min", "launch_us_back_to_back"):
        out.pop(k, None)
    # HBM bytes per launch from rocprofv3 PMC passes of these launches (tools/pmc_traffic.sh), if
    # recorded for every batch of the mix: the count-weighted mean per launch, like achieved
    tfile = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "roofline_traffic.json")
    if os.path.exists(tfile):
        t = json.load(open(tfile))
        tb = t.get("per_batch", {})
        if t.get("kernel") == out["kernel"] and all(str(p["batch"]) in tb for p in per):
            out["traffic"] = sum(p["count"] * tb[str(p["batch"])]["bytes_per_launch"] for p in per) / n
            out["algorithmic_bytes_per_launch"] = sum(p["count"] * tb[str(p["batch"])]["algorithmic_bytes"]
                                                      for p in per) / n
            out["traffic_source"] = t.get("source")
    out["critic_probe"] = probe_kernel(dev, PROBES["probe"])
    out["top_instance"] = TOP_INSTANCE
    return out


# Algorithmic GFLOP per image of each phase graph of the pipelined iteration:
# fake = the no-grad generator forward, critic = the rest of a critic step (critic on real + fake,
# gradient penalty with its double backward), gen = the generator step.
PHASE_GFLOP_PER_IMAGE = {"fake": 101.99, "critic": 245.93 - 101.99, "gen": 329.81}


def bf16_algo(algo, issued, bf16_issued):
    """Algorithmic FLOPs of the bf16 part (issued bf16 scaled by the algorithmic/issued ratio)."""
    return bf16_issued * (algo / issued) if issued else 0.0


def gemm_census(dev, rec, top=8):
    """Per-shape speed of the iteration's conv GEMMs: every distinct (op, geometry, scales) recorded
    in one eager iteration is timed in isolation (HIP events around 5 back-to-back launches after a
    warm-up) on the bench's own stream; est time = count x time.  Returns the GEMM-weighted
    achieved TF/s (algorithmic FLOPs / est time), its fraction of the fp32 MFMA peak, and the top
    shapes by estimated time with their own fractions."""
    import collections
    import gan_amd.ops as ops
    cnt = collections.Counter(rec)
    rows = []
    s = torch.cuda.current_stream()
    for (op, g, xs, ys, math), n in cnt.items():
        xin = torch.randn(g.Cin, g.B, g.H, g.W, device=dev)
        yout = torch.randn(g.Cout, g.B, g.OH, g.OW, device=dev)
        w = torch.nn.Parameter(torch.randn((g.Cin, g.Cout, g.K, g.K) if g.transposed else (g.Cout, g.Cin, g.K, g.K),
                                           device=dev))
        sx = torch.rand(g.Cin, g.B, device=dev) if xs else None
        sy = torch.rand(g.Cout, g.B, device=dev) if ys else None
        if op == "fwd":
            f = lambda: ops._conv_fwd(g, xin, w, None, sx, sy, 1.0)
        elif op == "dgrad":      # the recorded flag is the gy (Cout-side) scale
            sgy = torch.rand(g.Cout, g.B, device=dev) if xs else None
            f = lambda: ops._conv_dgrad(g, yout, w, sgy, 1.0)
        else:
            f = lambda: ops._conv_wgrad(g, xin, yout, sx, sy, 1.0)
        with torch.no_grad(), ops.math_mode(math):
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                f()
            e1.record(s)
            torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 5e3
        flop = ops.FlopCounter.algorithmic(g)
        rows.append((n * t, n, t, flop, op, g, xs or ys, math))
        del xin, yout, w, sx, sy
    rows.sort(key=lambda r: -r[0])
    tot_t = sum(r[0] for r in rows)
    if os.environ.get("GANAMD_CENSUS_OUT"):         # full per-shape table (profiles/)
        with open(os.environ["GANAMD_CENSUS_OUT"], "w") as f:
            f.write(f"{'share':>6} {'n':>5} {'us':>9} {'TF/s':>7}  op     B  Cin  H   W  Cout OH  OW k s p T sc math\n")
            for r in rows:
                g = r[5]
                f.write(f"{100 * r[0] / tot_t:6.2f} {r[1]:5d} {1e6 * r[2]:9.1f} {r[3] / r[2] / 1e12:7.2f}  {r[4]:5s} "
                        f"{g.B:3d} {g.Cin:4d} {g.H:3d} {g.W:3d} {g.Cout:4d} {g.OH:3d} {g.OW:3d} {g.K} {g.stride} {g.pad} "
                        f"{int(g.transposed)} {int(bool(r[6]))} {r[7]}\n")
    tot_f = sum(r[1] * r[3] for r in rows)
    tf = tot_f / tot_t / 1e12

    def shape(r):
        g = r[5]
        return (f"{r[4]} B={g.B} {g.Cin}->{g.Cout} {g.H}x{g.W}->{g.OH}x{g.OW} k{g.K} s{g.stride}"
                f"{' T' if g.transposed else ''}{' scaled' if r[6] else ''}{' bf16' if r[7] == 'bf16' else ''}")

    def peak(r, fp32=False):
        """the ceiling of the pipe the shape runs on: bf16 MFMA, or split6 for fp32 work (fp32=True: the
        fp32 MFMA peak instead, the fraction quoted before round 4)"""
        return BF16_MFMA_PEAK_TFLOPS if r[7] == "bf16" else (FP32_MFMA_PEAK_TFLOPS if fp32 else SPLIT6_PIPE_PEAK_TFLOPS)
    return {"distinct_shapes": len(rows), "launches_per_iter": sum(r[1] for r in rows),
            "est_gemm_s_per_iter": tot_t, "gemm_tflops": tf,
            "gemm_frac": sum(r[1] * r[3] / (peak(r) * 1e12) for r in rows) / tot_t,
            "gemm_frac_fp32": sum(r[1] * r[3] / (peak(r, True) * 1e12) for r in rows) / tot_t,
            "method": "every distinct conv GEMM of one iteration timed in isolation (HIP events, 5 launches); "
                      "algorithmic FLOPs / (count x time); includes each op's split-K reduce / fold launches",
            "top": [{"shape": shape(r), "count": r[1], "us": 1e6 * r[2], "tflops": r[3] / r[2] / 1e12,
                     "frac": r[3] / r[2] / 1e12 / peak(r), "frac_fp32": r[3] / r[2] / 1e12 / peak(r, True),
                     "share": r[0] / tot_t} for r in rows[:top]]}


CONFIGS = {
    # name: (metric, default per-GPU batch, description)
    "wgangp": (METRIC, 64, "G13_5+D9_4 WGAN-GP iteration (5 critic steps with GP + 1 generator step), 64x64x3"),
    "lazy": ("images/sec per lazy-GP+R1/R2 period (G13_5+D9_4, 64x64, wganlazygpR2, 5 batches)", 128,
             "G13_5+D9_4 train/wganlazygpR2.py: 5 batches = 5 x (critic step + generator step), R1/R2/GP on the "
             "first, Adam; config 4 of BASELINE.json"),
    "progan": ("images/sec per WGAN-GP iter (generator_3_progan ngf=256 + discriminator_3_wgangp_progan ndf=64, "
               "64x64, n_critic=5)", 64,
               "progan pair under train/wgangp.py, fixed 64x64 nets (the reference has no progressive schedule); "
               "config 5 of BASELINE.json at 64 images per GPU"),
}


def build(args, dev, rank, world):
    """Models, trainer, and the timed iteration: a pipeline.Iteration for the WGAN-GP configs
    (the tested graph schedule, tests/test_pipeline_gpu.py), else a list of optimizer phases
    (graph key, backward callable, optimizer)."""
    import gan_amd
    from gan_amd.pipeline import Iteration
    torch.manual_seed(1234)                         # identical initial weights on every rank
    if args.config == "progan":
        G = gan_amd.generator_3_progan.Generator(1, 256, 256, 3).to(dev)
        D = gan_amd.discriminator_3_wgangp_progan.Discriminator(1, 64, 3).to(dev)
    else:
        G = gan_amd.Generator(256).to(dev)
        D = gan_amd.Discriminator().to(dev)
    rng = gan_amd.DeviceRNG(dev, 4321 + rank)       # per-rank data / z / noise / eps streams
    if args.config == "lazy":
        tr = gan_amd.wganlazygpR2.Train([], dev, 1, 256, G, args.config, D, args.config, rng=rng,
                                        precision=args.precision)
    else:
        tr = gan_amd.Train([], dev, 1, 256, G, args.config, D, args.config, rng=rng)
    B = args.batch
    if args.config != "lazy":
        return G, D, tr, Iteration(tr, B, N_CRITIC, world, *fake_schedule(args, B, world))
    data = rng.fork(2)

    def real():
        return data.randn((B, 3, 64, 64))

    gen = ("gen", lambda: tr.generator_backward(B), tr.optimizer_G)
    phases = []
    for idx in range(5):     # one lazy period: the regularised critic step, then 4 plain ones
        key = "critic_reg" if idx == 0 else "critic"
        phases += [(key, (lambda i=idx: tr.discriminator_backward(real(), B, i)), tr.optimizer_D), gen]
    return G, D, tr, phases


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.batch is None:
        args.batch = CONFIGS[args.config][1]
    if args.precision is None:
        args.precision = "bf16" if args.config == "lazy" else "fp32"
    if args.precision == "bf16" and args.config != "lazy":
        raise SystemExit("--precision bf16 applies to --config lazy (config 4); the headline is fp32")
    world, rank, local = setup_dist(args.gpus, args.backend)
    dev = torch.device("cuda", torch.cuda.current_device())
    from gan_amd import ops
    from gan_amd.dist import allreduce_mean_
    ops.set_patch(15 if args.patch == "on" else 0)    # patch fwd + dgrad, row-blocked wgrad, direct Cout<=4 conv (kernel_off)

    G, D, tr, it = build(args, dev, rank, world)
    B = args.batch
    headline = args.config == "wgangp"
    pipelined = not isinstance(it, list)
    # images per iteration per GPU: the generator-step batches (wgangp: 1 per n_critic critic steps)
    imgs_per_iter = B if pipelined else B * sum(1 for k, *_ in it if k == "gen")

    def iteration():
        if pipelined:
            it.eager()
            return
        for _key, bwd, opt in it:
            bwd()
            if world > 1:
                allreduce_mean_(opt.flat.grad)
            opt.step()

    # warm-up (eager); the first one also counts the conv FLOPs this build issues
    ops.FlopCounter.enabled = True
    census_rec = ops.FlopCounter.record = []
    iteration()
    ops.FlopCounter.enabled = False
    ops.FlopCounter.record = None
    issued_flops = ops.FlopCounter.flops
    algo_flops, bf16_flops = ops.FlopCounter.algo_flops, ops.FlopCounter.flops_bf16
    def mem_note(i):
        # live bytes after each eager warm-up iteration, and after a cyclic GC (what survives an
        # iteration: DESIGN.md §2 "peak HBM vs warm-ups")
        import gc
        torch.cuda.synchronize()
        a0 = torch.cuda.memory_allocated() / 2**30
        gc.collect()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warm-up {i}: live {a0:.1f} GiB, after gc.collect {torch.cuda.memory_allocated() / 2**30:.1f} "
                  f"GiB, peak {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB", file=sys.stderr, flush=True)
    mem_note(0)
    for i in range(max(0, args.warmup - 1)):
        iteration()
        mem_note(i + 1)
    torch.cuda.synchronize()
    if rank == 0:
        print(f"[bench] warm-up done ({args.config}, B={B}/GPU, {world} rank(s))", file=sys.stderr, flush=True)

    step = iteration
    graphs = {}
    if args.mode == "graph" and pipelined:
        it.count_nodes = True          # the iteration's dispatch count (graph nodes per replay)
        it.capture()
        step = it.step
        if rank == 0:
            kind = f"fake groups {it.groups}, {'overlapped' if it.overlap else 'serial'}"
            print(f"[bench] captured the iteration graphs ({kind})",
                  file=sys.stderr, flush=True)
    elif args.mode == "graph":
        # one HIP graph per distinct phase (synthetic real batch, z, noise and eps are drawn
        # inside; the device Philox stream offsets advance on every replay).  N = 1: backward +
        # optimizer in one graph.  N > 1: the all-reduce of the flat gradient runs eagerly between
        # a backward graph and an optimizer graph (collectives are kept out of capture).  All
        # phase graphs share ONE memory pool (they replay one after another).
        pool = torch.cuda.graph_pool_handle()
        torch.cuda.empty_cache()

        def capture(fn):
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                fn()
            return g

        for key, bwd, opt in it:
            if key in graphs:
                continue
            if world == 1:
                graphs[key] = (capture(lambda b=bwd, o=opt: (b(), o.step())), None, opt)
            else:
                graphs[key] = (capture(bwd), capture(opt.step), opt)
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] captured {len(graphs)} phase graphs", file=sys.stderr, flush=True)

        def step():
            for key, *_ in it:
                gb, go, opt = graphs[key]
                gb.replay()
                if go is not None:
                    allreduce_mean_(opt.flat.grad)
                    go.replay()

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
        # breakdown (outside the timed region): one replay per phase graph
        if pipelined:
            parts = it.phase_ms()
        else:
            parts = {}
            for key, (g, _, _) in graphs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                parts[key] = round(e0.elapsed_time(e1), 1)
        print(f"[bench] ms per phase graph: {parts}", file=sys.stderr, flush=True)
        phase_frac = None
        if headline and pipelined and it.grouped:
            # GFLOP / ms = TFLOP/s; the batched fake phase makes n_critic batches
            imgs = {k: B * (it.groups[0] if k == "fake" else 1) for k in parts}
            phase_frac = {k: {"ms": v, "tflops": PHASE_GFLOP_PER_IMAGE[k] * imgs[k] / v,
                              "frac": PHASE_GFLOP_PER_IMAGE[k] * imgs[k] / v / SPLIT6_PIPE_PEAK_TFLOPS,
                              "frac_fp32": PHASE_GFLOP_PER_IMAGE[k] * imgs[k] / v / FP32_MFMA_PEAK_TFLOPS}
                          for k, v in parts.items() if k in PHASE_GFLOP_PER_IMAGE}
    probe = census = None
    if "phase_frac" not in locals():
        phase_frac = None
    if rank == 0 and world == 1 and headline and not args.no_extras:
        probe = roofline_probe(dev, census_rec)
    if rank == 0 and world == 1 and not args.no_extras:
        census = gemm_census(dev, census_rec)
    if rank == 0:
        print(f"[bench] peak HBM allocated {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB "
              f"(reserved {torch.cuda.max_memory_reserved() / 2**30:.1f}), "
              f"issued GEMM launches/iter {ops.FlopCounter.launches}", file=sys.stderr, flush=True)
        n_img = imgs_per_iter * world * args.steps
        t_iter = secs / args.steps
        metric, _, desc = CONFIGS[args.config]
        out = {
            "metric": metric,
            "value": n_img / secs,
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * t_iter,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if args.precision == "fp32" else "bf16 GEMM operands, fp32 accumulate/storage; fp32 R1/R2/GP steps",
            "data": "synthetic N(0,1) real batches drawn on device each critic step; random reference-init weights",
            "config": {"workload": desc, "global_batch": B * world, "per_gpu_batch": B,
                       "parallelism": f"dp{world}", "mode": args.mode, "patch_conv": args.patch},
        }
        if headline:
            out["config"]["n_critic"] = N_CRITIC
            if pipelined:
                out["config"]["fake_groups"] = it.groups
                out["config"]["fake_overlap"] = it.overlap
                if it.nodes:
                    # kernel dispatches (graph kernel nodes) of one replayed iteration, and the rest
                    out["dispatches_per_iter"] = it.dispatches()
            achieved = ALGO_GFLOP_PER_IMAGE * 1e9 * B / t_iter / 1e12      # per GPU
            out["roofline"] = dict(probe or {}, **{
                # whole iteration: algorithmic FLOPs / iteration time, per GPU
                "iteration_tflops": achieved, "iteration_frac": achieved / SPLIT6_PIPE_PEAK_TFLOPS,
                "iteration_frac_fp32": achieved / FP32_MFMA_PEAK_TFLOPS,
                "algorithmic_gflop_per_iter": ALGO_GFLOP_PER_IMAGE * B,
                "algorithmic_gemm_gflop_per_iter": algo_flops / 1e9,
                "issued_gemm_gflop_per_iter": issued_flops / 1e9})
        else:
            # bf16 and fp32 GEMMs priced at their own peaks: frac = (time the issued-precision mix
            # needs at peak) / iteration time; "peak" is that mix's effective rate
            t_peak = (algo_flops - bf16_algo(algo_flops, issued_flops, bf16_flops)) / (FP32_MFMA_PEAK_TFLOPS * 1e12) + \
                bf16_algo(algo_flops, issued_flops, bf16_flops) / (BF16_MFMA_PEAK_TFLOPS * 1e12)
            eff_peak = algo_flops / t_peak / 1e12
            out["roofline"] = {"bound": "mfma", "algorithmic_gemm_gflop_per_iter": algo_flops / 1e9,
                               "issued_gemm_gflop_per_iter": issued_flops / 1e9,
                               "bf16_issued_gemm_gflop_per_iter": bf16_flops / 1e9,
                               "achieved": algo_flops / t_iter / 1e12, "peak": eff_peak, "unit": "TFLOP/s",
                               "frac": algo_flops / t_iter / 1e12 / eff_peak,
                               "note": "algorithmic conv-GEMM FLOPs per iteration / iteration time, against the "
                                       "fp32 (157.3) / bf16 (2500) MFMA peaks weighted by the FLOPs each precision runs"}
        if census is not None:
            out["roofline"]["gemm_census"] = census
        if phase_frac:
            out["roofline"]["phases"] = phase_frac
        out["wall_s"] = wall
        if world == 1 and headline and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
