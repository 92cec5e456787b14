"""One rank of the data-parallel WGAN-GP rehearsal (run under torchrun by
tests/test_dp_gpu.py; world 2, gloo, every rank on cuda:0).

Each rank runs the REAL gan_amd trainer on its own 4-image shard with its own replayed random
stream (z, StyleConv noise, eps): a critic step (generator forward, critic on real+fake, GP
double backward) whose flat gradient is all-reduced (gan_amd.dist.allreduce_mean_) before the
fused AdamW step, then a generator backward whose flat gradient is all-reduced too -- the order
bench.py runs for N > 1.  Rank 0 writes the all-reduced gradients and the
critic's parameters after its step to the path given as argv[1].

``dp_worker.py OUT progan``: config 5's split (BASELINE.json: the progan pair, 4 ranks): the bench's
progan schedule (pipeline.Iteration, fake batches one per critic step on a side stream) at
B = 64 per rank, one iteration; rank 0 writes both models' parameters and gradients.

``dp_worker.py OUT graph SCHEDULE [B]`` (2 ranks; 8 ranks for config 3's world size): the bench's
N > 1 graph-mode path instead -- one pipelined
WGAN-GP iteration (gan_amd.pipeline.Iteration: captured fake-batch / critic / AdamW / generator
graphs, the next fake batch on a side stream, the flat-gradient all-reduce eagerly between graphs)
at B per rank (default 8; 64 = config 3's per-GPU batch) with device Philox streams seeded per rank;
rank 0 writes both models' parameters and gradients after the iteration, and the first all-reduced
critic gradient (before any AdamW step).

Every mode records the FIRST all-reduced critic gradient of the timed iteration (``d_grad0``): the
shard mean before any optimizer step, where a DP bug would show without the iteration's
amplification of rounding differences.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

B = 4
B_GRAPH = 8


def graph_seed(rank):
    return 960 + rank


def shard_inputs(rank):
    """Per-shard real images and the seed of the shard's replayed random stream."""
    images = torch.randn(B, 3, 64, 64, generator=torch.Generator().manual_seed(900 + rank))
    return images, 950 + rank


def make_models(gan, dev):
    from oracle.params import fill_module
    from tests._util import plan
    P = plan()
    G = gan.Generator(256)
    fill_module(G, P["g_seed"])
    D = gan.Discriminator()
    fill_module(D, P["d_seed"])
    return G.to(dev), D.to(dev)


def main(out):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import gan_amd
    from gan_amd.dist import allreduce_mean_
    dev = torch.device("cuda", 0)
    G, D = make_models(gan_amd, dev)
    images, seed = shard_inputs(rank)
    tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.ReplayRNG(seed, dev))
    tr.discriminator_backward(images.to(dev), B)
    allreduce_mean_(tr.optimizer_D.flat.grad)
    d_grad = tr.optimizer_D.flat.grad.detach().cpu().clone()
    tr.optimizer_D.step()
    d_data = tr.optimizer_D.flat.data.detach().cpu().clone()
    tr.generator_backward(B)
    allreduce_mean_(tr.optimizer_G.flat.grad)
    g_grad = tr.optimizer_G.flat.grad.detach().cpu().clone()
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"d_grad": d_grad, "d_data": d_data, "g_grad": g_grad, "world": world}, out)
    dist.barrier()
    dist.destroy_process_group()


GRAPH_FAKE_GROUPS = (4, 1)


class FirstAllreduce:
    """The trainer's all-reduce (dist.allreduce_mean_) that keeps a copy of the first buffer it
    reduces once ``armed`` -- the first critic gradient of the timed iteration."""

    def __init__(self):
        from gan_amd.dist import allreduce_mean_
        self.fn, self.armed, self.first = allreduce_mean_, False, None

    def __call__(self, flat):
        self.fn(flat)
        if self.armed and self.first is None:
            self.first = flat.detach().cpu().clone()
        return flat


def _mem(tag):
    if os.environ.get("DP_MEMLOG") == "1":
        torch.cuda.synchronize()
        print(f"[mem] {tag}: allocated {torch.cuda.memory_allocated() / 2**30:.1f} GiB, reserved "
              f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB, peak {torch.cuda.max_memory_reserved() / 2**30:.1f}",
              flush=True)


def main_graph(out):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import gan_amd
    from gan_amd.pipeline import Iteration, restore, snapshot
    dev = torch.device("cuda", 0)
    G, D = make_models(gan_amd, dev)
    tr = gan_amd.Train([], dev, 1, 256, G, "G13_5", D, "D9_4", rng=gan_amd.DeviceRNG(dev, graph_seed(rank)))
    # bench.py's N > 1 schedule: fake groups (4, 1), the second group made on the side stream while
    # the first group's critic steps and all-reduces run ("serial": the N = 1 order)
    serial = len(sys.argv) > 3 and sys.argv[3] == "serial"
    bs = int(sys.argv[4]) if len(sys.argv) > 4 else B_GRAPH
    ar = FirstAllreduce()
    it = Iteration(tr, bs, 5, world, overlap=not serial, fake_groups=GRAPH_FAKE_GROUPS, allreduce=ar)
    snap = snapshot(tr, "cpu")     # two B = 64 ranks and the test share one GPU: host copies
    _mem("models")
    it.eager()                     # warm-up (all-reduces included), then capture
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    _mem("eager warm-up")
    # the ranks capture one after another: they share one GPU here, and a capture peaks at the
    # graph pools plus one phase's eager warm-up (~140 GB per rank at B = 64; with eight ranks the
    # captures of the others' would add up)
    for r in range(world):
        if r == rank:
            if os.environ.get("DP_MEMLOG") == "1":
                print(f"[rank {rank}] before capture: device free {torch.cuda.mem_get_info()[0] / 2**30:.1f} GiB, "
                      f"reserved {torch.cuda.memory_reserved() / 2**30:.1f} GiB", flush=True)
            it.capture()
            # hand the eager warm-up's cached blocks back before the next rank captures (the graph
            # pools stay): rank 0 at 139 GiB reserved left the second rank's capture 3 GiB short
            torch.cuda.synchronize()
            if os.environ.get("DP_NO_EMPTY") != "1":
                torch.cuda.empty_cache()
            free, _ = torch.cuda.mem_get_info()
            print(f"[rank {rank}] captured: reserved {torch.cuda.memory_reserved() / 2**30:.1f} GiB, device free "
                  f"{free / 2**30:.1f} GiB", flush=True)
        dist.barrier()
    _mem("captured")
    restore(tr, snap)
    dist.barrier()
    ar.armed = True
    it.step()
    torch.cuda.synchronize()
    res = {k: v.detach().cpu().clone() for k, v in
           (("g_data", tr.optimizer_G.flat.data), ("g_grad", tr.optimizer_G.flat.grad),
            ("d_data", tr.optimizer_D.flat.data), ("d_grad", tr.optimizer_D.flat.grad))}
    if rank == 0:
        torch.save(dict(res, world=world, d_grad0=ar.first, batch=bs, peak_reserved=torch.cuda.max_memory_reserved(),
                        reserved=torch.cuda.memory_reserved()), out)
    dist.barrier()
    dist.destroy_process_group()


B_PROGAN = 64
PROGAN_WORLD = int(os.environ.get("GANAMD_TEST_PROGAN_WORLD", "4"))


def progan_seed(rank):
    return 1960 + rank


def make_progan(gan, dev):
    import json
    from oracle.params import fill_module
    from tests._util import GOLDEN
    with open(os.path.join(GOLDEN, "plan_progan.json")) as f:
        pp = json.load(f)
    G = gan.generator_3_progan.Generator(1, 256, pp["ngf"], 3)
    D = gan.discriminator_3_wgangp_progan.Discriminator(1, pp["ndf"], 3)
    fill_module(G, pp["g_seed"])
    fill_module(D, pp["d_seed"])
    return G.to(dev), D.to(dev)


def main_progan(out):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    import gan_amd
    from gan_amd.pipeline import Iteration, restore, snapshot
    if os.environ.get("GANAMD_TEST_PATCH_MASK"):      # diagnosis: kernel selection A/B
        gan_amd.ops.set_patch(int(os.environ["GANAMD_TEST_PATCH_MASK"]))
    dev = torch.device("cuda", 0)
    G, D = make_progan(gan_amd, dev)
    tr = gan_amd.Train([], dev, 1, 256, G, "G3_progan", D, "D3_progan", rng=gan_amd.DeviceRNG(dev, progan_seed(rank)))
    overlap = os.environ.get("GANAMD_TEST_PROGAN_OVERLAP", "1") != "0"     # diagnosis override
    ar = FirstAllreduce()
    it = Iteration(tr, B_PROGAN, 5, world, overlap=overlap, allreduce=ar)    # bench.py's progan schedule
    snap = snapshot(tr)
    it.eager()
    it.capture()
    restore(tr, snap)
    dist.barrier()
    ar.armed = True
    it.step()
    torch.cuda.synchronize()
    res = {k: v.detach().cpu().clone() for k, v in
           (("g_data", tr.optimizer_G.flat.data), ("g_grad", tr.optimizer_G.flat.grad),
            ("d_data", tr.optimizer_D.flat.data), ("d_grad", tr.optimizer_D.flat.grad))}
    if rank == 0:
        torch.save(dict(res, world=world, d_grad0=ar.first), out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    mode = sys.argv[2] if len(sys.argv) > 2 else ""
    {"graph": main_graph, "progan": main_progan}.get(mode, main)(sys.argv[1])
