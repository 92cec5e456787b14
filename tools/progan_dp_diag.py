"""Diagnosis of tests/test_dp_gpu.py::test_dp_progan_four_ranks_match_shard_mean on ONE process:
the progan pair's iteration as (a) pipeline.Iteration replay, (b) Iteration.eager, (c) the test's
shard-mean loop with one shard -- on the same start state -- and the relative differences of the
flat parameters / gradients between them.   usage: python tools/progan_dp_diag.py [overlap 0|1]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests import dp_worker  # noqa: E402


def rel(a, b):
    return float((a - b).double().norm() / max(b.double().norm(), 1e-30))


def poison():
    """Fill the caching allocator's free blocks with NaN: a kernel that reads workspace it did not
    write then shows up as NaN or a mismatch instead of reading the same leftovers every run."""
    free = torch.cuda.mem_get_info()[0]
    blocks = []
    try:
        for _ in range(64):
            blocks.append(torch.full((1 << 28,), float("nan"), device="cuda"))   # 1 GiB each
            if torch.cuda.mem_get_info()[0] < free // 4:
                break
    finally:
        del blocks
    torch.cuda.synchronize()


def main():
    overlap = (sys.argv[1] != "0") if len(sys.argv) > 1 else True
    do_poison = len(sys.argv) > 2 and sys.argv[2] == "poison"
    import gan_amd
    from gan_amd.pipeline import Iteration, restore, snapshot
    dev = torch.device("cuda", 0)
    B = dp_worker.B_PROGAN
    G, D = dp_worker.make_progan(gan_amd, dev)
    rng = gan_amd.DeviceRNG(dev, dp_worker.progan_seed(0))
    tr = gan_amd.Train([], dev, 1, 256, G, "G3_progan", D, "D3_progan", rng=rng)
    it = Iteration(tr, B, 5, 1, overlap=overlap)
    snap = snapshot(tr)

    def grab():
        torch.cuda.synchronize()
        return {k: v.detach().cpu().clone() for k, v in
                (("g_data", tr.optimizer_G.flat.data), ("g_grad", tr.optimizer_G.flat.grad),
                 ("d_data", tr.optimizer_D.flat.data), ("d_grad", tr.optimizer_D.flat.grad))}

    it.eager()
    it.capture()
    restore(tr, snap)
    it.step()
    replay = grab()
    restore(tr, snap)
    if do_poison:
        poison()
    it.eager()
    eager = grab()
    restore(tr, snap)
    if do_poison:
        poison()
    _shard_mean_iteration_1(tr, rng, B)
    loop = grab()
    for k, v in loop.items():
        print(f"[diag] non-finite in {k}: {int((~torch.isfinite(v)).sum())}", flush=True)
    for name, (x, y) in {"replay vs eager": (replay, eager), "eager vs shard loop": (eager, loop),
                         "replay vs shard loop": (replay, loop)}.items():
        print(f"[diag] overlap={int(overlap)} poison={int(do_poison)} {name}: " + "  ".join(f"{k} {rel(x[k], y[k]):.3e}" for k in x), flush=True)


def _shard_mean_iteration_1(tr, rng, B):
    """The test's reference loop with one shard (no assertion that shards differ)."""
    tr.rng = rng
    fakes = [f for _ in range(5) for f in tr.generate_fakes(1, B)]
    for i in range(5):
        tr.discriminator_backward(rng.fork(2).randn((B, 3, 64, 64)), B, gen_imgs=fakes[i])
        tr.optimizer_D.step()
    tr.generator_backward(B)
    tr.optimizer_G.step()


if __name__ == "__main__":
    main()
