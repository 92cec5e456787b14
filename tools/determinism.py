"""Run-to-run determinism of the training iteration (diagnostic, GPU).

  python tools/determinism.py [B]          # the generator step twice, under four configurations
  DET_FULL=1 python tools/determinism.py   # + the eager iteration twice, the captured ones twice

From one snapshot of the training state each pair of runs is compared bit for bit.  On a
generator mismatch it names the first module outputs that differ (forward, execution order), whether
the gradient reaching G's output differs (the critic's input-gradient sweep), and the parameters
whose gradients differ."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from tests import dp_worker  # noqa: E402

DEV = torch.device("cuda", 0)


def _state(tr):
    from gan_amd.pipeline import training_state
    return [t.detach().clone() for t in training_state(tr)] + [o.clone() for o in tr.rng.state().values()]


def _cmp(tag, a, b):
    names = ["G.data", "G.grad", "G.m", "G.v", "G.step", "D.data", "D.grad", "D.m", "D.v", "D.step"]
    bad = []
    for i, (x, y) in enumerate(zip(a, b)):
        if not torch.equal(x, y):
            bad.append((names[i] if i < len(names) else f"buf{i}", float((x.double() - y.double()).abs().max())))
    print(f"{tag}: {'bit-identical' if not bad else bad}", flush=True)
    return not bad


class _Recorder:
    """Forward outputs of every module of G (execution order) and the gradient reaching G's output."""

    def __init__(self, G):
        self.out, self.hs, self.gout = [], [], None
        for n, m in G.named_modules():
            self.hs.append(m.register_forward_hook(self._hook(n)))

    def _hook(self, name):
        def f(mod, inp, out):
            if torch.is_tensor(out):
                self.out.append((name, out.detach().clone()))
                if name == "" and out.requires_grad:
                    out.register_hook(lambda g: setattr(self, "gout", g.detach().clone()))
        return f

    def remove(self):
        for h in self.hs:
            h.remove()


def _g_twice(tr, snap, G, B):
    from gan_amd.pipeline import restore
    grads, recs = [], []
    for _ in range(2):
        restore(tr, snap)
        rec = _Recorder(G)
        tr.generator_backward(B)
        torch.cuda.synchronize()
        rec.remove()
        grads.append([(n, None if p.grad is None else p.grad.detach().clone()) for n, p in G.named_parameters()])
        recs.append(rec)
    bad = [(n, float((a - b).abs().max())) for (n, a), (_, b) in zip(recs[0].out, recs[1].out)
           if not torch.equal(a, b)]
    print(f"G forward twice: {len(bad)} of {len(recs[0].out)} module outputs differ; first: {bad[:12]}", flush=True)
    ga, gb = recs[0].gout, recs[1].gout
    print("gradient at G's output:", "same" if (ga is not None and torch.equal(ga, gb)) else
          f"DIFFERENT {None if ga is None else float((ga - gb).abs().max())}", flush=True)
    rows = []
    for (n, a), (_, b) in zip(grads[0], grads[1]):
        if a is not None and b is not None and not torch.equal(a, b):
            rows.append((n, tuple(a.shape), float((a - b).abs().max()), float(a.abs().max())))
    print(f"G step twice: {len(rows)} of {len(grads[0])} parameter gradients differ", flush=True)
    for r in rows[:80]:
        print("   ", r, flush=True)


def main(B):
    import gan_amd as gan
    from gan_amd import ops
    from gan_amd.pipeline import Iteration, restore, snapshot
    G, D = dp_worker.make_models(gan, DEV)
    tr = gan.Train([], DEV, 1, 256, G, "G13_5", D, "D9_4", rng=gan.DeviceRNG(DEV, 2024))
    it = Iteration(tr, B, n_critic=5, overlap=True)
    it.eager()
    torch.cuda.synchronize()
    snap = snapshot(tr)

    for tag, br, mask in (("default", True, 7), ("no branch streams", False, 7), ("patch off", True, 0),
                          ("no branch streams, patch off", False, 0)):
        ops.BRANCH_STREAMS[0] = br
        ops.set_patch(mask)
        print(f"== {tag}", flush=True)
        _g_twice(tr, snap, G, B)
    ops.BRANCH_STREAMS[0] = True
    ops.set_patch(15)
    if os.environ.get("DET_FULL") != "1":
        return

    st = []
    for _ in range(2):
        restore(tr, snap)
        it.eager()
        torch.cuda.synchronize()
        st.append(_state(tr))
    _cmp("eager iteration twice", st[0], st[1])
    eager = st[0]
    for overlap in (True, False):
        restore(tr, snap)
        it2 = Iteration(tr, B, n_critic=5, overlap=overlap)
        it2.capture()
        rs = []
        for _ in range(2):
            restore(tr, snap)
            it2.step()
            torch.cuda.synchronize()
            rs.append(_state(tr))
        _cmp(f"graph overlap={overlap} replay twice", rs[0], rs[1])
        _cmp(f"graph overlap={overlap} vs eager", rs[0], eager)
        del it2
        torch.cuda.synchronize()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
