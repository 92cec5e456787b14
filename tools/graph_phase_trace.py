"""Kernel-time breakdown of the bench's captured phase graphs (the timed path), one phase at a time.

    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python3 tools/graph_phase_trace.py
    python3 tools/graph_phase_trace.py --analyse DIR/.../run_kernel_trace.csv > summary.txt

Run mode: builds bench.py's default Iteration, captures it, replays one full iteration, then
replays each phase graph alone (fake group 0, critic, dstep, gen) REPS times with a device sync and
a 100 ms pause around each replay, so the trace splits into windows at the pauses.

Analyse mode: for each window, span, the time with at least one kernel running, and each kernel's
ATTRIBUTED time: every instant is split equally among the kernels running at it, so the
attributions sum to the busy time and concurrent kernels are not double counted (a trace's
per-kernel durations stretch when streams overlap).  Windows are labelled by the order above."""
import argparse
import collections
import csv
import os
import sys
import time

PHASES = ["fake", "critic", "dstep", "gen"]
REPS = 2


def run():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.argv = [sys.argv[0]]
    import torch
    import bench
    args = bench.parse()
    args.batch = bench.CONFIGS[args.config][1]
    args.precision = "fp32"
    from gan_amd import ops
    ops.set_patch(15)
    dev = torch.device("cuda", 0)
    G, D, tr, it = bench.build(args, dev, 0, 1)
    it.eager()
    it.capture()
    it.step()
    torch.cuda.synchronize()
    for key in PHASES:
        g = it.graphs[key]
        g = g[0] if isinstance(g, list) else g
        for _ in range(REPS):
            time.sleep(0.1)
            g.replay()
            torch.cuda.synchronize()
        print(f"[trace] {key} x{REPS}", flush=True)
    time.sleep(0.1)


def analyse(path, top):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # windows: split at gaps > 50 ms; keep the last len(PHASES) * REPS
    wins, cur, last_end = [], [], None
    for s, e, n in ev:
        if last_end is not None and s - last_end > 50_000_000:
            wins.append(cur)
            cur = []
        cur.append((s, e, n))
        last_end = e if last_end is None else max(last_end, e)
    wins.append(cur)
    wins = wins[-len(PHASES) * REPS:]
    for wi, w in enumerate(wins):
        if wi % REPS != REPS - 1:            # the last replay of each phase (warm)
            continue
        label = PHASES[wi // REPS]
        pts = []
        for i, (s, e, n) in enumerate(w):
            pts.append((s, 1, i))
            pts.append((e, -1, i))
        pts.sort()
        active, attr, busy, conc = set(), collections.Counter(), 0, collections.Counter()
        prev = pts[0][0]
        for t, d, i in pts:
            if active and t > prev:
                dt = t - prev
                busy += dt
                conc[min(len(active), 4)] += dt
                for j in active:
                    attr[j] += dt / len(active)
            prev = t
            if d > 0:
                active.add(i)
            else:
                active.discard(i)
        span = max(e for _, e, _ in w) - min(s for s, _, _ in w)
        byk, cnt = collections.Counter(), collections.Counter()
        for i, (s, e, n) in enumerate(w):
            k = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]
            byk[k] += attr[i]
            cnt[k] += 1
        print(f"== {label}: {len(w)} dispatches, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms "
              f"(idle {100 * (1 - busy / span):.1f} %); time at concurrency 1/2/3/4+: "
              + " / ".join(f"{conc[c] / 1e6:.1f}" for c in (1, 2, 3, 4)) + " ms")
        for k, v in byk.most_common(top):
            print(f"  {v / 1e6:8.2f} ms {100 * v / busy:5.1f}%  {cnt[k]:6d}  {k}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--analyse":
        ap = argparse.ArgumentParser()
        ap.add_argument("--analyse", required=True)
        ap.add_argument("--top", type=int, default=40)
        a = ap.parse_args()
        analyse(a.analyse, a.top)
    else:
        run()
