"""Summarise a rocprofv3 kernel trace CSV: busy vs span, time by kernel family and by kernel.

    python tools/trace_summary.py TRACE.csv [--last SECONDS]

--last keeps only the dispatches that start in the final SECONDS of the trace (e.g. the timed
bench iteration: pass its ms_per_step/1000), so warmup and capture are excluded."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=float, default=0.0)
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()

rows = list(csv.DictReader(open(a.trace)))
st = [int(r["Start_Timestamp"]) for r in rows]
en = [int(r["End_Timestamp"]) for r in rows]
if a.last > 0:
    t0 = max(en) - int(a.last * 1e9)
    keep = [i for i, s in enumerate(st) if s >= t0]
    rows = [rows[i] for i in keep]
    st = [st[i] for i in keep]
    en = [en[i] for i in keep]
span = (max(en) - min(st)) / 1e9
busy = sum(e - s for s, e in zip(st, en)) / 1e9
fam = collections.Counter()
cnt = collections.Counter()
kern = collections.Counter()
kcnt = collections.Counter()
for r, s, e in zip(rows, st, en):
    n = r["Kernel_Name"]
    k = ("gemm" if ("conv_gemm" in n or "wgrad_gemm" in n) else
         "grouped_gemm" if "grouped_gemm" in n else
         "split_reduce" if "split_reduce" in n else
         "bn" if "bn_" in n or "reduce3" in n else
         "prelu" if "prelu" in n else
         "resample" if "resample" in n else
         "torch:" + n.split("(")[0].split("<")[0].split("::")[-1][:40] if ("at::" in n or "native" in n) else
         n.split("(")[0][:48])
    fam[k] += (e - s) / 1e9
    cnt[k] += 1
    short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]
    kern[short] += (e - s) / 1e9
    kcnt[short] += 1
print(f"dispatches {len(rows)}  span {span:.3f}s  busy {busy:.3f}s  idle {span - busy:.3f}s")
print("-- by family")
for k, v in fam.most_common(25):
    print(f"{v:8.3f}s {100 * v / busy:5.1f}%  {cnt[k]:7d}  {k}")
print("-- by kernel")
for k, v in kern.most_common(a.top):
    print(f"{v:8.3f}s {100 * v / busy:5.1f}%  {kcnt[k]:7d}  {1e6 * v / kcnt[k]:9.1f}us  {k}")
