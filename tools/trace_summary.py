"""Summarise a rocprofv3 kernel trace CSV: busy vs span, and time by kernel family."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0        # drop the first N dispatches (init)
rows = rows[skip:]
st = [int(r["Start_Timestamp"]) for r in rows]
en = [int(r["End_Timestamp"]) for r in rows]
span = (max(en) - min(st)) / 1e9
busy = sum(e - s for s, e in zip(st, en)) / 1e9
fam = collections.Counter()
cnt = collections.Counter()
for r, s, e in zip(rows, st, en):
    n = r["Kernel_Name"]
    k = ("gemm" if ("conv_gemm" in n or "wgrad_gemm" in n) else
         "split_reduce" if "split_reduce" in n else
         "bn" if "bn_" in n or "reduce3" in n else
         "prelu" if "prelu" in n else
         "resample" if "resample" in n else
         "torch:" + n.split("(")[0].split("<")[0].split("::")[-1][:40] if ("at::" in n or "native" in n) else
         n.split("(")[0][:48])
    fam[k] += (e - s) / 1e9
    cnt[k] += 1
print(f"dispatches {len(rows)}  span {span:.3f}s  busy {busy:.3f}s  idle {span - busy:.3f}s")
for k, v in fam.most_common(25):
    print(f"{v:8.3f}s {100 * v / busy:5.1f}%  {cnt[k]:7d}  {k}")
