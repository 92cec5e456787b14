"""The roofline probe's launches in a rocprofv3 kernel trace of bench.py.

bench.py's probe issues 3 + 20 back-to-back launches of conv_gemm_kernel<128,128,2,2,1,false,false>
at 768 blocks (D9_4's 128->128 3x3 conv at 32x32, B=96).  Other launches of that kernel can have
768 blocks too (split-K tails, the census' 5-launch runs), so the probe is the run of >= 20
consecutive dispatches (by start time) of that kernel and grid; its last 20 are averaged.

    python tools/probe_from_trace.py TRACE.csv[.gz]
"""
import csv
import gzip
import sys

KERNEL = "conv_gemm_kernel<128, 128, 2, 2, 1, false, false>"
path = sys.argv[1]
rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
best = []
run = []
for r in rows:
    if KERNEL in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 768 * 256:
        run.append(r)
    else:
        if len(run) >= 20:
            best = run
        run = []
if len(run) >= 20:
    best = run
if not best:
    sys.exit("no run of >= 20 consecutive probe launches in the trace")
last = best[-20:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in last]
avg = sum(d) / len(d)
print(f"roofline probe: the last 20 of a run of {len(best)} back-to-back dispatches of {KERNEL} at 768 blocks")
print(f"average {avg:.1f} us  min {min(d):.1f}  max {max(d):.1f}  -> {28.991029248e9 / (avg * 1e-6) / 1e12:.1f} TF/s "
      f"(28.99 GFLOP per launch), {28.991029248e9 / (avg * 1e-6) / 1e12 / 157.3:.3f} of 157.3")
