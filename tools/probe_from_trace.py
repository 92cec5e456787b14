"""The roofline probes' launches in a rocprofv3 kernel trace of bench.py.

bench.py times each roofline kernel (PROBES in bench.py) with 3 warm-up + 20 individually-timed
+ 20 back-to-back launches -- the dominant one at each batch of its launch mix (DOMINANT_MIX).  Other launches of those kernels with the same grid exist (the
iteration's own, the census' 6-launch runs), so a probe is the longest run of >= 20 consecutive
dispatches (by start time) of that kernel and grid; its launches after the first 3 are averaged.

    python tools/probe_from_trace.py TRACE.csv[.gz] [--mix=256:10,64:20]
"""
import csv
import gzip
import sys

PROBES = [  # (kernel name as rocprof prints it, threads per block, images per launched block, GFLOP per image,
    # label); the probe batch is the one bench.py picks at run time (_whole_tile_geo), read back from the grid
    ("conv_patch_x3_kernel<96, 12, 512, 5, 64, true, false>", 768, 1 / 8, 2.0 * 64 * 64 * 96 * 96 * 25 / 1e9,
     "dominant: G13_5 modulated conv fwd 96->96 5x5 64x64 (split6 LDS-patch conv, 12 waves)"),
    ("conv_patch_x3_kernel<96, 8, 512, 5, 64, true, false>", 512, 1 / 8, 2.0 * 64 * 64 * 96 * 96 * 25 / 1e9,
     "dominant: G13_5 modulated conv fwd 96->96 5x5 64x64 (split6 LDS-patch conv, 8 waves)"),
    ("conv_gemm_kernel<128, 128, 2, 2, 1, false, false>", 256, 128 / (32 * 32), 2.0 * 32 * 32 * 128 * 128 * 9 / 1e9,
     "critic probe: D9_4 conv fwd 128->128 3x3 32x32"),
]
PEAK = 157.3 * 16 / 6      # the split6 pipe (bench.py SPLIT6_PIPE_PEAK_TFLOPS)

path = sys.argv[1]
# the dominant kernel's launch mix {batch: launches per iteration} (bench.py DOMINANT_MIX)
MIX = {256: 10, 64: 20}
for a in sys.argv[2:]:
    if a.startswith("--mix="):
        MIX = {int(k): int(v) for k, v in (x.split(":") for x in a[6:].split(","))}
rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for kernel, threads, per_block, gflop_img, label in PROBES:
    best, run = {}, []            # grid -> longest run of consecutive launches at that grid

    def close(run):
        if run and len(run) > len(best.get(run[0]["Grid_Size_X"], [])):
            best[run[0]["Grid_Size_X"]] = run
    for r in rows:
        if kernel in r["Kernel_Name"] and (not run or r["Grid_Size_X"] == run[0]["Grid_Size_X"]):
            run.append(r)
        elif kernel in r["Kernel_Name"]:
            close(run)
            run = [r]
        else:
            close(run)
            run = []
    close(run)
    found = {}
    for grid, b in sorted(best.items(), key=lambda kv: -int(kv[0])):
        if len(b) < 20:
            continue
        blocks = int(grid) // threads
        B = round(blocks * per_block)
        gflop = gflop_img * B
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in b[3:]]
        avg = sum(d) / len(d)
        found[B] = (gflop, avg)
        print(f"{label}: {kernel} at {blocks} blocks (B={B}), {len(d)} launches (run of {len(b)}, first 3 skipped)")
        print(f"  average {avg:.1f} us  min {min(d):.1f}  max {max(d):.1f}  -> {gflop / avg * 1e3:.1f} TF/s "
              f"({gflop:.2f} GFLOP per launch), {gflop / avg * 1e3 / PEAK:.3f} of the split6 pipe {PEAK:.1f}, "
              f"{gflop / avg * 1e3 / 157.3:.3f} of the fp32 MFMA peak 157.3")
    if not found:
        print(f"{label}: no run of >= 20 consecutive launches of {kernel}")
    elif label.startswith("dominant") and all(b in found for b in MIX):
        n = sum(MIX.values())
        gf = sum(MIX[b] * found[b][0] for b in MIX) / n
        us = sum(MIX[b] * found[b][1] for b in MIX) / n
        print(f"  launch mix {MIX}: average launch {gf:.2f} GFLOP in {us:.1f} us -> {gf / us * 1e3:.1f} TF/s, "
              f"{gf / us * 1e3 / PEAK:.3f} of the split6 pipe")
