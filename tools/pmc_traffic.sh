#!/bin/bash
# HBM traffic of bench.py's roofline kernel -- the dominant one, the split6 LDS-patch conv
# conv_patch_x3_kernel<96,...,5,64,true,false>: G13_5's modulated conv fwd 96->96 5x5 64x64 at bench.py's
# whole-tile probe batches (the iteration's launch mix) -- from rocprofv3 PMC counters, one counter per pass (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950).  FETCH_SIZE is doubled (gfx950 reports half the bytes
# of wide coalesced reads: MI355X_MICROARCH.md, HBM section).  Writes profiles/roofline_traffic.json.
set -e
export TMPDIR=/tmp
# the probe's batches: bench.py's launch mix of the dominant shape (DOMINANT_MIX), each at the planner's
# whole-tile batch
BS=$(python3 -c "import bench, gan_amd.ops as ops; print(' '.join(str(bench._whole_tile_geo(ops, dict(bench.PROBES['dominant'], B=b))[0].B) for b in bench.DOMINANT_MIX))" 2>/dev/null | tail -1)
for B in $BS; do
  ARGS="--op fwd --B $B --cin 96 --H 64 --cout 96 --k 5 --pad 2 --scaled --reps 5"
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf /tmp/pmc_${C}_$B
    timeout -k 10 300 rocprofv3 --pmc $C -d /tmp/pmc_${C}_$B -o run --output-format csv -- python3 tools/gemm_micro.py $ARGS > /dev/null 2>&1
  done
done
BS="$BS" python3 - <<'PY'
import csv, glob, json, os
per_batch = {}
for B in map(int, os.environ["BS"].split()):
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"/tmp/pmc_{c}_{B}/**/*counter_collection.csv", recursive=True)[0]
        rows = [r for r in csv.DictReader(open(f)) if "conv_patch_x3_kernel<96, " in r["Kernel_Name"]]
        per = {}
        for r in rows:
            per.setdefault(r["Dispatch_Id"], 0.0)
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        vals[c] = sum(per.values()) / len(per)          # KiB per dispatch
    fetch_b = 2 * vals["FETCH_SIZE"] * 1024
    write_b = vals["WRITE_SIZE"] * 1024
    # x read + packed W read + x/y scales + y write, once
    alg = 4 * (96 * B * 64 * 64 + 96 * 96 * 25 + 2 * 96 * B + 96 * B * 64 * 64)
    per_batch[str(B)] = {"bytes_per_launch": fetch_b + write_b, "fetch_bytes_x2": fetch_b, "write_bytes": write_b,
                         "raw_kib_per_dispatch": vals, "algorithmic_bytes": alg}
out = {"kernel": "conv_patch_x3_kernel<96,...,5,64,true,false>", "per_batch": per_batch,
       "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes per batch), tools/pmc_traffic.sh; "
                 "FETCH doubled per the gfx950 correction"}
json.dump(out, open("gpurun_out/roofline_traffic.json", "w"), indent=1)
print(json.dumps(out))
PY
