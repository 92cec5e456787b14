# fp32 MFMA ceiling on random vs constant operands (in-kernel clock), and the MFMA-busy counter
# calibrated on that probe vs the conv roofline-probe launch.
set -e
export TMPDIR=/tmp
timeout -k 10 120 tools/variants/mfma_peak_rand > gpurun_out/mfma_ceiling.txt 2>&1
cat gpurun_out/mfma_ceiling.txt
rm -rf /tmp/pmc_peak /tmp/pmc_conv
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d /tmp/pmc_peak -o run --output-format csv -- tools/variants/mfma_peak_rand > /dev/null 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d /tmp/pmc_conv -o run --output-format csv -- python3 tools/gemm_micro.py --op fwd --B 96 --cin 128 --H 32 --cout 128 --k 3 --pad 1 --reps 5 > /dev/null 2>&1
python3 - <<'PY' | tee -a gpurun_out/mfma_ceiling.txt
import csv, glob, collections
for d in ("/tmp/pmc_peak", "/tmp/pmc_conv"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        k = r["Dispatch_Id"]
        names[k] = r["Kernel_Name"][:60]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k in list(per)[-3:]:
        print(d, names[k], dict(per[k]))
PY
