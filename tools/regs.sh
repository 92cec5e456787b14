#!/bin/bash
# Register usage / spills / occupancy per kernel of one unit:  tools/regs.sh UNIT "-DFLAGS..."
cd /tmp && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC $2 -Rpass-analysis=kernel-resource-usage \
  -c /root/repo/-gan-_amd/csrc/$1.hip -o /tmp/regs_$$.o 2>&1 | python3 -c '
import sys, re, subprocess
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"remark: ([A-Za-z ]+): (\S+)", line)
    if not m: continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}; rows.append(cur)
    elif cur is not None: cur[k] = v
for r in rows:
    n = re.sub(r"\(.*", "", r["name"]).replace("ganamd_patch::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    print(f"{n[:80]:80s} V{r.get(\"VGPRs\",\"?\"):>4} A{r.get(\"AGPRs\",\"?\"):>4} spillV{r.get(\"VGPRs Spill\",\"?\"):>4} occ{r.get(\"Occupancy [waves/SIMD]\",\"?\")} lds{r.get(\"LDS Size [bytes/block]\",\"?\")}")
'
rm -f /tmp/regs_$$.o
