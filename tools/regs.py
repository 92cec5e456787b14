"""Register usage / spills / occupancy per kernel of one unit:  python tools/regs.py UNIT [-DFLAGS...]"""
import os
import re
import subprocess
import sys

src = f"/root/repo/-gan-_amd/csrc/{sys.argv[1]}.hip"
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", *sys.argv[2:],
                      "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", f"/tmp/regs_{os.getpid()}.o"],
                     capture_output=True, text=True, cwd="/tmp").stderr
os.remove(f"/tmp/regs_{os.getpid()}.o")
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: ([A-Za-z \[\]/]+): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    n = re.sub(r"\(.*", "", r["name"].replace("(anonymous namespace)::", "")).replace("void ", "")
    g = r.get
    print(f"{n[:78]:78s} V{g('VGPRs', '?'):>4} A{g('AGPRs', '?'):>4} spill{g('VGPRs Spill', '?'):>4} "
          f"occ {g('Occupancy [waves/SIMD]', '?')} lds {g('LDS Size [bytes/block]', '?')}")
