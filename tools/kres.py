#!/usr/bin/env python3
"""Per-kernel resource usage (VGPRs, SGPR/VGPR spills, scratch, occupancy, LDS) of a HIP
source for gfx950, from the compiler's kernel-resource-usage remarks.
usage: tools/kres.py csrc/encode.hip [-DFOO=1 ...] [--filter seg]"""
import re
import subprocess
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--filter")]
flt = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--filter=")), "")
src, defs = args[0], args[1:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-DTKZ_MAXB=24",
       "-Wno-unused-result", "-Wno-unused-value", "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage", *defs]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1).split(" [")[0], m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
print(f"{'kernel':60s} {'VGPR':>5s} {'SGPR':>5s} {'sSpill':>6s} {'vSpill':>6s} {'scr':>5s} {'occ':>4s} {'LDS':>6s}")
for r in rows:
    n = re.sub(r"\(.*", "", r["name"]).replace("tkz::", "")
    if flt and flt not in n:
        continue
    print(f"{n[:60]:60s} {r.get('VGPRs','?'):>5s} {r.get('TotalSGPRs','?'):>5s} {r.get('SGPRs Spill','?'):>6s} "
          f"{r.get('VGPRs Spill','?'):>6s} {r.get('ScratchSize','?'):>5s} {r.get('Occupancy','?'):>4s} {r.get('LDS Size','?'):>6s}")
