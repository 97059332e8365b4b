#!/usr/bin/env python3
"""Kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage remarks.

    python tools/resource_usage.py mm-vae_amd/csrc/nb_kernels.hip [filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-munsafe-fp-atomics",
       "-I/opt/rocm/include", "-c", src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", "-n", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>3} vspill {r.get('VGPRs Spill','?'):>4} "
              f"sspill {r.get('SGPRs Spill','?'):>4} occ {r.get('Occupancy [waves/SIMD]','?')}  {r['name'][:150]}")
