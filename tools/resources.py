#!/usr/bin/env python3
"""Per-kernel resource usage of one HIP source (VGPRs, spills, LDS, occupancy) from the
compiler's kernel-resource-usage remarks:
    python tools/resources.py csrc/fft3.hip [name filter] [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-fno-slp-vectorize", "-I../include", "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"]
cmd += sys.argv[3:]
out = subprocess.run(cmd, capture_output=True, text=True, cwd="ocean-simulation_amd").stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        cur = {"name": re.sub(r"ocean::\(anonymous namespace\)::", "", dm).split("(")[0]}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        print(f'{r["name"]:60s} VGPR {r.get("VGPRs", "?"):>4} AGPR {r.get("AGPRs", "?"):>3} '
              f'spill {r.get("VGPRs Spill", "?"):>3} LDS {r.get("LDS Size [bytes/block]", "?"):>6} '
              f'occ {r.get("Occupancy [waves/SIMD]", "?")}')
