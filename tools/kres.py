#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per kernel."""
import re, subprocess, sys
src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
       "-Icsrc/kernels", "-c", src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None; rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark: +([A-Za-z /\[\]]+): (\S+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for k, v in rows.items():
    if filt in k:
        dm = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
        print(f"{dm[:90]:90s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} spill={v.get('VGPRs Spill')} scratch={v.get('ScratchSize [bytes/lane]')} occ={v.get('Occupancy [waves/SIMD]')} lds={v.get('LDS Size [bytes/block]')}")
