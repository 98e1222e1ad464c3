#!/usr/bin/env python3
"""VGPR / scratch / occupancy per kernel of one HIP source (compile-time,
-Rpass-analysis=kernel-resource-usage).  python tools/resusage.py csrc/hip/sgd.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-ffp-contract=fast", *(["-mllvm", "-amdgpu-mfma-vgpr-form"] if src.endswith("kmeans.hip") else []),
       "-Wno-unused-result", "-fvisibility=hidden", "-I/opt/rocm/include", "-Icsrc", "-x", "hip", "-c", src,
       "-o", "/tmp/resusage.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    if "error" in line:
        print(line)
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    name = re.sub(r"^_ZN5twtml\d+", "", k)
    name = re.sub(r"EEEvNS_.*$", "", name)
    if flt in name:
        print(f"{name:48s} vgpr {v.get('VGPRs', '?'):>4} agpr {v.get('AGPRs', '?'):>3} "
              f"scratch {v.get('ScratchSize', '?'):>4} occ {v.get('Occupancy', '?')}")
