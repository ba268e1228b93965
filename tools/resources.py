"""Kernel resource table (VGPRs, scratch, occupancy) of libhiprag's kernels: python tools/resources.py [filter]"""
import os
import re
import subprocess
import sys

src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "youtu-rag_amd", "csrc")
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "hr_index.hip", "-o",
                      "/tmp/hr_index_res.o", "-Rpass-analysis=kernel-resource-usage"], cwd=src, capture_output=True,
                     text=True).stderr
rows, cur = [], None
keys = {"VGPRs": "vgpr", "ScratchSize [bytes/lane]": "scratch", "Occupancy [waves/SIMD]": "occ", "VGPRs Spill": "vspill"}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for k, short in keys.items():
        m = re.search(re.escape(k) + r": (\d+)", line)
        if m and cur is not None and short not in cur:
            cur[short] = m.group(1)
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:52]:52s} vgpr={r.get('vgpr')} scratch={r.get('scratch')} occ={r.get('occ')} "
              f"vspill={r.get('vspill')}")
