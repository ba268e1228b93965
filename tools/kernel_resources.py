"""Per-kernel register and spill counts of the built libhiprag.so, read from its gfx950 code objects' metadata.

The library's .hip_fatbin section holds one clang offload bundle per translation unit; each bundle's gfx950 code
object carries the AMDHSA metadata note (.vgpr_count, .vgpr_spill_count, .sgpr_spill_count, ...) of its kernels.
Used by tests/test_kernel_resources.py: the scan kernels sit at the 256-VGPR limit of two waves per SIMD, where the
register allocator's choices flip with unrelated edits -- a scratch spill in the FILTER's tile loop cost 9 % at
1.25M rows (round 4) -- so a spill must fail the CPU suite, not show up on the GPU.
Usage: python tools/kernel_resources.py [libhiprag.so] [name-regex]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def kernel_resources(lib: str) -> dict[str, dict]:
    """{kernel symbol: {"vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "agpr_count"}} over every bundle."""
    out: dict[str, dict] = {}
    with tempfile.TemporaryDirectory() as td:
        sec = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={sec}", lib, os.path.join(td, "x")],
                       check=True, capture_output=True)
        data = open(sec, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, a in enumerate(starts):
            b = starts[i + 1] if i + 1 < len(starts) else len(data)
            bun, co = os.path.join(td, f"b{i}"), os.path.join(td, f"c{i}.o")
            open(bun, "wb").write(data[a:b])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={bun}",
                                f"--targets={TARGET}", f"--output={co}", "--allow-missing-bundles"], capture_output=True)
            if r.returncode or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            cur = None
            for line in notes.splitlines():
                m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
                if not m:
                    continue
                key, val = m.groups()
                if key == "name" and not val.endswith(".kd"):
                    cur = out.setdefault(val, {})
                elif cur is not None and key in ("vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "agpr_count",
                                                     "private_segment_fixed_size"):
                    cur[key] = int(val)
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                             "youtu-rag_amd", "hiprag", "libhiprag.so")
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for name, r in sorted(kernel_resources(lib).items()):
        if pat.search(name):
            print(f"{r.get('vgpr_count', '?'):>4} vgpr  {r.get('vgpr_spill_count', '?'):>3} vspill  "
                  f"{r.get('sgpr_spill_count', '?'):>4} sspill  {name}")
