"""CPU: register budget of the hot scan kernels in the built libhiprag.so (gfx950 code-object metadata, read by
tools/kernel_resources.py -- no GPU needed).

The FILTER kernels run two waves per SIMD and sit at (or near) the 256-VGPR limit, where the register allocator's
choices flip with unrelated edits: in round 4 removing a few lines of diagnostics made k_scan_filter spill 42 VGPRs
to scratch inside its tile loop and cost 9 % at 1.25M rows.  A VGPR spill in these kernels fails here, on the CPU,
before it reaches a GPU.  (SGPR spills go to VGPR lanes and are not scratch traffic.)
"""
import os
import re
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "youtu-rag_amd", "hiprag", "libhiprag.so")
sys.path.insert(0, os.path.join(REPO, "tools"))

pytestmark = pytest.mark.skipif(not os.path.exists(LIB) or not shutil.which("/opt/rocm/lib/llvm/bin/llvm-readelf"),
                                reason="libhiprag.so or the ROCm LLVM tools are missing")

# kernels that must not spill VGPRs at all, and the 128-query FILTER's known spills (not to grow)
NO_SPILL = re.compile(r"k_scan_(filter|sample|collect|persist)")
WIDE = re.compile(r"k_filter_wide8")
Q256 = re.compile(r"k_filter_q256")


@pytest.fixture(scope="module")
def resources():
    from kernel_resources import kernel_resources

    return kernel_resources(LIB)


def test_scan_kernels_do_not_spill(resources):
    hot = {k: v for k, v in resources.items() if NO_SPILL.search(k)}
    assert len(hot) >= 40, sorted(hot)  # every instantiation was found
    spilled = {k: v["vgpr_spill_count"] for k, v in hot.items() if v.get("vgpr_spill_count", 0)}
    assert not spilled, spilled
    persist = [v for k, v in hot.items() if "k_scan_persist" in k]
    assert len(persist) == 4


def test_wide_filter_spills_bounded(resources):
    wide = {k: v for k, v in resources.items() if WIDE.search(k)}
    assert len(wide) == 32, sorted(wide)
    worst = max(v.get("vgpr_spill_count", 0) for v in wide.values())
    assert worst <= 35, worst


def test_q256_filter_does_not_spill(resources):
    """The 256-query FILTER holds 256 accumulators in AGPRs and the corpus ring in VGPRs at one wave per SIMD: its
    first builds spilled the ring to scratch (a rolled span loop) and then the accumulators (the register allocator
    copying whole accumulators out of the AGPRs ahead of the epilogue) -- neither may come back."""
    q = {k: v for k, v in resources.items() if Q256.search(k)}
    assert len(q) == 16, sorted(q)  # bf16 / f16 rows + fp32 rows with either MFMA type, 4 depths each
    spilled = {k: v.get("vgpr_spill_count", 0) for k, v in q.items() if v.get("vgpr_spill_count", 0)}
    assert not spilled, spilled
    assert all(v.get("private_segment_fixed_size", 0) == 0 for v in q.values()), q


def test_no_bit_cast_of_a_vector_element():
    """hipcc (ROCm 7.2 clang) lowers __builtin_bit_cast(float, v[c]) -- v an ext_vector_type -- to v[0] for every c
    (it loads only that dword).  The first 256-query FILTER read its per-query thresholds that way and compared every
    register against one query's threshold; bit_cast the whole vector, then index.  No source may use the form."""
    import glob

    pat = re.compile(r"__builtin_bit_cast\(\s*(float|u?int32_t|int|unsigned)\s*,\s*[A-Za-z_][A-Za-z_0-9]*\s*(\[[^\]]+\])+\s*\)")
    csrc = os.path.join(REPO, "youtu-rag_amd", "csrc")
    hits = []
    for f in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp")):
        for i, line in enumerate(open(f), 1):
            if pat.search(line):
                hits.append(f"{os.path.basename(f)}:{i}: {line.strip()}")
    assert not hits, hits
