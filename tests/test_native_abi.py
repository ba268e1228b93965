"""CPU: libhiprag.so loads and exports every entry point include/hiprag.h (the drop-in boundary) and
include/hiprag_diag.h (diagnostics) declare (no compute call is made without a GPU)."""
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "hiprag.h")
DIAG_HEADER = os.path.join(REPO, "include", "hiprag_diag.h")


def _decls(path):
    return set(re.findall(r"^\s*(?:int|void|const char\*)\s+(hr_\w+)\s*\(", open(path).read(), re.M))


def declared_symbols():
    return sorted(_decls(HEADER) | _decls(DIAG_HEADER))


def test_header_declares_the_abi():
    syms = declared_symbols()
    assert "hr_index_search" in syms and "hr_merge_candidates" in syms and len(syms) >= 20
    # the boundary header holds no diagnostics, and no symbol is declared twice
    boundary, diag = _decls(HEADER), _decls(DIAG_HEADER)
    assert not boundary & diag
    assert {"hr_index_debug_approx", "hr_index_last_candidates", "hr_index_set_scan_timing", "hr_index_wave_tiles",
            "hr_index_persist_trace"} <= diag


def test_library_exports_every_declared_symbol():
    from hiprag import _native

    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libhiprag.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {line.split()[-1] for line in out.stdout.splitlines() if line.strip()}
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    assert sorted(_native.EXPORTS) == declared_symbols()


def test_library_loads_and_reports_errors():
    from hiprag import _native

    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libhiprag.so not built")
    L = _native.load_library()
    assert L.hr_abi_version() == 2
    assert [L.hr_kc_for_k(k) for k in range(1, _native.HR_MAX_K + 1)] == \
        [_native.kc_for_k(k) for k in range(1, _native.HR_MAX_K + 1)]
    assert _native.kc_for_k(_native.HR_MAX_K) <= _native.HR_MAX_KC and _native.kc_for_k(45) == 96 and _native.kc_for_k(100) == 160
    assert _native.kc_for_k(10) == 32 and _native.kc_for_k(32) == 64 and _native.kc_for_k(128) == 192
    for dim in (64, 1024, 1100, 2000, 2048, 2304):
        assert [L.hr_kc_for_k_dim(k, dim) for k in range(1, _native.HR_MAX_K + 1)] == \
            [_native.kc_for_k(k, dim) for k in range(1, _native.HR_MAX_K + 1)]
    assert _native.kc_for_k(10, 2304) == 32 and _native.kc_for_k(16, 2304) == 64 and _native.kc_for_k(64, 2304) == 128 and _native.kc_for_k(128, 2304) == 256
    with pytest.raises(ValueError):  # argument validation happens before any device call
        _native.NativeIndex(0, "bf16", "cosine")
    with pytest.raises(ValueError):
        _native.NativeIndex(64, "int8", "cosine")
