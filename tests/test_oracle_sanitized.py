"""CPU: the oracle restatement (hr_oracle.c) built with AddressSanitizer + UBSan (oracle/Makefile
target ``asan``) and driven over its edge cases by oracle/asan_driver.c in a child process: no
sanitizer finding, synthetic and stored searches bit-identical (SURVEY §5 "Race detection /
sanitizers")."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "asan"], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([os.path.join(REPO, "oracle", "_build", "hr_oracle_asan")], env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all consistent" in p.stdout
    assert "AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr
