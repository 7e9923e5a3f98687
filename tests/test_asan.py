"""Sanitizers on the host code (GPU sanitizers are not available on this pool):
tools/asan_check.sh builds the C oracle and libclassmate_hip's host side with ASan + UBSan and runs
(1) a seeded driver through every oracle entry point, (2) a driver through every C-ABI entry
point's validation / error paths, (3) the C-oracle pytest cases with the sanitized oracle loaded
into Python.  Any sanitizer report fails the script (halt_on_error)."""
import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("gcc") is None or not Path("/opt/rocm/bin/hipcc").exists(),
                    reason="needs gcc and hipcc")
def test_host_code_under_asan_ubsan():
    r = subprocess.run(["bash", str(REPO / "tools" / "asan_check.sh")], capture_output=True, text=True,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "oracle under ASan/UBSan: OK" in out and "host ABI validation paths: OK" in out
    assert "runtime error" not in out and "ERROR: AddressSanitizer" not in out
