"""C-ABI library: loads, exports every symbol include/classmate_hip.h declares,
and the ctypes binding covers them.  No compute calls (CPU-only container)."""
import re
import subprocess
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
HEADER = REPO / "include" / "classmate_hip.h"
LIB = REPO / "classmate-rag_amd" / "classmate_hip" / "libclassmate_hip.so"


def declared():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(cm_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (cm_[a-z0-9_]+)", out))
    missing = [s for s in declared() if s not in exported]
    assert not missing, missing


def test_ctypes_binding_covers_header():
    from classmate_hip import _lib
    assert sorted(_lib.SIGNATURES) == declared()
    assert _lib.fn["cm_version"]() >= 100
    assert _lib.max_topk() == 256


def test_gpu_object_is_gfx950():
    # the device code object is embedded in .hip_fatbin; its target id names the arch
    data = LIB.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_errors_map_to_python_exceptions():
    import ctypes
    import pytest
    from classmate_hip import _lib
    h = ctypes.c_void_p()
    rc = _lib.fn["cm_dense_create"](0, 0, 0, ctypes.byref(h))     # dim 0 -> EINVAL before any HIP call
    with pytest.raises(ValueError):
        _lib.check(rc)
    assert "dim" in _lib.last_error()
