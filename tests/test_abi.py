"""C-ABI surface checks that need no GPU: the library loads and exports every entry point
include/gcslam.h declares; the Python binding covers them; argument errors map to ValueError."""

import os
import re
import ctypes

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gcslam.h")
LIB = os.path.join(ROOT, "fl-slam_amd", "gcslam", "libgcslam.so")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|const char\*)\s+(gc_[a-z0-9_]+)\s*\(", txt, re.M)))


def test_header_declares_entries():
    names = declared()
    assert "gc_ctx_create" in names and "gc_scan_bins_fused" in names
    assert len(names) >= 20


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgcslam.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    from gcslam import _abi
    names = set(declared()) - {"gc_last_error"}
    assert names <= set(_abi.SIGNATURES), sorted(names - set(_abi.SIGNATURES))


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgcslam.so not built")
def test_version_and_null_ctx_errors():
    from gcslam import _abi
    assert _abi.lib().gc_version() >= 10000
    with pytest.raises(ValueError):
        _abi.check(_abi.lib().gc_ctx_synchronize(None))
