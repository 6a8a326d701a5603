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


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgcslam.so not built")
def test_packed_map_record_layout():
    """gc_primitive_map_record_layout (host-only): the fuse's read-modify-write fields in the first
    two 128-B lines of a 128-B-multiple record, no two fields overlapping, any lobe count; the Python
    map struct matches the header's field order and size."""
    import numpy as np
    from gcslam import _abi
    from gcslam.primitive_map import _MapStruct
    widths = lambda L: [72, 24, 24 * L, 8, 8, 8, 8, 8, 8, 24, 8, 24, 24, 1, 8, 8]  # struct field order
    for L in range(1, 9):
        off = np.zeros(16, np.int64)
        sb = ctypes.c_int64(0)
        _abi.call("gc_primitive_map_record_layout", L, off.ctypes.data, ctypes.byref(sb))
        w = widths(L)
        spans = sorted((int(o), int(o) + w[k]) for k, o in enumerate(off))
        assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])), (L, spans)
        assert sb.value % 128 == 0 and spans[-1][1] <= sb.value
        if L <= 3:  # Λ θ η w stamp seqs cam lidar accum denom: the first two lines
            assert max(int(off[k]) + w[k] for k in range(11)) <= 256
        # rgb and colors each own a whole 32-B sector (the fuse writes them as such)
        assert off[11] % 32 == 0 and off[12] % 32 == 0 and off[12] - off[11] >= 32
        assert all(not (off[11] < o < off[11] + 32 or off[12] < o < off[12] + 32) for o in off)
    with pytest.raises(ValueError):
        _abi.call("gc_primitive_map_record_layout", 9, off.ctypes.data, ctypes.byref(sb))
    # int64 m_slots, int32 n_lobes, int32 colors_current, 16 pointers, int64 slot_bytes
    assert ctypes.sizeof(_MapStruct) == 8 + 4 + 4 + 16 * 8 + 8
