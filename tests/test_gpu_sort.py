"""The library's device radix sort (gc_sort.hip, through gc_test_radix_sort) against NumPy's stable
argsort: the order the PrimitiveMap cull / insert / merge and the map view rely on (primitive_map.py
:1222-1229 top-k by weight, the insert's replacement order, the merge's ascending pair distances). Keys
ascending or descending, equal keys (and -0.0 / +0.0) in input order, values permuted alike, keys
returned bit for bit, within equal-length segments; sizes around the 2048-key tile."""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-slam_amd"))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from gcslam import _abi
    c = _abi.Context(0)
    yield c
    c.close()


def _keys(rng, n, kind):
    if kind == "ties":  # few distinct values, both zeros, both infinities, subnormals
        pool = np.array([0.0, -0.0, 1.0, -1.0, 2.5, -2.5, np.inf, -np.inf, 5e-324, -5e-324, 1e300, -1e300])
        return pool[rng.integers(0, pool.size, n)]
    if kind == "wide":
        return rng.standard_normal(n) * 10.0 ** rng.integers(-300, 300, n)
    return np.round(rng.standard_normal(n), 2)  # "rounded": many duplicates among ordinary values


def _expect(keys, vals, n_seg, L, desc):
    ko, vo = np.empty_like(keys), np.empty_like(vals)
    for g in range(n_seg):
        k = keys[g * L:(g + 1) * L]
        perm = np.argsort(-k if desc else k, kind="stable")
        ko[g * L:(g + 1) * L] = k[perm]
        vo[g * L:(g + 1) * L] = vals[g * L:(g + 1) * L][perm]
    return ko, vo


def _run(ctx, keys, vals, n_seg, L, desc):
    from gcslam import _abi
    dk = _abi.DeviceArray.from_host(ctx, keys)
    dko = _abi.DeviceArray(ctx, keys.shape)
    dv = _abi.DeviceArray.from_host(ctx, vals, np.uint32) if vals is not None else None
    dvo = _abi.DeviceArray(ctx, keys.shape, np.uint32) if vals is not None else None
    _abi.call("gc_test_radix_sort", ctx.handle, dk.ptr, dv.ptr if dv else None, n_seg, L, 1 if desc else 0, dko.ptr,
              dvo.ptr if dvo else None, ctx=ctx)
    return dko.download(), (dvo.download() if dvo else None)


@pytest.mark.parametrize("L", [1, 7, 2047, 2048, 2049, 5000, 70001])
@pytest.mark.parametrize("n_seg", [1, 3])
@pytest.mark.parametrize("desc", [False, True])
@pytest.mark.parametrize("kind", ["ties", "wide", "rounded"])
def test_radix_sort_matches_stable_argsort(ctx, L, n_seg, desc, kind):
    rng = np.random.default_rng(L * 7 + n_seg * 3 + int(desc) + len(kind))
    keys = _keys(rng, n_seg * L, kind)
    vals = np.arange(n_seg * L, dtype=np.uint32) ^ np.uint32(0x5A5A5A5A)
    ko, vo = _run(ctx, keys, vals, n_seg, L, desc)
    ek, ev = _expect(keys, vals, n_seg, L, desc)
    np.testing.assert_array_equal(ko.view(np.uint64), ek.view(np.uint64))  # the keys' bits, -0.0 kept
    np.testing.assert_array_equal(vo, ev)


@pytest.mark.parametrize("desc", [False, True])
def test_radix_sort_keys_only(ctx, desc):
    rng = np.random.default_rng(11)
    keys = _keys(rng, 9000, "wide")
    ko, _ = _run(ctx, keys, None, 1, keys.size, desc)
    ek, _ = _expect(keys, np.zeros(keys.size, np.uint32), 1, keys.size, desc)
    np.testing.assert_array_equal(ko.view(np.uint64), ek.view(np.uint64))


def test_radix_sort_rejects_bad_sizes(ctx):
    from gcslam import _abi
    with pytest.raises(ValueError):
        _abi.call("gc_test_radix_sort", ctx.handle, None, None, 1 << 20, 1 << 13, 0, None, None, ctx=ctx)
