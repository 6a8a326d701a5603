"""Device-resident PrimitiveMap and its operators (backend/structures/primitive_map.py):
primitive_map_fuse (:992-1163) with the world pushforward of transform_gaussian_to_world
(backend/pipeline.py:1248-1256) fused in (the C5 map update), and the maintenance operators
primitive_map_insert_masked (:807-982), primitive_map_cull (:1175-1305), primitive_map_forget
(:1314-1390), primitive_map_recency_inflate (:1400-1490) and primitive_map_merge_reduce
(:1809-2030). The map lives in HBM as one flat array of n_tiles * m_tile slots (tile t, local
slot j -> t * m_tile + j); every operator runs in place on its tile. The AtlasMap bookkeeping
(next_global_id, total_count, per-tile count) stays on the host, as in the reference."""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import _abi
from .certificates import CertBundle, ExpectedEffect, InfluenceCert
from .constants import (GC_CHART_ID, GC_EPS_LIFT, GC_EPS_MASS, GC_EPS_PSD, GC_K_MERGE_PAIRS_PER_TILE,
                        GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD, GC_PRIMITIVE_FORGETTING_FACTOR,
                        GC_PRIMITIVE_MERGE_MAX_TILE_SIZE, GC_PRIMITIVE_MERGE_THRESHOLD, GC_RECENCY_DECAY_LAMBDA,
                        GC_RECENCY_MIN_SCALE)

GC_VMF_N_LOBES = 3

_F64 = ("Lambdas", "thetas", "etas", "weights", "timestamps")
_I64 = ("last_supported_scan_seq", "last_update_scan_seq")
_COL = ("cam_mass", "lidar_mass", "rgb_cam_accum", "rgb_cam_denom", "rgb", "colors")
_MAINT = ("valid_mask", "created_timestamps", "primitive_ids")


class _MapStruct(C.Structure):
    _fields_ = [("m_slots", C.c_int64), ("n_lobes", C.c_int32), ("colors_current", C.c_int32)] + \
               [(k, C.c_void_p) for k in _F64 + _I64 + _COL + _MAINT] + [("slot_bytes", C.c_int64)]


class _InsertStruct(C.Structure):
    _fields_ = [("K", C.c_int64)] + [(k, C.c_void_p) for k in (
        "Lambdas", "thetas", "etas", "weights", "valid_mask", "colors", "sources")]


class _FuseStruct(C.Structure):
    _fields_ = [("K", C.c_int64)] + [(k, C.c_void_p) for k in (
        "target_slots", "Lambdas", "thetas", "etas", "weights", "responsibilities", "valid_mask", "colors",
        "sources")]


class DevicePrimitiveMap:
    """n_tiles x m_tile slots of PrimitiveMapTile fields (create_empty_tile, primitive_map.py:148-175).

    packed=True (default) keeps one record per slot in HBM (gc_primitive_map_record_layout: the
    fuse's read-modify-write fields in the record's first two 128-B lines); upload / download
    transpose to and from the reference's per-field arrays on the device (gc_copy_strided).
    packed=False keeps the per-field arrays themselves."""

    def __init__(self, n_tiles: int, m_tile: int, n_lobes: int = GC_VMF_N_LOBES, track_colors: bool = True,
                 ctx=None, packed: bool = True):
        self.ctx = ctx or _abi.default_context()
        self.n_tiles, self.m_tile, self.n_lobes = int(n_tiles), int(m_tile), int(n_lobes)
        M = self.M = self.n_tiles * self.m_tile
        self.shapes = dict(Lambdas=(M, 3, 3), thetas=(M, 3), etas=(M, n_lobes, 3), weights=(M,), timestamps=(M,),
                           last_supported_scan_seq=(M,), last_update_scan_seq=(M,), cam_mass=(M,), lidar_mass=(M,),
                           rgb_cam_accum=(M, 3), rgb_cam_denom=(M,), rgb=(M, 3), colors=(M, 3),
                           valid_mask=(M,), created_timestamps=(M,), primitive_ids=(M,))
        self.dtypes = {k: np.dtype(np.float64) for k in self.shapes}
        self.dtypes.update(last_supported_scan_seq=np.dtype(np.int64), last_update_scan_seq=np.dtype(np.int64),
                           primitive_ids=np.dtype(np.int64), valid_mask=np.dtype(np.uint8))
        names = [k for k in _F64 + _I64 + _COL + _MAINT if track_colors or k not in _COL]
        self.packed = bool(packed)
        self.ptrs: Dict[str, int] = {}
        self.fields: Dict[str, _abi.DeviceArray] = {}  # per-field arrays (packed=False)
        if self.packed:
            off = np.zeros(16, np.int64)
            sb = C.c_int64(0)
            _abi.call("gc_primitive_map_record_layout", self.n_lobes, off.ctypes.data, C.byref(sb))
            self.slot_bytes = int(sb.value)
            self.records = _abi.DeviceArray(self.ctx, M * self.slot_bytes, np.uint8)
            self.records.zero()
            order = _F64 + _I64 + _COL + _MAINT
            for k in names:
                self.ptrs[k] = self.records.ptr + int(off[order.index(k)])
        else:
            self.slot_bytes = 0
            for k in names:
                self.fields[k] = _abi.DeviceArray(self.ctx, self.shapes[k], self.dtypes[k])
                self.fields[k].zero()
                self.ptrs[k] = self.fields[k].ptr
        self._struct = _MapStruct(M, self.n_lobes, 0, *[self.ptrs.get(k) for k in _F64 + _I64 + _COL + _MAINT],
                                  self.slot_bytes)
        # per tile: every slot's rgb and colors = the fuse's estimate of its camera accumulators. Not so
        # for an empty tile (create_empty_tile: rgb gray, colors 0); a fuse leaves its tile current,
        # insert / merge / a colour upload do not
        self._tile_cc = [False] * self.n_tiles
        # pipelines with this map attached (BatchedScanPipeline.attach_primitive_map): told when a host
        # operation makes the colours stale, so their next in-scan update recomputes every slot's
        self._listeners: List[Any] = []
        if track_colors:
            self.upload(rgb=np.full((M, 3), 0.5))
        # AtlasMap bookkeeping (primitive_map.py:183-201): host integers, as in the reference
        self.next_global_id = 0
        self.total_count = 0
        self.tile_count: Dict[int, int] = {}
        # tile keys of the dense tiles (the reference's packed MA-hex tile ids); default 0..n-1
        self.tile_keys: List[int] = list(range(self.n_tiles))

    @property
    def colors_current(self) -> bool:
        """True while every slot's rgb / colors equal the fuse's estimate of its camera accumulators
        (a fuse then recomputes only the slots it touches, as gc_primitive_map.colors_current)."""
        return all(self._tile_cc)

    @colors_current.setter
    def colors_current(self, v: bool) -> None:
        if not v:
            self.colors_stale()
        else:
            self._tile_cc = [True] * self.n_tiles

    def colors_stale(self, tile_id: Optional[int] = None) -> None:
        """A host operation wrote colour fields (insert, merge, a colour upload): rgb / colors of the
        tile (None: every tile) are no longer the fuse's estimate. Attached pipelines are told, so
        their next in-scan update recomputes them (gc_pipeline_map_colors_stale)."""
        if tile_id is None:
            self._tile_cc = [False] * self.n_tiles
        else:
            self._tile_cc[int(tile_id)] = False
        alive = []
        for ref in self._listeners:
            pipe = ref()
            if pipe is not None and getattr(pipe, "_smap", None) is self:
                pipe._map_colors_stale()
                alive.append(ref)
        self._listeners = alive

    def struct(self) -> "_MapStruct":
        """The whole flat map (all tiles) for a C entry, its colour flag up to date."""
        self._struct.colors_current = 1 if self.colors_current else 0
        return self._struct

    def tile_struct(self, tile_id: int) -> "_MapStruct":
        """One tile as a map of m_tile slots (tile-local slot indices), as the reference's per-tile
        operators see it."""
        s0, n = self.tile_range(tile_id)
        st = _MapStruct.from_buffer_copy(self._struct)
        st.m_slots = n
        st.colors_current = 1 if self._tile_cc[int(tile_id)] else 0
        for k, p in self.ptrs.items():
            setattr(st, k, p + s0 * (self.slot_bytes or self._row_bytes(k)))
        return st

    def set_tile_keys(self, keys) -> None:
        keys = [int(k) for k in keys]
        if len(keys) != self.n_tiles or len(set(keys)) != len(keys):
            raise ValueError("tile keys must be n_tiles distinct ids")
        self.tile_keys = keys

    def dense_tile(self, key: int) -> int:
        """Dense tile index holding tile key `key`, or -1 (an empty tile for the view)."""
        try:
            return self.tile_keys.index(int(key))
        except ValueError:
            return -1

    def _row_bytes(self, k: str) -> int:
        return int(np.prod(self.shapes[k][1:], dtype=np.int64)) * self.dtypes[k].itemsize

    def upload(self, **arrays):
        for k, v in arrays.items():
            if k not in self.ptrs:
                raise KeyError(k)
            if k in _COL:
                self.colors_stale()  # arbitrary colours / accumulators: the next fuse recomputes all
            if not self.packed:
                self.fields[k].upload(v)
                continue
            tmp = _abi.DeviceArray.from_host(self.ctx, np.asarray(v).reshape(self.shapes[k]), self.dtypes[k])
            rb = self._row_bytes(k)
            _abi.call("gc_copy_strided", self.ctx.handle, self.ptrs[k], self.slot_bytes, tmp.ptr, rb, rb, self.M,
                      ctx=self.ctx)
            self.ctx.sync()

    def download(self, *names):
        if not self.packed:
            return {k: self.fields[k].download() for k in (names or self.fields.keys())}
        out = {}
        for k in (names or self.ptrs.keys()):
            tmp = _abi.DeviceArray(self.ctx, self.shapes[k], self.dtypes[k])
            rb = self._row_bytes(k)
            _abi.call("gc_copy_strided", self.ctx.handle, tmp.ptr, rb, self.ptrs[k], self.slot_bytes, rb, self.M,
                      ctx=self.ctx)
            out[k] = tmp.download()
        return out

    def tile_slot(self, tile_id: int, slots) -> np.ndarray:
        return int(tile_id) * self.m_tile + np.asarray(slots, dtype=np.int64)

    def tile_range(self, tile_id: int) -> Tuple[int, int]:
        t = int(tile_id)
        if not 0 <= t < self.n_tiles:
            raise ValueError(f"tile_id {t} outside [0, {self.n_tiles})")
        return t * self.m_tile, self.m_tile

    def download_tile(self, tile_id: int, *names) -> Dict[str, np.ndarray]:
        s0, n = self.tile_range(tile_id)
        return {k: v[s0:s0 + n] for k, v in self.download(*names).items()}


@dataclass
class PrimitiveMapFuseResult:
    atlas_map: DevicePrimitiveMap
    tile_id: int
    n_fused: int


class DeviceFuseBatch:
    """K measurement rows resident in HBM (flat map slots), reusable across fuse calls."""

    def __init__(self, ctx, slots, Lambdas, thetas, etas, weights, responsibilities, valid_mask=None, colors=None,
                 sources=None, n_lobes: int = GC_VMF_N_LOBES):
        sl = np.ascontiguousarray(slots, dtype=np.int32).reshape(-1)
        K = self.K = sl.shape[0]
        arrs = [sl, np.ascontiguousarray(Lambdas, np.float64).reshape(K, 9),
                np.ascontiguousarray(thetas, np.float64).reshape(K, 3),
                np.ascontiguousarray(etas, np.float64).reshape(K, 3 * n_lobes),
                np.ascontiguousarray(weights, np.float64).reshape(K),
                np.ascontiguousarray(responsibilities, np.float64).reshape(K)]
        opt = [None if valid_mask is None else np.ascontiguousarray(valid_mask, np.uint8).reshape(K),
               None if colors is None else np.ascontiguousarray(colors, np.float64).reshape(K, 3),
               None if sources is None else np.ascontiguousarray(sources, np.int32).reshape(K)]
        self.dev = [_abi.DeviceArray.from_host(ctx, a, a.dtype) for a in arrs] + \
                   [_abi.DeviceArray.from_host(ctx, a, a.dtype) if a is not None else None for a in opt]
        self.struct = _FuseStruct(K, *[d.ptr if d is not None else None for d in self.dev])


def fuse_device(dmap: DevicePrimitiveMap, batch: DeviceFuseBatch, timestamp: float, scan_seq: int = 0,
                world_pose=None, eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS,
                count: bool = True, tile_id: Optional[int] = None) -> int:
    """Fuse a resident batch in place; returns the distinct slots touched (count=False: -1, no sync).
    tile_id=None: the rows hold flat slots of the whole map; else tile-local slots of that tile (the
    colour estimate then covers that tile, as the reference's per-tile fuse)."""
    pose = None if world_pose is None else np.ascontiguousarray(world_pose, np.float64).reshape(6)
    n = C.c_int64(-1)
    st = dmap.struct() if tile_id is None else dmap.tile_struct(tile_id)
    _abi.call("gc_primitive_map_fuse", dmap.ctx.handle, C.byref(st), C.byref(batch.struct),
              None if pose is None else pose.ctypes.data, float(eps_lift), float(eps_mass), float(timestamp),
              int(scan_seq), C.byref(n) if count else None, ctx=dmap.ctx)
    if "cam_mass" in dmap.ptrs:  # the fuse leaves every slot's colour (of the tile) at its estimate
        if tile_id is None:
            dmap.colors_current = True
        else:
            dmap._tile_cc[int(tile_id)] = True
    return int(n.value)


def fuse_rows(dmap: DevicePrimitiveMap, slots, Lambdas, thetas, etas, weights, responsibilities, timestamp: float,
              scan_seq: int = 0, valid_mask=None, colors=None, sources=None, world_pose=None,
              eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS, tile_id: Optional[int] = None) -> int:
    """K host rows (flat map slots, or tile-local with tile_id) -> fused in place; returns the number of
    distinct slots touched."""
    if np.asarray(slots).reshape(-1).shape[0] == 0:
        return 0
    b = DeviceFuseBatch(dmap.ctx, slots, Lambdas, thetas, etas, weights, responsibilities, valid_mask, colors,
                        sources, dmap.n_lobes)
    return fuse_device(dmap, b, timestamp, scan_seq, world_pose, eps_lift, eps_mass, tile_id=tile_id)


def primitive_map_fuse(atlas_map: DevicePrimitiveMap, tile_id: int, target_slots, Lambdas_meas, thetas_meas,
                       etas_meas, weights_meas, responsibilities, timestamp: float, scan_seq: int = 0,
                       valid_mask=None, colors_meas=None, sources_meas=None, eps_psd: float = GC_EPS_PSD,
                       eps_mass: float = GC_EPS_MASS, fuse_chunk_size: int = 0, chart_id: str = GC_CHART_ID,
                       anchor_id: str = "primitive_map", world_pose=None, eps_lift: float = GC_EPS_LIFT
                       ) -> Tuple[PrimitiveMapFuseResult, CertBundle, ExpectedEffect]:
    """Reference signature; fuse_chunk_size is accepted for compatibility (the device reduce-by-key
    has no chunking). world_pose (optional [t, rotvec]) applies transform_gaussian_to_world."""
    sl = np.asarray(target_slots, dtype=np.int64).reshape(-1)
    K = sl.shape[0]
    if K == 0:
        return (PrimitiveMapFuseResult(atlas_map, int(tile_id), 0),
                CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
                ExpectedEffect(objective_name="primitive_map_fuse", predicted=0.0, realized=0.0))
    atlas_map.tile_range(tile_id)  # validates the tile
    local = np.where((sl >= 0) & (sl < atlas_map.m_tile), sl, -1)
    n = fuse_rows(atlas_map, local, Lambdas_meas, thetas_meas, etas_meas, weights_meas, responsibilities, timestamp,
                  scan_seq, valid_mask, colors_meas if sources_meas is not None else None, sources_meas, world_pose,
                  eps_lift, eps_mass, tile_id=tile_id)
    return (PrimitiveMapFuseResult(atlas_map, int(tile_id), n),
            CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
            ExpectedEffect(objective_name="primitive_map_fuse", predicted=float(K), realized=float(n)))


# ----------------------------------------------------------------------------- maintenance
def _no_op(result, chart_id: str, anchor_id: str, name: str, predicted: float = 0.0):
    """_exact_no_op_result (primitive_map.py:624-640)."""
    return (result, CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
            ExpectedEffect(objective_name=name, predicted=predicted, realized=0.0))


@dataclass
class PrimitiveMapForgetResult:
    atlas_map: DevicePrimitiveMap
    tile_id: int


def primitive_map_forget(atlas_map: DevicePrimitiveMap, tile_id: int,
                         forgetting_factor: float = GC_PRIMITIVE_FORGETTING_FACTOR, chart_id: str = GC_CHART_ID,
                         anchor_id: str = "primitive_map"
                         ) -> Tuple[PrimitiveMapForgetResult, CertBundle, ExpectedEffect]:
    """primitive_map_forget (primitive_map.py:1314-1390): weights *= γ on the tile."""
    s0, n = atlas_map.tile_range(tile_id)
    gamma = float(forgetting_factor)
    _abi.call("gc_primitive_map_forget", atlas_map.ctx.handle, C.byref(atlas_map.struct()), s0, n, gamma,
              ctx=atlas_map.ctx)
    return (PrimitiveMapForgetResult(atlas_map, int(tile_id)),
            CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
            ExpectedEffect(objective_name="primitive_map_forget", predicted=1.0 - gamma, realized=1.0 - gamma))


@dataclass
class PrimitiveMapRecencyInflateStats:
    staleness_inflation_strength: float
    staleness_cov_inflation_trace: float
    stale_precision_downscale_total: float


def primitive_map_recency_inflate(atlas_map: DevicePrimitiveMap, tile_ids: List[int], scan_seq: int,
                                  recency_decay_lambda: float = GC_RECENCY_DECAY_LAMBDA,
                                  min_scale: float = GC_RECENCY_MIN_SCALE, chart_id: str = GC_CHART_ID,
                                  anchor_id: str = "primitive_map_recency_inflate"):
    """primitive_map_recency_inflate (primitive_map.py:1400-1490) -> (atlas_map, cert, effect, stats)."""
    n_valid = downscale = trace = 0.0
    for tid in tile_ids:
        s0, n = atlas_map.tile_range(tid)
        st = np.zeros(3)
        _abi.call("gc_primitive_map_recency_inflate", atlas_map.ctx.handle, C.byref(atlas_map.struct()), s0, n,
                  int(scan_seq), float(recency_decay_lambda), float(min_scale), st.ctypes.data, ctx=atlas_map.ctx)
        n_valid += st[0]
        downscale += st[1]
        trace += st[2]
    stats = PrimitiveMapRecencyInflateStats(staleness_inflation_strength=float(downscale / max(n_valid, 1.0)),
                                            staleness_cov_inflation_trace=float(trace),
                                            stale_precision_downscale_total=float(downscale))
    return (atlas_map, CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
            ExpectedEffect(objective_name="primitive_map_recency_inflate", predicted=float(n_valid),
                           realized=float(n_valid)), stats)


@dataclass
class PrimitiveMapCullResult:
    atlas_map: DevicePrimitiveMap
    tile_id: int
    n_culled: int
    mass_dropped: float


def primitive_map_cull(atlas_map: DevicePrimitiveMap, tile_id: int,
                       weight_threshold: float = GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD,
                       max_primitives: Optional[int] = None, chart_id: str = GC_CHART_ID,
                       anchor_id: str = "primitive_map") -> Tuple[PrimitiveMapCullResult, CertBundle, ExpectedEffect]:
    """primitive_map_cull (primitive_map.py:1175-1305)."""
    s0, n = atlas_map.tile_range(tile_id)
    out = np.zeros(4)
    _abi.call("gc_primitive_map_cull", atlas_map.ctx.handle, C.byref(atlas_map.struct()), s0, n,
              float(weight_threshold), -1 if max_primitives is None else int(max_primitives), out.ctypes.data,
              ctx=atlas_map.ctx)
    n_culled, mass_dropped, sum_w, n_valid = int(out[0]), float(out[1]), float(out[2]), int(out[3])
    if n_valid == 0 or n_culled == 0:
        return _no_op(PrimitiveMapCullResult(atlas_map, int(tile_id), 0, 0.0), chart_id, anchor_id,
                      "primitive_map_cull")
    atlas_map.tile_count[int(tile_id)] = n_valid - n_culled
    atlas_map.total_count -= n_culled
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["budgeting", "mass_drop"],
                                    influence=InfluenceCert.identity().with_overrides(
                                        mass_epsilon_ratio=mass_dropped / (sum_w + GC_EPS_MASS)))
    return (PrimitiveMapCullResult(atlas_map, int(tile_id), n_culled, mass_dropped), cert,
            ExpectedEffect(objective_name="primitive_map_cull", predicted=float(n_culled), realized=float(n_culled)))


@dataclass
class PrimitiveMapInsertResult:
    atlas_map: DevicePrimitiveMap
    tile_id: int
    n_inserted: int
    new_ids: np.ndarray
    target_slots: Optional[np.ndarray] = None  # tile-local eviction slots (extra field)


def primitive_map_insert_masked(atlas_map: DevicePrimitiveMap, tile_id: int, Lambdas_new, thetas_new, etas_new,
                                weights_new, timestamp: float, valid_new_mask, scan_seq: int = 0,
                                recency_decay_lambda: float = GC_RECENCY_DECAY_LAMBDA, colors_new=None,
                                sources_new=None, chart_id: str = GC_CHART_ID,
                                anchor_id: str = "primitive_map_insert_masked"
                                ) -> Tuple[PrimitiveMapInsertResult, CertBundle, ExpectedEffect]:
    """primitive_map_insert_masked (primitive_map.py:807-982)."""
    s0, n = atlas_map.tile_range(tile_id)
    L = atlas_map.n_lobes
    w = np.ascontiguousarray(weights_new, np.float64).reshape(-1)
    K = w.shape[0]
    mask = np.ascontiguousarray(valid_new_mask).reshape(-1).astype(np.uint8)
    if mask.shape[0] != K or K > n or K == 0:
        raise ValueError(f"insert_masked: K={K} proposals, mask {mask.shape[0]}, tile {n}")
    ctx = atlas_map.ctx
    arrs = [np.ascontiguousarray(Lambdas_new, np.float64).reshape(K, 9),
            np.ascontiguousarray(thetas_new, np.float64).reshape(K, 3),
            np.ascontiguousarray(etas_new, np.float64).reshape(K, 3 * L), w, mask,
            None if colors_new is None else np.ascontiguousarray(colors_new, np.float64).reshape(K, 3),
            None if sources_new is None else np.ascontiguousarray(sources_new, np.int32).reshape(K)]
    dev = [None if a is None else _abi.DeviceArray.from_host(ctx, a, a.dtype) for a in arrs]
    batch = _InsertStruct(K, *[None if d is None else d.ptr for d in dev])
    d_slots = _abi.DeviceArray(ctx, K, np.int32)
    d_ids = _abi.DeviceArray(ctx, K, np.int64)
    out = np.zeros(2, np.int64)
    _abi.call("gc_primitive_map_insert_masked", ctx.handle, C.byref(atlas_map.struct()), s0, n, C.byref(batch),
              float(timestamp), int(scan_seq), float(recency_decay_lambda), int(atlas_map.next_global_id),
              d_slots.ptr, d_ids.ptr, out.ctypes.data, ctx=ctx)
    n_ins, count = int(out[0]), int(out[1])
    if n_ins > 0:
        atlas_map.colors_stale(tile_id)  # inserted colours are clip(c), not the estimate clip(c·cam / cam)
    atlas_map.next_global_id += n_ins
    atlas_map.total_count += n_ins
    atlas_map.tile_count[int(tile_id)] = count
    dropped = int(np.sum(mask == 0))
    cert = (CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["insert_unfilled_budget"],
                                     frobenius_applied=False) if dropped > 0
            else CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id))
    return (PrimitiveMapInsertResult(atlas_map, int(tile_id), n_ins, d_ids.download(), d_slots.download()), cert,
            ExpectedEffect(objective_name="primitive_map_insert_masked", predicted=float(int(mask.sum())),
                           realized=float(n_ins)))


@dataclass
class PrimitiveMapMergeReduceResult:
    atlas_map: DevicePrimitiveMap
    tile_id: int
    n_merged: int
    frobenius_correction: float


def primitive_map_merge_reduce(atlas_map: DevicePrimitiveMap, tile_id: int,
                               merge_threshold: float = GC_PRIMITIVE_MERGE_THRESHOLD,
                               max_pairs: int = GC_K_MERGE_PAIRS_PER_TILE,
                               max_tile_size: int = GC_PRIMITIVE_MERGE_MAX_TILE_SIZE, eps_psd: float = GC_EPS_PSD,
                               eps_lift: float = GC_EPS_LIFT, chart_id: str = GC_CHART_ID,
                               anchor_id: str = "primitive_map"
                               ) -> Tuple[PrimitiveMapMergeReduceResult, CertBundle, ExpectedEffect]:
    """primitive_map_merge_reduce (primitive_map.py:1809-2030)."""
    s0, M = atlas_map.tile_range(tile_id)

    def no_op(predicted, triggers=None, influence=None):
        res = PrimitiveMapMergeReduceResult(atlas_map, int(tile_id), 0, 0.0)
        cert = (CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=triggers,
                                         frobenius_applied=True, influence=influence or InfluenceCert.identity())
                if triggers else CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id))
        return res, cert, ExpectedEffect(objective_name="primitive_map_merge_reduce", predicted=predicted,
                                         realized=0.0)

    if int(max_tile_size) > 0 and M > int(max_tile_size):
        # the budget cap (:1881-1890) applies after the M / valid count / max_pairs no-op test (:1879)
        n_valid = int(atlas_map.download_tile(tile_id, "valid_mask")["valid_mask"].sum())
        if M < 2 or n_valid < 2 or int(max_pairs) <= 0:
            return no_op(float(max_pairs))
        over = float(M - int(max_tile_size)) / float(max(M, 1))
        return no_op(float(max_pairs), ["merge_reduce_budget_cap"],
                     InfluenceCert.identity().with_overrides(mass_epsilon_ratio=over))
    out = np.zeros(2, np.int64)
    _abi.call("gc_primitive_map_merge_reduce", atlas_map.ctx.handle, C.byref(atlas_map.struct()), s0, M,
              float(merge_threshold), int(max_pairs), float(eps_psd), float(eps_lift), out.ctypes.data,
              ctx=atlas_map.ctx)
    n_merged, count = int(out[0]), int(out[1])
    if n_merged <= 0:
        return no_op(float(max_pairs))
    atlas_map.colors_stale(tile_id)  # merged colours use max(denom, eps_psd) (primitive_map.py:1976-1983)
    atlas_map.tile_count[int(tile_id)] = count
    atlas_map.total_count -= n_merged
    cert = CertBundle.create_approx(chart_id=chart_id, anchor_id=anchor_id, triggers=["primitive_map_merge_reduce"],
                                    frobenius_applied=True, influence=InfluenceCert.identity().with_overrides(
                                        mass_epsilon_ratio=float(n_merged) / float(max(M, 1))))
    return (PrimitiveMapMergeReduceResult(atlas_map, int(tile_id), n_merged, float(n_merged)), cert,
            ExpectedEffect(objective_name="primitive_map_merge_reduce", predicted=float(max_pairs),
                           realized=float(n_merged)))
