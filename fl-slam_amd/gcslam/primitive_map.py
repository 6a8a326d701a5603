"""Device-resident PrimitiveMap and primitive_map_fuse (backend/structures/primitive_map.py:
992-1163) with the world pushforward of transform_gaussian_to_world (backend/pipeline.py:
1248-1256) fused in: the C5 map update. The map lives in HBM as one flat array of
n_tiles * m_tile slots (tile t, local slot j -> t * m_tile + j); the fuse runs in place."""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Tuple

import numpy as np

from . import _abi
from .certificates import CertBundle, ExpectedEffect
from .constants import GC_CHART_ID, GC_EPS_LIFT, GC_EPS_MASS, GC_EPS_PSD

GC_VMF_N_LOBES = 3

_F64 = ("Lambdas", "thetas", "etas", "weights", "timestamps")
_I64 = ("last_supported_scan_seq", "last_update_scan_seq")
_COL = ("cam_mass", "lidar_mass", "rgb_cam_accum", "rgb_cam_denom", "rgb", "colors")


class _MapStruct(C.Structure):
    _fields_ = [("m_slots", C.c_int64), ("n_lobes", C.c_int32), ("pad_", C.c_int32)] + \
               [(k, C.c_void_p) for k in _F64 + _I64 + _COL]


class _FuseStruct(C.Structure):
    _fields_ = [("K", C.c_int64)] + [(k, C.c_void_p) for k in (
        "target_slots", "Lambdas", "thetas", "etas", "weights", "responsibilities", "valid_mask", "colors",
        "sources")]


class DevicePrimitiveMap:
    """n_tiles x m_tile slots of PrimitiveMapTile fields (create_empty_tile, primitive_map.py:148-175)."""

    def __init__(self, n_tiles: int, m_tile: int, n_lobes: int = GC_VMF_N_LOBES, track_colors: bool = True,
                 ctx=None):
        self.ctx = ctx or _abi.default_context()
        self.n_tiles, self.m_tile, self.n_lobes = int(n_tiles), int(m_tile), int(n_lobes)
        M = self.M = self.n_tiles * self.m_tile
        shapes = dict(Lambdas=(M, 3, 3), thetas=(M, 3), etas=(M, n_lobes, 3), weights=(M,), timestamps=(M,),
                      last_supported_scan_seq=(M,), last_update_scan_seq=(M,), cam_mass=(M,), lidar_mass=(M,),
                      rgb_cam_accum=(M, 3), rgb_cam_denom=(M,), rgb=(M, 3), colors=(M, 3))
        self.fields: Dict[str, _abi.DeviceArray] = {}
        for k, shp in shapes.items():
            if k in _COL and not track_colors:
                continue
            self.fields[k] = _abi.DeviceArray(self.ctx, shp, np.int64 if k in _I64 else np.float64)
            self.fields[k].zero()
        if track_colors:
            self.fields["rgb"].upload(np.full((M, 3), 0.5))
        self._struct = _MapStruct(M, self.n_lobes, 0, *[self.fields[k].ptr if k in self.fields else None
                                                        for k in _F64 + _I64 + _COL])

    def upload(self, **arrays):
        for k, v in arrays.items():
            self.fields[k].upload(v)

    def download(self, *names):
        return {k: self.fields[k].download() for k in (names or self.fields.keys())}

    def tile_slot(self, tile_id: int, slots) -> np.ndarray:
        return int(tile_id) * self.m_tile + np.asarray(slots, dtype=np.int64)


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
                count: bool = True) -> int:
    """Fuse a resident batch in place; returns the distinct slots touched (count=False: -1, no sync)."""
    pose = None if world_pose is None else np.ascontiguousarray(world_pose, np.float64).reshape(6)
    n = C.c_int64(-1)
    _abi.call("gc_primitive_map_fuse", dmap.ctx.handle, C.byref(dmap._struct), C.byref(batch.struct),
              None if pose is None else pose.ctypes.data, float(eps_lift), float(eps_mass), float(timestamp),
              int(scan_seq), C.byref(n) if count else None, ctx=dmap.ctx)
    return int(n.value)


def fuse_rows(dmap: DevicePrimitiveMap, slots, Lambdas, thetas, etas, weights, responsibilities, timestamp: float,
              scan_seq: int = 0, valid_mask=None, colors=None, sources=None, world_pose=None,
              eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS) -> int:
    """K host rows (flat map slots) -> fused in place; returns the number of distinct slots touched."""
    if np.asarray(slots).reshape(-1).shape[0] == 0:
        return 0
    b = DeviceFuseBatch(dmap.ctx, slots, Lambdas, thetas, etas, weights, responsibilities, valid_mask, colors,
                        sources, dmap.n_lobes)
    return fuse_device(dmap, b, timestamp, scan_seq, world_pose, eps_lift, eps_mass)


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
    flat = np.where((sl >= 0) & (sl < atlas_map.m_tile), atlas_map.tile_slot(tile_id, sl), -1)
    n = fuse_rows(atlas_map, flat, Lambdas_meas, thetas_meas, etas_meas, weights_meas, responsibilities, timestamp,
                  scan_seq, valid_mask, colors_meas if sources_meas is not None else None, sources_meas, world_pose,
                  eps_lift, eps_mass)
    return (PrimitiveMapFuseResult(atlas_map, int(tile_id), n),
            CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
            ExpectedEffect(objective_name="primitive_map_fuse", predicted=float(K), realized=float(n)))
