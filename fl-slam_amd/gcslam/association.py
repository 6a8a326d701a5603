"""Map view extraction and OT association on the GPU (the current
PrimitiveMap pose-evidence path):

- extract_atlas_map_view (backend/structures/primitive_map.py:356-451): the top m_tile_view slots
  of each listed tile, stitched into one candidate pool resident in HBM (DeviceMapView);
- associate_primitives_ot (backend/operators/primitive_association.py:239-553): per-measurement
  MA-hex stencil candidates, sparse cost, top-K by a stable cost sort, recency bias, and the
  fixed-iteration unbalanced Sinkhorn;
- block_associations_for_fuse (:561-588), host reshaping of the result for the fuse.

All arithmetic runs in libgcslam (gc_extract_map_view, gc_associate_primitives_ot); the host
marshals arguments and reads results back."""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from enum import Enum
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _abi
from .certificates import CertBundle, ComputeCert, ExpectedEffect, InfluenceCert, OTCert, SupportCert
from .constants import GC_CHART_ID, GC_EPS_LIFT, GC_EPS_MASS, GC_RECENCY_DECAY_LAMBDA
from .primitive_map import DevicePrimitiveMap

GC_K_ASSOC = 8                 # constants.py:356
GC_K_SINKHORN = 50             # constants.py:357
GC_H_TILE = 2.0                # constants.py:408
GC_R_STENCIL_TILES_XY = 1      # constants.py:415
GC_R_STENCIL_TILES_Z = 0       # constants.py:416
GC_M_TILE_VIEW = 1024          # constants.py:436
GC_ASSOC_BLOCK_SIZE = 256      # constants.py:473

_PACK_BITS, _PACK_BIAS = 21, 1 << 20
_PACK_MASK = (1 << _PACK_BITS) - 1


def tile_id_from_cell_3d(c1: int, c2: int, cz: int) -> int:
    """tiling.py:91-105 (PackedTileIdSpec: 21 bits per axis after a 2^20 bias)."""
    u1, u2, uz = ((int(x) + _PACK_BIAS) & _PACK_MASK for x in (c1, c2, cz))
    return (u1 << (2 * _PACK_BITS)) | (u2 << _PACK_BITS) | uz


class MeasurementMassPolicy(Enum):
    UNIFORM = "uniform"
    WEIGHT_PROPORTIONAL = "weight_proportional"
    FEATURE_CONFIDENCE = "feature_confidence"


class MapMassPolicy(Enum):
    UNIFORM = "uniform"
    PRIMITIVE_MASS = "primitive_mass"
    MASS_TEMPERED = "mass_tempered"


@dataclass
class AssociationConfig:
    """primitive_association.py:205-236."""
    k_assoc: int = GC_K_ASSOC
    k_sinkhorn: int = GC_K_SINKHORN
    beta: float = 0.5
    epsilon: float = 0.1
    tau_a: float = 0.5
    tau_b: float = 0.5
    cost_subtract_row_min: bool = True
    cost_scale_by_median: bool = False
    a_policy: MeasurementMassPolicy = MeasurementMassPolicy.UNIFORM
    b_policy: MapMassPolicy = MapMassPolicy.UNIFORM
    eps_mass: float = GC_EPS_MASS
    h_tile: float = GC_H_TILE
    r_stencil_tiles_xy: int = GC_R_STENCIL_TILES_XY
    r_stencil_tiles_z: int = GC_R_STENCIL_TILES_Z
    scan_seq: int = 0
    recency_decay_lambda: float = GC_RECENCY_DECAY_LAMBDA


class _ViewStruct(C.Structure):
    _fields_ = [("n_tiles", C.c_int32), ("m_tile_view", C.c_int32), ("n_lobes", C.c_int32), ("pad_", C.c_int32)] + \
               [(k, C.c_void_p) for k in (
                   "tile_ids", "candidate_tile_ids", "candidate_slots", "valid_mask", "positions", "covariances",
                   "directions", "kappas", "weights", "primitive_ids", "last_supported_scan_seq", "etas", "colors")]


class DeviceMapView:
    """AtlasMapView (primitive_map.py:270-300) resident in HBM; `download()` gives the arrays."""

    _SHAPES = dict(candidate_tile_ids=((), np.int64), candidate_slots=((), np.int64), valid_mask=((), np.uint8),
                   positions=((3,), np.float64), covariances=((3, 3), np.float64), directions=((3,), np.float64),
                   kappas=((), np.float64), weights=((), np.float64), primitive_ids=((), np.int64),
                   last_supported_scan_seq=((), np.int64), colors=((3,), np.float64))

    def __init__(self, ctx, tile_ids, m_tile_view: int, n_lobes: int):
        self.ctx = ctx
        self.tile_ids = np.asarray(tile_ids, np.int64).reshape(-1)
        self.n_tiles, self.m_tile_view, self.n_lobes = self.tile_ids.shape[0], int(m_tile_view), int(n_lobes)
        V = self.count = self.n_tiles * self.m_tile_view
        self.arrays: Dict[str, _abi.DeviceArray] = {"tile_ids": _abi.DeviceArray(ctx, self.n_tiles, np.int64)}
        for k, (shp, dt) in self._SHAPES.items():
            self.arrays[k] = _abi.DeviceArray(ctx, (V,) + shp, dt)
        self.arrays["etas"] = _abi.DeviceArray(ctx, (V, self.n_lobes, 3), np.float64)
        order = [f[0] for f in _ViewStruct._fields_[4:]]
        self.struct = _ViewStruct(self.n_tiles, self.m_tile_view, self.n_lobes, 0,
                                  *[self.arrays[k].ptr for k in order])

    def download(self, *names) -> Dict[str, np.ndarray]:
        out = {k: self.arrays[k].download() for k in (names or self.arrays.keys())}
        if "valid_mask" in out:
            out["valid_mask"] = out["valid_mask"].astype(bool)
        return out


def extract_atlas_map_view(atlas_map: DevicePrimitiveMap, tile_ids: List[int], m_tile_view: int,
                           eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS) -> DeviceMapView:
    """primitive_map.py:356-451. tile_ids are the map's tile keys (atlas_map.tile_key); keys the map
    does not hold are empty tiles, as in the reference."""
    if m_tile_view <= 0:
        raise ValueError(f"extract_atlas_map_view: m_tile_view must be > 0, got {m_tile_view}")
    view = DeviceMapView(atlas_map.ctx, tile_ids, m_tile_view, atlas_map.n_lobes)
    dense = np.array([atlas_map.dense_tile(int(t)) for t in view.tile_ids], np.int64)
    _abi.call("gc_extract_map_view", atlas_map.ctx.handle, C.byref(atlas_map.struct()), int(atlas_map.m_tile),
              dense.ctypes.data, view.tile_ids.ctypes.data, float(eps_lift), float(eps_mass), C.byref(view.struct),
              ctx=atlas_map.ctx)
    return view


@dataclass
class PrimitiveAssociationResult:
    """primitive_association.py:71-92."""
    responsibilities: np.ndarray
    candidate_pool_indices: np.ndarray
    candidate_tile_ids: np.ndarray
    candidate_slots: np.ndarray
    row_masses: np.ndarray
    cost_matrix: np.ndarray


def _p95(x: np.ndarray) -> float:
    s = np.sort(np.asarray(x).reshape(-1))
    return float(s[min(int(0.95 * s.shape[0]), s.shape[0] - 1)]) if s.shape[0] else 0.0


def associate_primitives_ot(measurement_batch, map_view: DeviceMapView, config: Optional[AssociationConfig] = None,
                            eps_lift: float = GC_EPS_LIFT, eps_mass: float = GC_EPS_MASS, chart_id: str = GC_CHART_ID,
                            anchor_id: str = "primitive_ot"
                            ) -> Tuple[PrimitiveAssociationResult, CertBundle, ExpectedEffect]:
    """primitive_association.py:239-553. measurement_batch is duck-typed like MeasurementBatch:
    Lambdas (N,3,3), thetas (N,3), etas (N,L,3), weights (N), valid_mask (N)."""
    cfg = config or AssociationConfig()
    if cfg.a_policy not in (MeasurementMassPolicy.UNIFORM, MeasurementMassPolicy.WEIGHT_PROPORTIONAL):
        raise ValueError(f"Unsupported measurement mass policy: {cfg.a_policy}. "
                         "Only UNIFORM and WEIGHT_PROPORTIONAL are implemented.")
    if cfg.b_policy != MapMassPolicy.UNIFORM:
        raise ValueError(f"Unsupported map mass policy: {cfg.b_policy}. Only UNIFORM is implemented.")
    if cfg.cost_scale_by_median:
        raise ValueError("cost_scale_by_median is not supported by the device path")
    ctx = map_view.ctx
    valid = np.ascontiguousarray(measurement_batch.valid_mask).reshape(-1).astype(np.uint8)
    N = valid.shape[0]
    L = int(np.asarray(measurement_batch.etas).shape[1])
    K = int(cfg.k_assoc)
    arrs = [np.ascontiguousarray(measurement_batch.Lambdas, np.float64).reshape(N, 9),
            np.ascontiguousarray(measurement_batch.thetas, np.float64).reshape(N, 3),
            np.ascontiguousarray(measurement_batch.etas, np.float64).reshape(N, L * 3),
            np.ascontiguousarray(measurement_batch.weights, np.float64).reshape(N), valid]
    dev = [_abi.DeviceArray.from_host(ctx, a, a.dtype) for a in arrs]
    out = dict(responsibilities=_abi.DeviceArray(ctx, (N, K)), candidate_pool_indices=_abi.DeviceArray(ctx, (N, K), np.int32),
               candidate_tile_ids=_abi.DeviceArray(ctx, (N, K), np.int64),
               candidate_slots=_abi.DeviceArray(ctx, (N, K), np.int64), row_masses=_abi.DeviceArray(ctx, N),
               cost_matrix=_abi.DeviceArray(ctx, (N, K)))
    h_cfg = np.array([K, cfg.k_sinkhorn, cfg.beta, cfg.epsilon, cfg.tau_a, cfg.tau_b, float(cfg.cost_subtract_row_min),
                      float(cfg.a_policy == MeasurementMassPolicy.WEIGHT_PROPORTIONAL), cfg.eps_mass, cfg.h_tile,
                      cfg.r_stencil_tiles_xy, cfg.r_stencil_tiles_z, cfg.scan_seq, cfg.recency_decay_lambda, eps_lift],
                     np.float64)
    cert_v = np.zeros(13)
    _abi.call("gc_associate_primitives_ot", ctx.handle, N, L, dev[0].ptr, dev[1].ptr, dev[2].ptr, dev[3].ptr,
              dev[4].ptr, C.byref(map_view.struct), h_cfg.ctypes.data, out["responsibilities"].ptr,
              out["candidate_pool_indices"].ptr, out["candidate_tile_ids"].ptr, out["candidate_slots"].ptr,
              out["row_masses"].ptr, out["cost_matrix"].ptr, cert_v.ctypes.data, ctx=ctx)
    res = PrimitiveAssociationResult(**{k: v.download() for k, v in out.items()})
    if cert_v[11] == 0 or cert_v[12] == 0:
        return (res, CertBundle.create_exact(chart_id=chart_id, anchor_id=anchor_id),
                ExpectedEffect(objective_name="primitive_association_ot", predicted=0.0, realized=0.0))
    (defect_a, defect_b, transport, sum_a, sum_b, sum_m, sum_novel, ess, nz_a, nz_b, total_cost) = cert_v[:11]
    # p95 diagnostics (sorted marginals / recency rows), host-side as in the reference's cert build
    vf = valid.astype(np.float64)
    a = (vf * arrs[3] if cfg.a_policy == MeasurementMassPolicy.WEIGHT_PROPORTIONAL else vf) / sum_a
    last = map_view.download("last_supported_scan_seq")["last_supported_scan_seq"][res.candidate_pool_indices]
    dt = np.maximum(0, int(cfg.scan_seq) - last).astype(np.float64)
    rd = np.exp(-cfg.recency_decay_lambda * dt)
    rd = np.where(rd > 0.0, rd, 0.0)
    b_row = rd / np.maximum(rd.sum(axis=1, keepdims=True), cfg.eps_mass)
    cert = CertBundle.create_approx(
        chart_id=chart_id, anchor_id=anchor_id, triggers=["sinkhorn_fixed_iter", "sinkhorn_unbalanced_kl_relax"],
        frobenius_applied=False, support=SupportCert(ess_total=float(ess), support_frac=float(nz_a) / float(max(N, 1))),
        influence=InfluenceCert.identity().with_overrides(mass_epsilon_ratio=float(cfg.eps_mass) / (transport + cfg.eps_mass)),
        compute=ComputeCert(alloc_bytes_est=int(N * K * 8 * 4), largest_tensor_shape=(int(N), K), segment_sum_k=K))
    cert.ot = OTCert(marginal_defect_a=float(defect_a), marginal_defect_b=float(defect_b),
                     transport_mass_total=float(transport), sum_a=float(sum_a), sum_b=float(sum_b), sum_m=float(sum_m),
                     sum_novel=float(sum_novel), p95_a=_p95(a), p95_b=1.0 / K, nonzero_a=int(nz_a), nonzero_b=int(nz_b),
                     epsilon=float(cfg.epsilon), tau_a=float(cfg.tau_a), tau_b=float(cfg.tau_b),
                     n_iters=int(cfg.k_sinkhorn), b_policy=str(cfg.b_policy.value),
                     b_recency_decay_lambda=float(cfg.recency_decay_lambda), b_recency_p95=_p95(b_row))
    return (res, cert, ExpectedEffect(objective_name="primitive_association_ot", predicted=float(total_cost),
                                      realized=float(total_cost)))


def block_associations_for_fuse(result: PrimitiveAssociationResult, valid_mask,
                                block_size: int = GC_ASSOC_BLOCK_SIZE):
    """primitive_association.py:561-588 (index bookkeeping on the host result)."""
    N, _ = result.responsibilities.shape
    block = int(max(1, block_size))
    nb = (N + block - 1) // block
    idx = np.arange(nb * block, dtype=np.int32).reshape(nb, block)
    clipped = np.minimum(idx, N - 1)
    valid_rows = (idx < N) & np.asarray(valid_mask, bool).reshape(-1)[clipped]
    return (clipped, result.candidate_tile_ids[clipped], result.candidate_slots[clipped],
            result.responsibilities[clipped] * valid_rows[:, :, None], valid_rows)
