"""Operator-contract certificate types (field-compatible with fl_slam_poc/common/certificates.py).

Every operator returns ``(Result, CertBundle, ExpectedEffect)`` (docs/OPERATOR_CONTRACTS.md:3).
The numeric surface that feeds back into the pipeline is ``total_trigger_magnitude``
(certificates.py:439-455), which the recompose step turns into its Frobenius strength. The
field names, defaults and aggregation rules (certificates.py:511-600) are the reference's, so
code that reads a reference CertBundle reads these unchanged.
"""

from __future__ import annotations

from dataclasses import dataclass, field, fields, replace
from typing import Any, Dict, List, Optional

import numpy as np


def _as_dict(obj) -> Dict[str, Any]:
    return {f.name: getattr(obj, f.name) for f in fields(obj)}


@dataclass
class ConditioningCert:
    eig_min: float = 1.0
    eig_max: float = 1.0
    cond: float = 1.0
    near_null_count: int = 0

    to_dict = _as_dict


@dataclass
class SupportCert:
    ess_total: float = 0.0
    support_frac: float = 1.0

    to_dict = _as_dict


@dataclass
class MismatchCert:
    nll_per_ess: float = 0.0
    directional_score: float = 1.0

    to_dict = _as_dict


@dataclass
class ExcitationCert:
    dt_effect: float = 0.0
    extrinsic_effect: float = 0.0

    to_dict = _as_dict


@dataclass
class InfluenceCert:
    lift_strength: float = 0.0
    psd_projection_delta: float = 0.0
    nu_projection_delta: float = 0.0
    mass_epsilon_ratio: float = 0.0
    anchor_drift_rho: float = 0.0
    dt_scale: float = 1.0
    extrinsic_scale: float = 1.0
    trust_alpha: float = 1.0
    power_beta: float = 1.0

    @classmethod
    def identity(cls) -> "InfluenceCert":
        return cls()

    def with_overrides(self, **kw: Any) -> "InfluenceCert":
        return replace(self, **kw)

    to_dict = _as_dict


@dataclass
class OverconfidenceCert:
    excitation_total: float = 0.0
    ess_to_excitation: float = 0.0
    cond_to_support: float = 0.0
    dt_asymmetry: float = 0.0
    z_to_xy_ratio: float = 0.0
    ess_growth_rate: float = 0.0
    excitation_growth_rate: float = 0.0
    nullspace_energy_ratio: float = 0.0

    to_dict = _as_dict


@dataclass
class DeviceRuntimeCert:
    host_sync_count_est: int = 0
    device_to_host_bytes_est: int = 0
    host_to_device_bytes_est: int = 0
    jit_recompile_count: int = 0

    to_dict = _as_dict


@dataclass
class ScanIOCert:
    scan_seq: int = 0
    scan_stamp_sec: float = 0.0
    scan_window_start_sec: float = 0.0
    scan_window_end_sec: float = 0.0
    streams: Dict[str, Dict[str, float]] = field(default_factory=dict)

    to_dict = _as_dict


@dataclass
class ComputeCert:
    alloc_bytes_est: int = 0
    largest_tensor_shape: tuple = (0, 0)
    segment_sum_k: int = 0
    psd_projection_count: int = 0
    chol_solve_count: int = 0
    scan_io: ScanIOCert = field(default_factory=ScanIOCert)
    device_runtime: DeviceRuntimeCert = field(default_factory=DeviceRuntimeCert)

    def to_dict(self) -> Dict[str, Any]:
        d = _as_dict(self)
        d["scan_io"] = self.scan_io.to_dict()
        d["device_runtime"] = self.device_runtime.to_dict()
        return d


@dataclass
class OTCert:
    """OT association block (certificates.py OTCert; filled by primitive_association.py:524-544)."""
    marginal_defect_a: float = 0.0
    marginal_defect_b: float = 0.0
    transport_mass_total: float = 0.0
    dual_gap_proxy: float = 0.0
    sum_a: float = 0.0
    sum_b: float = 0.0
    sum_m: float = 0.0
    sum_novel: float = 0.0
    p95_a: float = 0.0
    p95_b: float = 0.0
    nonzero_a: int = 0
    nonzero_b: int = 0
    epsilon: float = 0.0
    tau_a: float = 0.0
    tau_b: float = 0.0
    n_iters: int = 0
    b_policy: str = "uniform"
    b_recency_decay_lambda: float = 0.0
    b_recency_p95: float = 0.0

    to_dict = _as_dict


@dataclass
class MapUpdateCert:
    """Map-maintenance block (certificates.py MapUpdateCert)."""
    n_active_tiles: int = 0
    tile_ids_active: List[int] = field(default_factory=list)
    n_inactive_tiles: int = 0
    tile_ids_inactive: List[int] = field(default_factory=list)
    tile_cache_hits: int = 0
    tile_cache_misses: int = 0
    candidate_tiles_per_meas_mean: float = 0.0
    candidate_primitives_per_meas_mean: float = 0.0
    candidate_primitives_per_meas_p95: float = 0.0
    insert_count_total: int = 0
    insert_mass_total: float = 0.0
    insert_mass_p95: float = 0.0
    evicted_count: int = 0
    evicted_mass_total: float = 0.0
    fused_count: int = 0
    fused_mass_total: float = 0.0
    merged_count: int = 0
    staleness_inflation_strength: float = 0.0
    staleness_cov_inflation_trace: float = 0.0
    stale_precision_downscale_total: float = 0.0

    to_dict = _as_dict


_TRIGGER_UNIT = ("dt_scale", "extrinsic_scale", "trust_alpha", "power_beta")
_TRIGGER_ADD = ("lift_strength", "psd_projection_delta", "nu_projection_delta",
                "mass_epsilon_ratio", "anchor_drift_rho")


def trigger_magnitude(inf: InfluenceCert) -> float:
    """Σ additive influence magnitudes + Σ |1 - unit scales| (certificates.py:439-455)."""
    return (sum(getattr(inf, k) for k in _TRIGGER_ADD)
            + sum(abs(1.0 - getattr(inf, k)) for k in _TRIGGER_UNIT))


@dataclass
class CertBundle:
    chart_id: str
    anchor_id: str
    exact: bool
    approximation_triggers: List[str] = field(default_factory=list)
    frobenius_applied: bool = False
    conditioning: ConditioningCert = field(default_factory=ConditioningCert)
    support: SupportCert = field(default_factory=SupportCert)
    mismatch: MismatchCert = field(default_factory=MismatchCert)
    excitation: ExcitationCert = field(default_factory=ExcitationCert)
    influence: InfluenceCert = field(default_factory=InfluenceCert)
    overconfidence: OverconfidenceCert = field(default_factory=OverconfidenceCert)
    compute: ComputeCert = field(default_factory=ComputeCert)
    ot: Optional["OTCert"] = None
    map_update: Optional["MapUpdateCert"] = None

    @classmethod
    def create_exact(cls, chart_id: str, anchor_id: str, **parts) -> "CertBundle":
        return cls(chart_id=chart_id, anchor_id=anchor_id, exact=True,
                   **{k: v for k, v in parts.items() if v is not None})

    @classmethod
    def create_approx(cls, chart_id: str, anchor_id: str, triggers: List[str],
                      frobenius_applied: bool = False, **parts) -> "CertBundle":
        return cls(chart_id=chart_id, anchor_id=anchor_id, exact=False,
                   approximation_triggers=list(triggers), frobenius_applied=frobenius_applied,
                   **{k: v for k, v in parts.items() if v is not None})

    def total_trigger_magnitude(self) -> float:
        return trigger_magnitude(self.influence)

    def to_dict(self) -> Dict[str, Any]:
        d = {"chart_id": self.chart_id, "anchor_id": self.anchor_id, "exact": self.exact,
             "approximation_triggers": self.approximation_triggers,
             "frobenius_applied": self.frobenius_applied}
        for k in ("conditioning", "support", "mismatch", "excitation", "influence",
                  "overconfidence", "compute"):
            d[k] = getattr(self, k).to_dict()
        d["total_trigger_magnitude"] = self.total_trigger_magnitude()
        for k in ("ot", "map_update"):
            if getattr(self, k) is not None:
                d[k] = getattr(self, k).to_dict()
        return d


@dataclass
class ExpectedEffect:
    objective_name: str
    predicted: float
    realized: Optional[float] = None

    to_dict = _as_dict


def aggregate_certificates(certs: List[CertBundle]) -> CertBundle:
    """Pipeline-level summary (certificates.py:511-600): worst-case conditioning, mean support,
    summed mismatch, max excitation, summed/maxed/minned influence per field."""
    if not certs:
        return CertBundle.create_exact(chart_id="unknown", anchor_id="unknown")
    n = float(len(certs))
    c0 = certs[0]
    col = lambda path: [getattr(getattr(c, path[0]), path[1]) for c in certs]  # noqa: E731
    inf = InfluenceCert(
        lift_strength=sum(col(("influence", "lift_strength"))),
        psd_projection_delta=sum(col(("influence", "psd_projection_delta"))),
        nu_projection_delta=sum(col(("influence", "nu_projection_delta"))),
        mass_epsilon_ratio=max(col(("influence", "mass_epsilon_ratio"))),
        anchor_drift_rho=max(col(("influence", "anchor_drift_rho"))),
        dt_scale=min(col(("influence", "dt_scale"))),
        extrinsic_scale=min(col(("influence", "extrinsic_scale"))),
        trust_alpha=min(col(("influence", "trust_alpha"))),
        power_beta=min(col(("influence", "power_beta"))))
    over = OverconfidenceCert(**{f.name: max(col(("overconfidence", f.name)))
                                 for f in fields(OverconfidenceCert)})
    triggers: List[str] = []
    for c in certs:
        triggers.extend(c.approximation_triggers)

    def nelem(shape) -> int:  # ranking key of largest_tensor_shape (non-integer entries rank 0)
        try:
            return int(np.prod([int(v) for v in shape])) if len(shape) else 0
        except (TypeError, ValueError):
            return 0

    comp = [c.compute for c in certs]
    dev = [cc.device_runtime for cc in comp]
    compute = ComputeCert(
        alloc_bytes_est=max(cc.alloc_bytes_est for cc in comp),
        largest_tensor_shape=max((cc.largest_tensor_shape for cc in comp), key=nelem),
        segment_sum_k=max(cc.segment_sum_k for cc in comp),
        psd_projection_count=max(cc.psd_projection_count for cc in comp),
        chol_solve_count=max(cc.chol_solve_count for cc in comp),
        scan_io=max((cc.scan_io for cc in comp), key=lambda io: io.scan_seq),  # latest scan, first on ties
        device_runtime=DeviceRuntimeCert(max(d.host_sync_count_est for d in dev),
                                         max(d.device_to_host_bytes_est for d in dev),
                                         max(d.host_to_device_bytes_est for d in dev),
                                         max(d.jit_recompile_count for d in dev)))
    ots = [c.ot for c in certs if c.ot is not None]
    ot = None
    if ots:  # maxima of defects / p95s, sums of masses and counts, parameters of the first
        o0 = ots[0]
        mx = ("marginal_defect_a", "marginal_defect_b", "dual_gap_proxy", "p95_a", "p95_b", "b_recency_p95")
        sm = ("transport_mass_total", "sum_a", "sum_b", "sum_m", "sum_novel", "nonzero_a", "nonzero_b")
        ot = replace(o0, **{k: max(getattr(o, k) for o in ots) for k in mx},
                     **{k: sum(getattr(o, k) for o in ots) for k in sm})
    mus = [c.map_update for c in certs if c.map_update is not None]
    mu = None
    if mus:  # union of tile ids, sums of counts / masses, maxima of rates and strengths
        act = sorted(set(i for m in mus for i in m.tile_ids_active))
        ina = sorted(set(i for m in mus for i in m.tile_ids_inactive))
        sm = ("tile_cache_hits", "tile_cache_misses", "insert_count_total", "insert_mass_total", "evicted_count",
              "evicted_mass_total", "fused_count", "fused_mass_total", "merged_count",
              "stale_precision_downscale_total")
        mx = ("candidate_tiles_per_meas_mean", "candidate_primitives_per_meas_mean",
              "candidate_primitives_per_meas_p95", "insert_mass_p95", "staleness_inflation_strength",
              "staleness_cov_inflation_trace")
        mu = MapUpdateCert(n_active_tiles=len(act), tile_ids_active=act, n_inactive_tiles=len(ina),
                           tile_ids_inactive=ina, **{k: sum(getattr(m, k) for m in mus) for k in sm},
                           **{k: max(getattr(m, k) for m in mus) for k in mx})
    return CertBundle(
        chart_id=c0.chart_id, anchor_id=c0.anchor_id, exact=all(c.exact for c in certs),
        approximation_triggers=triggers, frobenius_applied=any(c.frobenius_applied for c in certs),
        conditioning=ConditioningCert(min(col(("conditioning", "eig_min"))),
                                      max(col(("conditioning", "eig_max"))),
                                      max(col(("conditioning", "cond"))),
                                      sum(col(("conditioning", "near_null_count")))),
        support=SupportCert(sum(col(("support", "ess_total"))) / n,
                            sum(col(("support", "support_frac"))) / n),
        mismatch=MismatchCert(sum(col(("mismatch", "nll_per_ess"))),
                              sum(col(("mismatch", "directional_score"))) / n),
        excitation=ExcitationCert(max(col(("excitation", "dt_effect"))),
                                  max(col(("excitation", "extrinsic_effect")))),
        influence=inf, overconfidence=over, compute=compute, ot=ot, map_update=mu)
