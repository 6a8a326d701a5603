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
    ot: Optional[Any] = None
    map_update: Optional[Any] = None

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
        influence=inf, overconfidence=over)
