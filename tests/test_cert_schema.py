"""The CertBundle boundary type against the reference's own schema tests
(fl_ws/src/fl_slam_poc/test/test_cert_schema.py:60-280, JAX-free in the reference too): every
component certificate and compute sub-block exists with the reference's types, ``to_dict`` carries
the reference's key set, ``aggregate_certificates`` keeps the schema and its max / latest-scan
rules, and a JSON snapshot of a cert is deterministic. Plus the trigger-magnitude rule that feeds
recompose (common/certificates.py:439-455). CPU only."""

import hashlib
import json

import pytest

from gcslam.certificates import (CertBundle, ComputeCert, ConditioningCert, DeviceRuntimeCert, ExcitationCert,
                                 ExpectedEffect, InfluenceCert, MapUpdateCert, MismatchCert, OTCert,
                                 OverconfidenceCert, ScanIOCert, SupportCert, aggregate_certificates)


def _exact(chart="chart", anchor="anchor"):
    return CertBundle.create_exact(chart_id=chart, anchor_id=anchor)


def _approx(chart="chart", anchor="anchor", triggers=("test",), frob=False):
    return CertBundle.create_approx(chart_id=chart, anchor_id=anchor, triggers=list(triggers), frobenius_applied=frob)


def _snapshot(c: CertBundle) -> str:
    """A content hash of the cert's dict form (test_cert_schema.py:233-238)."""
    return hashlib.sha256(json.dumps(c.to_dict(), sort_keys=True, default=str).encode()).hexdigest()[:16]


def test_compute_block_types():
    """test_cert_schema.py:60-87: ComputeCert, its ScanIOCert and DeviceRuntimeCert, with types."""
    c = _exact()
    cc = c.compute
    assert isinstance(cc, ComputeCert)
    assert isinstance(cc.alloc_bytes_est, int) and isinstance(cc.segment_sum_k, int)
    assert isinstance(cc.largest_tensor_shape, tuple) and len(cc.largest_tensor_shape) == 2
    assert isinstance(cc.psd_projection_count, int) and isinstance(cc.chol_solve_count, int)
    assert isinstance(cc.scan_io, ScanIOCert)
    assert isinstance(cc.scan_io.scan_seq, int) and isinstance(cc.scan_io.scan_stamp_sec, float)
    assert isinstance(cc.scan_io.streams, dict)
    dr = cc.device_runtime
    assert isinstance(dr, DeviceRuntimeCert)
    for k in ("host_sync_count_est", "device_to_host_bytes_est", "host_to_device_bytes_est", "jit_recompile_count"):
        assert isinstance(getattr(dr, k), int)
    d = c.to_dict()
    assert {"scan_io", "device_runtime"} <= set(d["compute"])


def test_overconfidence_growth_sentinels():
    """test_cert_schema.py:90-117: the original five fields plus the three growth sentinels
    (floats), all in to_dict."""
    oc = _exact().overconfidence
    assert isinstance(oc, OverconfidenceCert)
    for k in ("excitation_total", "ess_to_excitation", "cond_to_support", "dt_asymmetry", "z_to_xy_ratio"):
        assert hasattr(oc, k)
    for k in ("ess_growth_rate", "excitation_growth_rate", "nullspace_energy_ratio"):
        assert isinstance(getattr(oc, k), float)
        assert k in oc.to_dict()


def test_all_component_certs_present():
    """test_cert_schema.py:120-139."""
    c = _exact()
    for k in ("chart_id", "anchor_id", "exact", "approximation_triggers", "frobenius_applied"):
        assert hasattr(c, k)
    for k, t in (("conditioning", ConditioningCert), ("support", SupportCert), ("mismatch", MismatchCert),
                 ("excitation", ExcitationCert), ("influence", InfluenceCert),
                 ("overconfidence", OverconfidenceCert), ("compute", ComputeCert)):
        assert isinstance(getattr(c, k), t), k


def test_to_dict_key_set():
    """test_cert_schema.py:142-185: the top-level and nested keys of to_dict."""
    d = _approx("test_chart", "test_anchor", ["test_trigger"], True).to_dict()
    top = {"chart_id", "anchor_id", "exact", "approximation_triggers", "frobenius_applied", "conditioning",
           "support", "mismatch", "excitation", "influence", "overconfidence", "compute", "total_trigger_magnitude"}
    assert top <= set(d)
    assert {"eig_min", "eig_max", "cond"} <= set(d["conditioning"])
    assert {"ess_total", "support_frac"} <= set(d["support"])
    assert {"ess_growth_rate", "excitation_growth_rate", "nullspace_energy_ratio"} <= set(d["overconfidence"])
    assert {"alloc_bytes_est", "scan_io", "device_runtime"} <= set(d["compute"])
    assert d["frobenius_applied"] is True and d["approximation_triggers"] == ["test_trigger"]


def test_to_dict_with_ot_and_map_blocks():
    """The optional OT / map-update blocks serialise too (CertBundle.to_dict, certificates.py)."""
    c = _exact()
    c.ot = OTCert(sum_a=1.0, nonzero_a=3)
    c.map_update = MapUpdateCert(n_active_tiles=1, tile_ids_active=[7])
    d = c.to_dict()
    assert d["ot"]["sum_a"] == 1.0 and d["ot"]["nonzero_a"] == 3
    assert d["map_update"]["tile_ids_active"] == [7]
    json.dumps(d)


def test_aggregation_takes_the_latest_scan_io():
    """test_cert_schema.py:193-200: the aggregate's scan_io is that of the highest scan_seq."""
    c1, c2 = _exact(), _exact()
    c1.compute.scan_io.scan_seq, c2.compute.scan_io.scan_seq = 1, 2
    assert aggregate_certificates([c1, c2]).compute.scan_io.scan_seq == 2
    assert aggregate_certificates([c2, c1]).compute.scan_io.scan_seq == 2


def test_aggregation_keeps_schema_and_maxima():
    """test_cert_schema.py:203-219 plus the compute rules of aggregate_certificates
    (certificates.py:597-633): maxima of counts / bytes, the largest tensor shape."""
    c1, c2 = _exact(), _approx(triggers=["test"])
    c1.overconfidence.ess_growth_rate = 0.1
    c2.overconfidence.excitation_growth_rate = 0.2
    c1.compute.alloc_bytes_est, c2.compute.alloc_bytes_est = 10, 5
    c1.compute.largest_tensor_shape, c2.compute.largest_tensor_shape = (4, 4), (2, 100)
    c2.compute.device_runtime.host_sync_count_est = 3
    agg = aggregate_certificates([c1, c2])
    for k in ("ess_growth_rate", "excitation_growth_rate", "nullspace_energy_ratio"):
        assert hasattr(agg.overconfidence, k)
    assert agg.overconfidence.ess_growth_rate == 0.1 and agg.overconfidence.excitation_growth_rate == 0.2
    assert agg.exact is False and agg.approximation_triggers == ["test"]
    assert agg.compute.alloc_bytes_est == 10 and agg.compute.largest_tensor_shape == (2, 100)
    assert agg.compute.device_runtime.host_sync_count_est == 3


def test_aggregation_of_ot_and_map_blocks():
    """OT: maxima of defects, sums of masses, the first cert's parameters; map: union of tiles."""
    c1, c2, c3 = _exact(), _exact(), _exact()
    c1.ot = OTCert(marginal_defect_a=0.1, sum_a=1.0, epsilon=0.5, nonzero_a=2)
    c2.ot = OTCert(marginal_defect_a=0.3, sum_a=2.0, epsilon=0.9, nonzero_a=1)
    c1.map_update = MapUpdateCert(tile_ids_active=[1, 2], fused_count=3)
    c3.map_update = MapUpdateCert(tile_ids_active=[2, 5], fused_count=4, staleness_inflation_strength=0.7)
    agg = aggregate_certificates([c1, c2, c3])
    assert agg.ot.marginal_defect_a == 0.3 and agg.ot.sum_a == 3.0 and agg.ot.epsilon == 0.5
    assert agg.ot.nonzero_a == 3
    assert agg.map_update.n_active_tiles == 3 and sorted(agg.map_update.tile_ids_active) == [1, 2, 5]
    assert agg.map_update.fused_count == 7 and agg.map_update.staleness_inflation_strength == 0.7
    assert aggregate_certificates([_exact()]).ot is None


def test_aggregate_of_nothing():
    """test_cert_schema.py:222-227."""
    agg = aggregate_certificates([])
    assert (agg.chart_id, agg.anchor_id, agg.exact) == ("unknown", "unknown", True)


@pytest.mark.parametrize("make", [lambda: _exact(), lambda: _approx(triggers=["test", "another"], frob=True)])
def test_snapshot_is_deterministic(make):
    """test_cert_schema.py:241-262: equal inputs, equal snapshot id."""
    assert _snapshot(make()) == _snapshot(make())


def test_snapshot_separates_inputs():
    """test_cert_schema.py:265-274."""
    assert _snapshot(_exact(chart="chart1")) != _snapshot(_exact(chart="chart2"))


def test_expected_effect_schema():
    """test_cert_schema.py:282-294."""
    d = ExpectedEffect(objective_name="test_objective", predicted=1.0, realized=0.9).to_dict()
    assert d == {"objective_name": "test_objective", "predicted": 1.0, "realized": 0.9}


def test_total_trigger_magnitude_rule():
    """certificates.py:439-455: Σ of the additive influences + Σ |1 - scale| of the unit ones."""
    inf = InfluenceCert(lift_strength=0.1, psd_projection_delta=0.2, nu_projection_delta=0.3, mass_epsilon_ratio=0.4,
                        anchor_drift_rho=0.5, dt_scale=0.9, extrinsic_scale=1.2, trust_alpha=0.7, power_beta=1.0)
    c = CertBundle.create_approx("c", "a", ["x"], influence=inf)
    assert c.total_trigger_magnitude() == pytest.approx(1.5 + 0.1 + 0.2 + 0.3 + 0.0)
    assert _exact().total_trigger_magnitude() == 0.0
