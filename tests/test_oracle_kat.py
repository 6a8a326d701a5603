"""Pins the CPU oracle (oracle/gc_oracle.py) against the known-answer and property tests the
reference's own suites hold for this path. Each test cites the reference test it restates;
inputs drawn there from jax.random are replaced by seeded NumPy draws of the same shape."""

import math

import numpy as np
import pytest

from oracle import gc_oracle as O

REF_PRIM = "fl_ws/src/fl_slam_poc/test/test_primitives.py"
REF_AUDIT = "fl_ws/src/fl_slam_poc/test/test_audit_invariants.py"
REF_OPS = "archive/legacy_tests/test_operators.py"


# ---- test_primitives.py:56-94 (TestDomainProjectionPSD)
def test_psd_identity_unchanged():
    Mp, c = O.psd_project(np.eye(3))
    assert np.allclose(Mp, np.eye(3), atol=1e-10) and c[0] < 1e-10


def test_psd_negative_eigenvalue_clamped():
    Mp, c = O.psd_project(np.array([[1.0, 0.0], [0.0, -0.5]]))
    assert np.all(np.linalg.eigvalsh(Mp) >= 1e-12) and c[0] > 0


def test_psd_conditioning():
    _, c = O.psd_project(np.eye(3))
    assert c[2] > 0 and c[3] >= c[2] and c[4] >= 1.0


@pytest.mark.parametrize("M", [np.array([[1.0, 0.0], [0.0, -1.0]]), np.zeros((3, 3)),
                               np.array([[1.0, 2.0], [3.0, 4.0]])])
def test_psd_always_psd(M):
    Mp, _ = O.psd_project(M)
    assert np.all(np.linalg.eigvalsh(Mp) >= 1e-12 - 1e-15)


# ---- test_audit_invariants.py:119-135
def test_psd_extreme_negative():
    Mp, c = O.psd_project(np.diag([1.0, -1000.0, 1.0]), eps_psd=1e-6)
    assert np.min(np.linalg.eigvalsh(Mp)) >= 1e-6 - 1e-12 and c[0] > 0


# ---- test_primitives.py:100-125 / test_audit_invariants.py:148-164 (lifted solve)
def test_lifted_solve_identity():
    x, lift = O.chol_solve_lifted(np.eye(3), np.array([1.0, 2.0, 3.0]))
    assert np.allclose(x, [1.0, 2.0, 3.0], atol=1e-8) and lift > 0


def test_lifted_solve_singular_and_near_singular():
    x, _ = O.chol_solve_lifted(np.array([[1.0, 0.0], [0.0, 0.0]]), np.ones(2), eps_lift=1e-6)
    assert np.all(np.isfinite(x))
    x, lift = O.chol_solve_lifted(np.diag([1.0, 1e-15, 1.0]), np.ones(3), eps_lift=1e-9)
    assert np.all(np.isfinite(x)) and lift > 0


# ---- test_audit_invariants.py:77-117 (kappa order independence, smoothness)
def test_kappa_order_independent():
    a = O.kappa_batch(np.array([0.3, 0.5, 0.7, 0.2, 0.8]))
    b = O.kappa_batch(np.array([0.7, 0.3, 0.8, 0.5, 0.2]))
    np.testing.assert_allclose(np.sort(a), np.sort(b), atol=1e-12)


def test_kappa_smooth():
    k = O.kappa_batch(np.linspace(0.01, 0.99, 100))
    d = np.abs(np.diff(k))
    assert d.max() < 100 * np.median(d)


# ---- test_audit_invariants.py:412-426 (batch == scalar, rtol 1e-10); test_operators.py:97-114
def test_kappa_batch_matches_scalar():
    R = np.array([0.1, 0.3, 0.5, 0.7, 0.85])
    kb = O.kappa_batch(R)
    for i, r in enumerate(R):
        np.testing.assert_allclose(kb[i], O.kappa_scalar(r), rtol=1e-10)


def test_kappa_nonnegative_and_monotone():
    assert all(O.kappa_scalar(r) >= 0 for r in (0.0, 0.5, 0.9, 0.99))
    k = [O.kappa_scalar(r) for r in (0.1, 0.5, 0.8)]
    assert k[0] < k[1] < k[2]


# ---- test_audit_invariants.py:137-146 (softmax at ±1000)
def test_softmax_extreme():
    x = np.array([1000.0, -1000.0, 0.0, 500.0, -500.0])
    e = np.exp(x - x.max())
    p = e / e.sum()
    assert np.all(np.isfinite(p)) and abs(p.sum() - 1.0) < 1e-6


# ---- test_audit_invariants.py:224-328 (Lie round trips on the reference's fixed vectors)
@pytest.mark.parametrize("w,atol", [([0.01, -0.02, 0.015], 1e-10), ([0.5, -0.7, 0.3], 1e-10),
                                    ([1.5, -1.2, 0.8], 1e-9), ([math.pi - 0.01, 0.0, 0.0], 1e-8)])
def test_so3_roundtrip(w, atol):
    R = O.so3_exp(np.array(w))
    np.testing.assert_allclose(O.so3_exp(O.so3_log(R)), R, atol=atol)


@pytest.mark.parametrize("xi,atol", [([0.1, -0.05, 0.02, 0.2, -0.1, 0.05], 1e-9),
                                     ([1.0, -0.5, 0.3, 0.8, -0.6, 0.4], 1e-8)])
def test_se3_roundtrip(xi, atol):
    T = O.se3_exp(np.array(xi))
    np.testing.assert_allclose(O.se3_exp(O.se3_log(T)), T, atol=atol)


def test_so3_log_exp_random():
    rng = np.random.default_rng(456)
    for _ in range(10):
        w = rng.normal(size=3) * 0.5
        np.testing.assert_allclose(O.so3_log(O.so3_exp(w)), w, atol=1e-9)


def test_se3_V_inv():
    phi = np.array([0.3, -0.2, 0.1])
    np.testing.assert_allclose(O.se3_V_inv(phi) @ O.se3_V(phi), np.eye(3), atol=1e-10)
    tiny = np.array([1e-9, -1e-9, 1e-9])
    np.testing.assert_allclose(O.se3_V(tiny), np.eye(3), atol=1e-7)
    np.testing.assert_allclose(O.se3_V_inv(tiny) @ O.se3_V(tiny), np.eye(3), atol=1e-10)


# ---- test_operators.py:29-73 (PointBudgetResample)
def test_budget_respects_cap_and_mass():
    rng = np.random.default_rng(42)
    P = rng.normal(size=(10000, 3))
    r = O.point_budget_resample(P, np.linspace(0, 1, 10000), np.ones(10000), n_points_cap=8192)
    assert r["points"].shape[0] <= 8192
    r = O.point_budget_resample(P[:100], np.linspace(0, 1, 100), np.ones(100), n_points_cap=8192)
    assert abs(r["total_mass_out"] - r["total_mass_in"]) < 1e-6


# ---- test_operators.py:117-166 (BinSoftAssign rows sum to 1; exact)
def test_soft_assign_rows_sum_to_one():
    rng = np.random.default_rng(42)
    d = rng.normal(size=(50, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = O.bin_soft_assign(d, O.fibonacci_atlas(20))
    assert np.allclose(r["resp"].sum(1), 1.0, atol=1e-6) and r["trig"] == 0.0


# ---- test_operators.py:330-395 (Predict stamp), :398-447 (InfoFusion trace), :450-511 (floor)
def test_predict_timestamp_updated():
    b = O.Belief(np.zeros(6), np.zeros(22), np.eye(22), np.zeros(22), 1.0)
    out, _ = O.predict_diffusion(b, np.eye(22), 0.5)
    assert out.stamp_sec == 1.5


def test_info_fusion_trace_increases():
    L, h, _ = O.info_fusion_additive(np.eye(22), np.zeros(22), 0.5 * np.eye(22), np.zeros(22), 1.0)
    assert np.trace(L) >= 22.0


def test_hypothesis_weight_floor():
    Ls = np.stack([np.eye(22)] * 4)
    r = O.hypothesis_barycenter(Ls, np.zeros((4, 22)), np.zeros((4, 22)),
                                np.array([0.998, 0.001, 0.0005, 0.0005]), 0.0025)
    assert r["floor_adjustment"] > 0


# ---- test_geometric_compositional_invariants.py:197-212
def test_total_trigger_at_least_lift_plus_psd():
    assert O.trigger(lift=1e-8, psd=0.3) >= 1e-8 + 0.3


# ---- archive/legacy_tests/test_operators.py:300-327 (gyro residual direction: pred^{-1} ∘ meas)
def test_gyro_residual_is_pred_inverse_composed_with_meas():
    pred = np.array([0.01, -0.02, 0.005])
    r = O.imu_gyro_rotation_evidence(np.zeros(3), pred, np.zeros(3), np.eye(3), 1.0)
    assert np.allclose(r["r_rot"], -pred, atol=1e-6)


@pytest.mark.gpu
def test_gpu_gyro_residual_direction(ctx):
    from gcslam.ops import imu_gyro_rotation_evidence
    pred = np.array([0.01, -0.02, 0.005])
    res, _, _ = imu_gyro_rotation_evidence(np.zeros(3), pred, np.zeros(3), np.eye(3), 1.0, ctx=ctx)
    assert np.allclose(res.r_rot, -pred, atol=1e-6)
