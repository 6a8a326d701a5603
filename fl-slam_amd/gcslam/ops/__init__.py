"""Drop-in replacements for the reference operators on the GC-SLAM v2 hot path
(fl_slam_poc.backend.operators + archive/legacy_operators). Same names, arguments, defaults,
result dataclasses and (Result, CertBundle, ExpectedEffect) returns; compute runs in libgcslam."""

from .point_budget import PointBudgetResult, point_budget_resample
from .deskew_constant_twist import DeskewConstantTwistResult, deskew_constant_twist
from .binning import (BinAtlas, BinSoftAssignResult, ScanBinStats, bin_soft_assign,
                      create_fibonacci_atlas, point_directions, scan_bin_moment_match)
from .kappa import kappa_from_resultant_batch
from .primitives import domain_projection_psd, domain_projection_psd_batch, spd_cholesky_inverse_lifted
from .predict import predict_diffusion
from .imu_preintegration import (imu_accel_meas_iw_suffstats_from_gravity_dir_jax,
                                 imu_gyro_meas_iw_suffstats_from_avg_rate_jax,
                                 preintegrate_imu_relative_pose_jax, smooth_window_weights)
from .matrix_fisher_evidence import (MatrixFisherResult, PlanarTranslationResult, ScatterMetrics,
                                     matrix_fisher_rotation_evidence, planar_translation_evidence)
from .excitation import apply_excitation_prior_scaling_jax, compute_excitation_scales_jax
from .fusion import FusionScaleResult, fusion_scale_from_certificates, info_fusion_additive
from .recompose import (AnchorDriftResult, RecomposeResult, anchor_drift_update,
                        pose_update_frobenius_recompose)
from .inverse_wishart import (MeasurementNoiseIWState, ProcessNoiseIWState,
                              measurement_noise_apply_suffstats_jax,
                              process_noise_iw_apply_suffstats_jax,
                              process_noise_iw_suffstats_from_info_jax, process_noise_state_to_Q_jax)
from .hypothesis import HypothesisProjectionResult, hypothesis_barycenter_projection
from .pointcloud import PointCloud2Msg, PointField, imu_message_to_base, imu_window_padded, parse_pointcloud2_vlp16
from .imu_odom_evidence import (ImuDependenceInflationResult, ImuGyroEvidenceResult, ImuPreintegrationFactorResult,
                                OdomDependenceInflationResult, OdomEvidenceResult, OdomVelocityEvidenceResult,
                                OdomYawRateEvidenceResult, PlanarPriorResult, PoseTwistConsistencyResult,
                                TimeResolvedImuResult, VelocityZPriorResult, imu_dependence_inflation,
                                imu_gyro_rotation_evidence, imu_preintegration_factor,
                                imu_vmf_gravity_evidence_time_resolved, odom_dependence_inflation,
                                odom_quadratic_evidence, odom_velocity_evidence, odom_yawrate_evidence,
                                planar_z_prior, pose_twist_kinematic_consistency, velocity_z_prior)

__all__ = [
    "PointBudgetResult", "point_budget_resample", "DeskewConstantTwistResult",
    "deskew_constant_twist", "BinAtlas", "BinSoftAssignResult", "ScanBinStats",
    "bin_soft_assign", "create_fibonacci_atlas", "point_directions", "scan_bin_moment_match",
    "kappa_from_resultant_batch", "domain_projection_psd", "domain_projection_psd_batch", "spd_cholesky_inverse_lifted",
    "predict_diffusion", "smooth_window_weights", "preintegrate_imu_relative_pose_jax",
    "imu_gyro_meas_iw_suffstats_from_avg_rate_jax", "imu_accel_meas_iw_suffstats_from_gravity_dir_jax",
    "MatrixFisherResult", "PlanarTranslationResult", "ScatterMetrics", "matrix_fisher_rotation_evidence",
    "planar_translation_evidence", "compute_excitation_scales_jax", "apply_excitation_prior_scaling_jax",
    "FusionScaleResult", "fusion_scale_from_certificates", "info_fusion_additive", "RecomposeResult",
    "AnchorDriftResult", "pose_update_frobenius_recompose", "anchor_drift_update", "ProcessNoiseIWState",
    "MeasurementNoiseIWState", "process_noise_iw_suffstats_from_info_jax", "process_noise_iw_apply_suffstats_jax",
    "process_noise_state_to_Q_jax", "measurement_noise_apply_suffstats_jax", "HypothesisProjectionResult",
    "hypothesis_barycenter_projection", "OdomEvidenceResult", "odom_quadratic_evidence", "TimeResolvedImuResult",
    "imu_vmf_gravity_evidence_time_resolved", "ImuDependenceInflationResult", "imu_dependence_inflation",
    "ImuGyroEvidenceResult", "imu_gyro_rotation_evidence", "ImuPreintegrationFactorResult",
    "imu_preintegration_factor", "PlanarPriorResult", "planar_z_prior", "VelocityZPriorResult", "velocity_z_prior",
    "OdomVelocityEvidenceResult", "odom_velocity_evidence", "OdomYawRateEvidenceResult", "odom_yawrate_evidence",
    "PoseTwistConsistencyResult", "pose_twist_kinematic_consistency", "OdomDependenceInflationResult",
    "odom_dependence_inflation", "PointCloud2Msg", "PointField", "parse_pointcloud2_vlp16", "imu_window_padded", "imu_message_to_base",
]
