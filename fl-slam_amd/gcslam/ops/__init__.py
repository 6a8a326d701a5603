"""Drop-in replacements for the reference operators on the GC-SLAM v2 hot path
(fl_slam_poc.backend.operators + archive/legacy_operators). Same names, arguments, defaults,
result dataclasses and (Result, CertBundle, ExpectedEffect) returns; compute runs in libgcslam."""

from .point_budget import PointBudgetResult, point_budget_resample
from .deskew_constant_twist import DeskewConstantTwistResult, deskew_constant_twist
from .binning import (BinAtlas, BinSoftAssignResult, ScanBinStats, bin_soft_assign,
                      create_fibonacci_atlas, scan_bin_moment_match)
from .kappa import kappa_from_resultant_batch
from .primitives import domain_projection_psd, domain_projection_psd_batch

__all__ = [
    "PointBudgetResult", "point_budget_resample", "DeskewConstantTwistResult",
    "deskew_constant_twist", "BinAtlas", "BinSoftAssignResult", "ScanBinStats",
    "bin_soft_assign", "create_fibonacci_atlas", "scan_bin_moment_match",
    "kappa_from_resultant_batch", "domain_projection_psd", "domain_projection_psd_batch",
]
