"""GC-SLAM v2 constants used on the hot path.

Values mirror fl_slam_poc/common/constants.py:54-143, :259-281 and PipelineConfig defaults
(backend/pipeline.py:96-160). Names keep the reference's GC_* spelling so code written
against the reference reads the same. Build-declared values the reference never records
(GC_B_BINS, GC_TAU_SOFT_ASSIGN) are marked.
"""

GC_CHART_ID = "GC-RIGHT-01"
GC_D_Z = 22
D_Z = GC_D_Z
GC_K_HYP = 4
GC_HYP_WEIGHT_FLOOR = 0.0025  # 0.01 / K_HYP (docs/GC_SLAM.md:122); batched driver uses 0.01/H
GC_N_POINTS_CAP = 8192
GC_MAX_IMU_PREINT_LEN = 512

GC_EPS_PSD = 1e-12
GC_EPS_LIFT = 1e-9
GC_EPS_MASS = 1e-12
GC_EPS_R = 1e-6
GC_EXC_EPS = 1e-12
GC_GRAVITY_W = (0.0, 0.0, -9.81)

GC_ALPHA_MIN = 1.0
GC_ALPHA_MAX = 1.0
GC_KAPPA_SCALE = 1.0
GC_C0_COND = 1e6
GC_KAPPA_BLEND_R0 = 0.8
GC_KAPPA_BLEND_TAU = 0.03
GC_C_DT = 1.0
GC_C_EX = 1.0
GC_C_FROB = 1.0
GC_ANCHOR_DRIFT_M0 = 0.5
GC_ANCHOR_DRIFT_R0 = 0.2
GC_TIME_WARP_SIGMA_FRAC = 0.1
GC_OU_DAMPING_LAMBDA = 0.1
GC_WEIGHT_FLOOR = 1e-12
GC_RANGE_WEIGHT_SIGMA = 0.25
GC_RANGE_WEIGHT_MIN_R = 0.5
GC_RANGE_WEIGHT_MAX_R = 50.0
GC_IW_NU_WEAK_ADD = 0.5
GC_IMU_GYRO_NOISE_DENSITY = 8.7e-7   # constants.py:190
GC_IMU_ACCEL_NOISE_DENSITY = 9.5e-5  # constants.py:201
GC_PLANAR_Z_REF = 0.0                # constants.py:294
GC_PLANAR_Z_SIGMA = 0.1              # constants.py:305
GC_PLANAR_VZ_SIGMA = 0.01            # constants.py:310
# PrimitiveMap maintenance (constants.py:392-477)
GC_PRIMITIVE_MAP_MAX_SIZE = 50000
GC_RECENCY_DECAY_LAMBDA = 0.02
GC_RECENCY_MIN_SCALE = 0.05
GC_PRIMITIVE_FORGETTING_FACTOR = 0.995
GC_PRIMITIVE_MERGE_THRESHOLD = 0.1
GC_K_MERGE_PAIRS_PER_TILE = 4
GC_PRIMITIVE_MERGE_MAX_TILE_SIZE = 2048
GC_PRIMITIVE_CULL_WEIGHT_THRESHOLD = 1e-4
GC_K_INSERT_TILE = 64

# PipelineConfig defaults (pipeline.py:118-131; gc_unified.yaml:41-57)
POWER_BETA_MIN = 0.25
POWER_BETA_EXC_C = 50.0
POWER_BETA_Z_C = 1.0
FORGETTING_FACTOR = 0.99

# Build-declared (absent from the reference; parity of these two values is unpinned)
GC_B_BINS = 48
GC_TAU_SOFT_ASSIGN = 0.1

# gc_unified.yaml:18-24
T_BASE_LIDAR = (-0.065447, -0.100474, 0.108987, -0.002723, -0.069383, 0.028979)
