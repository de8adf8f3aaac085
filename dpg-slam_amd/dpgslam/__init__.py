"""dpgslam -- MI355X-native DPG-SLAM hot path (ICP scan matching + pose-graph Gauss-Newton).

Python face of the C ABI in include/dpg_slam_c.h (libdpg.so, HIP kernels for gfx950).
"""
from ._abi import (DpgError, FACTOR_DTYPE, RESULT_DTYPE, default_gn_params, default_icp_params,  # noqa: F401
                   lib, LIB_PATH)
from .api import (Context, Node, calculate_ICP_COV, downsample, icp_guess, inverse_transform_point,  # noqa: F401
                  prior_factor, between_factor, odometry_factor, scan_to_cloud, scans_to_clouds, transform_point)
