"""ctypes view of the C ABI in include/dpg_slam_c.h and include/dpg_icp_cov.h.

The shared library is dpg-slam_amd/lib/libdpg.so (built by `make -C dpg-slam_amd`, or
`__graft_entry__.build()`).  There is no fallback implementation: if the library is missing,
`lib()` raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPGSLAM_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libdpg.so")

DPG_OK = 0
DPG_FACTOR_PRIOR = 0
DPG_FACTOR_BETWEEN = 1
DPG_ICP_OK = 0
DPG_ICP_TOO_FEW_CORR = 1
DPG_ICP_LANES = 512


class IcpParams(C.Structure):
    """dpg_icp_params -- PoseGraphParameters ICP fields (parameters.h:105-141)."""

    _fields_ = [
        ("icp_maximum_iterations", C.c_int32),
        ("icp_use_reciprocal_correspondences", C.c_int32),
        ("icp_maximum_transformation_epsilon", C.c_double),
        ("icp_max_correspondence_distance", C.c_double),
        ("ransac_iterations", C.c_int32),
        ("downsample_icp_points_ratio", C.c_int32),
        ("laser_x_variance", C.c_float),
        ("laser_y_variance", C.c_float),
        ("laser_theta_variance", C.c_float),
        ("min_number_correspondences", C.c_int32),
        ("mse_threshold_absolute", C.c_double),
    ]


class IcpResult(C.Structure):
    _fields_ = [
        ("T", C.c_float * 6),
        ("z", C.c_float * 3),
        ("converged", C.c_int32),
        ("iterations", C.c_int32),
        ("n_corr", C.c_int32),
        ("status", C.c_int32),
        ("pad", C.c_int32),
        ("fitness", C.c_double),
    ]


class Factor(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("i", C.c_int32),
        ("j", C.c_int32),
        ("pad", C.c_int32),
        ("z", C.c_double * 3),
        ("info", C.c_double * 3),
    ]


class GnParams(C.Structure):
    _fields_ = [
        ("max_iterations", C.c_int32),
        ("use_error_criteria", C.c_int32),
        ("delta_tol", C.c_double),
        ("relative_error_tol", C.c_double),
        ("absolute_error_tol", C.c_double),
        ("pcg_rel_tol", C.c_double),
        ("pcg_max_iterations", C.c_int32),
        ("pcg_check_every", C.c_int32),
        ("linear_solver", C.c_int32),
        ("reuse_factorization", C.c_int32),
        ("refactor_delta", C.c_double),
    ]


DPG_SOLVER_CHOLESKY = 0
DPG_SOLVER_PCG = 1


class GnStats(C.Structure):
    _fields_ = [
        ("iterations", C.c_int32),
        ("pcg_iterations", C.c_int32),
        ("initial_error", C.c_double),
        ("final_error", C.c_double),
        ("last_delta_inf", C.c_double),
        ("ms_total", C.c_double),
        ("ms_per_iteration", C.c_double),
    ]


class ReoptParams(C.Structure):
    _fields_ = [
        ("max_node_dist_within_pass", C.c_float),
        ("max_node_dist_across_passes", C.c_float),
        ("new_pass_std_dev", C.c_float * 3),
        ("motion_model", C.c_float * 4),
        ("odometry_constraints", C.c_int32),
    ]


class ReoptStats(C.Structure):
    _fields_ = [
        ("n_factors", C.c_int64),
        ("n_icp_edges", C.c_int64),
        ("n_candidates", C.c_int64),
        ("n_loop_closures", C.c_int64),
        ("ms_candidates", C.c_double),
        ("ms_icp", C.c_double),
        ("ms_gn", C.c_double),
        ("gn", GnStats),
    ]


DPG_INC_ISAM2 = 0
DPG_INC_BATCH = 1


class IncParams(C.Structure):
    """dpg_inc_params -- the incremental per-node solve (ISAM2 defaults)."""

    _fields_ = [
        ("mode", C.c_int32),
        ("relinearize_skip", C.c_int32),
        ("relinearize_threshold", C.c_double),
        ("duplicate_factors", C.c_int32),
        ("reorder_every", C.c_int32),
        ("reorder_lead", C.c_int32),
        ("full_refactor", C.c_int32),
        ("gn", GnParams),
    ]


class SolverOptions(C.Structure):
    """dpg_solver_options -- the supernodal Cholesky's options (per context)."""

    _fields_ = [(n, C.c_int32) for n in ("order", "fused", "solve_stage", "solve_maxseg", "solve_dinv",
                                          "merge_single", "max_supernode_cols", "solve_inv_cols")] + [("relax_fraction", C.c_double)]


class IncStats(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int64),
        ("n_factors", C.c_int64),
        ("nnz_l", C.c_int64),
        ("reordered", C.c_int32),
        ("relinearized", C.c_int32),
        ("gn_iterations", C.c_int32),
        ("fronts_kept", C.c_int32),
        ("error", C.c_double),
        ("last_delta_inf", C.c_double),
        ("ms_total", C.c_double),
        ("ms_symbolic", C.c_double),
        ("ms_numeric", C.c_double),
    ]


class AddNodeStats(C.Structure):
    _fields_ = [
        ("n_icp_edges", C.c_int64),
        ("n_loop_closures", C.c_int64),
        ("ms_icp", C.c_double),
        ("update", IncStats),
    ]


# numpy mirrors of the array-of-struct types (same layout as the C structs)
RESULT_DTYPE = np.dtype(
    [("T", "<f4", (6,)), ("z", "<f4", (3,)), ("converged", "<i4"), ("iterations", "<i4"),
     ("n_corr", "<i4"), ("status", "<i4"), ("pad", "<i4"), ("fitness", "<f8")], align=True)
FACTOR_DTYPE = np.dtype(
    [("kind", "<i4"), ("i", "<i4"), ("j", "<i4"), ("pad", "<i4"), ("z", "<f8", (3,)),
     ("info", "<f8", (3,))], align=True)
assert RESULT_DTYPE.itemsize == C.sizeof(IcpResult) == 64
assert FACTOR_DTYPE.itemsize == C.sizeof(Factor) == 64

P = C.c_void_p
F32P = C.POINTER(C.c_float)
F64P = C.POINTER(C.c_double)
I32P = C.POINTER(C.c_int32)
I64P = C.POINTER(C.c_int64)
U8P = C.POINTER(C.c_uint8)

# name -> (restype, argtypes); the full exported surface of include/*.h

class ChangeParams(C.Structure):
    """dpg_change_params -- DpgParameters (parameters.h:37-87) + the laser pose (parameters.h:319-339)."""

    _fields_ = [
        ("num_sectors", C.c_int32),
        ("current_pose_chain_len", C.c_int32),
        ("num_bins_for_change_detection", C.c_int32),
        ("pad", C.c_int32),
        ("delta_change_threshold", C.c_double),
        ("current_pose_graph_coverage_threshold", C.c_double),
        ("occ_grid_resolution", C.c_double),
        ("minimum_percent_active_sectors", C.c_float),
        ("distance_threshold_for_local_submap_nodes", C.c_float),
        ("laser", C.c_float * 3),
        ("pad2", C.c_float),
    ]


class ChangeStats(C.Structure):
    """dpg_change_stats -- counters and timings of one dpg_execute_dpg."""

    _fields_ = [(n, C.c_int64) for n in (
        "n_chain", "n_candidates", "n_submap_nodes", "n_chain_cells", "n_uncovered", "n_added", "n_removed",
        "n_committed", "n_sectors_deactivated", "n_nodes_deactivated", "grid_cells", "n_samples")] + [
        ("ms_total", C.c_double), ("ms_kernels", C.c_double)]

    COUNTERS = ("n_chain", "n_candidates", "n_submap_nodes", "n_chain_cells", "n_uncovered", "n_added",
                "n_removed", "n_committed", "n_sectors_deactivated", "n_nodes_deactivated")

    def counters(self) -> dict:
        return {k: int(getattr(self, k)) for k in self.COUNTERS}


ALLREDUCE_F64 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64)
ALLREDUCE_F32 = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_float), C.c_int64)
ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)


class CollOps(C.Structure):
    """dpg_coll_ops -- the caller's blocking host-memory collectives (dpg_ctx_create_rank_ops)."""

    _fields_ = [("user", C.c_void_p), ("allreduce_sum_f64", ALLREDUCE_F64), ("allreduce_sum_f32", ALLREDUCE_F32),
                ("allgather", ALLGATHER)]


SIGNATURES = {
    "dpg_last_error": (C.c_char_p, []),
    "dpg_version": (C.c_char_p, []),
    "dpg_icp_params_default": (None, [C.POINTER(IcpParams)]),
    "dpg_gn_params_default": (None, [C.POINTER(GnParams)]),
    "dpg_ctx_create": (P, [C.c_int]),
    "dpg_ctx_create_multi": (P, [C.c_int32, I32P]),
    "dpg_ctx_num_gpus": (C.c_int32, [P]),
    "dpg_ctx_create_virtual": (P, [C.c_int32, C.c_int32]),
    "dpg_ctx_create_rank": (P, [C.c_int32, P, C.c_int32, C.c_int32]),
    "dpg_ctx_create_rank_ops": (P, [C.c_int32, C.POINTER(CollOps), C.c_int32, C.c_int32]),
    "dpg_shard_plan": (C.c_int, [F32P, C.c_int64, C.c_int32, I32P, I64P, I64P]),
    "dpg_shard_reassemble": (C.c_int, [I32P, C.c_int64, C.c_int32, C.c_int64, C.c_int64, P, P]),
    "dpg_nccl_unique_id": (C.c_int, [P]),
    "dpg_ctx_num_ranks": (C.c_int32, [P]),
    "dpg_ctx_rank": (C.c_int32, [P]),
    "dpg_ctx_set_icp_schedule": (C.c_int, [P, C.c_int32]),
    "dpg_solver_options_default": (None, [C.POINTER(SolverOptions)]),
    "dpg_ctx_set_solver_options": (C.c_int, [P, C.POINTER(SolverOptions)]),
    "dpg_ctx_destroy": (None, [P]),
    "dpg_ctx_set_stream": (C.c_int, [P, P]),
    "dpg_ctx_synchronize": (C.c_int, [P]),
    "dpg_scan_to_cloud": (C.c_int64, [F32P, C.c_int64, C.c_float, C.c_float, C.c_float, C.c_float,
                                      C.c_float, C.c_float, F32P]),
    "dpg_scans_to_clouds": (C.c_int64, [F32P, C.c_int64, C.c_int64, C.c_float, C.c_float, C.c_float,
                                        C.c_float, C.c_float, C.c_float, F32P, I64P]),
    "dpg_downsample_cloud": (C.c_int64, [F32P, C.c_int64, C.c_int32, F32P]),
    "dpg_inverse_transform_point": (None, [F32P, F32P, F32P]),
    "dpg_transform_point": (None, [F32P, F32P, F32P]),
    "dpg_icp_guess": (None, [F32P, F32P, F32P]),
    "dpg_odometry_factors": (C.c_int, [F32P, C.c_int64, I32P, I32P, C.c_int64, C.c_float, C.c_float, C.c_float,
                                      C.c_float, C.c_void_p]),
    "dpg_odometry_factor": (C.c_int, [F32P, F32P, C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float,
                                      C.c_float, C.POINTER(Factor)]),
    "dpg_icp_factor": (None, [C.POINTER(IcpResult), C.c_int32, C.c_int32, C.POINTER(IcpParams),
                              C.POINTER(Factor)]),
    "dpg_synth_world": (C.c_int64, [C.c_uint64, C.c_float, F32P, C.c_int64]),
    "dpg_synth_trajectory": (C.c_int, [C.c_uint64, C.c_int64, F32P, C.c_int64, C.c_float, C.c_float, F64P]),
    "dpg_synth_scans": (C.c_int, [F64P, C.c_int64, F32P, C.c_int64, C.c_int32, C.c_float, C.c_float,
                                  C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, C.c_uint64,
                                  C.c_int32, F32P]),
    "dpg_run_icp": (C.c_int, [P, F32P, C.c_int64, F32P, C.c_int64, F32P, F32P, C.POINTER(IcpParams),
                              C.POINTER(IcpResult), F64P, F64P]),
    "dpg_scans_upload": (C.c_int, [P, F32P, I64P, C.c_int64, C.c_int32]),
    "dpg_icp_batch_prepare": (C.c_int, [P, I32P, C.c_int64, F32P, C.POINTER(IcpParams)]),
    "dpg_icp_batch_run": (C.c_int, [P, C.c_int32, C.c_int32]),
    "dpg_icp_batch_fetch": (C.c_int, [P, P, F64P, C.c_int64]),
    "dpg_icp_batch_fetch_trace": (C.c_int, [P, I32P, C.c_int64, I64P]),
    "dpg_icp_batch_size": (C.c_int64, [P]),
    "dpg_icp_batch_kernel_ms": (C.c_float, [P]),
    "dpg_cov_batch_kernel_ms": (C.c_float, [P]),
    "dpg_cov_batch_overlapped": (C.c_int32, [P]),
    "dpg_kdtree_build_ms": (C.c_float, [P]),
    "dpg_ctx_set_icp_variant": (C.c_int, [P, C.c_int32]),
    "dpg_ctx_set_icp_defer_cap": (C.c_int, [P, C.c_int32]),
    "dpg_ctx_set_cov_workgroups": (C.c_int, [P, C.c_int32]),
    "dpg_ctx_set_icp_kernel_variant": (C.c_int, [P, C.c_int32]),
    "dpg_icp_batch_algorithmic_bytes": (C.c_double, [P]),
    "dpg_optimize_graph": (C.c_int, [P, F64P, C.c_int64, P, C.c_int64, C.POINTER(GnParams),
                                     C.POINTER(GnStats)]),
    "dpg_gn_setup": (C.c_int, [P, C.c_int64, P, C.c_int64, C.c_int64, C.c_int64, C.POINTER(GnParams)]),
    "dpg_gn_take_icp_measurements": (C.c_int, [P, C.c_int64, C.c_int64, C.c_int64, C.POINTER(IcpParams)]),
    "dpg_gn_hb_size": (C.c_int64, [P]),
    "dpg_gn_setup_profile": (C.c_int, [P, F64P]),
    "dpg_gn_set_poses": (C.c_int, [P, F64P]),
    "dpg_gn_get_poses": (C.c_int, [P, F64P]),
    "dpg_gn_assemble": (C.c_int, [P, P]),
    "dpg_gn_solve_retract": (C.c_int, [P, P, F64P, F64P, I32P]),
    "dpg_gn_solve_retract_async": (C.c_int, [P, P]),
    "dpg_gn_fetch": (C.c_int, [P, P, F64P]),
    "dpg_gn_factorizations": (C.c_int32, [P]),
    "dpg_gn_run": (C.c_int, [P, F64P, C.POINTER(GnStats)]),
    "dpg_gn_last_assemble_ms": (C.c_float, [P]),
    "dpg_gn_last_solve_ms": (C.c_float, [P]),
    "icp_cov_calculate": (C.c_int, [P, F32P, C.c_int64, F32P, C.c_int64, F32P, C.c_float, C.c_float,
                                    C.c_float, F64P, F64P]),
    "icp_cov_sandwich": (C.c_int, [P, F32P, C.c_int64, F32P, C.c_int64, F32P, F64P, F64P]),
    "dpg_reopt_params_default": (None, [C.POINTER(ReoptParams)]),
    "dpg_get_map": (C.c_int64, [P, F32P, C.c_int32, F32P, C.c_int64]),
    "dpg_get_map_kernel_ms": (C.c_float, [P]),
    "dpg_loop_closure_candidates": (C.c_int64, [P, C.c_int64, I32P, F32P, C.c_float, C.c_float, I32P, C.c_int64]),
    "dpg_change_params_default": (None, [C.POINTER(ChangeParams)]),
    "dpg_dpg_create": (P, [P, C.c_int64, I64P, F32P, F32P, C.POINTER(ChangeParams)]),
    "dpg_dpg_destroy": (None, [P]),
    "dpg_dpg_append": (C.c_int, [P, C.c_int64, I64P, F32P, F32P]),
    "dpg_execute_dpg": (C.c_int, [P, C.c_int64, C.c_int64, F32P, C.POINTER(ChangeStats)]),
    "dpg_execute_dpg_chain": (C.c_int, [P, C.c_int64, C.c_int64, F32P, F32P, C.POINTER(ChangeStats)]),
    "dpg_dpg_fetch": (C.c_int, [P, U8P, U8P, U8P]),
    "dpg_dpg_load": (C.c_int, [P, U8P, U8P, U8P]),
    "dpg_active_dynamic_points": (C.c_int64, [P, C.c_int64, F32P, F32P, C.c_int64, I64P]),
    "dpg_reoptimize": (C.c_int, [P, C.c_int64, I32P, F32P, F32P, C.POINTER(IcpParams), C.POINTER(GnParams),
                                 C.POINTER(ReoptParams), F64P, C.POINTER(ReoptStats)]),
    "dpg_reoptimize_inc": (C.c_int, [P, C.c_int64, I32P, F32P, F32P, C.POINTER(IcpParams), C.POINTER(ReoptParams),
                                     F64P, C.POINTER(ReoptStats)]),
    "dpg_inc_params_default": (None, [C.POINTER(IncParams)]),
    "dpg_inc_create": (P, [P, C.POINTER(IncParams)]),
    "dpg_inc_destroy": (None, [P]),
    "dpg_inc_reset": (C.c_int, [P]),
    "dpg_inc_update": (C.c_int, [P, C.c_int64, F64P, P, C.c_int64, C.POINTER(IncStats)]),
    "dpg_inc_num_nodes": (C.c_int64, [P]),
    "dpg_inc_get_poses": (C.c_int, [P, F64P, C.c_int64]),
    "dpg_inc_save": (C.c_int, [P, C.c_char_p]),
    "dpg_inc_load": (P, [P, C.c_char_p]),
    "dpg_inc_export": (C.c_int64, [P, I64P, P, I32P, C.c_int64, F64P, F64P, F64P]),
    "dpg_scans_append": (C.c_int, [P, F32P, I64P, C.c_int64, C.c_int32]),
    "dpg_add_node": (C.c_int, [P, F32P, C.c_int64, I32P, F32P, P, C.c_int64, C.POINTER(IcpParams),
                               C.POINTER(ReoptParams), C.c_int32, C.POINTER(AddNodeStats)]),
    "dpg_add_node_pairs": (C.c_int, [P, F32P, C.c_int64, F32P, P, C.c_int64, I32P, C.c_int64, C.c_int32,
                                     C.POINTER(IcpParams), C.POINTER(AddNodeStats)]),
}


def default_inc_params() -> IncParams:
    p = IncParams()
    lib().dpg_inc_params_default(C.byref(p))
    return p


def default_solver_options() -> SolverOptions:
    o = SolverOptions()
    lib().dpg_solver_options_default(C.byref(o))
    return o


def default_reopt_params() -> ReoptParams:
    p = ReoptParams()
    lib().dpg_reopt_params_default(C.byref(p))
    return p

_LIB = None


def lib() -> C.CDLL:
    """Load libdpg.so (raises OSError/RuntimeError when it is not built -- no fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built; run `make -C dpg-slam_amd` or __graft_entry__.build()")
        # One HIP runtime per process: PyTorch ships its own libamdhip64 (same soname), so load it
        # first and libdpg binds to it; loaded the other way round torch would bring a second
        # runtime that finds no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def ptr(a: np.ndarray, ctype):
    """Pointer to a contiguous numpy array (None for None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(C.POINTER(ctype))


def vptr(a: np.ndarray):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return C.c_void_p(a.ctypes.data)


class DpgError(RuntimeError):
    pass


def check(rc: int, what: str = "dpg call"):
    if rc != DPG_OK:
        msg = lib().dpg_last_error()
        raise DpgError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def default_icp_params() -> IcpParams:
    p = IcpParams()
    lib().dpg_icp_params_default(C.byref(p))
    return p


def default_change_params() -> ChangeParams:
    p = ChangeParams()
    lib().dpg_change_params_default(C.byref(p))
    return p


default_change_params_host = default_change_params


def default_gn_params() -> GnParams:
    p = GnParams()
    lib().dpg_gn_params_default(C.byref(p))
    return p
