/*
 * dpg_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the DPG-SLAM hot path, used as the parity checker for the HIP
 * product path and as the CPU baseline ("kind": "port") in bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product library
 * (dpg-slam_amd/) never links or calls it.
 *
 * Pinning status (see DESIGN.md "Oracle"):
 *   - pinned by the reference's own known answers: the gtsam_test graph
 *     (src/dpg_slam/dpg_slam_main.cc:224-251, analytic optimum), the constant ICP_COV
 *     (cov_func_point_to_point.h:572-575 with parameters.h:374,385,396), and the covariance
 *     [x,y,yaw] block against the reference's own d2J expressions (cov :133-165, fixture
 *     tests/golden/cov_expr.npz generated from the reference text);
 *   - UNPINNED: the PCL ICP / FLANN / Umeyama arithmetic and the GTSAM factor/solver arithmetic
 *     (third-party, absent from /root/reference; restated from their public semantics).
 */
#ifndef DPG_ORACLE_H
#define DPG_ORACLE_H
#include "../include/dpg_slam_c.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_NN_BRUTE 0
#define ORACLE_NN_GRID 1

int64_t oracle_scan_to_cloud(const float* ranges, int64_t n, float angle_min, float angle_max,
                             float range_max, float lx, float ly, float lth, float* xy_out);
int64_t oracle_downsample(const float* xy, int64_t n, int32_t ratio, float* xy_out);
void oracle_inverse_transform_point(const float a[3], const float b[3], float out[3]);
void oracle_transform_point(const float p[3], const float f[3], float out[3]);
void oracle_icp_guess(const float pose_src[3], const float pose_tgt[3], float guess[6]);

/* PCL IterativeClosestPoint::align restated on downsampled clouds. trace: [trace_iters][n_src]. */
int oracle_icp_align(const float* src, int64_t n_src, const float* tgt, int64_t n_tgt,
                     const float guess[6], const dpg_icp_params* p, int nn_mode,
                     dpg_icp_result* res, int32_t* trace, int32_t trace_iters);
/* calculate_ICP_COV: constant output + diagnostic [x,y,yaw] block (fp64). */
void oracle_icp_cov(const float* data, int64_t nd, const float* model, int64_t nm, const float T6[6],
                    float vx, float vy, float vth, double cov[9], double hess[9]);
/* Literal (non-simplified) evaluation of the reference's d2J_da2 / d2J_dxda / d2J_dyda at
 * b = c = 0, z = 0 -- used only to cross-check oracle_icp_cov's closed form. */
void oracle_cov_block_literal(const float* data, int64_t nd, const float* model, int64_t nm,
                              const float T6[6], double hess[9]);
/* runIcp (dpg_slam.cc:362-446) over full clouds. */
int oracle_run_icp(const float* src_full, int64_t n_src, const float* tgt_full, int64_t n_tgt,
                   const float pose_src[3], const float pose_tgt[3], const dpg_icp_params* p,
                   int nn_mode, dpg_icp_result* res, double cov[9], double hess[9]);
/* Batch over edges (OpenMP over edges when n_threads > 1). */
int oracle_icp_batch(const float* pts, const int64_t* offs, int64_t n_nodes, const int32_t* edges,
                     int64_t n_edges, const float* poses, const dpg_icp_params* p, int nn_mode,
                     int n_threads, dpg_icp_result* res, double* hess);

/* GTSAM semantics (GaussNewton over PriorFactor<Pose2>/BetweenFactor<Pose2>). */
void oracle_linearize(const dpg_factor* f, const double* poses, double e[3], double Ai[9],
                      double Aj[9]);
double oracle_graph_error(const double* poses, const dpg_factor* f, int64_t nf);
int oracle_optimize_graph(double* poses, int64_t n_nodes, const dpg_factor* f, int64_t nf,
                          const dpg_gn_params* gp, dpg_gn_stats* st);
/* One linear solve H delta = -g at the given poses (for solver-level parity tests). */
int oracle_icp_cov_sandwich(const float* data, int64_t nd, const float* model, int64_t nm, const float T6[6],
                            double cov6[36], double cov3[9]);
int oracle_gn_delta(const double* poses, int64_t n_nodes, const dpg_factor* f, int64_t nf,
                    double* delta, double* error);

#ifdef __cplusplus
}
#endif
#endif
