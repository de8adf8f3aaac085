/*
 * dpg_slam_c.h -- C ABI of the MI355X-native DPG-SLAM hot path.
 *
 * This library replaces the numerically hot part of BharathMasetty/DPG-SLAM:
 *   - DpgSLAM::runIcp            (src/dpg_slam/dpg_slam.cc:362-446, decl dpg_slam.h:630)
 *     which wraps pcl::IterativeClosestPoint<PointXYZ,PointXYZ>::align (dpg_slam.cc:387-416)
 *     and calculate_ICP_COV (src/icp_cov/cov_func_point_to_point.h:24, see dpg_icp_cov.h);
 *   - DpgSLAM::optimizeGraph     (src/dpg_slam/dpg_slam.cc:316-329, decl dpg_slam.h:464)
 *     which runs GTSAM ISAM2 / Gauss-Newton over PriorFactor<Pose2> / BetweenFactor<Pose2>
 *     built at dpg_slam.cc:44-75,178-183,227-238,331-338.
 *
 * All entry points are extern "C", take plain pointers + sizes, and return an int status
 * (0 = OK, negative = error; dpg_last_error() gives the message).  Buffers are caller-owned
 * HOST memory unless the parameter name ends in _dev (device memory on the context's GPU).
 * A context is thread-compatible (one per thread), not thread-safe -- the reference calls
 * all of these from the single ros::spin thread (dpg_slam_main.cc:328).
 */
#ifndef DPG_SLAM_C_H
#define DPG_SLAM_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPG_OK 0
#define DPG_ERR_ARG (-1)
#define DPG_ERR_HIP (-2)
#define DPG_ERR_STATE (-3)
#define DPG_ERR_SIZE (-4)
#define DPG_ERR_NUMERIC (-5)
#define DPG_ERR_INTERNAL (-6) /* a kernel failed its own consistency check (DPG_ICP_INTERNAL) */

/* Fixed reduction geometry of the ICP rigid fit (part of the algorithm's definition so that
 * CPU oracle and GPU agree bit for bit): lane l accumulates source points l, l+512, ... in
 * increasing order (fp64); each 64-lane wave folds acc[k] += acc[k + off], off = 32 ... 1, and
 * the eight wave totals combine as ((W0 + W1) + (W2 + W3)) + ((W4 + W5) + (W6 + W7)). */
#define DPG_ICP_LANES 512

/* ICP parameters: field names follow PoseGraphParameters (src/dpg_slam/parameters.h:105-141,
 * defaults :146,159,173,191,201,374,385,396,402) plus the PCL defaults the reference inherits
 * (Registration::min_number_correspondences_ = 3, DefaultConvergenceCriteria mse abs 1e-12). */
typedef struct dpg_icp_params {
    int32_t icp_maximum_iterations;              /* 500 */
    int32_t icp_use_reciprocal_correspondences;  /* 1 */
    double icp_maximum_transformation_epsilon;   /* 5e-9 */
    double icp_max_correspondence_distance;      /* 0.6 */
    int32_t ransac_iterations;                   /* 50 -- inert, as in PCL ICP */
    int32_t downsample_icp_points_ratio;         /* 5 */
    float laser_x_variance;                      /* 0.5 */
    float laser_y_variance;                      /* 0.5 */
    float laser_theta_variance;                  /* 0.3 */
    int32_t min_number_correspondences;          /* 3 (pcl::Registration default) */
    double mse_threshold_absolute;               /* 1e-12 (pcl DefaultConvergenceCriteria) */
} dpg_icp_params;

/* Per-edge ICP outcome (runIcp's out-param + return value, dpg_slam.cc:433-445). */
typedef struct dpg_icp_result {
    float T[6];          /* final transformation, rows: T00 T01 T03 / T10 T11 T13 (z row = e3) */
    float z[3];          /* measurement (T03, T13, atan2(T10, T00)) -- dpg_slam.cc:434-439 */
    int32_t converged;   /* icp.hasConverged() (max iterations counts as converged, as in PCL) */
    int32_t iterations;  /* nr_iterations_ */
    int32_t n_corr;      /* correspondences of the last iteration */
    int32_t status;      /* DPG_ICP_* below */
    int32_t pad;
    double fitness;      /* MSE of the last iteration's correspondences */
} dpg_icp_result;

#define DPG_ICP_OK 0
#define DPG_ICP_TOO_FEW_CORR 1   /* fewer than min_number_correspondences -> converged = 0 */
#define DPG_ICP_NON_PLANAR 2     /* est_transform(2,2) != 1 (dpg_slam.cc:422-426); never produced by
                                    the planar closed form, kept for ABI parity */
#define DPG_ICP_INTERNAL 3       /* kernel self-check failed (a bug: never expected) */

/* Factors (R9/R10).  info = diagonal information (1/sigma^2 for noiseModel::Diagonal::Sigmas,
 * 1/variance for noiseModel::Gaussian::Covariance of a diagonal matrix, dpg_slam.cc:335). */
#define DPG_FACTOR_PRIOR 0
#define DPG_FACTOR_BETWEEN 1
typedef struct dpg_factor {
    int32_t kind;      /* DPG_FACTOR_PRIOR | DPG_FACTOR_BETWEEN */
    int32_t i;         /* first key (prior: the key) */
    int32_t j;         /* second key (between) */
    int32_t pad;
    double z[3];       /* measured Pose2 (x, y, theta): prior mean or between measurement */
    double info[3];    /* diagonal information */
} dpg_factor;          /* 64 bytes */

typedef struct dpg_gn_params {
    int32_t max_iterations;      /* 100 (GaussNewtonParams.maxIterations, dpg_slam_main.cc:262) */
    int32_t use_error_criteria;  /* 1: GTSAM checkConvergence on the error; 0: stop on max|delta| */
    double delta_tol;            /* 1e-10: batch-GN target */
    double relative_error_tol;   /* 1e-5 (GaussNewtonParams.relativeErrorTol) */
    double absolute_error_tol;   /* 1e-5 (NonlinearOptimizerParams default) */
    double pcg_rel_tol;          /* 1e-12: PCG stops when |r| <= tol * |b| */
    int32_t pcg_max_iterations;  /* 20000 */
    int32_t pcg_check_every;     /* PCG iterations between host convergence checks (GPU only) */
    int32_t linear_solver;       /* DPG_SOLVER_CHOLESKY (default, GTSAM's CHOLESKY) | DPG_SOLVER_PCG */
    int32_t reuse_factorization; /* 1 (default): once the last step's max|delta| < refactor_delta, solve
                                    with the previous Cholesky factor (a chord step: same fixed point
                                    g(X) = 0, H barely changes that close to it); 0: refactor every
                                    iteration (plain Gauss-Newton) */
    double refactor_delta;       /* 1e-3 (tools/refactor_sweep.sh: config 4 converges in 8 iterations
                                    with 3 factorizations instead of 7 with 4, 2.4 % less per step) */
} dpg_gn_params;

#define DPG_SOLVER_CHOLESKY 0    /* supernodal multifrontal Cholesky on the GPU */
#define DPG_SOLVER_PCG 1         /* block-Jacobi preconditioned CG on the GPU */

typedef struct dpg_gn_stats {
    int32_t iterations;
    int32_t pcg_iterations;      /* total over all GN iterations */
    double initial_error;        /* 0.5 * sum ||e||^2_info at the initial values */
    double final_error;
    double last_delta_inf;
    double ms_total;
    double ms_per_iteration;
} dpg_gn_stats;

typedef struct dpg_ctx dpg_ctx;

/* ---- library / context ---- */
const char* dpg_last_error(void);
const char* dpg_version(void);
void dpg_icp_params_default(dpg_icp_params* p);
void dpg_gn_params_default(dpg_gn_params* p);
/* device = HIP device ordinal; returns NULL (and sets dpg_last_error) when no GPU is usable. */
dpg_ctx* dpg_ctx_create(int device);
/* Also destroys every incremental graph (dpg_inc_create / dpg_inc_load) and DPG store
 * (dpg_dpg_create) still alive on ctx; their handles are invalid afterwards. */
void dpg_ctx_destroy(dpg_ctx* ctx);
/* Multi-GPU context (SURVEY 8b "dpg_ctx_create(int n_gpus)", 8e): ONE host process drives n_gpus
 * devices (devices[k], or 0 .. n_gpus-1 when devices is NULL), one stream per device and one RCCL
 * communicator per device (ncclCommInitAll over xGMI).  The same entry points then run sharded,
 * so a single-threaded host -- the reference's ROS node (dpg_slam_main.cc:284-331) -- uses N GPUs
 * through the unchanged call sites:
 *   dpg_scans_upload / dpg_scans_append   every device holds every scan;
 *   dpg_icp_batch_prepare / _run / _fetch edge e is aligned on device e mod n_gpus, all devices
 *                                         concurrently; results (and covariance blocks) come back
 *                                         in the caller's order; _kernel_ms is the slowest device
 *                                         (dpg_ctx_set_icp_schedule: once every edge's cost is
 *                                         known from an earlier run, a longest-processing-time
 *                                         assignment instead);
 *   dpg_optimize_graph, dpg_reoptimize,   every device holds the factor list and linearizes its
 *   dpg_gn_setup + _take_icp_measurements share (factor f mod n, and each ICP slot on the device
 *   + _set_poses + dpg_gn_run             that aligned its edge); per Gauss-Newton iteration ONE
 *                                         ncclAllReduce(sum, fp64) of the packed [H upper | g |
 *                                         chi2]; every device factors and solves the identical
 *                                         system and takes its own (identical) stop / chord
 *                                         decisions on the device (poses bitwise equal on all
 *                                         devices; the loop checks their reports agree).
 * dpg_run_icp, icp_cov_calculate / icp_cov_sandwich, dpg_get_map and dpg_loop_closure_candidates
 * run on the first device.  The per-iteration step API (dpg_gn_assemble / _solve_retract* /
 * _fetch), the trace and the incremental graph (dpg_inc_create: per-node updates are
 * latency-bound, one GPU) need a single-device context.  n_gpus = 1 gives a context whose calls
 * take the sharded paths with one rank (RCCL included): its results equal dpg_ctx_create's byte
 * for byte. */
dpg_ctx* dpg_ctx_create_multi(int32_t n_gpus, const int32_t* devices);
/* One process per GPU (torchrun and the like): this process's `device` is global rank `rank` of
 * `world`; the RCCL communicator is built from the id rank 0 made with dpg_nccl_unique_id and the
 * caller handed to every rank (ncclCommInitRank).  The batched calls above then act on the whole
 * job: dpg_icp_batch_prepare takes ALL edges and aligns this rank's share, dpg_icp_batch_fetch
 * returns every edge's result (a collective: every rank calls it), the Gauss-Newton calls
 * all-reduce across ranks.  Every rank must make the same calls with the same arguments. */
#define DPG_NCCL_ID_BYTES 128
int dpg_nccl_unique_id(void* id_out /*[DPG_NCCL_ID_BYTES]*/);
dpg_ctx* dpg_ctx_create_rank(int32_t device, const void* nccl_id, int32_t rank, int32_t world);
/* The same one-process-per-GPU form over the CALLER's collectives instead of RCCL: a host that
 * already runs a communicator (MPI, gloo), or ranks that share one card (RCCL refuses a second rank
 * on a device -- the one-GPU test box runs the world > 1 rank form this way).  Three blocking calls
 * on host memory, made by every rank in the same order with the same sizes, each returning 0 on
 * success: the float sum of the alignment costs (the LPT plan), the all-gather of the results, the
 * fp64 sum of the packed [H upper | g | chi2 | votes] per Gauss-Newton iteration. */
typedef struct dpg_coll_ops {
    void* user;
    int (*allreduce_sum_f64)(void* user, double* buf, int64_t n);               /* in place */
    int (*allreduce_sum_f32)(void* user, float* buf, int64_t n);                /* in place */
    int (*allgather)(void* user, const void* send, void* recv, int64_t bytes);  /* recv: world * bytes, rank order */
} dpg_coll_ops;
dpg_ctx* dpg_ctx_create_rank_ops(int32_t device, const dpg_coll_ops* ops, int32_t rank, int32_t world);
/* Host helpers of the multi-device forms (no device call): the batch's assignment over `world` ranks
 * -- cost == NULL: edge e on rank e mod world in the caller's order; else longest-processing-time
 * (longest first to the least-loaded rank; ties: lower index, lower rank) -- as owner[e] and every
 * rank's dispatch order (rank 0's counts[0] edges first, then rank 1's, ...); and the rank form's
 * all-gathered results (slice r = rank r's records, its edges ascending, `slice` records reserved
 * per rank) back into the caller's order. */
int dpg_shard_plan(const float* cost, int64_t n_edges, int32_t world, int32_t* owner, int64_t* dispatch,
                   int64_t* counts);
int dpg_shard_reassemble(const int32_t* owner, int64_t n_edges, int32_t world, int64_t slice, int64_t rec_bytes,
                         const void* gathered, void* out);
/* Test / rehearsal form: k "devices" that are k contexts on ONE device sharing one stream, the
 * all-reduce a device-side sum in rank order.  Every sharded path of the multi-device forms runs
 * with k > 1 on one card (k <= 16). */
dpg_ctx* dpg_ctx_create_virtual(int32_t k, int32_t device);
int32_t dpg_ctx_num_gpus(dpg_ctx* ctx);   /* local devices: 1 for dpg_ctx_create and the rank form */
int32_t dpg_ctx_num_ranks(dpg_ctx* ctx);  /* ranks of the collective (ncclCommCount; k virtual; 1) */
int32_t dpg_ctx_rank(dpg_ctx* ctx);       /* global rank of the first local device */
/* Batched ICP dispatch (results are identical for both): DPG_ICP_SCHEDULE_CALLER -- edge e on rank
 * e mod ranks, in the caller's order; DPG_ICP_SCHEDULE_MEASURED (default) -- the same until every
 * edge of the staged batch has a measured cost (iterations x points, from an earlier run of the
 * same (target, source) pair: a batch run again, or the next sweep), then a longest-processing-time
 * assignment over the ranks and longest-first dispatch on each, so that the alignments that bound
 * a launch start first. */
#define DPG_ICP_SCHEDULE_CALLER 0
#define DPG_ICP_SCHEDULE_MEASURED 1
int dpg_ctx_set_icp_schedule(dpg_ctx* ctx, int32_t schedule);
/* Options of the supernodal Cholesky (per context; every device of a multi-device context), taken
 * by the next graph set up on it (dpg_gn_setup, dpg_optimize_graph, dpg_reoptimize, dpg_inc_create).
 * The defaults are the measured choices; the others are cross-checks and A/B
 * references that must give the same solution to rounding. */
#define DPG_ORDER_AUTO 0   /* nested dissection: the shorter critical path of two separator rules */
#define DPG_ORDER_MD 1     /* minimum degree */
#define DPG_ORDER_ND 2     /* nested dissection, round 2's separator rule alone */
typedef struct dpg_solver_options {
    int32_t order;               /* DPG_ORDER_AUTO */
    int32_t fused;               /* 1: one-launch DAG factorization + solves when every front fits LDS;
                                    0: the level-scheduled factorization */
    int32_t solve_stage;         /* doubles of L staged in LDS by the DAG solves; -1: what fills 80 KB */
    int32_t solve_maxseg;        /* ancestor row segments per front in the backward solve; -1: all */
    int32_t solve_dinv;          /* 1: the solves use inverted diagonal blocks (0: substitution chains) */
    int32_t merge_single;        /* 1: supernodes merge only along single-child chains (round 1's rule) */
    int32_t max_supernode_cols;  /* 64 block columns */
    int32_t solve_inv_cols;      /* 0 (never): fronts with at least this many pivot columns get their
                                    diagonal block's inverse L11^-1 after each factorization (beside
                                    the backward solve in the pipelined loop), and the chord steps'
                                    triangular solves apply it as one product instead of a
                                    substitution chain -- 14 us off each solve, but the inversion and
                                    its stream hand-offs cost more */
    double relax_fraction;       /* 0.3: explicit-zero budget of relaxed supernodes */
} dpg_solver_options;
void dpg_solver_options_default(dpg_solver_options* o);
int dpg_ctx_set_solver_options(dpg_ctx* ctx, const dpg_solver_options* o);
/* Run all work of this context on an external hipStream_t (e.g. torch's current stream); on a
 * multi-GPU context it applies to the first device only. */
int dpg_ctx_set_stream(dpg_ctx* ctx, void* hip_stream);
int dpg_ctx_synchronize(dpg_ctx* ctx);

/* ---- host-side data path helpers (R1-R3, no GPU) ---- */
/* MeasurementPoint + createNode + getCachedPointCloudFromNode (dpg_measurement.h:41-46,102-104,
 * dpg_slam.cc:488-513, dpg_node.cc:8-25): polar scan -> base_link cloud, MAX_RANGE dropped.
 * Returns the number of points written to xy_out (capacity n_ranges points). */
int64_t dpg_scan_to_cloud(const float* ranges, int64_t n_ranges, float angle_min, float angle_max,
                          float range_max, float laser_x, float laser_y, float laser_theta,
                          float* xy_out);
/* R1 over a scan set: ranges[V][n_beams] -> concatenated clouds, offsets_out[V+1] (capacity
 * V * n_beams points).  Returns the total number of points. */
int64_t dpg_scans_to_clouds(const float* ranges, int64_t n_nodes, int64_t n_beams, float angle_min,
                            float angle_max, float range_max, float laser_x, float laser_y,
                            float laser_theta, float* xy_out, int64_t* offsets_out);
/* downsamplePointCloud (dpg_slam.cc:346-360). Returns the number of points written. */
int64_t dpg_downsample_cloud(const float* xy, int64_t n, int32_t ratio, float* xy_out);
/* math_utils::inverseTransformPoint (math_utils.cc:21-35): pose of a in b's frame. */
void dpg_inverse_transform_point(const float a[3], const float b[3], float out[3]);
/* math_utils::transformPoint (math_utils.cc:6-19). */
void dpg_transform_point(const float p[3], const float frame[3], float out[3]);
/* runIcp guess (dpg_slam.cc:364-378): 2x3 float matrix rows (c,-s,tx / s,c,ty). */
void dpg_icp_guess(const float pose_src[3], const float pose_tgt[3], float guess_out[6]);
/* R9 factor builders: odometry BetweenFactor with the motion-model sigmas (dpg_slam.cc:53-75),
 * ICP BetweenFactor with the calculate_ICP_COV diagonal (dpg_slam.cc:331-338). */
int dpg_odometry_factor(const float odom_prev[3], const float odom_cur[3], int32_t i_prev, int32_t i_cur,
                        float transl_from_transl, float transl_from_rot, float rot_from_transl,
                        float rot_from_rot, dpg_factor* out);
void dpg_icp_factor(const dpg_icp_result* r, int32_t from_node, int32_t to_node,
                    const dpg_icp_params* p, dpg_factor* out);
/* dpg_odometry_factor over n pairs: factor k between odometry poses odom[i_prev[k]] and
 * odom[i_cur[k]] (odom: [n_odom][3]), into out[k] -- the reference's per-node loop of reoptimize
 * (dpg_slam.cc:53-75) in one call; returns the first error (out[k] of a failed pair unset). */
int dpg_odometry_factors(const float* odom, int64_t n_odom, const int32_t* i_prev, const int32_t* i_cur, int64_t n,
                         float transl_from_transl, float transl_from_rot, float rot_from_transl, float rot_from_rot,
                         dpg_factor* out);

/* ---- synthetic workload generator (seeded, deterministic) ---- */
/* World: axis-aligned rooms + random boxes in [0, world_size]^2; segments [n][4] (x0,y0,x1,y1). */
int64_t dpg_synth_world(uint64_t seed, float world_size, float* segs_out, int64_t max_segs);
/* Ground-truth trajectory: 1 m steps with heading noise, collision-free w.r.t. the world. */
int dpg_synth_trajectory(uint64_t seed, int64_t n_nodes, const float* segs, int64_t n_segs,
                         float world_size, float step, double* gt_out /*[n][3]*/);
/* Ray-cast laser scans (laser pose in base_link), Gaussian range noise, >= range_max kept as
 * range_max (MAX_RANGE).  ranges_out[n_nodes][n_beams]. */
int dpg_synth_scans(const double* gt, int64_t n_nodes, const float* segs, int64_t n_segs,
                    int32_t n_beams, float angle_min, float angle_max, float range_max,
                    float laser_x, float laser_y, float laser_theta, float noise_sigma,
                    uint64_t seed, int32_t n_threads, float* ranges_out);

/* ---- ICP (runIcp) ---- */
/* One alignment, mirroring DpgSLAM::runIcp(node_1 = target, node_2 = source, ...).
 * src_xy / tgt_xy are the FULL base_link clouds of node_2 / node_1 (the ICP downsamples them
 * by params->downsample_icp_points_ratio; the covariance uses the full clouds, dpg_slam.cc:430).
 * pose_src / pose_tgt: estimated poses (x, y, theta) of node_2 / node_1.
 * cov_out (3x3 row-major) receives ICP_COV; hess_out (nullable) the diagnostic [x,y,yaw] block.
 * Returns DPG_OK; the boolean runIcp result is result->converged && status == DPG_ICP_OK. */
int dpg_run_icp(dpg_ctx* ctx, const float* src_xy, int64_t n_src, const float* tgt_xy, int64_t n_tgt,
                const float pose_src[3], const float pose_tgt[3], const dpg_icp_params* params,
                dpg_icp_result* result, double cov_out[9], double hess_out[9]);

/* Batched, device-resident form (the GPU entry point).
 * 1) upload all node clouds once: pts_xy = concatenated full clouds, node_offsets[V+1]. */
int dpg_scans_upload(dpg_ctx* ctx, const float* pts_xy, const int64_t* node_offsets, int64_t n_nodes,
                     int32_t downsample_ratio);
/* 2) stage an edge batch: edges[e] = {node_1 (target), node_2 (source)}, poses[V][3] float. */
int dpg_icp_batch_prepare(dpg_ctx* ctx, const int32_t* edges, int64_t n_edges, const float* poses,
                          const dpg_icp_params* params);
/* 3) run ICP (+ covariance block when compute_cov) over the staged edges, asynchronously on the
 * context stream.  trace_iters > 0 records the per-iteration correspondence indices of every
 * edge (test mode; see dpg_icp_batch_fetch_trace). */
int dpg_icp_batch_run(dpg_ctx* ctx, int32_t compute_cov, int32_t trace_iters);
/* 4) copy results back (any pointer may be NULL).  cap: the number of records results (and
 * hess, [cap][9]) can hold; DPG_ERR_SIZE, with nothing written, when the staged batch is larger
 * (dpg_icp_batch_size tells how many are staged -- a sweep or dpg_add_node may have staged more
 * than the caller's own edges). */
int dpg_icp_batch_fetch(dpg_ctx* ctx, dpg_icp_result* results, double* hess /*[cap][9]*/, int64_t cap);
/* Edges of the staged batch -- dpg_icp_batch_prepare's, or the batch a sweep (dpg_reoptimize) or
 * dpg_add_node staged last: the number of records dpg_icp_batch_fetch writes. */
int64_t dpg_icp_batch_size(dpg_ctx* ctx);
/* trace_cap: int32 elements trace can hold; DPG_ERR_SIZE when E * trace_iters * max_src exceeds it
 * (call with trace = NULL first to learn max_src). */
int dpg_icp_batch_fetch_trace(dpg_ctx* ctx, int32_t* trace /*[E][trace_iters][max_src]*/, int64_t trace_cap,
                              int64_t* max_src_out);
/* Device time of the last ICP / covariance kernels (ms, HIP events on the context stream). */
float dpg_icp_batch_kernel_ms(dpg_ctx* ctx);
float dpg_cov_batch_kernel_ms(dpg_ctx* ctx);
/* 1: the last batch's covariance kernel ran on the context's second stream, beside what followed
 * the ICP on its stream (the pose graph does not read it; DPG_COV_OVERLAP=0 keeps stream order) */
int32_t dpg_cov_batch_overlapped(dpg_ctx* ctx);
/* Device time of the per-node index build (k-d trees / angle index) that precedes the ICP kernel. */
float dpg_kdtree_build_ms(dpg_ctx* ctx);
/* Nearest-neighbour machinery of the ICP kernel; all give bit-identical results. */
#define DPG_ICP_ANGULAR 3  /* per-node angle-sorted clouds + buckets, windowed scans (default) */
#define DPG_ICP_KDTREE 2   /* per-node k-d trees, seeded search, static-frame reciprocal test */
#define DPG_ICP_GRID 1     /* uniform LDS grid, all-pairs reverse keys by LDS atomics */
int dpg_ctx_set_icp_variant(dpg_ctx* ctx, int32_t variant);
/* Angular variant tuning (results are identical for every value): a point whose search window
 * holds more than `cap` candidates is handed to the workgroup's cooperative queue, where a whole
 * wave scans it; 0 scans every window in its own lane.  Default 256. */
int dpg_ctx_set_icp_defer_cap(dpg_ctx* ctx, int32_t cap);
/* The batched covariance that runs beside the pose graph (dpg_icp_batch_run with covariance, its own
 * stream): at most n workgroups, each taking edges in turn, so the pose graph's kernels find free
 * compute units while it runs; 0 = one workgroup per edge.  Default 256 -- one per compute unit
 * (config 4, one process A/B: 8.567 ms per step at 0, 8.524 at 256, 8.742 at 512; fewer than 64
 * stretch it past the pose graph).  Results are identical for every n. */
int dpg_ctx_set_cov_workgroups(dpg_ctx* ctx, int32_t n);
/* Diagnostic: the angular ICP kernel's form (0 = the default; others are A/B references that must give
 * byte-identical results, tools/icp_var_ab.py): 1 = the kernel's previous form (variant 4), 2 = the
 * default kernel after the angle index built by its previous bitonic network. */
int dpg_ctx_set_icp_kernel_variant(dpg_ctx* ctx, int32_t variant);
/* Sum over edges of iterations x (8N + 8M + 8N) -- algorithmic bytes of the correspondence
 * search for the last run, computed on device and copied back. */
double dpg_icp_batch_algorithmic_bytes(dpg_ctx* ctx);

/* ---- pose-graph Gauss-Newton (optimizeGraph) ---- */
/* Single call, batch GN to convergence.  poses_inout[V][3] double. */
int dpg_optimize_graph(dpg_ctx* ctx, double* poses_inout, int64_t n_nodes, const dpg_factor* factors,
                       int64_t n_factors, const dpg_gn_params* params, dpg_gn_stats* stats);

/* Step API for the edge-sharded multi-GPU solve (one RCCL all-reduce of the packed [H|b|chi2]
 * buffer per iteration, done by the caller between assemble and solve).
 * factors: ALL factors of the graph (the sparsity pattern is global); this rank assembles only
 * factors[shard_begin, shard_end). */
int dpg_gn_setup(dpg_ctx* ctx, int64_t n_nodes, const dpg_factor* factors, int64_t n_factors,
                 int64_t shard_begin, int64_t shard_end, const dpg_gn_params* params);
/* Overwrite the measurement/information of factors [first, first+count) with the ICP batch
 * results of edges [0, count) of the last dpg_icp_batch_run (device to device; multi-device forms:
 * count = the whole batch, each slot on the device that aligned it).  Edges
 * [0, n_always) always become factors (successive scans, dpg_slam.cc:85-89); the others only when
 * the alignment converged (loop closures, dpg_slam.cc:101-104) -- a dropped edge keeps its slot
 * with zero information, which adds nothing to H, g or the error. */
int dpg_gn_take_icp_measurements(dpg_ctx* ctx, int64_t first_factor, int64_t count, int64_t n_always,
                                 const dpg_icp_params* params);
int64_t dpg_gn_hb_size(dpg_ctx* ctx);   /* doubles in the packed buffer */
/* Host clock (ms) of the last dpg_gn_setup's parts, in this order: the pattern, contribution lists
 * and BSR rows; the Cholesky's symbolic analysis (ordering, supernodes); its plan (these three
 * before the setup waits for the context's stream; the lists and rows are built beside the other
 * two once the pairs are known); the wait + device allocations + uploads; the Cholesky's upload. */
int dpg_gn_setup_profile(dpg_ctx* ctx, double out[5]);
int dpg_gn_set_poses(dpg_ctx* ctx, const double* poses);
int dpg_gn_get_poses(dpg_ctx* ctx, double* poses);
/* Linearize the local shard at the current poses into hb_dev (overwritten, not accumulated). */
int dpg_gn_assemble(dpg_ctx* ctx, double* hb_dev);
/* Solve (sum of all shards in hb_dev) and retract.  Blocking: returns max|delta| and the error
 * 0.5*chi2 at the linearization point. */
int dpg_gn_solve_retract(dpg_ctx* ctx, const double* hb_dev, double* delta_inf, double* error,
                         int32_t* pcg_iterations);
/* The same, enqueued only (no host synchronisation with the Cholesky solver): the GN loop then
 * re-linearizes (dpg_gn_assemble, [all-reduce]) and reads everything it decides on with ONE
 * dpg_gn_fetch: out = {max|delta| of the last retraction, error of hb_dev, solver status
 * (0 = ok, 1 = H not positive definite, 2 = solver timeout)}. */
int dpg_gn_solve_retract_async(dpg_ctx* ctx, const double* hb_dev);
int dpg_gn_fetch(dpg_ctx* ctx, const double* hb_dev, double out[3]);
/* The whole Gauss-Newton loop of the setup (its parameters) from the poses of the last
 * dpg_gn_set_poses, natively: assemble, then per iteration solve + retract + re-linearize with the
 * stop and chord decisions taken on the device (multi-device forms: sharded assembly and one
 * all-reduce per iteration); poses_out[V][3] (may be NULL) receives the result. */
int dpg_gn_run(dpg_ctx* ctx, double* poses_out, dpg_gn_stats* stats);
/* Cholesky factorizations since the last dpg_gn_set_poses (the other solves reused one). */
int32_t dpg_gn_factorizations(dpg_ctx* ctx);
float dpg_gn_last_assemble_ms(dpg_ctx* ctx);
float dpg_gn_last_solve_ms(dpg_ctx* ctx);

/* ---- re-linearisation sweep (DpgSLAM::reoptimize, dpg_slam.cc:35-120) ---- */
typedef struct dpg_reopt_params {
    float max_node_dist_within_pass;    /* 5.0 (parameters.h:212) */
    float max_node_dist_across_passes;  /* 2.0 (parameters.h:224) */
    float new_pass_std_dev[3];          /* prior sigmas x, y, theta: 0.2, 0.2, 0.15 (parameters.h:264-274) */
    float motion_model[4];              /* transl<-transl, transl<-rot, rot<-transl, rot<-rot: 0.4 each
                                           (parameters.h:279-309) */
    int32_t odometry_constraints;       /* 1 (parameters.h:364) */
} dpg_reopt_params;

typedef struct dpg_reopt_stats {
    int64_t n_factors;          /* priors + odometry + ICP factor slots */
    int64_t n_icp_edges;        /* successive + loop-closure candidates (all aligned) */
    int64_t n_candidates;       /* loop-closure candidates (j, i), j < i - 1, within the distance rule */
    int64_t n_loop_closures;    /* candidates whose alignment converged (became factors) */
    double ms_candidates;       /* GPU candidate search incl. the copy back of the pair list */
    double ms_icp;              /* batched ICP (angle index + kernel) */
    double ms_gn;               /* graph setup (symbolic analysis) + Gauss-Newton */
    dpg_gn_stats gn;
} dpg_reopt_stats;

void dpg_reopt_params_default(dpg_reopt_params* p);

/* The candidate pairs of the sweep (dpg_slam.cc:91-98): for i ascending, j = 0 .. i-2 ascending,
 * (j, i) when the float distance of the estimated positions est_poses[j] - est_poses[i] (Eigen
 * Vector2f::norm) is <= max_node_dist_within_pass (same pass_numbers) or
 * <= max_node_dist_across_passes.  Computed on the GPU; writes min(count, cap) pairs {j, i} and
 * returns the count (negative: error). */
int64_t dpg_loop_closure_candidates(dpg_ctx* ctx, int64_t n_nodes, const int32_t* pass_numbers,
                                    const float* est_poses /*[V][3]*/, float max_dist_within_pass,
                                    float max_dist_across_passes, int32_t* pairs_out /*[cap][2]*/, int64_t cap);

/* The whole sweep on the uploaded scans (dpg_scans_upload of all V nodes):
 *   factors per node i in order: a prior (0, 0, 0) on the first node of each pass, otherwise the
 *   odometry Between (i-1, i) from odom_only (if odometry_constraints); the ICP edges: every
 *   successive pair (i-1, i) (always a factor, dpg_slam.cc:85-89) and every loop-closure
 *   candidate (j, i) (a factor when the alignment converged, dpg_slam.cc:101-104) -- one batched
 *   ICP of all of them from the estimated poses; then batch Gauss-Newton from est_poses (the
 *   ISAM2 update of optimizeGraph, run to convergence: SURVEY Q1/Q6).
 * poses_out[V][3] (double) receives the optimised poses. */
/* DpgSLAM::GetMap (dpg_slam.cc:555-575) over the uploaded full clouds: every node's base_link
 * points in the map frame (transformPoint with the node's estimated pose), one point in
 * display_points_fraction (10, parameters.h:22) by the running index over all nodes.  Writes
 * min(count, cap) points and returns the count, ceil(P / fraction) (negative: error). */
int64_t dpg_get_map(dpg_ctx* ctx, const float* est_poses /*[V][3]*/, int32_t display_points_fraction,
                    float* map_out /*[cap][2]*/, int64_t cap);
float dpg_get_map_kernel_ms(dpg_ctx* ctx);   /* device time of the last dpg_get_map kernel */

int dpg_reoptimize(dpg_ctx* ctx, int64_t n_nodes, const int32_t* pass_numbers, const float* est_poses,
                   const float* odom_only, const dpg_icp_params* icp_params, const dpg_gn_params* gn_params,
                   const dpg_reopt_params* params, double* poses_out, dpg_reopt_stats* stats);

/* DpgSLAM::reoptimize for a live incremental graph g (dpg_slam.cc:35-120): the sweep of
 * dpg_reoptimize (candidates, ONE batched ICP, the factors in the reference's order: pass prior or
 * odometry per node, every successive alignment, the converged loop closures) on g's context, then g
 * is rebuilt from exactly those factors -- dpg_inc_reset + ONE dpg_inc_update of all V nodes from
 * est_poses: the reference's new ISAM2 + new graph_ and its one update (:36-39, :111-119), under g's
 * own update semantics (DPG_INC_ISAM2: one step; DPG_INC_BATCH: to convergence).  Later
 * dpg_add_node calls then build on the swept graph, as the reference's per-node updates do after
 * reoptimize.  The context's scan store must hold the V nodes (it does after V dpg_add_node).
 * poses_out[V][3] = g's estimate; stats.gn carries the update's iterations and error. */
struct dpg_inc;
int dpg_reoptimize_inc(struct dpg_inc* g, int64_t n_nodes, const int32_t* pass_numbers, const float* est_poses,
                       const float* odom_only, const dpg_icp_params* icp_params, const dpg_reopt_params* params,
                       double* poses_out, dpg_reopt_stats* stats);

/* ---- incremental per-node solve (updatePoseGraphObsConstraints -> optimizeGraph -> isam_->update,
 *      dpg_slam.cc:255-329, ISAM2 built at :22 with default parameters) ----
 * A device-resident pose graph that grows by one isam_->update per call.  The elimination order of
 * the Cholesky is kept and extended (new nodes at its end, new edges add their fill along the
 * elimination tree); a fresh minimum-degree order is computed every reorder_every nodes or when the
 * fill grows 1.5x.  DPG_INC_ISAM2: ISAM2 semantics with its defaults (relinearize variables whose
 * max |delta| >= 0.1 on every 10th update, one Gauss-Newton step from the linearization point per
 * update; exact solve instead of the 0.001 wildfire threshold).  DPG_INC_BATCH: Gauss-Newton to
 * convergence on every update.  duplicate_factors = 1 reproduces SURVEY Q1 (the reference re-adds
 * the whole accumulated graph_ on every update: a factor's information is scaled by the number of
 * updates it has been part of). */
#define DPG_INC_ISAM2 0
#define DPG_INC_BATCH 1
typedef struct dpg_inc_params {
    int32_t mode;                    /* DPG_INC_ISAM2 | DPG_INC_BATCH */
    int32_t relinearize_skip;        /* 10 (ISAM2Params::relinearizeSkip) */
    double relinearize_threshold;    /* 0.1 (ISAM2Params::relinearizeThreshold) */
    int32_t duplicate_factors;       /* 0; 1: SURVEY Q1 */
    int32_t reorder_every;           /* 32: a fresh fill-reducing order every this many new nodes */
    int32_t reorder_lead;            /* 8: that order is computed on a worker thread from a snapshot of
                                        the graph this many nodes before it is due, then extended by the
                                        nodes and edges that arrived since; 0: on the calling thread */
    int32_t full_refactor;           /* 0: ISAM2 updates refactor only the fronts the update touches
                                        (new nodes, new factors' and pairs' nodes, structure changes,
                                        and everything above them) -- isam_->update's partial
                                        re-elimination, bit-identical to a full refactorization;
                                        1: every front, every update */
    dpg_gn_params gn;                /* DPG_INC_BATCH: the Gauss-Newton loop (Cholesky) */
} dpg_inc_params;

typedef struct dpg_inc_stats {
    int64_t n_nodes, n_factors;
    int64_t nnz_l;                   /* 3x3 blocks below the diagonal of L */
    int32_t reordered;               /* 1: this update computed a fresh order */
    int32_t relinearized;            /* ISAM2: variables relinearized by this update */
    int32_t gn_iterations;           /* ISAM2: 1 */
    int32_t fronts_kept;             /* ISAM2: Cholesky fronts this update kept from the last one
                                        (0: a full refactorization) */
    double error;                    /* 0.5 chi2 at the last linearization point */
    double last_delta_inf;
    double ms_total, ms_symbolic, ms_numeric;
} dpg_inc_stats;

typedef struct dpg_inc dpg_inc;
void dpg_inc_params_default(dpg_inc_params* p);
dpg_inc* dpg_inc_create(dpg_ctx* ctx, const dpg_inc_params* params);
void dpg_inc_destroy(dpg_inc* g);
/* reoptimize() (dpg_slam.cc:36-39): a new ISAM2 and a new graph */
int dpg_inc_reset(dpg_inc* g);
/* isam_->update(new factors, new values): n_new nodes appended (keys V .. V+n_new-1, initial values
 * init[n_new][3]) and the factors added since the last update (keys < V + n_new). */
int dpg_inc_update(dpg_inc* g, int64_t n_new, const double* init, const dpg_factor* factors, int64_t n_factors,
                   dpg_inc_stats* stats);
int64_t dpg_inc_num_nodes(const dpg_inc* g);
/* calculateEstimate() of the first n nodes: poses[n][3] */
int dpg_inc_get_poses(dpg_inc* g, double* poses, int64_t n);

/* Graph checkpoint ("optional binary dump of the graph (poses, edges,
 * measurements)"; the reference keeps dpg_nodes_ with their scans, graph_ and isam_ only in memory,
 * dpg_slam.h:362,367,372).  dpg_inc_save writes the graph's factors, node pairs (arrival order),
 * linearization points, estimate, per-variable |delta|, update count and parameters, and the
 * context's scan store (full clouds, downsample ratio) when it holds the graph's nodes (the
 * dpg_add_node path; a graph fed by dpg_inc_update alone is saved without scans), to one binary
 * file.  dpg_inc_load restores it on ctx (single device; a saved scan store replaces ctx's and is
 * indexed, else ctx's store is left as it is): the next
 * dpg_add_node / dpg_inc_update continues the saved run, ISAM2's relinearization schedule
 * included; the elimination order is recomputed from the saved pattern, so later estimates agree
 * with an uninterrupted run to rounding.  dpg_inc_load returns NULL on error (dpg_last_error);
 * a file of another version or layout is rejected. */
int dpg_inc_save(dpg_inc* g, const char* path);
dpg_inc* dpg_inc_load(dpg_ctx* ctx, const char* path);
/* The graph's state as host copies (the checkpoint's arrays without the scans): the update count,
 * the factors and the update that added each (up to cap_factors of them), the linearization points
 * theta [3 V], the estimate [3 V] and the last max |delta| per node [V] (V = dpg_inc_num_nodes);
 * any pointer may be NULL.  Returns the number of factors, negative on error. */
int64_t dpg_inc_export(dpg_inc* g, int64_t* updates, dpg_factor* factors, int32_t* created, int64_t cap_factors,
                       double* theta, double* est, double* maxd);

/* Append nodes to the uploaded scan store (dpg_scans_upload's layout): pts_xy = the new nodes' full
 * clouds concatenated, node_offsets[n_new + 1] relative to pts_xy; the downsample ratio must match
 * the store's.  Only the new nodes' neighbour indexes are built. */
int dpg_scans_append(dpg_ctx* ctx, const float* pts_xy, const int64_t* node_offsets, int64_t n_new,
                     int32_t downsample_ratio);

typedef struct dpg_add_node_stats {
    int64_t n_icp_edges;             /* successive + loop-closure alignments run for this node */
    int64_t n_loop_closures;         /* loop-closure factors added (converged alignments) */
    double ms_icp;                   /* batched ICP of the node's edges (incl. its index build) */
    dpg_inc_stats update;
} dpg_add_node_stats;

/* One new node (id V = dpg_inc_num_nodes(g)) with explicit alignments: the node's base_link cloud
 * joins the scan store; ONE batched ICP aligns the successive pair (V-1, V) when `successive` and
 * every pair in pairs[n_pairs][2] = {node_1 (target), node_2 (source)}, keys <= V; the successive
 * factor always joins the graph, the other pairs' factors when converged (dpg_slam.cc:263-267,
 * 295-301), after the caller's `extra` factors, in one dpg_inc_update (initial pose init_pose).
 * The update's symbolic work runs on the host while the GPU aligns, with every pair in the pattern:
 * a pair whose alignment does not converge stays an explicit zero block of H (no factor; the
 * solution is unchanged, the update's nnz statistics count it). */
int dpg_add_node_pairs(dpg_inc* g, const float* cloud_xy, int64_t n_pts, const float init_pose[3],
                       const dpg_factor* extra, int64_t n_extra, const int32_t* pairs, int64_t n_pairs,
                       int32_t successive, const dpg_icp_params* icp_params, dpg_add_node_stats* stats);
/* One new node, as updatePoseGraphObsConstraints + optimizeGraph run it (dpg_slam.cc:255-314):
 * the node's base_link cloud is appended to the scan store (node id = dpg_inc_num_nodes(g)); ONE
 * batched ICP aligns the successive pair (prev, new) and every loop-closure candidate (i, prev),
 * i < V - 2 (V = nodes before this one), whose float distance to prev's estimate is within
 * max_node_dist_within_pass (same pass_numbers) or max_node_dist_across_passes; the successive
 * factor is always added, loop closures when converged; together with the caller's `extra`
 * factors (the pass prior or the odometry Between) they go into one dpg_inc_update with the node's
 * initial pose init_pose (createRelativePositionedNode, float).  pass_numbers[V + 1]: every node's
 * pass, the new one last.  non_successive = 0 skips the loop closures
 * (non_successive_scan_constraints_, parameters.h:349-354).  The ICP guesses use the estimates of
 * dpg_inc_get_poses rounded to float (the reference's dpg_nodes_ positions are float). */
int dpg_add_node(dpg_inc* g, const float* cloud_xy, int64_t n_pts, const int32_t* pass_numbers, const float init_pose[3],
                 const dpg_factor* extra, int64_t n_extra, const dpg_icp_params* icp_params,
                 const dpg_reopt_params* params, int32_t non_successive, dpg_add_node_stats* stats);

/* ---- DPG change detection (DpgSLAM::executeDPG, dpg_slam.cc:865-886) ----
 * The dynamic node state (DpgNode/Measurement: per-beam label and sector, per-node sector
 * activation and active flag) lives on the device in a dpg_dpg store; executeDPG runs on it.
 * Semantics are the reference's with its Q8 defects fixed ("DPG"): a grid point is
 * transformed into the map frame once; unlabelled points count as STATIC; the uncovered-cell set
 * loses every cell the candidate covers; the bin ratio is a real division; the bin score uses the
 * pose-chain node whose grid is tested and its own scan's angle range; removed points are labelled
 * on their own node; a deactivated sector skips one removed point (continue, not break); the pose
 * chain is placed at the nodes' CURRENT estimates (est_poses) everywhere -- the reference's
 * current_pass_nodes_ holds by-value DpgNode copies made at creation (dpg_slam.cc:195,307,598,
 * dpg_node.h:163) that optimizeGraph never updates, so its chain grids and proximity search sit at
 * creation-time poses while its bin score (:793-800) and sector update (:893-898) use the
 * optimised ones (DPG item 8). */
enum { DPG_LABEL_STATIC = 0, DPG_LABEL_ADDED = 1, DPG_LABEL_REMOVED = 2, DPG_LABEL_NOT_YET_LABELED = 3,
       DPG_LABEL_MAX_RANGE = 4 };   /* PointLabel, dpg_measurement.h:21 */

typedef struct dpg_change_params {
    int32_t num_sectors;                        /* 5 (parameters.h:44) */
    int32_t current_pose_chain_len;             /* 5 (parameters.h:57), <= 15 */
    int32_t num_bins_for_change_detection;      /* uninitialised in the reference (parameters.h:62); 36 */
    int32_t pad;
    double delta_change_threshold;              /* 0.20 (parameters.h:67) */
    double current_pose_graph_coverage_threshold; /* 1.0 (parameters.h:72) */
    double occ_grid_resolution;                 /* 0.05 (parameters.h:77) */
    float minimum_percent_active_sectors;       /* 0.5 (parameters.h:82) */
    float distance_threshold_for_local_submap_nodes; /* 5.0 (parameters.h:87) */
    float laser[3];                             /* laser pose in base_link: 0.2, 0, 0 (parameters.h:319-339) */
    float pad2;
} dpg_change_params;

typedef struct dpg_change_stats {
    int64_t n_chain;            /* current pose chain length used */
    int64_t n_candidates;       /* active past nodes within the proximity threshold */
    int64_t n_submap_nodes;     /* candidates merged into the local submap */
    int64_t n_chain_cells;      /* cells of the pose-chain grids (the uncovered set at the start) */
    int64_t n_uncovered;        /* chain cells left uncovered by the submap */
    int64_t n_added;            /* points labelled ADDED (committed nodes only) */
    int64_t n_removed;          /* distinct points labelled REMOVED */
    int64_t n_committed;        /* pose-chain nodes whose bin score passed */
    int64_t n_sectors_deactivated; /* by updateNodesAndSectorStatus */
    int64_t n_nodes_deactivated;
    int64_t grid_cells;         /* dense window cells (W x H) */
    int64_t n_samples;          /* ray samples marched (all rasterisation passes) */
    double ms_total;            /* wall time of dpg_execute_dpg */
    double ms_kernels;          /* device time, HIP events around the device work */
} dpg_change_stats;

typedef struct dpg_dpg dpg_dpg;

void dpg_change_params_default(dpg_change_params* p);
/* Node store: n_nodes scans (ranges[beam_offsets[v] .. beam_offsets[v+1]), geom[v] = angle_min,
 * angle_max, range_max).  Labels start as MeasurementPoint's constructor sets them
 * (dpg_measurement.h:41-46), sectors as createNode numbers them (dpg_slam.cc:499-507), every sector
 * and node active.  NULL on error (dpg_last_error). */
dpg_dpg* dpg_dpg_create(dpg_ctx* ctx, int64_t n_nodes, const int64_t* beam_offsets, const float* ranges,
                        const float* geom /*[V][3]*/, const dpg_change_params* params);
void dpg_dpg_destroy(dpg_dpg* d);
/* Add n_new nodes' scans at the end (createNode of each new node, dpg_slam.cc:488-513):
 * beam_offsets[n_new + 1] relative to ranges[0]; existing labels, sectors and activity are kept. */
int dpg_dpg_append(dpg_dpg* d, int64_t n_new, const int64_t* beam_offsets, const float* ranges,
                   const float* geom /*[n_new][3]*/);
/* executeDPG after node n_nodes-1 was added: dpg_nodes_ = nodes [0, n_nodes), current_pass_nodes_ =
 * the last current_pass_len of them; est_poses[n_nodes][3] the estimated node poses. */
int dpg_execute_dpg(dpg_dpg* d, int64_t n_nodes, int64_t current_pass_len, const float* est_poses,
                    dpg_change_stats* stats);
/* The same with the pose chain placed where the reference places it: chain_poses[chain_n][3] are the
 * poses of the last chain_n = min(current_pass_len, current_pose_chain_len) nodes as the host's
 * current_pass_nodes_ copies hold them (dpg_slam.cc:195,307,598: by-value copies taken at creation
 * and never refreshed by optimizeGraph).  They place the chain grids (computeLocalSubMap,
 * :591-620) and the submap proximity search (:646-668); the bin score (:786-800) and the sector
 * update (:893-898) keep est_poses, as dpg_nodes_ does.  chain_poses == NULL is dpg_execute_dpg
 * (every use at est_poses, Q8 fix 8 of DESIGN.md section 3). */
int dpg_execute_dpg_chain(dpg_dpg* d, int64_t n_nodes, int64_t current_pass_len, const float* est_poses,
                          const float* chain_poses, dpg_change_stats* stats);
/* Copy the node state back (any pointer may be NULL): labels[B], sector_active[V] (bit s = sector s
 * active), node_active[V]. */
int dpg_dpg_fetch(dpg_dpg* d, uint8_t* labels, uint8_t* sector_active, uint8_t* node_active);
/* Overwrite the node state (tests, checkpoint restore); NULL leaves that part unchanged. */
int dpg_dpg_load(dpg_dpg* d, const uint8_t* labels, const uint8_t* sector_active, const uint8_t* node_active);
/* DpgSLAM::getActiveAndDynamicMapPoints (dpg_slam.cc:832-863) over nodes [0, n_nodes): the four
 * point lists in node/beam order, concatenated into out[cap][2] as active_static | active_added |
 * dynamic_removed | dynamic_added; counts[4] receives their sizes.  Returns the total (negative:
 * error); writes nothing past cap. */
int64_t dpg_active_dynamic_points(dpg_dpg* d, int64_t n_nodes, const float* est_poses, float* out,
                                  int64_t cap, int64_t counts[4]);

#ifdef __cplusplus
}
#endif
#endif /* DPG_SLAM_C_H */
