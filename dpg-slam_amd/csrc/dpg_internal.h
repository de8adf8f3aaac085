/*
 * dpg_internal.h -- private structures shared by the C-ABI layer (dpg_api.hip) and the HIP
 * kernel translation units (dpg_icp.hip, dpg_gn.hip).  Not part of the public ABI.
 */
#ifndef DPG_INTERNAL_H
#define DPG_INTERNAL_H

#include <stdint.h>

#include "../../include/dpg_slam_c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* error message + code for dpg_last_error; the context's stream / device (dpg_api.hip) */
int dpg_set_error(int code, const char* msg);
dpg_ctx* dpg_inc_ctx(dpg_inc* g);   /* the context an incremental graph runs on (dpg_inc.hip) */
/* the structural half of the next dpg_inc_update (host only: n_new nodes, node pairs that may carry
 * its Between factors), so that it can run while the GPU aligns the node's edges (dpg_inc.hip) */
int dpg_inc_prepare(dpg_inc* g, int64_t n_new, const int32_t* pairs, int64_t n_pairs);
int dpg_inc_abort_prepare(dpg_inc* g);
int dpg_ctx_is_multi(dpg_ctx* c);
/* the scan store as host copies, and the neighbour index of every stored node (the graph
 * checkpoint, dpg_inc_save / dpg_inc_load in dpg_inc.hip) */
int dpg_scans_export(dpg_ctx* c, int64_t* n_nodes, int32_t* ratio, int64_t* off, float* pts);
int dpg_scans_index_all(dpg_ctx* c);
void* dpg_ctx_stream_of(dpg_ctx* c);
int dpg_ctx_device_of(dpg_ctx* c);
/* children of a context (incremental graphs, DPG stores): dpg_ctx_destroy destroys the ones still
 * alive, newest first; a child's own destroy releases it from the list */
void dpg_ctx_adopt(dpg_ctx* c, void* child, void (*destroy)(void*));
void dpg_ctx_release_child(dpg_ctx* c, void* child);
/* one lane waits (system-scope loads of a host-mapped word) until *flag - tag >= 0 as int32; after
 * ~120 s it gives up and sets *timed_out (dpg_gn.hip; the rank form's host collective thread) */
int dpg_launch_host_wait(const uint32_t* flag, uint32_t tag, uint32_t* timed_out, void* stream);

/* One ICP edge as the kernel sees it (64 B).  Offsets/counts are in points (float2). */
typedef struct dpg_icp_edge {
    int32_t src_ds_off, n_src_ds;    /* downsampled node_2 cloud (ICP source) */
    int32_t tgt_ds_off, n_tgt_ds;    /* downsampled node_1 cloud (ICP target) */
    int32_t src_full_off, n_src_full;  /* full node_2 cloud (covariance data_pi) */
    int32_t tgt_full_off, n_tgt_full;  /* full node_1 cloud (covariance model_qi) */
    float guess[6];                  /* runIcp transform_guess rows (dpg_slam.cc:374-378) */
    int32_t src_node, tgt_node;      /* cloud ids (angle-index bucket tables) */
    int32_t pad[2];                  /* pad[0]: index of the edge in the caller's list (results go
                                        there); the array itself is in dispatch order */
} dpg_icp_edge;

/* Scalars of the ICP/convergence rule, precomputed on the host in double. */
typedef struct dpg_icp_kparams {
    double r2;          /* max_dist_sqr = d * d (determineReciprocalCorrespondences) */
    double eps;         /* transformation_epsilon_ (translation threshold) */
    double rot_thr;     /* 1 - transformation_epsilon_ (rotation threshold) */
    double mse_abs;     /* mse_threshold_absolute_ */
    float r2_f;         /* largest float <= r2: (double)d <= r2  <=>  d <= r2_f for float d */
    float h_min;        /* smallest grid cell: 1.05 * r */
    int32_t max_iter;
    int32_t min_corr;
    int32_t reciprocal;
    int32_t cells_max;  /* LDS grid capacity */
    int32_t lds_tgt;    /* LDS target capacity (points) */
    int32_t trace_iters;
    int32_t trace_stride;
    int32_t defer_cap;  /* angular kernel: windows of more candidates go to the workgroup's
                           cooperative queue (0: never) */
    int32_t kernel_variant;   /* angular kernel form (dpg_ctx_set_icp_kernel_variant, A/B only) */
} dpg_icp_kparams;

/* Launchers (defined in dpg_icp.hip).  Return 0 or a negative DPG_ERR_*. */
int dpg_launch_icp(const float* ds_pts_dev, const dpg_icp_edge* edges_dev, int64_t n_edges,
                   const dpg_icp_kparams* kp, int32_t max_points, dpg_icp_result* results_dev,
                   int32_t* trace_dev, void* stream);
int dpg_launch_cov(const float* full_pts_dev, const dpg_icp_edge* edges_dev, int64_t n_edges,
                   const dpg_icp_result* results_dev, double* hess_dev, int32_t max_workgroups, void* stream);
size_t dpg_icp_lds_bytes(int32_t lds_tgt, int32_t cells_max);
/* the 6x6 covariance sums of icp_cov_sandwich (dpg_icp.hip cov6_kernel): out[16] */
int dpg_launch_cov6(const float* pts_dev, int32_t n_data, int32_t n_model, const float* T6_dev, double* out_dev,
                    void* stream);
/* k-d tree variant (dpg_icp_kd.hip): per-node trees over the downsampled clouds, then ICP. */
int dpg_launch_kdtree_build(const float* ds_pts_dev, const int64_t* ds_off_dev, int64_t n_nodes,
                            int32_t max_points, float* tree_pts_dev, uint16_t* tree_idx_dev, void* stream);
int dpg_launch_icp_kd(const float* ds_pts_dev, const float* tree_pts_dev, const uint16_t* tree_idx_dev,
                      const dpg_icp_edge* edges_dev, int64_t n_edges, const dpg_icp_kparams* kp,
                      int32_t max_points, dpg_icp_result* results_dev, int32_t* trace_dev, void* stream);
size_t dpg_icp_kd_lds_bytes(int32_t cap);
/* angular-index variant (dpg_icp_ang.hip, the default): per-node angle-sorted clouds + buckets. */
int32_t dpg_angle_buckets(void);
/* loop-closure candidate search of the re-linearisation sweep (dpg_reopt.hip) */
int dpg_launch_lc_count(const float* poses_dev, const int32_t* pass_dev, int64_t V, float within, float across,
                        int32_t* count_dev, void* stream);
int dpg_launch_lc_write(const float* poses_dev, const int32_t* pass_dev, int64_t V, float within, float across,
                        const int64_t* off_dev, int32_t* pairs_dev, void* stream);
/* map assembly (GetMap): frames_dev[V][4] = x, y, cos, sin (dpg_reopt.hip) */
int dpg_launch_map_points(const float* pts_dev, const int64_t* off_dev, const float* frames_dev, int64_t V,
                          int32_t fraction, float* out_dev, void* stream);
int dpg_launch_angle_index(const float* ds_pts_dev, const int64_t* ds_off_dev, int64_t n_nodes,
                           int32_t max_points, float* idx_pts_dev, uint16_t* idx_orig_dev,
                           uint16_t* buckets_dev, int32_t bitonic, void* stream);
/* clouds of more than 4096 points: record slices in global scratch (scratch_bytes of it, used in
   chunks of scratch_bytes / dpg_icp_ang_scratch_per_edge(cap) edges); up to 16384 points */
int dpg_launch_icp_ang(const float* ds_pts_dev, const float* idx_pts_dev, const uint16_t* idx_orig_dev,
                       const uint16_t* buckets_dev, const dpg_icp_edge* edges_dev, int64_t n_edges,
                       const dpg_icp_kparams* kp, int32_t max_points, dpg_icp_result* results_dev,
                       int32_t* trace_dev, void* scratch, size_t scratch_bytes, void* stream);
size_t dpg_icp_ang_lds_bytes(int32_t cap);
size_t dpg_icp_ang_scratch_per_edge(int32_t cap);

/* Pose-graph system on device (defined in dpg_gn.hip). */
typedef struct dpg_gn_dev {
    int64_t n_nodes, n_factors, nnzb_upper, nnzb_full;
    int64_t shard_begin, shard_end;
    /* factors and their per-block contribution lists */
    dpg_factor* factors;           /* [n_factors] */
    /* upper pattern: block u (0..nnzb_upper) = (row, col) with row <= col; diag blocks first */
    int32_t* up_row;               /* [nnzb_upper] */
    int32_t* up_col;
    int32_t* up_cptr;              /* [nnzb_upper + 1] contribution list ptr */
    int32_t* up_clist;             /* factor index << 2 | role (0: ii, 1: jj, 2: ij, 3: ji) */
    int32_t* node_fptr;            /* [n_nodes + 1] factors whose FIRST key is the node (chi2/b) */
    int32_t* node_flist;
    /* full BSR for the solve */
    int32_t* rowptr;               /* [n_nodes + 1] */
    int32_t* colidx;               /* [nnzb_full] */
    int32_t* src_up;               /* [nnzb_full] upper block feeding this block; < 0: transposed (-1-u) */
    double* bsr;                   /* [nnzb_full][9] */
    double* minv;                  /* [n_nodes][9] block-Jacobi inverses */
    double* poses;                 /* [n_nodes][3] */
    double* x, *r, *z, *p0, *p1, *q; /* PCG vectors [3 n_nodes] */
    double* partials;              /* PCG per-block partial sums */
    double* scal;                  /* PCG scalars */
    double* hb_own;                /* packed [H upper | b | chi2] buffer for single-GPU solves */
    void* chol;                    /* supernodal Cholesky (dpg_chol.hip), NULL if analysis failed */
    double* scal3;                 /* [4] device scalars: max |delta|, chi2, status, pad */
    double* scal3_host;            /* pinned mirror of scal3 */
    int32_t n_blocks_rows;         /* grid size for row kernels */
    int32_t last_pcg_iters;
    int32_t last_used_chol;        /* the last solve ran the Cholesky (its status word is meaningful) */
    double last_delta_inf;         /* host: max |delta| of the last fetched retraction */
    double prev_delta_inf;         /* host: the one before it */
    int32_t have_factor;           /* the Cholesky holds a factorization of this graph */
    int32_t last_was_chord;        /* the last solve reused the factor */
    int32_t n_factorizations;      /* since dpg_gn_set_poses */
    /* multi-device forms: this device linearizes the factors f with mine[f] != 0 (instead of the
       range [shard_begin, shard_end)) into hb_part; the all-reduce of hb_part gives hb_own */
    uint8_t* mine;                 /* [n_factors] or NULL */
    double* hb_part;               /* [hb size] or NULL */
    int32_t world, rank;
    /* world > 1: the packed buffer ends in 2 world "vote" words -- this device's max |delta| at
       [rank] and its solver status at [world + rank], zeros elsewhere -- so after the sum every
       device holds every device's pair and takes its stop / chord decision from the same numbers
       (dpg_gn_pipe.h): the ranks cannot disagree on the iteration count, and with it on the number
       of collectives they issue */
    int32_t n_vote;
    /* host clock of the last dpg_gn_dev_alloc (ms): pattern + contribution lists + BSR rows, the
       Cholesky's symbolic analysis, its host plan (these three before the stream wait), the wait +
       device allocations + uploads, the Cholesky's upload */
    double setup_ms[5];
} dpg_gn_dev;

/* Supernodal multifrontal Cholesky of the block system (dpg_chol.hip); opts (dpg_chol.h, NULL =
   defaults) are the context's solver options */
struct dpg_chol_opts;
int dpg_chol_create(void** chol, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                    const struct dpg_chol_opts* opts);
void dpg_chol_destroy(void* chol);
/* factor H (upper blocks of hb) and solve H x = -g; x (block positions) stays on device */
int dpg_chol_solve(void* chol, const double* hb, void* stream);
/* solve H x = -g with the factorization of the last dpg_chol_solve (g from hb) */
int dpg_chol_resolve(void* chol, const double* hb, void* stream);
/* keep L11^-1 of the large fronts after each ungated factorization for dpg_chol_resolve (GN graphs) */
void dpg_chol_keep_inverse(void* chol, int on);
/* Partial refactorization (the incremental graph's ISAM2 updates, dpg_inc.hip): with tracking on,
   the solver remembers the analysis its fronts were last factored under.  dpg_chol_solve_partial
   then refactors only the fronts that hold a dirty node's column (a new node, an endpoint of a new
   factor or pair), whose structure changed, or that lie above such a front; the others keep their
   factored values (moved to the new layout where it shifted them), then the forward and backward
   solves run over every front.  Falls back to dpg_chol_solve when nothing can be kept.  Valid only
   when the H blocks of the kept fronts are unchanged since that factorization (same linearization
   point, same factors). */
void dpg_chol_track_factor(void* chol, int on);
void dpg_chol_forget_factor(void* chol);
int dpg_chol_solve_partial(void* chol, const double* hb, const int32_t* dirty_nodes, int64_t n_dirty, void* stream);
/* the last solve: fronts refactored, fronts kept, doubles moved (all fronts refactored: kept = 0),
   host ns of the partial solve's pick + launches */
void dpg_chol_partial_stats(void* chol, int64_t out[4]);
const int32_t* dpg_chol_pos_dev(void* chol);
const double* dpg_chol_x_dev(void* chol);
const int32_t* dpg_chol_status_dev(void* chol);
void dpg_chol_stats(void* chol, double out[6]);

/* host work first (pattern, lists, the Cholesky's analysis and plan), then -- after
   hipStreamSynchronize(sync_stream) when given -- the device allocations and uploads */
int dpg_gn_dev_alloc(dpg_gn_dev* g, int64_t n_nodes, const dpg_factor* factors, int64_t n_factors,
                     int64_t shard_begin, int64_t shard_end, const struct dpg_chol_opts* opts, void* sync_stream);
/* the context's solver options (dpg_ctx_set_solver_options) */
const struct dpg_chol_opts* dpg_ctx_chol_opts(dpg_ctx* c);
void dpg_gn_dev_free(dpg_gn_dev* g);
int64_t dpg_gn_dev_hb_size(const dpg_gn_dev* g);
int64_t dpg_gn_dev_vote_offset(const dpg_gn_dev* g);   /* first vote word of the packed buffer */
int dpg_gn_dev_assemble(dpg_gn_dev* g, double* hb_dev, void* stream);
/* enqueue the solve + retraction (max |delta| kept on device); no host synchronisation for the
   Cholesky solver */
int dpg_gn_dev_solve_async(dpg_gn_dev* g, const double* hb_dev, const dpg_gn_params* gp, void* stream);
/* one synchronisation: out = {max |delta| of the last retraction, chi2 of hb, solver status} */
int dpg_gn_dev_fetch(dpg_gn_dev* g, const double* hb_dev, void* stream, double out[3]);
int dpg_gn_dev_solve(dpg_gn_dev* g, const double* hb_dev, const dpg_gn_params* gp, void* stream,
                     double* delta_inf, double* error, int32_t* pcg_iters);
int dpg_gn_dev_icp_to_factors(dpg_gn_dev* g, const dpg_icp_result* results_dev, int64_t first,
                              int64_t count, int64_t n_always, double info_x, double info_y,
                              double info_th, void* stream);
/* multi-device forms: factor f is this device's when f mod world == rank (allocates mine + hb_part) */
int dpg_gn_dev_set_ownership(dpg_gn_dev* g, int32_t world, int32_t rank, void* stream);
/* ICP slots [first, first + count) of the batch: this device's n_local results (caller indices
   idx_dev) become its factors, every other slot in the range another device's */
int dpg_gn_dev_icp_to_factors_scatter(dpg_gn_dev* g, const dpg_icp_result* results_dev, const int32_t* idx_dev,
                                      int64_t n_local, int64_t first, int64_t count, int64_t n_always, double info_x,
                                      double info_y, double info_th, void* stream);
/* this device's share of [H upper | g | chi2] into hb_part (gate: the pipelined loop's, or NULL) */
int dpg_gn_dev_assemble_part(dpg_gn_dev* g, const int32_t* gate, void* stream);
/* virtual devices: outs[r] = sum over q in rank order of parts[q], n doubles, r < k <= 16 */
int dpg_launch_vsum(const double* const* parts, double* const* outs, int32_t k, int64_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif
