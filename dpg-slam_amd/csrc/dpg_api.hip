// dpg_api.hip -- the extern "C" boundary (include/dpg_slam_c.h, include/dpg_icp_cov.h).
//
// Entry points replace (reference file:line):
//   icp_cov_calculate     -> calculate_ICP_COV            src/icp_cov/cov_func_point_to_point.h:24
//   dpg_run_icp           -> DpgSLAM::runIcp               src/dpg_slam/dpg_slam.cc:362-446
//   dpg_icp_batch_*       -> the runIcp calls of reoptimize / updatePoseGraphObsConstraints
//                            (dpg_slam.cc:85,101,263,295), batched
//   dpg_optimize_graph    -> DpgSLAM::optimizeGraph        src/dpg_slam/dpg_slam.cc:316-329
//   dpg_gn_*              -> the same solve, split for the edge-sharded multi-GPU driver
// Host memory in, host memory out; device work is asynchronous on the context stream except
// where a host value must be returned.  No fallback: without a usable GPU dpg_ctx_create returns
// NULL and every call that needs one fails with DPG_ERR_HIP.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/dpg_icp_cov.h"
#include "../../include/dpg_slam_c.h"
#include "dpg_chol.h"
#include "dpg_gn_pipe.h"
#include "dpg_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) return fail(DPG_ERR_HIP, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

double now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
    int reserve(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return -1;
        cap = n;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    // grow to n elements keeping the first `keep` (stream-ordered copy, synchronised)
    int grow(size_t n, size_t keep, hipStream_t s) {
        if (n <= cap) return 0;
        const size_t nc = std::max(n, cap + cap / 2);
        T* q = nullptr;
        if (hipMalloc(reinterpret_cast<void**>(&q), nc * sizeof(T)) != hipSuccess) return -1;
        if (p && keep && (hipMemcpyAsync(q, p, std::min(keep, cap) * sizeof(T), hipMemcpyDeviceToDevice, s) != hipSuccess ||
                          hipStreamSynchronize(s) != hipSuccess)) {
            (void)hipFree(q);
            return -1;
        }
        if (p) (void)hipFree(p);
        p = q;
        cap = nc;
        return 0;
    }
};

}  // namespace

struct dpg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipEvent_t ev[8] = {};
    // the batch covariance runs on `aux` beside what follows the ICP on `stream` (the pose graph
    // does not read it): ev[2] marks its end, cov_pending until `stream` has been made to wait
    hipStream_t aux = nullptr;
    bool cov_pending = false, cov_on_aux = false;
    int32_t icp_variant = DPG_ICP_ANGULAR;
    int32_t defer_cap = 256;        // angular ICP: cooperative-queue threshold (dpg_ctx_set_icp_defer_cap)
    int32_t cov_wg = 256;           // covariance kernel workgroups beside the pose graph (dpg_ctx_set_cov_workgroups)
    int32_t kernel_variant = 0;     // angular ICP kernel form (dpg_ctx_set_icp_kernel_variant, A/B)
    float map_ms = 0.f;             // last dpg_get_map kernel (HIP events map_ev)
    hipEvent_t map_ev[2] = {};
    // scan store (batch form)
    DevBuf<float> full, ds;
    DevBuf<int64_t> ds_off_dev;
    DevBuf<int64_t> full_off_dev;  // the full clouds' offsets (the upload's device-side downsampling)
    DevBuf<float> tree_pts;        // per-node index over the downsampled clouds (k-d tree or angle order)
    DevBuf<uint16_t> tree_idx;
    DevBuf<uint16_t> buckets;      // angle variant: [V][B+1] bucket starts
    DevBuf<unsigned char> icp_scratch;   // angle variant, clouds above 4096 points: record slices
    std::vector<int64_t> full_off, ds_off;
    int64_t n_nodes = 0;
    int64_t idx_valid = 0;         // angular variant: nodes [0, idx_valid) of the store have their index
    int32_t ratio = 1;
    int32_t max_ds = 0;
    // staged edge batch
    std::vector<dpg_icp_edge> h_edges;
    DevBuf<dpg_icp_edge> edges;
    DevBuf<dpg_icp_result> res;
    DevBuf<double> hess;
    DevBuf<int32_t> trace;
    int64_t n_edges = 0;
    int32_t max_src = 0, max_tgt = 0;
    int32_t trace_iters = 0;
    dpg_icp_kparams kp{};
    bool have_cov = false;
    // single-call scratch (dpg_run_icp / icp_cov_calculate)
    DevBuf<float> s_pts;
    DevBuf<dpg_icp_edge> s_edge;
    DevBuf<dpg_icp_result> s_res;
    DevBuf<double> s_hess;
    DevBuf<int64_t> s_off;
    DevBuf<float> s_tree_pts;
    DevBuf<uint16_t> s_tree_idx;
    DevBuf<uint16_t> s_buckets;
    // pose graph
    dpg_gn_dev gn{};
    bool gn_ready = false;
    dpg_gn_params gp{};
    float asm_ms = 0.f, solve_ms = 0.f;
    // the pipelined GN loop (dpg_gn_pipe.h): control block, two host-mapped report slots + events
    dpg_gn_ctl* pipe_ctl = nullptr;
    dpg_gn_slot* pipe_slot = nullptr;
    uint32_t pipe_loop = 0;            // loops run on this device (tags their reports)
    // multi-device forms (dpg_ctx_create_multi / _rank / _virtual): this context drives local
    // device 0 and holds the batch as the caller sees it; `peers` are full single-device contexts
    // of the other local devices.  Local device k is global rank rank0 + k of `world`.
    std::vector<dpg_ctx*> peers;
    // incremental graphs and DPG stores created on this context: dpg_ctx_destroy destroys them
    // first (their buffers, helper thread and events all use the context's stream)
    std::vector<std::pair<void*, void (*)(void*)>> children;
    std::vector<ncclComm_t> comms;   // RCCL: one communicator per local device
    dpg_coll_ops host_ops{};         // kCollHost: the caller's host-memory collectives
    std::vector<double> host_hb;     // kCollHost: the packed system in host memory
    struct HostColl;                 // kCollHost, pipelined GN: the collective thread (below)
    std::unique_ptr<HostColl> hc;
    int32_t coll = 0;                // kCollNone | kCollRccl | kCollVirtual | kCollHost
    int32_t world = 1, rank0 = 0;
    int32_t rank = 0;                // global rank of THIS device context (peers too)
    // the staged batch, every form: the edges in the caller's order and their assignment --
    // batch_owner[e] = global rank aligning edge e; shard[k] = the caller indices aligned on local
    // device k, ascending (local result j of device k is edge shard[k][j])
    std::vector<dpg_icp_edge> batch;
    std::vector<int32_t> batch_owner;
    std::vector<std::vector<int64_t>> shard;
    bool batch_measured = false;     // assignment + dispatch order from measured costs
    int32_t batch_runs = 0;          // runs of the staged batch so far
    int32_t schedule = DPG_ICP_SCHEDULE_MEASURED;
    // measured alignment cost (iterations x (source + target points)) by (target, source) pair,
    // from earlier runs: the LPT assignment over ranks and the longest-first dispatch order
    std::unordered_map<uint64_t, float> cost;
    DevBuf<int32_t> shard_idx;       // per device context: its shard's caller indices
    DevBuf<float> cost_dev;          // rank form: the all-reduced cost vector of a batch
    dpg_chol_opts copts;             // solver options (dpg_ctx_set_solver_options)
};

// The rank form over the caller's collectives (kCollHost) in the pipelined Gauss-Newton loop: the
// packed system's all-reduce of iteration i runs on this thread, so the host can queue iteration
// i + 1 before iteration i's report, as over RCCL.  Per iteration, on the context stream: the
// assembly's partial system -> pinned host buffer, an event; then a one-lane kernel that waits
// until the thread has stored the iteration's tag in a host-mapped word (system-scope loads); then
// the summed system -> hb_own.  The thread waits for the event, calls the caller's all-reduce in
// place and stores the tag.  Stream order serializes the buffer's uses (the next copy into it
// follows this iteration's copy out of it).  A failed collective still stores the tag (the stream
// moves on) and sets `failed`, which the loop checks at every report.
struct dpg_ctx::HostColl {
    double* buf = nullptr;           // pinned: the packed system, summed in place
    size_t cap = 0;                  // doubles
    uint32_t* flag = nullptr;        // host-mapped: the last tag the thread completed
    uint32_t* timed_out = nullptr;   // host-mapped: the wait kernel gave up (no tag in 120 s)
    hipEvent_t ev[2] = {nullptr, nullptr};
    uint32_t next_tag = 0;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<uint32_t, hipEvent_t>> jobs;
    size_t count = 0;                // doubles of the current system
    uint64_t posted = 0, done = 0;
    bool stop = false;
    std::atomic<int> failed{0};
};

namespace {
enum { kCollNone = 0, kCollRccl = 1, kCollVirtual = 2, kCollHost = 3, kMaxVirtual = 16 };
inline int n_dev(const dpg_ctx* c) { return 1 + (int)c->peers.size(); }
// one process per GPU with more than one rank (dpg_ctx_create_rank / _rank_ops): the batch's
// results and costs travel between processes
inline bool is_rank_form(const dpg_ctx* c) {
    return (c->coll == kCollRccl || c->coll == kCollHost) && c->peers.empty() && c->world > 1;
}
inline dpg_ctx* dev_ctx(dpg_ctx* c, int k) { return k == 0 ? c : c->peers[(size_t)k - 1]; }
// made by dpg_ctx_create_multi / _rank / _virtual (even for one GPU: its calls then take the
// sharded paths, the all-reduce included, with one rank)
inline bool is_multi(const dpg_ctx* c) { return c->coll != kCollNone; }
// order `stream` after the last batch covariance (before anything rewrites its inputs or reads it)
inline int join_cov(dpg_ctx* c) {
    if (!c->cov_pending) return DPG_OK;
    c->cov_pending = false;
    return hipStreamWaitEvent(c->stream, c->ev[2], 0) == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}
}  // namespace

namespace {

int set_kparams(dpg_icp_kparams* kp, const dpg_icp_params* p) {
    if (!p) return fail(DPG_ERR_ARG, "params is NULL");
    if (!(p->icp_max_correspondence_distance > 0.0)) return fail(DPG_ERR_ARG, "icp_max_correspondence_distance must be > 0");
    memset(kp, 0, sizeof(*kp));
    const double r = p->icp_max_correspondence_distance;
    kp->r2 = r * r;
    float f = (float)kp->r2;
    if ((double)f > kp->r2) f = nextafterf(f, 0.0f);
    kp->r2_f = f;
    kp->h_min = (float)(r * 1.05);
    kp->eps = p->icp_maximum_transformation_epsilon;
    kp->rot_thr = 1.0 - p->icp_maximum_transformation_epsilon;
    kp->mse_abs = p->mse_threshold_absolute;
    kp->max_iter = p->icp_maximum_iterations;
    kp->min_corr = p->min_number_correspondences;
    kp->reciprocal = p->icp_use_reciprocal_correspondences ? 1 : 0;
    kp->cells_max = 4096;
    return DPG_OK;
}

int32_t round_up(int32_t v, int32_t m) { return (v + m - 1) / m * m; }

// Per-node indexes (k-d trees / angle order) are built over `n_tree_nodes` clouds (offsets
// ds_off_dev) before the ICP kernel of those variants.
int launch_batch(dpg_ctx* c, const float* ds_dev, const float* full_dev, const int64_t* ds_off_dev,
                 int64_t n_tree_nodes, int32_t max_node_pts, float* tree_pts, uint16_t* tree_idx,
                 uint16_t* buckets, const dpg_icp_edge* edges_dev, int64_t ne, dpg_icp_kparams kp,
                 int32_t max_src, int32_t max_tgt, dpg_icp_result* res_dev, double* hess_dev, int32_t* trace_dev,
                 bool timed, int64_t tree_from = 0) {
    if (c->icp_variant != DPG_ICP_ANGULAR) tree_from = 0;   // the other variants rebuild everything
    const int32_t maxp = std::max(max_src, max_tgt);
    if (maxp > 16384) return fail(DPG_ERR_SIZE, "downsampled cloud of %d points exceeds 16384", maxp);
    if (maxp > 4096 && c->icp_variant != DPG_ICP_ANGULAR)
        return fail(DPG_ERR_SIZE, "downsampled cloud of %d points: only the angular ICP variant takes more than 4096", maxp);
    int rc = join_cov(c);
    if (rc) return fail(rc, "stream wait failed");
    if (timed) HIP_TRY(hipEventRecord(c->ev[6], c->stream));
    if (c->icp_variant == DPG_ICP_KDTREE) {
        rc = dpg_launch_kdtree_build(ds_dev, ds_off_dev, n_tree_nodes, max_node_pts, tree_pts, tree_idx, c->stream);
        if (rc) return fail(rc, "k-d tree build launch failed (%d)", rc);
    } else if (c->icp_variant == DPG_ICP_ANGULAR && tree_from < n_tree_nodes) {
        rc = dpg_launch_angle_index(ds_dev, ds_off_dev + tree_from, n_tree_nodes - tree_from, max_node_pts, tree_pts,
                                    tree_idx, buckets + tree_from * (int64_t)(dpg_angle_buckets() + 1),
                                    c->kernel_variant == 2, c->stream);
        if (rc) return fail(rc, "angle index build launch failed (%d)", rc);
    }
    if (ds_dev == c->ds.p)   // the store's own indexes: current for every node now, or (other variants) overwritten
        c->idx_valid = c->icp_variant != DPG_ICP_ANGULAR ? 0 : tree_from <= c->idx_valid ? n_tree_nodes : c->idx_valid;
    if (timed) HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    if (c->icp_variant == DPG_ICP_ANGULAR) {
        kp.lds_tgt = round_up(std::max<int32_t>(maxp, 1), 16);   // record capacity
        kp.defer_cap = c->defer_cap;
        kp.kernel_variant = c->kernel_variant;
        // large clouds: a record slice per resident edge in global scratch, edges in chunks of <= 2048
        const size_t per_edge = dpg_icp_ang_scratch_per_edge(kp.lds_tgt);
        size_t sbytes = 0;
        if (per_edge) {
            sbytes = per_edge * (size_t)std::min<int64_t>(ne, 2048);
            if (c->icp_scratch.reserve(sbytes)) return fail(DPG_ERR_HIP, "out of device memory for the ICP scratch");
        }
        rc = dpg_launch_icp_ang(ds_dev, tree_pts, tree_idx, buckets, edges_dev, ne, &kp, maxp, res_dev, trace_dev,
                                per_edge ? c->icp_scratch.p : nullptr, sbytes, c->stream);
    } else if (c->icp_variant == DPG_ICP_KDTREE) {
        kp.lds_tgt = round_up(std::max<int32_t>(maxp, 1), 64);
        rc = dpg_launch_icp_kd(ds_dev, tree_pts, tree_idx, edges_dev, ne, &kp, maxp, res_dev, trace_dev, c->stream);
    } else {
        kp.lds_tgt = round_up(std::max<int32_t>(max_tgt, 1), 64);
        rc = dpg_launch_icp(ds_dev, edges_dev, ne, &kp, maxp, res_dev, trace_dev, c->stream);
    }
    if (rc) return fail(rc, "ICP kernel launch failed (%d): %s", rc, hipGetErrorString(hipGetLastError()));
    if (timed) HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    if (hess_dev && timed) {   // beside the pose graph: on aux, after the ICP
        if (!c->aux) HIP_TRY(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
        HIP_TRY(hipStreamWaitEvent(c->aux, c->ev[1], 0));
        rc = dpg_launch_cov(full_dev, edges_dev, ne, res_dev, hess_dev, c->cov_wg, c->aux);
        if (rc) return fail(rc, "covariance kernel launch failed");
        HIP_TRY(hipEventRecord(c->ev[2], c->aux));
        c->cov_pending = true;
        c->cov_on_aux = true;
        return DPG_OK;
    }
    if (timed) c->cov_on_aux = false;
    if (hess_dev) {
        rc = dpg_launch_cov(full_dev, edges_dev, ne, res_dev, hess_dev, 0, c->stream);
        if (rc) return fail(rc, "covariance kernel launch failed");
    }
    if (timed) HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    return DPG_OK;
}

void const_cov(const dpg_icp_params* p, double cov[9]) {
    memset(cov, 0, 9 * sizeof(double));
    cov[0] = (double)p->laser_x_variance;
    cov[4] = (double)p->laser_y_variance;
    cov[8] = (double)p->laser_theta_variance;
}

dpg_ctx* g_default_ctx = nullptr;

}  // namespace

extern "C" {

const char* dpg_last_error(void) { return g_err.c_str(); }

// internal (dpg_internal.h): error reporting and the context's stream for the other TUs
int dpg_set_error(int code, const char* msg) { return fail(code, "%s", msg); }
void* dpg_ctx_stream_of(dpg_ctx* c) { return c ? reinterpret_cast<void*>(c->stream) : nullptr; }
int dpg_ctx_device_of(dpg_ctx* c) { return c ? c->device : -1; }
const char* dpg_version(void) { return "dpg-mi355x 0.1 (gfx950)"; }

// The batch over the ranks (host only).  cost != NULL: longest-processing-time -- edges by cost,
// longest first (stable: lower index first among equals), each to the least-loaded rank (lower rank
// among equals), dispatched on its rank in that order, so the alignments that bound a launch start
// first.  cost == NULL: edge e on rank e mod world in the caller's order (the caller's lists come
// grouped -- successive pairs, then loop closures nearest first -- so every rank gets the same mix).
int dpg_shard_plan(const float* cost, int64_t ne, int32_t world, int32_t* owner, int64_t* dispatch, int64_t* counts) {
    if (ne < 0 || world < 1 || (ne > 0 && (!owner || !dispatch)) || !counts) return fail(DPG_ERR_ARG, "dpg_shard_plan: bad arguments");
    std::vector<std::vector<int64_t>> disp((size_t)world);
    if (cost) {
        std::vector<int64_t> ord((size_t)ne);
        for (int64_t e = 0; e < ne; ++e) ord[(size_t)e] = e;
        std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return cost[a] > cost[b]; });
        std::vector<double> load((size_t)world, 0.0);
        for (int64_t e : ord) {
            int r = 0;
            for (int q = 1; q < world; ++q)
                if (load[(size_t)q] < load[(size_t)r]) r = q;
            owner[e] = r;
            load[(size_t)r] += cost[e];
            disp[(size_t)r].push_back(e);
        }
    } else {
        for (int64_t e = 0; e < ne; ++e) {
            owner[e] = (int32_t)(e % world);
            disp[(size_t)(e % world)].push_back(e);
        }
    }
    int64_t o = 0;
    for (int r = 0; r < world; ++r) {
        counts[r] = (int64_t)disp[(size_t)r].size();
        for (int64_t e : disp[(size_t)r]) dispatch[o++] = e;
    }
    return DPG_OK;
}

// The rank form's all-gathered results back in the caller's order (host only): slice r holds rank
// r's records -- its edges ascending, `slice` records of rec_bytes reserved per rank
int dpg_shard_reassemble(const int32_t* owner, int64_t ne, int32_t world, int64_t slice, int64_t rec_bytes,
                         const void* gathered, void* out) {
    if (ne < 0 || world < 1 || slice < 0 || rec_bytes <= 0 || (ne > 0 && (!owner || !gathered || !out)))
        return fail(DPG_ERR_ARG, "dpg_shard_reassemble: bad arguments");
    std::vector<int64_t> pos((size_t)world, 0);
    const char* g = static_cast<const char*>(gathered);
    char* o = static_cast<char*>(out);
    for (int64_t e = 0; e < ne; ++e) {
        const int32_t r = owner[e];
        if (r < 0 || r >= world || pos[(size_t)r] >= slice) return fail(DPG_ERR_ARG, "dpg_shard_reassemble: edge %lld owner %d out of range", (long long)e, r);
        memcpy(o + e * rec_bytes, g + (r * slice + pos[(size_t)r]++) * rec_bytes, (size_t)rec_bytes);
    }
    return DPG_OK;
}

dpg_ctx* dpg_ctx_create(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        fail(DPG_ERR_HIP, "no HIP device available");
        return nullptr;
    }
    if (device < 0 || device >= n) {
        fail(DPG_ERR_ARG, "device %d out of range (%d devices)", device, n);
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        fail(DPG_ERR_HIP, "hipSetDevice(%d) failed", device);
        return nullptr;
    }
    dpg_ctx* c = new dpg_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        fail(DPG_ERR_HIP, "hipStreamCreate failed");
        return nullptr;
    }
    c->own_stream = true;
    // the side stream of the timed batch's covariance (beside the pose graph) is the context's too:
    // created with it, not inside the first solve (a stream creation costs ~7 ms on this stack)
    if (hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess) c->aux = nullptr;
    for (auto& e : c->ev) (void)hipEventCreate(&e);
    dpg_gn_params_default(&c->gp);
    return c;
}

dpg_ctx* dpg_ctx_create_multi(int32_t n_gpus, const int32_t* devices) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        fail(DPG_ERR_HIP, "no HIP device available");
        return nullptr;
    }
    if (n_gpus < 1 || n_gpus > n) {
        fail(DPG_ERR_ARG, "dpg_ctx_create_multi: %d GPUs asked, %d present", n_gpus, n);
        return nullptr;
    }
    std::vector<int> dl((size_t)n_gpus);
    for (int k = 0; k < n_gpus; ++k) {
        dl[(size_t)k] = devices ? devices[k] : k;
        for (int j = 0; j < k; ++j)
            if (dl[(size_t)j] == dl[(size_t)k]) {
                fail(DPG_ERR_ARG, "dpg_ctx_create_multi: device %d listed twice", dl[(size_t)k]);
                return nullptr;
            }
    }
    dpg_ctx* c = dpg_ctx_create(dl[0]);
    if (!c) return nullptr;
    for (int k = 1; k < n_gpus; ++k) {
        dpg_ctx* q = dpg_ctx_create(dl[(size_t)k]);
        if (!q) {
            dpg_ctx_destroy(c);
            return nullptr;
        }
        q->rank = k;
        c->peers.push_back(q);
    }
    c->comms.assign((size_t)n_gpus, nullptr);
    const ncclResult_t r = ncclCommInitAll(c->comms.data(), n_gpus, dl.data());
    if (r != ncclSuccess) {
        c->comms.clear();
        dpg_ctx_destroy(c);
        fail(DPG_ERR_HIP, "ncclCommInitAll over %d devices failed: %s", n_gpus, ncclGetErrorString(r));
        return nullptr;
    }
    c->coll = kCollRccl;
    c->world = n_gpus;
    (void)hipSetDevice(c->device);
    return c;
}

// Test / rehearsal form: k device contexts on ONE device, all on one stream (so the DAG solves of
// the k "devices" never run concurrently), the all-reduce a device-side sum in rank order.  Every
// sharded code path of the multi-device forms runs, with k > 1, on one card.
dpg_ctx* dpg_ctx_create_virtual(int32_t k, int32_t device) {
    if (k < 1 || k > kMaxVirtual) {
        fail(DPG_ERR_ARG, "dpg_ctx_create_virtual: %d virtual devices (1 .. %d)", k, kMaxVirtual);
        return nullptr;
    }
    dpg_ctx* c = dpg_ctx_create(device);
    if (!c) return nullptr;
    for (int r = 1; r < k; ++r) {
        dpg_ctx* q = dpg_ctx_create(device);
        if (!q) {
            dpg_ctx_destroy(c);
            return nullptr;
        }
        (void)hipStreamDestroy(q->stream);
        q->stream = c->stream;
        q->own_stream = false;
        q->rank = r;
        c->peers.push_back(q);
    }
    c->coll = kCollVirtual;
    c->world = k;
    return c;
}

int dpg_nccl_unique_id(void* id_out) {
    if (!id_out) return fail(DPG_ERR_ARG, "dpg_nccl_unique_id: NULL");
    static_assert(sizeof(ncclUniqueId) == DPG_NCCL_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(DPG_ERR_HIP, "ncclGetUniqueId failed: %s", ncclGetErrorString(r));
    memcpy(id_out, &id, sizeof(id));
    return DPG_OK;
}

// One process per GPU (torchrun): this process's device is global rank `rank` of `world`; the
// communicator comes from the id rank 0 made (dpg_nccl_unique_id), passed around by the caller.
dpg_ctx* dpg_ctx_create_rank(int32_t device, const void* nccl_id, int32_t rank, int32_t world) {
    if (!nccl_id || world < 1 || rank < 0 || rank >= world) {
        fail(DPG_ERR_ARG, "dpg_ctx_create_rank: rank %d of %d", rank, world);
        return nullptr;
    }
    dpg_ctx* c = dpg_ctx_create(device);
    if (!c) return nullptr;
    ncclUniqueId id;
    memcpy(&id, nccl_id, sizeof(id));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, world, id, rank);
    if (r != ncclSuccess) {
        dpg_ctx_destroy(c);
        fail(DPG_ERR_HIP, "ncclCommInitRank(rank %d of %d) failed: %s", rank, world, ncclGetErrorString(r));
        return nullptr;
    }
    c->comms.assign(1, comm);
    c->coll = kCollRccl;
    c->world = world;
    c->rank0 = rank;
    c->rank = rank;
    return c;
}

// One process per GPU over the caller's own collectives (blocking, host memory): a host that
// already runs a communicator (MPI, gloo), or ranks sharing one card (RCCL refuses a second rank
// on a device).  Every cross-process step of the rank form -- the cost all-reduce of the LPT plan,
// the results' all-gather, the packed system's all-reduce per Gauss-Newton iteration -- goes
// through `ops` instead of RCCL; the rest of the rank form is the same code.
dpg_ctx* dpg_ctx_create_rank_ops(int32_t device, const dpg_coll_ops* ops, int32_t rank, int32_t world) {
    if (!ops || !ops->allreduce_sum_f64 || !ops->allreduce_sum_f32 || !ops->allgather || world < 1 || rank < 0 ||
        rank >= world) {
        fail(DPG_ERR_ARG, "dpg_ctx_create_rank_ops: rank %d of %d (all three collectives are required)", rank, world);
        return nullptr;
    }
    dpg_ctx* c = dpg_ctx_create(device);
    if (!c) return nullptr;
    c->host_ops = *ops;
    c->coll = kCollHost;
    c->world = world;
    c->rank0 = rank;
    c->rank = rank;
    return c;
}

int32_t dpg_ctx_num_gpus(dpg_ctx* c) { return c ? n_dev(c) : -1; }
int dpg_ctx_is_multi(dpg_ctx* c) { return c && is_multi(c) ? 1 : 0; }
int32_t dpg_ctx_rank(dpg_ctx* c) { return c ? c->rank0 : -1; }

// ranks of the context's collective: ncclCommCount of its communicator (RCCL forms), k (virtual),
// 1 (single device)
int32_t dpg_ctx_num_ranks(dpg_ctx* c) {
    if (!c) return -1;
    if (c->coll == kCollRccl) {
        int n = -1;
        if (ncclCommCount(c->comms[0], &n) != ncclSuccess) return fail(DPG_ERR_HIP, "ncclCommCount failed");
        return n;
    }
    return c->world;
}

void dpg_solver_options_default(dpg_solver_options* o) {
    if (!o) return;
    const dpg_chol_opts d;
    memset(o, 0, sizeof(*o));
    o->order = d.order;
    o->fused = d.fused;
    o->solve_stage = d.solve_stage;
    o->solve_maxseg = d.solve_maxseg;
    o->solve_dinv = d.solve_dinv;
    o->merge_single = d.merge_single;
    o->max_supernode_cols = d.max_supernode_cols;
    o->relax_fraction = d.relax_fraction;
    o->solve_inv_cols = d.solve_inv_cols;
}

// per context (every device of a multi-device one): applies to the next graph set up on it
int dpg_ctx_set_solver_options(dpg_ctx* c, const dpg_solver_options* o) {
    if (!c || !o || o->order < DPG_ORDER_AUTO || o->order > DPG_ORDER_ND || o->max_supernode_cols < 1 || o->solve_inv_cols < 0 ||
        !(o->relax_fraction >= 0.0))
        return fail(DPG_ERR_ARG, "bad solver options");
    for (int k = 0; k < n_dev(c); ++k) {
        dpg_chol_opts& d = dev_ctx(c, k)->copts;
        d.order = o->order;
        d.fused = o->fused ? 1 : 0;
        d.solve_stage = o->solve_stage;
        d.solve_maxseg = o->solve_maxseg;
        d.solve_dinv = o->solve_dinv ? 1 : 0;
        d.merge_single = o->merge_single ? 1 : 0;
        d.max_supernode_cols = o->max_supernode_cols;
        d.relax_fraction = o->relax_fraction;
        d.solve_inv_cols = o->solve_inv_cols;
    }
    return DPG_OK;
}

const dpg_chol_opts* dpg_ctx_chol_opts(dpg_ctx* c) { return &c->copts; }

int dpg_ctx_set_icp_schedule(dpg_ctx* c, int32_t schedule) {
    if (!c || (schedule != DPG_ICP_SCHEDULE_CALLER && schedule != DPG_ICP_SCHEDULE_MEASURED))
        return fail(DPG_ERR_ARG, "bad ICP schedule");
    c->schedule = schedule;
    return DPG_OK;
}

void dpg_ctx_adopt(dpg_ctx* c, void* child, void (*destroy)(void*)) {
    if (c && child) c->children.emplace_back(child, destroy);
}
void dpg_ctx_release_child(dpg_ctx* c, void* child) {
    if (!c) return;
    for (size_t k = 0; k < c->children.size(); ++k)
        if (c->children[k].first == child) {
            c->children.erase(c->children.begin() + (std::ptrdiff_t)k);
            return;
        }
}

void dpg_ctx_destroy(dpg_ctx* c) {
    if (!c) return;
    while (!c->children.empty()) {   // each child's destroy releases itself from the list
        const auto ch = c->children.back();
        ch.second(ch.first);
        if (!c->children.empty() && c->children.back().first == ch.first) c->children.pop_back();
    }
    if (c->coll == kCollVirtual) (void)hipStreamSynchronize(c->stream);   // the peers' work is on it
    for (dpg_ctx* q : c->peers) dpg_ctx_destroy(q);
    c->peers.clear();
    for (ncclComm_t m : c->comms)
        if (m) (void)ncclCommDestroy(m);
    c->comms.clear();
    (void)hipSetDevice(c->device);
    (void)join_cov(c);
    (void)hipStreamSynchronize(c->stream);
    if (c->hc) {   // the collective thread: its queue is empty once the stream has drained
        {
            std::lock_guard<std::mutex> lk(c->hc->mu);
            c->hc->stop = true;
        }
        c->hc->cv.notify_all();
        if (c->hc->th.joinable()) c->hc->th.join();
        if (c->hc->buf) (void)hipHostFree(c->hc->buf);
        if (c->hc->flag) (void)hipHostFree(c->hc->flag);
        for (auto& e : c->hc->ev) if (e) (void)hipEventDestroy(e);
        c->hc.reset();
    }
    if (c->aux) (void)hipStreamDestroy(c->aux);
    c->full.release(); c->ds.release(); c->edges.release(); c->res.release(); c->hess.release();
    c->trace.release(); c->s_pts.release(); c->s_edge.release(); c->s_res.release(); c->s_hess.release();
    c->ds_off_dev.release(); c->tree_pts.release(); c->tree_idx.release(); c->full_off_dev.release();
    c->s_off.release(); c->s_tree_pts.release(); c->s_tree_idx.release();
    c->buckets.release(); c->s_buckets.release(); c->icp_scratch.release();
    c->shard_idx.release(); c->cost_dev.release();
    if (c->gn_ready) dpg_gn_dev_free(&c->gn);
    if (c->pipe_ctl) (void)hipFree(c->pipe_ctl);
    if (c->pipe_slot) (void)hipHostFree(c->pipe_slot);
    for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
    for (auto& e : c->map_ev) if (e) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    if (c == g_default_ctx) g_default_ctx = nullptr;
    delete c;
}

int dpg_ctx_set_stream(dpg_ctx* c, void* s) {
    if (!c) return fail(DPG_ERR_ARG, "ctx is NULL");
    if (join_cov(c)) return fail(DPG_ERR_HIP, "stream wait failed");
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->own_stream) (void)hipStreamDestroy(c->stream);
    c->stream = reinterpret_cast<hipStream_t>(s);
    c->own_stream = false;
    if (c->coll == kCollVirtual)   // the virtual devices keep sharing one stream
        for (dpg_ctx* q : c->peers) q->stream = c->stream;
    return DPG_OK;
}

int dpg_ctx_synchronize(dpg_ctx* c) {
    if (!c) return fail(DPG_ERR_ARG, "ctx is NULL");
    for (int k = 0; k < n_dev(c); ++k) {
        HIP_TRY(hipSetDevice(dev_ctx(c, k)->device));
        if (join_cov(dev_ctx(c, k))) return fail(DPG_ERR_HIP, "stream wait failed");
        HIP_TRY(hipStreamSynchronize(dev_ctx(c, k)->stream));
    }
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

// ------------------------------------------------------------------ ICP, batched
static int scans_upload_1(dpg_ctx* c, const float* pts, const int64_t* off, int64_t V, int32_t ratio);
static int scans_append_1(dpg_ctx* c, const float* pts, const int64_t* off, int64_t k, int32_t ratio);

// every device of a multi-GPU context holds every scan (5000 x 1000 points: 40 MB of downsampled
// clouds per device), so any edge can be aligned on any device
int dpg_scans_upload(dpg_ctx* c, const float* pts, const int64_t* off, int64_t V, int32_t ratio) {
    if (!c) return fail(DPG_ERR_ARG, "dpg_scans_upload: bad arguments");
    c->cost.clear();   // a new store: node ids name other scans
    for (int k = 0; k < n_dev(c); ++k) {
        const int rc = scans_upload_1(dev_ctx(c, k), pts, off, V, ratio);
        if (rc) return rc;
    }
    return hipSetDevice(c->device) == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

int dpg_scans_append(dpg_ctx* c, const float* pts, const int64_t* off, int64_t k, int32_t ratio) {
    if (!c) return fail(DPG_ERR_ARG, "dpg_scans_append: bad arguments");
    for (int d = 0; d < n_dev(c); ++d) {
        const int rc = scans_append_1(dev_ctx(c, d), pts, off, k, ratio);
        if (rc) return rc;
    }
    return hipSetDevice(c->device) == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

// R2 downsamplePointCloud of every node on the device (dpg_slam.cc:346-360, dpg_host.c
// dpg_downsample_cloud: every ratio-th point from the first, copied) -- one workgroup per node over
// the full clouds already uploaded, instead of a host pass over all of them
__global__ void downsample_kernel(const float2* __restrict__ full, const int64_t* __restrict__ full_off,
                                  const int64_t* __restrict__ ds_off, int32_t ratio, float2* __restrict__ ds) {
    const int64_t v = blockIdx.x;
    const int64_t f0 = full_off[v], d0 = ds_off[v], nd = ds_off[v + 1] - d0;
    for (int64_t k = threadIdx.x; k < nd; k += blockDim.x) ds[d0 + k] = full[f0 + k * ratio];
}

static int scans_upload_1(dpg_ctx* c, const float* pts, const int64_t* off, int64_t V, int32_t ratio) {
    if (!c || !pts || !off || V <= 0) return fail(DPG_ERR_ARG, "dpg_scans_upload: bad arguments");
    if (ratio < 1) ratio = 1;
    HIP_TRY(hipSetDevice(c->device));
    if (c->cov_pending) {   // the store may be re-allocated under a running covariance
        HIP_TRY(hipEventSynchronize(c->ev[2]));
        c->cov_pending = false;
    }
    const int64_t total = off[V];
    if (total >= ((int64_t)1 << 31)) return fail(DPG_ERR_SIZE, "too many points (%lld)", (long long)total);
    c->full_off.assign(off, off + V + 1);
    c->ds_off.assign((size_t)V + 1, 0);
    for (int64_t v = 0; v < V; ++v) {
        const int64_t n = off[v + 1] - off[v];
        if (n < 0) return fail(DPG_ERR_ARG, "node offsets must be non-decreasing");
        c->ds_off[(size_t)v + 1] = c->ds_off[(size_t)v] + (n + ratio - 1) / ratio;
    }
    const size_t n_ds = (size_t)(2 * std::max<int64_t>(c->ds_off[(size_t)V], 1));   // floats
    int64_t mx = 0;
    for (int64_t v = 0; v < V; ++v) mx = std::max(mx, c->ds_off[(size_t)v + 1] - c->ds_off[(size_t)v]);
    if (mx > 16384) return fail(DPG_ERR_SIZE, "a downsampled cloud has %lld points (max 16384)", (long long)mx);
    if (c->full.reserve((size_t)(2 * std::max<int64_t>(total, 1))) || c->ds.reserve(n_ds) ||
        c->ds_off_dev.reserve((size_t)V + 1) || c->full_off_dev.reserve((size_t)V + 1) || c->tree_pts.reserve(n_ds) ||
        c->tree_idx.reserve(n_ds / 2) || c->buckets.reserve((size_t)V * (size_t)(dpg_angle_buckets() + 1)))
        return fail(DPG_ERR_HIP, "out of device memory for scans");
    HIP_TRY(hipMemcpyAsync(c->full.p, pts, sizeof(float) * 2 * (size_t)total, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->full_off_dev.p, off, sizeof(int64_t) * ((size_t)V + 1), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->ds_off_dev.p, c->ds_off.data(), sizeof(int64_t) * ((size_t)V + 1), hipMemcpyHostToDevice,
                           c->stream));
    hipLaunchKernelGGL(downsample_kernel, dim3((unsigned)V), dim3(256), 0, c->stream, reinterpret_cast<const float2*>(c->full.p),
                       c->full_off_dev.p, c->ds_off_dev.p, ratio, reinterpret_cast<float2*>(c->ds.p));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->n_nodes = V;
    c->idx_valid = 0;
    c->ratio = ratio;
    c->max_ds = (int32_t)mx;
    return DPG_OK;
}

static int scans_append_1(dpg_ctx* c, const float* pts, const int64_t* off, int64_t k, int32_t ratio) {
    if (!c || !pts || !off || k <= 0) return fail(DPG_ERR_ARG, "dpg_scans_append: bad arguments");
    if (ratio < 1) ratio = 1;
    if (c->n_nodes == 0) return scans_upload_1(c, pts, off, k, ratio);
    if (c->cov_pending) {   // the store may be re-allocated under a running covariance
        HIP_TRY(hipSetDevice(c->device));
        HIP_TRY(hipEventSynchronize(c->ev[2]));
        c->cov_pending = false;
    }
    if (ratio != c->ratio) return fail(DPG_ERR_STATE, "scans were uploaded with downsample ratio %d", c->ratio);
    HIP_TRY(hipSetDevice(c->device));
    const int64_t V0 = c->n_nodes, V1 = V0 + k;
    const int64_t P0 = c->full_off[(size_t)V0], D0 = c->ds_off[(size_t)V0];
    const int64_t add = off[k] - off[0];
    if (P0 + add >= ((int64_t)1 << 31)) return fail(DPG_ERR_SIZE, "too many points");
    std::vector<int64_t> foff((size_t)k + 1), doff((size_t)k + 1);
    foff[0] = P0;
    doff[0] = D0;
    int64_t mx = c->max_ds;
    for (int64_t v = 0; v < k; ++v) {
        const int64_t n = off[v + 1] - off[v];
        if (n < 0) return fail(DPG_ERR_ARG, "node offsets must be non-decreasing");
        foff[(size_t)v + 1] = foff[(size_t)v] + n;
        doff[(size_t)v + 1] = doff[(size_t)v] + (n + ratio - 1) / ratio;
        mx = std::max(mx, (n + ratio - 1) / ratio);
    }
    if (mx > 16384) return fail(DPG_ERR_SIZE, "a downsampled cloud has %lld points (max 16384)", (long long)mx);
    const int64_t nds = doff[(size_t)k] - D0;
    std::vector<float> ds((size_t)(2 * std::max<int64_t>(nds, 1)));
    for (int64_t v = 0; v < k; ++v)
        dpg_downsample_cloud(pts + 2 * (off[v] - off[0]), off[v + 1] - off[v], ratio, ds.data() + 2 * (doff[(size_t)v] - D0));
    const size_t B = (size_t)(dpg_angle_buckets() + 1);
    if (c->full.grow((size_t)(2 * (P0 + add)), (size_t)(2 * P0), c->stream) ||
        c->ds.grow((size_t)(2 * (D0 + nds)), (size_t)(2 * D0), c->stream) ||
        c->ds_off_dev.grow((size_t)V1 + 1, (size_t)V0 + 1, c->stream) ||
        c->tree_pts.grow((size_t)(2 * (D0 + nds)), (size_t)(2 * D0), c->stream) ||
        c->tree_idx.grow((size_t)(D0 + nds), (size_t)D0, c->stream) ||
        c->buckets.grow((size_t)V1 * B, (size_t)V0 * B, c->stream))
        return fail(DPG_ERR_HIP, "out of device memory for scans");
    HIP_TRY(hipMemcpyAsync(c->full.p + 2 * P0, pts, sizeof(float) * 2 * (size_t)add, hipMemcpyHostToDevice, c->stream));
    if (nds > 0)
        HIP_TRY(hipMemcpyAsync(c->ds.p + 2 * D0, ds.data(), sizeof(float) * 2 * (size_t)nds, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->ds_off_dev.p + V0 + 1, doff.data() + 1, sizeof(int64_t) * (size_t)k, hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->full_off.insert(c->full_off.end(), foff.begin() + 1, foff.end());
    c->ds_off.insert(c->ds_off.end(), doff.begin() + 1, doff.end());
    c->n_nodes = V1;
    c->max_ds = (int32_t)mx;
    return DPG_OK;
}

// The scan store as host copies (the graph checkpoint, dpg_inc_save): node count, downsample
// ratio, and -- when the arrays are given -- the node offsets [n + 1] and the full clouds [off[n]][2]
int dpg_scans_export(dpg_ctx* c, int64_t* n_nodes, int32_t* ratio, int64_t* off, float* pts) {
    if (!c || !n_nodes || !ratio) return fail(DPG_ERR_ARG, "dpg_scans_export: bad arguments");
    *n_nodes = c->n_nodes;
    *ratio = c->ratio;
    if (c->n_nodes <= 0) return DPG_OK;
    if (off) std::copy(c->full_off.begin(), c->full_off.begin() + c->n_nodes + 1, off);
    if (pts) {
        HIP_TRY(hipSetDevice(c->device));
        const size_t total = (size_t)c->full_off[(size_t)c->n_nodes];
        if (total) HIP_TRY(hipMemcpyAsync(pts, c->full.p, sizeof(float) * 2 * total, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return DPG_OK;
}

// The neighbour index of every stored node (the incremental path builds it node by node as nodes
// arrive; a store restored from a checkpoint needs all of it before its next dpg_add_node)
int dpg_scans_index_all(dpg_ctx* c) {
    if (!c) return fail(DPG_ERR_ARG, "dpg_scans_index_all: ctx is NULL");
    if (c->n_nodes <= 0 || c->icp_variant != DPG_ICP_ANGULAR) return DPG_OK;   // the other variants index per batch
    HIP_TRY(hipSetDevice(c->device));
    const int rc = dpg_launch_angle_index(c->ds.p, c->ds_off_dev.p, c->n_nodes, c->max_ds, c->tree_pts.p, c->tree_idx.p,
                                          c->buckets.p, c->kernel_variant == 2, c->stream);
    if (rc) return fail(rc, "angle index build failed");
    c->idx_valid = c->n_nodes;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DPG_OK;
}

// the scan store back to its first V nodes (dpg_add_node_pairs' rollback); the device arrays keep
// their capacity, the entries past V are overwritten by the next append
static void scans_truncate(dpg_ctx* c, int64_t V) {
    if (!c) return;
    for (int k = 0; k < n_dev(c); ++k) {
        dpg_ctx* q = dev_ctx(c, k);
        if (V < 0 || V >= q->n_nodes) continue;
        q->full_off.resize((size_t)V + 1);
        q->ds_off.resize((size_t)V + 1);
        q->n_nodes = V;
        q->idx_valid = std::min(q->idx_valid, V);
    }
}

// The kernel's edge records of a batch in the caller's order (R3 guesses, dpg_slam.cc:364-378;
// pad[0] = the caller's index), the kernel scalars and the largest clouds.
static int build_batch(dpg_ctx* c, const int32_t* edges, int64_t ne, const float* poses, const dpg_icp_params* p,
                       std::vector<dpg_icp_edge>& out, dpg_icp_kparams& kp, int32_t& ms, int32_t& mt) {
    if (!c || (!edges && ne > 0) || ne < 0 || !poses || !p) return fail(DPG_ERR_ARG, "dpg_icp_batch_prepare: bad arguments");
    if (c->n_nodes <= 0) return fail(DPG_ERR_STATE, "no scans uploaded");
    if (p->downsample_icp_points_ratio != c->ratio && !(p->downsample_icp_points_ratio < 1 && c->ratio == 1))
        return fail(DPG_ERR_STATE, "scans were uploaded with downsample ratio %d", c->ratio);
    int rc = set_kparams(&kp, p);
    if (rc) return rc;
    out.resize((size_t)ne);
    ms = mt = 0;
    for (int64_t e = 0; e < ne; ++e) {
        const int32_t t = edges[2 * e], s = edges[2 * e + 1];  // node_1 = target, node_2 = source
        if (t < 0 || s < 0 || t >= c->n_nodes || s >= c->n_nodes)
            return fail(DPG_ERR_ARG, "edge %lld references a missing node", (long long)e);
        dpg_icp_edge& E = out[(size_t)e];
        memset(&E, 0, sizeof(E));
        E.src_node = s;
        E.tgt_node = t;
        E.src_ds_off = (int32_t)c->ds_off[(size_t)s];
        E.n_src_ds = (int32_t)(c->ds_off[(size_t)s + 1] - c->ds_off[(size_t)s]);
        E.tgt_ds_off = (int32_t)c->ds_off[(size_t)t];
        E.n_tgt_ds = (int32_t)(c->ds_off[(size_t)t + 1] - c->ds_off[(size_t)t]);
        E.src_full_off = (int32_t)c->full_off[(size_t)s];
        E.n_src_full = (int32_t)(c->full_off[(size_t)s + 1] - c->full_off[(size_t)s]);
        E.tgt_full_off = (int32_t)c->full_off[(size_t)t];
        E.n_tgt_full = (int32_t)(c->full_off[(size_t)t + 1] - c->full_off[(size_t)t]);
        dpg_icp_guess(poses + 3 * s, poses + 3 * t, E.guess);  // R3 (dpg_slam.cc:364-378)
        E.pad[0] = (int32_t)e;
        ms = std::max(ms, E.n_src_ds);
        mt = std::max(mt, E.n_tgt_ds);
    }
    return DPG_OK;
}

constexpr size_t kCostMemoryCap = (size_t)1 << 22;   // pairs remembered (~100 MB of hash map at most)
inline uint64_t pair_key(const dpg_icp_edge& E) { return (uint64_t)(uint32_t)E.tgt_node << 32 | (uint32_t)E.src_node; }
// what an alignment costs: its iterations, each a search over both clouds
inline float edge_cost(const dpg_icp_edge& E, int32_t iterations) {
    return (float)std::max(iterations, 1) * (float)(E.n_src_ds + E.n_tgt_ds);
}

// device q's share of the staged batch: h = its edges in dispatch order, pad[0] = the local result
// index; every device sizes its kernel by the batch-wide largest clouds (one kernel form)
static int stage_device(dpg_ctx* q, std::vector<dpg_icp_edge>& h, const dpg_icp_kparams& kp, int32_t ms, int32_t mt,
                        const std::vector<int64_t>* idx) {
    HIP_TRY(hipSetDevice(q->device));
    int rc = join_cov(q);
    if (rc) return fail(rc, "stream wait failed");
    const size_t ne = h.size();
    if (q->edges.reserve(std::max<size_t>(ne, 1)) || q->res.reserve(std::max<size_t>(ne, 1)) ||
        q->hess.reserve(9 * std::max<size_t>(ne, 1)))
        return fail(DPG_ERR_HIP, "out of device memory for %zu edges", ne);
    if (ne > 0)
        HIP_TRY(hipMemcpyAsync(q->edges.p, h.data(), sizeof(dpg_icp_edge) * ne, hipMemcpyHostToDevice, q->stream));
    if (idx) {   // multi-device: the caller's index of every local result (dpg_gn_take_icp_measurements)
        std::vector<int32_t> ix(idx->begin(), idx->end());
        if (q->shard_idx.reserve(std::max<size_t>(ix.size(), 1))) return fail(DPG_ERR_HIP, "out of device memory");
        if (!ix.empty())
            HIP_TRY(hipMemcpyAsync(q->shard_idx.p, ix.data(), sizeof(int32_t) * ix.size(), hipMemcpyHostToDevice, q->stream));
    }
    HIP_TRY(hipStreamSynchronize(q->stream));
    q->h_edges.swap(h);
    q->kp = kp;
    q->n_edges = (int64_t)ne;
    q->max_src = ms;
    q->max_tgt = mt;
    return DPG_OK;
}

// The staged batch over the ranks and each rank's dispatch order.  measured: every edge's cost is
// known from an earlier run -- longest-processing-time assignment (longest first to the least
// loaded rank; ties: lower index, lower rank) and longest-first dispatch on every rank, so the
// alignments that bound a launch start first.  Otherwise edge e goes to rank e mod world, in the
// caller's order (the caller's lists come grouped -- successive pairs, then loop closures nearest
// first -- so every rank gets the same mix of classes).  Results keep the caller's order either way.
static int plan_and_stage(dpg_ctx* c, bool measured) {
    const int64_t ne = (int64_t)c->batch.size();
    const int W = c->world;
    std::vector<float> w;
    if (measured) {
        w.resize((size_t)ne);
        for (int64_t e = 0; e < ne; ++e) w[(size_t)e] = c->cost.at(pair_key(c->batch[(size_t)e]));
    }
    c->batch_owner.assign((size_t)ne, 0);
    std::vector<int64_t> order((size_t)std::max<int64_t>(ne, 1)), counts((size_t)W, 0);
    int rc = dpg_shard_plan(measured ? w.data() : nullptr, ne, W, c->batch_owner.data(), order.data(), counts.data());
    if (rc) return rc;
    std::vector<int64_t> first((size_t)W + 1, 0);
    for (int r = 0; r < W; ++r) first[(size_t)r + 1] = first[(size_t)r] + counts[(size_t)r];
    const int32_t ms = c->max_src, mt = c->max_tgt;
    const dpg_icp_kparams kp = c->kp;
    c->shard.assign((size_t)n_dev(c), {});
    for (int k = 0; k < n_dev(c); ++k) {
        const int r = c->rank0 + k;
        const std::vector<int64_t> d(order.begin() + first[(size_t)r], order.begin() + first[(size_t)r + 1]);
        auto& sh = c->shard[(size_t)k];
        sh = d;
        std::sort(sh.begin(), sh.end());
        std::vector<dpg_icp_edge> h(d.size());
        for (size_t q = 0; q < d.size(); ++q) {
            h[q] = c->batch[(size_t)d[q]];
            h[q].pad[0] = (int32_t)(std::lower_bound(sh.begin(), sh.end(), d[q]) - sh.begin());
        }
        if ((rc = stage_device(dev_ctx(c, k), h, kp, ms, mt, is_multi(c) ? &sh : nullptr))) return rc;
    }
    c->batch_measured = measured;
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

static bool batch_costs_known(const dpg_ctx* c) {
    for (const dpg_icp_edge& E : c->batch)
        if (c->cost.find(pair_key(E)) == c->cost.end()) return false;
    return true;
}

// Stage an edge batch on every device.  The assignment uses measured costs when every edge of the
// batch has been aligned before (a sweep re-aligns the previous sweep's pairs from similar guesses).
int dpg_icp_batch_prepare(dpg_ctx* c, const int32_t* edges, int64_t ne, const float* poses, const dpg_icp_params* p) {
    if (!c) return fail(DPG_ERR_ARG, "dpg_icp_batch_prepare: bad arguments");
    int32_t ms = 0, mt = 0;
    dpg_icp_kparams kp;
    std::vector<dpg_icp_edge> all;
    int rc = build_batch(c, edges, ne, poses, p, all, kp, ms, mt);
    if (rc) return rc;
    c->batch.swap(all);
    c->kp = kp;
    c->max_src = ms;
    c->max_tgt = mt;
    c->batch_runs = 0;
    return plan_and_stage(c, c->schedule == DPG_ICP_SCHEDULE_MEASURED && ne > 0 && batch_costs_known(c));
}

static int batch_run_1(dpg_ctx* c, int32_t compute_cov, int32_t trace_iters) {
    if (!c) return fail(DPG_ERR_ARG, "ctx is NULL");
    HIP_TRY(hipSetDevice(c->device));
    dpg_icp_kparams kp = c->kp;
    int32_t* tr = nullptr;
    if (trace_iters > 0) {
        const size_t n = (size_t)c->n_edges * (size_t)trace_iters * (size_t)std::max(c->max_src, 1);
        if (c->trace.reserve(n)) return fail(DPG_ERR_HIP, "out of device memory for the trace");
        HIP_TRY(hipMemsetAsync(c->trace.p, 0xff, n * sizeof(int32_t), c->stream));
        kp.trace_iters = trace_iters;
        kp.trace_stride = std::max(c->max_src, 1);
        tr = c->trace.p;
    }
    c->trace_iters = trace_iters > 0 ? trace_iters : 0;
    c->have_cov = compute_cov != 0;
    // the angle index is a function of the stored scans alone: a batch run again on the same store
    // (the next sweep, the bench's steps) reuses it and builds only the nodes appended since
    return launch_batch(c, c->ds.p, c->full.p, c->ds_off_dev.p, c->n_nodes, c->max_ds, c->tree_pts.p, c->tree_idx.p,
                        c->buckets.p, c->edges.p, c->n_edges, kp, c->max_src, c->max_tgt, c->res.p,
                        compute_cov ? c->hess.p : nullptr, tr, true, std::min(c->idx_valid, c->n_nodes));
}

// ---- the rank form's cross-process steps (blocking; every rank makes them in the same order) ----
// in-place sum of host floats over the ranks
static int coll_allreduce_f32_host(dpg_ctx* c, float* w, size_t n) {
    if (c->coll == kCollHost) {
        if (c->host_ops.allreduce_sum_f32(c->host_ops.user, w, (int64_t)n))
            return fail(DPG_ERR_HIP, "the caller's float all-reduce failed");
        return DPG_OK;
    }
    HIP_TRY(hipSetDevice(c->device));
    if (c->cost_dev.reserve(n)) return fail(DPG_ERR_HIP, "out of device memory");
    HIP_TRY(hipMemcpyAsync(c->cost_dev.p, w, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
    const ncclResult_t nr = ncclAllReduce(c->cost_dev.p, c->cost_dev.p, n, ncclFloat, ncclSum, c->comms[0], c->stream);
    if (nr != ncclSuccess) return fail(DPG_ERR_HIP, "ncclAllReduce (costs) failed: %s", ncclGetErrorString(nr));
    HIP_TRY(hipMemcpyAsync(w, c->cost_dev.p, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DPG_OK;
}

// every rank's `slice_bytes` (the first mine_bytes of them from local_dev, this rank's records) into
// `all` on the host, rank order
static int coll_allgather_to_host(dpg_ctx* c, const void* local_dev, size_t mine_bytes, size_t slice_bytes,
                                  std::vector<char>& all) {
    const size_t W = (size_t)c->world;
    all.assign(slice_bytes * W, 0);
    HIP_TRY(hipSetDevice(c->device));
    if (c->coll == kCollHost) {
        std::vector<char> send(slice_bytes, 0);
        if (mine_bytes) HIP_TRY(hipMemcpyAsync(send.data(), local_dev, mine_bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->host_ops.allgather(c->host_ops.user, send.data(), all.data(), (int64_t)slice_bytes))
            return fail(DPG_ERR_HIP, "the caller's all-gather failed");
        return DPG_OK;
    }
    DevBuf<char> send, recv;
    int rc = DPG_OK;
    if (send.reserve(slice_bytes) || recv.reserve(slice_bytes * W)) rc = fail(DPG_ERR_HIP, "out of device memory for the gather");
    if (!rc && mine_bytes && hipMemcpyAsync(send.p, local_dev, mine_bytes, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
        rc = fail(DPG_ERR_HIP, "gather staging copy failed");
    if (!rc) {
        const ncclResult_t nr = ncclAllGather(send.p, recv.p, slice_bytes, ncclChar, c->comms[0], c->stream);
        if (nr != ncclSuccess) rc = fail(DPG_ERR_HIP, "ncclAllGather failed: %s", ncclGetErrorString(nr));
    }
    if (!rc && (hipMemcpyAsync(all.data(), recv.p, all.size(), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                hipStreamSynchronize(c->stream) != hipSuccess))
        rc = fail(DPG_ERR_HIP, "gather copy failed");
    send.release();
    recv.release();
    return rc;
}

// the measured cost of every edge of the last run into the cost memory (blocking); on the rank form
// the ranks' costs are summed into one vector (every edge has one owner, the others add 0), so every
// rank plans the next run from the same numbers
static int harvest_costs(dpg_ctx* c) {
    const int64_t ne = (int64_t)c->batch.size();
    std::vector<float> w((size_t)std::max<int64_t>(ne, 1), 0.f);
    std::vector<dpg_icp_result> r;
    for (int k = 0; k < (int)c->shard.size(); ++k) {
        dpg_ctx* q = dev_ctx(c, k);
        const auto& sh = c->shard[(size_t)k];
        if (sh.empty()) continue;
        r.resize(sh.size());
        HIP_TRY(hipSetDevice(q->device));
        if (join_cov(q)) return fail(DPG_ERR_HIP, "stream wait failed");
        HIP_TRY(hipMemcpyAsync(r.data(), q->res.p, sizeof(dpg_icp_result) * sh.size(), hipMemcpyDeviceToHost, q->stream));
        HIP_TRY(hipStreamSynchronize(q->stream));
        for (size_t j = 0; j < sh.size(); ++j) w[(size_t)sh[j]] = edge_cost(c->batch[(size_t)sh[j]], r[j].iterations);
    }
    int rc;
    if (is_rank_form(c) && ne > 0 && (rc = coll_allreduce_f32_host(c, w.data(), (size_t)ne))) return rc;
    for (int64_t e = 0; e < ne; ++e)
        if (w[(size_t)e] > 0.f) c->cost[pair_key(c->batch[(size_t)e])] = w[(size_t)e];
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

// Run the staged batch on every device (launches only: the devices run concurrently).  A batch
// run again after its first run (the bench's steps) is re-planned once from its measured costs.
int dpg_icp_batch_run(dpg_ctx* c, int32_t compute_cov, int32_t trace_iters) {
    if (!c) return fail(DPG_ERR_ARG, "ctx is NULL");
    if (trace_iters > 0 && is_multi(c)) return fail(DPG_ERR_STATE, "the correspondence trace is a single-device diagnostic");
    int rc;
    if (c->schedule == DPG_ICP_SCHEDULE_MEASURED && !c->batch_measured && c->batch_runs > 0 && trace_iters <= 0 &&
        !c->batch.empty()) {
        if (!batch_costs_known(c) && (rc = harvest_costs(c))) return rc;
        if (batch_costs_known(c) && (rc = plan_and_stage(c, true))) return rc;
    }
    for (int k = 0; k < n_dev(c); ++k)
        if ((rc = batch_run_1(dev_ctx(c, k), compute_cov, trace_iters))) return rc;
    c->have_cov = compute_cov != 0;
    ++c->batch_runs;
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

// the staged batch, building only the indexes of nodes [tree_from, n_nodes) (nodes appended since
// the last run: the others' indexes are still in place)
static int icp_batch_run_from(dpg_ctx* c, int64_t tree_from) {
    HIP_TRY(hipSetDevice(c->device));
    c->trace_iters = 0;
    c->have_cov = false;
    ++c->batch_runs;
    return launch_batch(c, c->ds.p, c->full.p, c->ds_off_dev.p, c->n_nodes, c->max_ds, c->tree_pts.p, c->tree_idx.p,
                        c->buckets.p, c->edges.p, c->n_edges, c->kp, c->max_src, c->max_tgt, c->res.p, nullptr,
                        nullptr, true, tree_from);
}

int dpg_ctx_set_icp_variant(dpg_ctx* c, int32_t variant) {
    if (!c || (variant != DPG_ICP_ANGULAR && variant != DPG_ICP_KDTREE && variant != DPG_ICP_GRID))
        return fail(DPG_ERR_ARG, "bad ICP variant");
    for (int k = 0; k < n_dev(c); ++k) {
        if (dev_ctx(c, k)->icp_variant != variant) dev_ctx(c, k)->idx_valid = 0;
        dev_ctx(c, k)->icp_variant = variant;
    }
    return DPG_OK;
}

int dpg_ctx_set_icp_defer_cap(dpg_ctx* c, int32_t cap) {
    if (!c || cap < 0) return fail(DPG_ERR_ARG, "bad defer cap");
    for (int k = 0; k < n_dev(c); ++k) dev_ctx(c, k)->defer_cap = cap;
    return DPG_OK;
}

int dpg_ctx_set_cov_workgroups(dpg_ctx* c, int32_t n) {
    if (!c || n < 0) return fail(DPG_ERR_ARG, "bad covariance workgroup count");
    for (int k = 0; k < n_dev(c); ++k) dev_ctx(c, k)->cov_wg = n;
    return DPG_OK;
}

int dpg_ctx_set_icp_kernel_variant(dpg_ctx* c, int32_t v) {
    if (!c || v < 0) return fail(DPG_ERR_ARG, "bad kernel variant");
    for (int k = 0; k < n_dev(c); ++k) {
        if ((dev_ctx(c, k)->kernel_variant == 2) != (v == 2)) dev_ctx(c, k)->idx_valid = 0;   // form 2: the bitonic builder
        dev_ctx(c, k)->kernel_variant = v;
    }
    return DPG_OK;
}

float dpg_kdtree_build_ms(dpg_ctx* c) {
    float ms = -1.f;
    if (!c || hipEventSynchronize(c->ev[0]) != hipSuccess) return -1.f;
    if (hipEventElapsedTime(&ms, c->ev[6], c->ev[0]) != hipSuccess) return -1.f;
    return ms;
}

// device q's results (+ covariance blocks) in local order, blocking
static int fetch_local(dpg_ctx* q, size_t n, dpg_icp_result* results, double* hess) {
    HIP_TRY(hipSetDevice(q->device));
    if (join_cov(q)) return fail(DPG_ERR_HIP, "stream wait failed");
    if (results && n > 0)
        HIP_TRY(hipMemcpyAsync(results, q->res.p, sizeof(dpg_icp_result) * n, hipMemcpyDeviceToHost, q->stream));
    if (hess && n > 0)
        HIP_TRY(hipMemcpyAsync(hess, q->hess.p, sizeof(double) * 9 * n, hipMemcpyDeviceToHost, q->stream));
    HIP_TRY(hipStreamSynchronize(q->stream));
    return DPG_OK;
}

// rank form: every rank's local results, gathered in equal-size slices (the largest share; each
// rank derives every other rank's share from the common plan), then put in the caller's order
static int fetch_allgather(dpg_ctx* c, void* out, size_t rec_bytes, const void* local_dev, std::vector<char>& all) {
    const int W = c->world;
    std::vector<size_t> cnt((size_t)W, 0);
    for (int32_t o : c->batch_owner) ++cnt[(size_t)o];
    const size_t slice = std::max<size_t>(*std::max_element(cnt.begin(), cnt.end()), 1);
    const size_t mine = c->shard.empty() ? 0 : c->shard[0].size();
    int rc = coll_allgather_to_host(c, local_dev, mine * rec_bytes, slice * rec_bytes, all);
    if (rc) return rc;
    return dpg_shard_reassemble(c->batch_owner.data(), (int64_t)c->batch_owner.size(), W, (int64_t)slice,
                                (int64_t)rec_bytes, all.data(), out);
}

// Results of the staged batch in the caller's order (and the covariance blocks).  On the rank form
// this is a collective: every rank receives every edge's result.  learn: the alignment costs go into
// the context's cost memory (the next plan of the same pairs); the per-node path, whose pairs are
// never re-planned, does not learn (the memory grew by every node's pairs).
static int batch_fetch(dpg_ctx* c, dpg_icp_result* results, double* hess, bool learn);
int dpg_icp_batch_fetch(dpg_ctx* c, dpg_icp_result* results, double* hess, int64_t cap) {
    if (!c) return fail(DPG_ERR_ARG, "ctx is NULL");
    if ((results || hess) && cap < (int64_t)c->batch.size())
        return fail(DPG_ERR_SIZE, "result buffers hold fewer records than the staged batch (dpg_icp_batch_size)");
    return batch_fetch(c, results, hess, true);
}

static int batch_fetch(dpg_ctx* c, dpg_icp_result* results, double* hess, bool learn) {
    if (!c) return fail(DPG_ERR_ARG, "ctx is NULL");
    if (hess && !c->have_cov && !c->batch.empty()) return fail(DPG_ERR_STATE, "last batch ran without compute_cov");
    const int64_t ne = (int64_t)c->batch.size();
    std::vector<dpg_icp_result> own;
    dpg_icp_result* R = results;
    if (!R) {   // the costs are learnt from every fetch
        own.resize((size_t)std::max<int64_t>(ne, 1));
        R = own.data();
    }
    int rc;
    if (is_rank_form(c)) {
        std::vector<char> buf;
        if (join_cov(c)) return fail(DPG_ERR_HIP, "stream wait failed");
        if ((rc = fetch_allgather(c, R, sizeof(dpg_icp_result), c->res.p, buf))) return rc;
        if (hess && (rc = fetch_allgather(c, hess, 9 * sizeof(double), c->hess.p, buf))) return rc;
    } else {
        std::vector<dpg_icp_result> r;
        std::vector<double> h;
        for (int k = 0; k < (int)c->shard.size(); ++k) {
            const auto& ids = c->shard[(size_t)k];
            r.resize(std::max<size_t>(ids.size(), 1));
            if (hess) h.resize(9 * std::max<size_t>(ids.size(), 1));
            if ((rc = fetch_local(dev_ctx(c, k), ids.size(), r.data(), hess ? h.data() : nullptr))) return rc;
            for (size_t j = 0; j < ids.size(); ++j) {
                R[ids[j]] = r[j];
                if (hess) memcpy(hess + 9 * ids[j], h.data() + 9 * j, 9 * sizeof(double));
            }
        }
    }
    if (learn) {
        if (c->cost.size() + (size_t)ne > kCostMemoryCap) c->cost.clear();   // bounded: a long session's old pairs go
        for (int64_t e = 0; e < ne; ++e) c->cost[pair_key(c->batch[(size_t)e])] = edge_cost(c->batch[(size_t)e], R[e].iterations);
    }
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

// edges of the staged batch (dpg_icp_batch_prepare's, or the one a sweep / dpg_add_node staged):
// what dpg_icp_batch_fetch writes
int64_t dpg_icp_batch_size(dpg_ctx* c) { return c ? (int64_t)c->batch.size() : fail(DPG_ERR_ARG, "ctx is NULL"); }

int dpg_icp_batch_fetch_trace(dpg_ctx* c, int32_t* trace, int64_t trace_cap, int64_t* max_src_out) {
    if (!c) return fail(DPG_ERR_ARG, "ctx is NULL");
    if (is_multi(c)) return fail(DPG_ERR_STATE, "the correspondence trace is a single-device diagnostic");
    if (max_src_out) *max_src_out = std::max(c->max_src, 1);
    if (!trace) return DPG_OK;
    if (c->trace_iters <= 0) return fail(DPG_ERR_STATE, "last batch ran without a trace");
    const size_t n = (size_t)c->n_edges * (size_t)c->trace_iters * (size_t)std::max(c->max_src, 1);
    if (trace_cap < 0 || (size_t)trace_cap < n) return fail(DPG_ERR_SIZE, "trace buffer smaller than E * trace_iters * max_src");
    HIP_TRY(hipMemcpyAsync(trace, c->trace.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DPG_OK;
}

// event pair (a, b) of the last batch: the slowest local device
static float batch_ms(dpg_ctx* c, int a, int b) {
    float worst = -1.f;
    for (int k = 0; k < (c ? n_dev(c) : 0); ++k) {
        dpg_ctx* q = dev_ctx(c, k);
        float ms = -1.f;
        if (hipSetDevice(q->device) != hipSuccess || hipEventSynchronize(q->ev[b]) != hipSuccess ||
            hipEventElapsedTime(&ms, q->ev[a], q->ev[b]) != hipSuccess)
            return -1.f;
        worst = std::max(worst, ms);
    }
    if (c) (void)hipSetDevice(c->device);
    return worst;
}

float dpg_icp_batch_kernel_ms(dpg_ctx* c) { return batch_ms(c, 0, 1); }

float dpg_cov_batch_kernel_ms(dpg_ctx* c) { return batch_ms(c, 1, 2); }

int32_t dpg_cov_batch_overlapped(dpg_ctx* c) { return c && c->cov_on_aux ? 1 : 0; }

// the last launch on device q, from its own records: sum over its edges of iterations x (8N + 8M + 8N)
static double batch_bytes_1(dpg_ctx* c) {
    if (!c || c->n_edges <= 0) return 0.0;
    std::vector<dpg_icp_result> r((size_t)c->n_edges);
    if (hipMemcpy(r.data(), c->res.p, sizeof(dpg_icp_result) * r.size(), hipMemcpyDeviceToHost) != hipSuccess) return -1.0;
    double bytes = 0.0;
    for (int64_t e = 0; e < c->n_edges; ++e) {
        const dpg_icp_edge& E = c->h_edges[(size_t)e];   // dispatch order; its result is r[E.pad[0]]
        // correspondence kernel per edge-iteration: 8N (source xy) + 8M (target xy) + 8N (idx + d^2)
        bytes += (double)r[(size_t)E.pad[0]].iterations * (16.0 * E.n_src_ds + 8.0 * E.n_tgt_ds);
    }
    return bytes;
}

// the local devices' launches (the rank form: this rank's share)
double dpg_icp_batch_algorithmic_bytes(dpg_ctx* c) {
    if (!c) return 0.0;
    double b = 0.0;
    for (int k = 0; k < n_dev(c); ++k) {
        (void)hipSetDevice(dev_ctx(c, k)->device);
        const double x = batch_bytes_1(dev_ctx(c, k));
        if (x < 0) return x;
        b += x;
    }
    (void)hipSetDevice(c->device);
    return b;
}

// ------------------------------------------------------------------ single alignment / covariance
int dpg_run_icp(dpg_ctx* c, const float* src, int64_t ns, const float* tgt, int64_t nt, const float pose_src[3],
                const float pose_tgt[3], const dpg_icp_params* p, dpg_icp_result* result, double cov_out[9],
                double hess_out[9]) {
    if (!c || !src || !tgt || ns < 0 || nt < 0 || !pose_src || !pose_tgt || !p || !result)
        return fail(DPG_ERR_ARG, "dpg_run_icp: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    dpg_icp_kparams kp;
    int rc = set_kparams(&kp, p);
    if (rc) return rc;
    const int32_t ratio = p->downsample_icp_points_ratio > 0 ? p->downsample_icp_points_ratio : 1;
    const int64_t nsd = (ns + ratio - 1) / ratio, ntd = (nt + ratio - 1) / ratio;
    // layout: [src full | tgt full | src ds | tgt ds]
    std::vector<float> buf((size_t)(2 * (ns + nt + nsd + ntd) + 2));
    memcpy(buf.data(), src, sizeof(float) * 2 * (size_t)ns);
    memcpy(buf.data() + 2 * ns, tgt, sizeof(float) * 2 * (size_t)nt);
    dpg_downsample_cloud(src, ns, ratio, buf.data() + 2 * (ns + nt));
    dpg_downsample_cloud(tgt, nt, ratio, buf.data() + 2 * (ns + nt + nsd));
    dpg_icp_edge E;
    memset(&E, 0, sizeof(E));
    E.src_node = 0;
    E.tgt_node = 1;
    E.src_full_off = 0; E.n_src_full = (int32_t)ns;
    E.tgt_full_off = (int32_t)ns; E.n_tgt_full = (int32_t)nt;
    // downsampled clouds (and their trees) are addressed relative to the ds part of the buffer
    E.src_ds_off = 0; E.n_src_ds = (int32_t)nsd;
    E.tgt_ds_off = (int32_t)nsd; E.n_tgt_ds = (int32_t)ntd;
    dpg_icp_guess(pose_src, pose_tgt, E.guess);
    const int64_t offs[3] = {0, nsd, nsd + ntd};
    if (c->s_pts.reserve(buf.size()) || c->s_edge.reserve(1) || c->s_res.reserve(1) || c->s_hess.reserve(9) ||
        c->s_off.reserve(3) || c->s_tree_pts.reserve((size_t)(2 * (nsd + ntd) + 2)) ||
        c->s_tree_idx.reserve((size_t)(nsd + ntd + 1)) || c->s_buckets.reserve((size_t)(2 * (dpg_angle_buckets() + 1))))
        return fail(DPG_ERR_HIP, "out of device memory");
    HIP_TRY(hipMemcpyAsync(c->s_pts.p, buf.data(), sizeof(float) * buf.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->s_edge.p, &E, sizeof(E), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->s_off.p, offs, sizeof(offs), hipMemcpyHostToDevice, c->stream));
    rc = launch_batch(c, c->s_pts.p + 2 * (ns + nt), c->s_pts.p, c->s_off.p, 2, (int32_t)std::max(nsd, ntd),
                      c->s_tree_pts.p, c->s_tree_idx.p, c->s_buckets.p, c->s_edge.p, 1, kp, (int32_t)nsd, (int32_t)ntd, c->s_res.p,
                      hess_out ? c->s_hess.p : nullptr, nullptr, false);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(result, c->s_res.p, sizeof(dpg_icp_result), hipMemcpyDeviceToHost, c->stream));
    if (hess_out) HIP_TRY(hipMemcpyAsync(hess_out, c->s_hess.p, 9 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (cov_out) const_cov(p, cov_out);
    return DPG_OK;
}

int icp_cov_calculate(dpg_ctx* c, const float* data, int64_t nd, const float* model, int64_t nm, const float T[16],
                      float vx, float vy, float vth, double cov_out[9], double hess_out[9]) {
    if (!cov_out || !T) return fail(DPG_ERR_ARG, "icp_cov_calculate: bad arguments");
    // :572-575 -- ICP_COV.resize(3,3) << laser_x_variance, 0, 0, 0, laser_y_variance, ...
    memset(cov_out, 0, 9 * sizeof(double));
    cov_out[0] = (double)vx;
    cov_out[4] = (double)vy;
    cov_out[8] = (double)vth;
    if (!hess_out) return DPG_OK;
    if (!data || !model || nd < 0 || nm < 0) return fail(DPG_ERR_ARG, "icp_cov_calculate: bad clouds");
    if (!c) {
        if (!g_default_ctx) g_default_ctx = dpg_ctx_create(0);
        c = g_default_ctx;
        if (!c) return DPG_ERR_HIP;
    }
    HIP_TRY(hipSetDevice(c->device));
    std::vector<float> buf((size_t)(2 * (nd + nm) + 2));
    memcpy(buf.data(), data, sizeof(float) * 2 * (size_t)nd);
    memcpy(buf.data() + 2 * nd, model, sizeof(float) * 2 * (size_t)nm);
    dpg_icp_edge E;
    memset(&E, 0, sizeof(E));
    E.src_full_off = 0; E.n_src_full = (int32_t)nd;
    E.tgt_full_off = (int32_t)nd; E.n_tgt_full = (int32_t)nm;
    dpg_icp_result R;
    memset(&R, 0, sizeof(R));
    R.T[0] = T[0]; R.T[1] = T[1]; R.T[2] = T[3];    // row-major 4x4 -> rows (T00 T01 T03 / T10 T11 T13)
    R.T[3] = T[4]; R.T[4] = T[5]; R.T[5] = T[7];
    if (c->s_pts.reserve(buf.size()) || c->s_edge.reserve(1) || c->s_res.reserve(1) || c->s_hess.reserve(9))
        return fail(DPG_ERR_HIP, "out of device memory");
    HIP_TRY(hipMemcpyAsync(c->s_pts.p, buf.data(), sizeof(float) * buf.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->s_edge.p, &E, sizeof(E), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->s_res.p, &R, sizeof(R), hipMemcpyHostToDevice, c->stream));
    int rc = dpg_launch_cov(c->s_pts.p, c->s_edge.p, 1, c->s_res.p, c->s_hess.p, 0, c->stream);
    if (rc) return fail(rc, "covariance kernel launch failed");
    HIP_TRY(hipMemcpyAsync(hess_out, c->s_hess.p, 9 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DPG_OK;
}

// d2J_dX2 and d2J_dZdX cov_z d2J_dZdX^T from the 16 sums of cov6_kernel (+ the pair counts), then
// cov6 = 0.01 inv(H) M inv(H) (Gauss-Jordan with partial pivoting, fp64, fixed order)
static int cov6_from_sums(const double* sm, int64_t nh, int64_t nb, double cov6[36]) {
    double H[36] = {0}, M[36] = {0};
    enum { X = 0, Y = 1, Z = 2, A = 3, B = 4, C = 5 };
    auto sym = [](double* m, int i, int j, double v) { m[6 * i + j] = v; m[6 * j + i] = v; };
    sym(H, X, X, 2.0 * (double)nh); sym(H, Y, Y, 2.0 * (double)nh); sym(H, Z, Z, 2.0 * (double)nh);
    sym(H, X, A, sm[0]); sym(H, Y, A, sm[1]); sym(H, A, A, sm[2]); sym(H, Z, B, sm[3]); sym(H, Z, C, sm[4]);
    sym(H, B, B, sm[5]); sym(H, B, C, sm[6]); sym(H, C, C, sm[7]);
    sym(M, X, X, 8.0 * (double)nb); sym(M, Y, Y, 8.0 * (double)nb); sym(M, Z, Z, 8.0 * (double)nb);
    sym(M, X, A, sm[8]); sym(M, Y, A, sm[9]); sym(M, A, A, sm[10]); sym(M, Z, B, sm[11]); sym(M, Z, C, sm[12]);
    sym(M, B, B, sm[13]); sym(M, B, C, sm[14]); sym(M, C, C, sm[15]);
    double I[36] = {0};
    for (int i = 0; i < 6; ++i) I[7 * i] = 1.0;
    for (int c = 0; c < 6; ++c) {
        int p = c;
        for (int r = c + 1; r < 6; ++r)
            if (fabs(H[6 * r + c]) > fabs(H[6 * p + c])) p = r;
        if (!(fabs(H[6 * p + c]) > 0.0)) return DPG_ERR_NUMERIC;
        if (p != c)
            for (int k = 0; k < 6; ++k) { std::swap(H[6 * p + k], H[6 * c + k]); std::swap(I[6 * p + k], I[6 * c + k]); }
        const double d = H[6 * c + c];
        for (int k = 0; k < 6; ++k) { H[6 * c + k] /= d; I[6 * c + k] /= d; }
        for (int r = 0; r < 6; ++r) {
            if (r == c) continue;
            const double f = H[6 * r + c];
            if (f == 0.0) continue;
            for (int k = 0; k < 6; ++k) { H[6 * r + k] -= f * H[6 * c + k]; I[6 * r + k] -= f * I[6 * c + k]; }
        }
    }
    double T1[36];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 6; ++k) acc += I[6 * i + k] * M[6 * k + j];
            T1[6 * i + j] = acc;
        }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 6; ++k) acc += T1[6 * i + k] * I[6 * k + j];
            cov6[6 * i + j] = 0.01 * acc;
        }
    return DPG_OK;
}

int icp_cov_sandwich(dpg_ctx* c, const float* data, int64_t nd, const float* model, int64_t nm, const float T[16],
                     double cov6_out[36], double cov3_out[9]) {
    if (!T || !data || !model || nd < 1 || nm < 1 || nd > INT32_MAX / 4 || nm > INT32_MAX / 4)
        return fail(DPG_ERR_ARG, "icp_cov_sandwich: bad arguments");
    // the closed forms hold at the planar operating point z = pitch = roll = 0 (the reference reads
    // z, roll, pitch from T's third row, cov_func_point_to_point.h:26-31): a non-planar T is refused
    // rather than silently evaluated at the wrong point
    if (T[2] != 0.f || T[6] != 0.f || T[8] != 0.f || T[9] != 0.f || T[10] != 1.f || T[11] != 0.f)
        return fail(DPG_ERR_ARG, "icp_cov_sandwich: T is not planar (needs T20 = T21 = T02 = T12 = T23 = 0, T22 = 1)");
    if (!c) {
        if (!g_default_ctx) g_default_ctx = dpg_ctx_create(0);
        c = g_default_ctx;
        if (!c) return DPG_ERR_HIP;
    }
    HIP_TRY(hipSetDevice(c->device));
    std::vector<float> buf((size_t)(2 * (nd + nm)) + 8);
    memcpy(buf.data(), data, sizeof(float) * 2 * (size_t)nd);
    memcpy(buf.data() + 2 * nd, model, sizeof(float) * 2 * (size_t)nm);
    float* T6 = buf.data() + 2 * (nd + nm);   // rows (T00 T01 T03 / T10 T11 T13), as the ICP result keeps them
    T6[0] = T[0]; T6[1] = T[1]; T6[2] = T[3]; T6[3] = T[4]; T6[4] = T[5]; T6[5] = T[7];
    if (c->s_pts.reserve(buf.size()) || c->s_hess.reserve(16)) return fail(DPG_ERR_HIP, "out of device memory");
    HIP_TRY(hipMemcpyAsync(c->s_pts.p, buf.data(), sizeof(float) * buf.size(), hipMemcpyHostToDevice, c->stream));
    int rc = dpg_launch_cov6(c->s_pts.p, (int32_t)nd, (int32_t)nm, c->s_pts.p + 2 * (nd + nm), c->s_hess.p, c->stream);
    if (rc) return fail(rc, "covariance kernel launch failed");
    double sm[16];
    HIP_TRY(hipMemcpyAsync(sm, c->s_hess.p, sizeof(sm), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const int64_t nh = std::min(nd, nm), nb = std::min<int64_t>(nh, 200);
    double cov6[36];
    if ((rc = cov6_from_sums(sm, nh, nb, cov6))) return fail(rc, "icp_cov_sandwich: d2J_dX2 is singular");
    if (cov6_out) memcpy(cov6_out, cov6, sizeof(cov6));
    if (cov3_out) {
        const int ix[3] = {0, 1, 3};
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) cov3_out[3 * i + j] = cov6[6 * ix[i] + ix[j]];
    }
    return DPG_OK;
}

// ------------------------------------------------------------------ pose graph
static int gn_setup_1(dpg_ctx* c, int64_t V, const dpg_factor* F, int64_t nf, int64_t b, int64_t e,
                      const dpg_gn_params* gp) {
    HIP_TRY(hipSetDevice(c->device));
    // the new graph's host work overlaps what still runs on the stream (a batch's ICP); the
    // stream is drained before the device allocations, and the previous graph freed after them
    dpg_gn_dev ng;
    int rc = dpg_gn_dev_alloc(&ng, V, F, nf, b, e, &c->copts, c->stream);
    if (rc) return fail(rc, "pose-graph setup failed (invalid factor or out of memory)");
    if (c->gn_ready) dpg_gn_dev_free(&c->gn);
    c->gn = ng;
    c->gn_ready = true;
    if (gp) c->gp = *gp;
    else dpg_gn_params_default(&c->gp);
    return DPG_OK;
}

// Multi-device forms: every local device holds the whole factor list (the sparsity pattern is
// global) and linearizes the factors f with f mod world == its rank; dpg_gn_take_icp_measurements
// then hands each ICP slot to the device that aligned the edge.
int dpg_gn_setup(dpg_ctx* c, int64_t V, const dpg_factor* F, int64_t nf, int64_t b, int64_t e,
                 const dpg_gn_params* gp) {
    if (!c || !F || V <= 0 || nf < 0) return fail(DPG_ERR_ARG, "dpg_gn_setup: bad arguments");
    if (!is_multi(c)) return gn_setup_1(c, V, F, nf, b, e, gp);
    if (b != 0 || e != nf) return fail(DPG_ERR_ARG, "dpg_gn_setup: a multi-device context shards the factors itself (0, n_factors)");
    for (int k = 0; k < n_dev(c); ++k) {
        dpg_ctx* q = dev_ctx(c, k);
        int rc = gn_setup_1(q, V, F, nf, 0, nf, gp);
        if (!rc && (rc = dpg_gn_dev_set_ownership(&q->gn, c->world, q->rank, q->stream)))
            rc = fail(rc, "pose-graph ownership setup failed");
        if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

int dpg_gn_take_icp_measurements(dpg_ctx* c, int64_t first, int64_t count, int64_t n_always,
                                 const dpg_icp_params* p) {
    if (!c || !c->gn_ready || !p) return fail(DPG_ERR_STATE, "graph not set up");
    const double ix = 1.0 / (double)p->laser_x_variance, iy = 1.0 / (double)p->laser_y_variance,
                 ith = 1.0 / (double)p->laser_theta_variance;
    if (!is_multi(c)) {
        if (count > c->n_edges) return fail(DPG_ERR_ARG, "only %lld ICP results available", (long long)c->n_edges);
        int rc = dpg_gn_dev_icp_to_factors(&c->gn, c->res.p, first, count, n_always, ix, iy, ith, c->stream);
        return rc ? fail(rc, "dpg_gn_take_icp_measurements failed") : DPG_OK;
    }
    // every slot of the batch: the aligning device's result, on that device only
    if (count != (int64_t)c->batch.size())
        return fail(DPG_ERR_ARG, "a multi-device context takes the whole batch (%lld results), not %lld",
                    (long long)c->batch.size(), (long long)count);
    for (int k = 0; k < n_dev(c); ++k) {
        dpg_ctx* q = dev_ctx(c, k);
        HIP_TRY(hipSetDevice(q->device));
        if (!q->gn_ready || !q->gn.mine) return fail(DPG_ERR_STATE, "graph not set up on device %d", k);
        const int64_t nl = (int64_t)c->shard[(size_t)k].size();
        const int rc = dpg_gn_dev_icp_to_factors_scatter(&q->gn, q->res.p, q->shard_idx.p, nl, first, count, n_always,
                                                         ix, iy, ith, q->stream);
        if (rc) return fail(rc, "dpg_gn_take_icp_measurements failed");
    }
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

int64_t dpg_gn_hb_size(dpg_ctx* c) { return (c && c->gn_ready) ? dpg_gn_dev_hb_size(&c->gn) : -1; }

int dpg_gn_setup_profile(dpg_ctx* c, double out[5]) {
    if (!c || !c->gn_ready || !out) return fail(DPG_ERR_STATE, "graph not set up");
    for (int k = 0; k < 5; ++k) out[k] = c->gn.setup_ms[k];
    return DPG_OK;
}

static int gn_set_poses_1(dpg_ctx* c, const double* poses) {
    if (!c->gn_ready) return fail(DPG_ERR_STATE, "graph not set up");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(c->gn.poses, poses, sizeof(double) * 3 * (size_t)c->gn.n_nodes, hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->gn.have_factor = 0;            // a new linearization point: the next solve refactors
    c->gn.last_delta_inf = 1e300;
    c->gn.prev_delta_inf = 1e300;
    c->gn.last_was_chord = 0;
    c->gn.n_factorizations = 0;
    return DPG_OK;
}

int dpg_gn_set_poses(dpg_ctx* c, const double* poses) {
    if (!c || !c->gn_ready || !poses) return fail(DPG_ERR_STATE, "graph not set up");
    for (int k = 0; k < n_dev(c); ++k) {
        const int rc = gn_set_poses_1(dev_ctx(c, k), poses);
        if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

int dpg_gn_get_poses(dpg_ctx* c, double* poses) {
    if (!c || !c->gn_ready || !poses) return fail(DPG_ERR_STATE, "graph not set up");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(poses, c->gn.poses, sizeof(double) * 3 * (size_t)c->gn.n_nodes, hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DPG_OK;
}

// the per-iteration step API: one device, the caller's collective between its calls
#define DPG_STEP_API_1(c)                                                                                        \
    do {                                                                                                         \
        if (!(c) || !(c)->gn_ready) return fail(DPG_ERR_STATE, "graph not set up");                             \
        if (is_multi(c)) return fail(DPG_ERR_STATE, "the step API is per device: a multi-device context runs "   \
                                                    "dpg_gn_run / dpg_optimize_graph / dpg_reoptimize");         \
    } while (0)

int dpg_gn_assemble(dpg_ctx* c, double* hb_dev) {
    DPG_STEP_API_1(c);
    if (!hb_dev) hb_dev = c->gn.hb_own;
    HIP_TRY(hipEventRecord(c->ev[3], c->stream));
    int rc = dpg_gn_dev_assemble(&c->gn, hb_dev, c->stream);
    if (rc) return fail(rc, "assembly launch failed");
    HIP_TRY(hipEventRecord(c->ev[4], c->stream));
    return DPG_OK;
}

int dpg_gn_solve_retract(dpg_ctx* c, const double* hb_dev, double* delta_inf, double* error, int32_t* pcg_iters) {
    DPG_STEP_API_1(c);
    if (!hb_dev) hb_dev = c->gn.hb_own;
    int rc = dpg_gn_dev_solve(&c->gn, hb_dev, &c->gp, c->stream, delta_inf, error, pcg_iters);
    if (rc) return fail(rc, "PCG solve failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipEventRecord(c->ev[5], c->stream));
    float a = 0.f, s = 0.f;
    if (hipEventSynchronize(c->ev[5]) == hipSuccess) {
        (void)hipEventElapsedTime(&a, c->ev[3], c->ev[4]);
        (void)hipEventElapsedTime(&s, c->ev[4], c->ev[5]);
    }
    c->asm_ms = a;
    c->solve_ms = s;
    return DPG_OK;
}

// enqueue solve + retract on one device (no multi check: the multi-device host loop uses it per device)
static int solve_retract_async_1(dpg_ctx* c, const double* hb_dev) {
    if (!hb_dev) hb_dev = c->gn.hb_own;
    HIP_TRY(hipEventRecord(c->ev[4], c->stream));
    int rc = dpg_gn_dev_solve_async(&c->gn, hb_dev, &c->gp, c->stream);
    if (rc) return fail(rc, "solve launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipEventRecord(c->ev[5], c->stream));
    return DPG_OK;
}

int dpg_gn_solve_retract_async(dpg_ctx* c, const double* hb_dev) {
    DPG_STEP_API_1(c);
    return solve_retract_async_1(c, hb_dev);
}

int32_t dpg_gn_factorizations(dpg_ctx* c) { return (c && c->gn_ready) ? c->gn.n_factorizations : -1; }

static int fetch_1(dpg_ctx* c, const double* hb_dev, double out[3]) {
    if (!hb_dev) hb_dev = c->gn.hb_own;
    int rc = dpg_gn_dev_fetch(&c->gn, hb_dev, c->stream, out);
    if (rc) return fail(rc, "fetch failed");
    float s = 0.f;
    if (hipEventElapsedTime(&s, c->ev[4], c->ev[5]) == hipSuccess) c->solve_ms = s;
    return DPG_OK;
}

int dpg_gn_fetch(dpg_ctx* c, const double* hb_dev, double out[3]) {
    DPG_STEP_API_1(c);
    if (!out) return fail(DPG_ERR_ARG, "dpg_gn_fetch: out is NULL");
    return fetch_1(c, hb_dev, out);
}

float dpg_gn_last_assemble_ms(dpg_ctx* c) { return c ? c->asm_ms : -1.f; }
float dpg_gn_last_solve_ms(dpg_ctx* c) { return c ? c->solve_ms : -1.f; }

static int read_error(dpg_ctx* c, double* err) {
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(err, c->gn.hb_own + 9 * c->gn.nnzb_upper + 3 * c->gn.n_nodes, sizeof(double),
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DPG_OK;
}

static int check_conv(const dpg_gn_params* gp, double cur, double nw) {
    if (nw <= 0.0) return 1;
    const double abs_dec = cur - nw;
    const double rel_dec = abs_dec / cur;
    return (gp->relative_error_tol != 0.0 && rel_dec <= gp->relative_error_tol) || (abs_dec <= gp->absolute_error_tol);
}

// The multi-device forms' all-reduce: every local device's hb_part summed into every hb_own --
// ONE ncclAllReduce(sum, fp64) per device on its own stream (grouped: one thread drives them), or
// the virtual devices' rank-order sum.  Out of place, so an iteration that a gate turned into
// no-ops sums the same partial buffers again and leaves hb_own as it was.
static int coll_sum_hb(dpg_ctx* c) {
    const size_t count = (size_t)dpg_gn_dev_hb_size(&c->gn);
    if (c->coll == kCollVirtual) {
        const double* parts[kMaxVirtual];
        double* outs[kMaxVirtual];
        for (int k = 0; k < n_dev(c); ++k) {
            parts[k] = dev_ctx(c, k)->gn.hb_part;
            outs[k] = dev_ctx(c, k)->gn.hb_own;
        }
        const int rc = dpg_launch_vsum(parts, outs, n_dev(c), (int64_t)count, c->stream);   // the shared stream
        return rc ? fail(rc, "virtual all-reduce launch failed") : DPG_OK;
    }
    if (c->coll == kCollHost) {   // the caller's collective, through host memory (blocking)
        c->host_hb.resize(count);
        HIP_TRY(hipSetDevice(c->device));
        HIP_TRY(hipMemcpyAsync(c->host_hb.data(), c->gn.hb_part, sizeof(double) * count, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->host_ops.allreduce_sum_f64(c->host_ops.user, c->host_hb.data(), (int64_t)count))
            return fail(DPG_ERR_HIP, "the caller's all-reduce of the packed system failed");
        HIP_TRY(hipMemcpyAsync(c->gn.hb_own, c->host_hb.data(), sizeof(double) * count, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return DPG_OK;
    }
    if (ncclGroupStart() != ncclSuccess) return fail(DPG_ERR_HIP, "ncclGroupStart failed");
    for (int k = 0; k < n_dev(c); ++k) {
        dpg_ctx* q = dev_ctx(c, k);
        const ncclResult_t r = ncclAllReduce(q->gn.hb_part, q->gn.hb_own, count, ncclDouble, ncclSum, c->comms[(size_t)k],
                                             q->stream);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return fail(DPG_ERR_HIP, "ncclAllReduce failed: %s", ncclGetErrorString(r));
        }
    }
    if (ncclGroupEnd() != ncclSuccess) return fail(DPG_ERR_HIP, "ncclGroupEnd failed");
    return DPG_OK;
}

// kCollHost, pipelined GN: the collective thread's loop (see dpg_ctx::HostColl)
static void host_coll_thread(dpg_ctx* c) {
    dpg_ctx::HostColl& h = *c->hc;
    (void)hipSetDevice(c->device);
    for (;;) {
        std::pair<uint32_t, hipEvent_t> job;
        {
            std::unique_lock<std::mutex> lk(h.mu);
            h.cv.wait(lk, [&] { return h.stop || !h.jobs.empty(); });
            if (h.jobs.empty()) return;   // stop, nothing left
            job = h.jobs.front();
            h.jobs.pop_front();
        }
        int bad = hipEventSynchronize(job.second) != hipSuccess;
        if (!bad && c->host_ops.allreduce_sum_f64(c->host_ops.user, h.buf, (int64_t)h.count)) bad = 1;
        if (bad) h.failed.store(1);
        std::atomic_thread_fence(std::memory_order_release);   // the sum before the tag
        __atomic_store_n(h.flag, job.first, __ATOMIC_RELEASE);
        {
            std::lock_guard<std::mutex> lk(h.mu);
            ++h.done;
        }
        h.cv.notify_all();
    }
}

// queue iteration's all-reduce on the collective thread and make the stream wait for it
static int coll_sum_hb_host_async(dpg_ctx* c) {
    const size_t count = (size_t)dpg_gn_dev_hb_size(&c->gn);
    HIP_TRY(hipSetDevice(c->device));
    if (!c->hc) {
        c->hc.reset(new dpg_ctx::HostColl());
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->hc->flag), 2 * sizeof(uint32_t),
                              hipHostMallocMapped | hipHostMallocCoherent));
        c->hc->flag[0] = 0;
        c->hc->flag[1] = 0;
        c->hc->timed_out = c->hc->flag + 1;
        for (auto& e : c->hc->ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->hc->th = std::thread(host_coll_thread, c);
    }
    dpg_ctx::HostColl& h = *c->hc;
    if (h.cap < count) {   // the thread is idle here: every posted job has completed (hc_drain)
        if (h.buf) HIP_TRY(hipHostFree(h.buf));
        h.buf = nullptr;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&h.buf), sizeof(double) * count, hipHostMallocDefault));
        h.cap = count;
    }
    h.count = count;
    const uint32_t tag = ++h.next_tag;
    hipEvent_t ev = h.ev[tag & 1];
    HIP_TRY(hipMemcpyAsync(h.buf, c->gn.hb_part, sizeof(double) * count, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipEventRecord(ev, c->stream));
    {
        std::lock_guard<std::mutex> lk(h.mu);
        h.jobs.emplace_back(tag, ev);
        ++h.posted;
    }
    h.cv.notify_all();
    int rc = dpg_launch_host_wait(h.flag, tag, h.timed_out, c->stream);
    if (rc) return fail(rc, "host-collective wait launch failed");
    HIP_TRY(hipMemcpyAsync(c->gn.hb_own, h.buf, sizeof(double) * count, hipMemcpyHostToDevice, c->stream));
    return DPG_OK;
}

// every all-reduce posted to the collective thread has completed (its stream work may still run)
static void hc_drain(dpg_ctx* c) {
    if (!c->hc) return;
    std::unique_lock<std::mutex> lk(c->hc->mu);
    c->hc->cv.wait(lk, [&] { return c->hc->done == c->hc->posted; });
}

static int ensure_pipe(dpg_ctx* q) {
    if (q->pipe_ctl) return DPG_OK;
    HIP_TRY(hipSetDevice(q->device));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&q->pipe_ctl), sizeof(dpg_gn_ctl)));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&q->pipe_slot), 3 * sizeof(dpg_gn_slot),   // + [2]: the initial error
                          hipHostMallocMapped | hipHostMallocCoherent));
    memset(q->pipe_slot, 0, 3 * sizeof(dpg_gn_slot));
    return DPG_OK;
}

// Wait for the report tagged `tag` in a host-mapped slot (the device stores the tag last, after a
// system-scope fence).  Spins, then yields; every ~2 ms checks the stream: a stream that has
// drained (or failed) without posting the tag is an error, not a hang.
static int wait_slot(dpg_ctx* q, const dpg_gn_slot* slot, uint64_t tag) {
    const volatile uint64_t* t = &slot->tag;
    auto t0 = std::chrono::steady_clock::now(), last = t0;
    for (unsigned n = 0;; ++n) {
        if (*t == tag) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return DPG_OK;
        }
        if (n < 4096) {
            __builtin_ia32_pause();
            continue;
        }
        std::this_thread::yield();
        const auto now = std::chrono::steady_clock::now();
        if (now - last > std::chrono::milliseconds(2)) {
            last = now;
            const hipError_t e = hipStreamQuery(q->stream);
            if (e != hipSuccess && e != hipErrorNotReady) return fail(DPG_ERR_HIP, "GN pipeline: %s", hipGetErrorString(e));
            if (e == hipSuccess && *t != tag) return fail(DPG_ERR_STATE, "GN pipeline: the stream drained without the report");
            if (now - t0 > std::chrono::seconds(60)) return fail(DPG_ERR_HIP, "GN pipeline: no report after 60 s");
        }
    }
}

// The Gauss-Newton iterations with the decisions on the device (dpg_gn_pipe.h): iteration k + 1 is
// queued before iteration k's report is read, so the GPU never waits for the host.  Multi-device
// forms: every device solves the identical all-reduced system and decides for itself (its own
// control block: the chord rule's bookkeeping stays per device); their reports must agree bit for
// bit, which the loop checks every iteration.
static int gn_loop_pipe_body(dpg_ctx* c, const dpg_gn_params& P, dpg_gn_stats& S, double& nw, double& dinf, int& it);
static int gn_loop_pipe(dpg_ctx* c, const dpg_gn_params& P, dpg_gn_stats& S, double& nw, double& dinf, int& it) {
    int rc = gn_loop_pipe_body(c, P, S, nw, dinf, it);
    if (c->coll == kCollHost && c->hc) {   // nothing of this loop left on the collective thread
        hc_drain(c);
        if (!rc && c->hc->failed.exchange(0)) rc = fail(DPG_ERR_HIP, "the caller's all-reduce of the packed system failed");
        if (!rc && __atomic_load_n(c->hc->timed_out, __ATOMIC_ACQUIRE))
            rc = fail(DPG_ERR_HIP, "GN pipeline: no all-reduce from the collective thread in 120 s");
    }
    return rc;
}
static int gn_loop_pipe_body(dpg_ctx* c, const dpg_gn_params& P, dpg_gn_stats& S, double& nw, double& dinf, int& it) {
    const int L = n_dev(c);
    const int part = is_multi(c) ? 1 : 0;
    int rc;
    for (int k = 0; k < L; ++k) {
        dpg_ctx* q = dev_ctx(c, k);
        if ((rc = ensure_pipe(q))) return rc;
        ++q->pipe_loop;
        const double* cur_dev = q->gn.hb_own + 9 * q->gn.nnzb_upper + 3 * q->gn.n_nodes;   // the assembled error
        if ((rc = dpg_gn_pipe_init(&q->gn, &P, q->pipe_ctl, cur_dev, q->pipe_slot + 2, q->pipe_loop, q->stream)))
            return fail(rc, "GN pipeline launch failed");
    }
    auto issue = [&](int i) -> int {   // iteration i (1-based) reports into slot i & 1
        int r;
        for (int k = 0; k < L; ++k) {
            dpg_ctx* q = dev_ctx(c, k);
            HIP_TRY(hipSetDevice(q->device));
            if ((r = dpg_gn_pipe_issue_solve(&q->gn, q->pipe_ctl, part, q->stream)))
                return fail(r, "GN pipeline launch failed: %s", hipGetErrorString(hipGetLastError()));
        }
        if (part && (r = (c->coll == kCollHost ? coll_sum_hb_host_async(c) : coll_sum_hb(c)))) return r;
        for (int k = 0; k < L; ++k) {
            dpg_ctx* q = dev_ctx(c, k);
            HIP_TRY(hipSetDevice(q->device));
            if ((r = dpg_gn_pipe_issue_ctl(&q->gn, &P, q->pipe_ctl, q->pipe_slot + (i & 1), part, q->stream)))
                return fail(r, "GN pipeline launch failed: %s", hipGetErrorString(hipGetLastError()));
        }
        return DPG_OK;
    };
    if ((rc = issue(1))) return rc;
    int issued = 1;
    std::vector<int> nfact((size_t)L, 0), reuse_last((size_t)L, 0);
    for (int k = 0; k < L; ++k) reuse_last[(size_t)k] = dev_ctx(c, k)->gn.last_was_chord;
    for (int i = 1;; ++i) {
        if (issued < P.max_iterations) {
            if ((rc = issue(i + 1))) return rc;
            ++issued;
        }
        dpg_gn_slot o0{};
        for (int k = 0; k < L; ++k) {
            dpg_ctx* q = dev_ctx(c, k);
            HIP_TRY(hipSetDevice(q->device));
            if (i == 1) {   // the initial error, as the device read it (pipe_init_kernel)
                if ((rc = wait_slot(q, q->pipe_slot + 2, (uint64_t)q->pipe_loop << 32))) return rc;
                const double e0 = static_cast<const volatile dpg_gn_slot*>(q->pipe_slot + 2)->error;
                if (e0 <= 0.0) {   // nothing to do: no iteration runs (pipe_init_kernel's test, NaN runs)
                    for (int j = 0; j < L; ++j) (void)hipStreamSynchronize(dev_ctx(c, j)->stream);
                    S.initial_error = e0;
                    nw = e0;
                    dinf = 0.0;
                    it = 0;
                    HIP_TRY(hipSetDevice(c->device));
                    return DPG_OK;
                }
            }
            if ((rc = wait_slot(q, q->pipe_slot + (i & 1), ((uint64_t)q->pipe_loop << 32) | (uint32_t)i))) return rc;
            dpg_gn_slot o;   // host-mapped, written by the device: read through volatile
            {
                const volatile dpg_gn_slot* v = q->pipe_slot + (i & 1);
                o.dinf = v->dinf;
                o.error = v->error;
                o.status = v->status;
                o.reuse = v->reuse;
                o.active = v->active;
                o.final_ = v->final_;
                o.it = v->it;
            }
            if (i == 1 && k == 0) S.initial_error = static_cast<const volatile dpg_gn_slot*>(q->pipe_slot + 2)->error;
            if (!o.active || o.it != i) return fail(DPG_ERR_STATE, "GN pipeline out of step (device %d, iteration %d)", k, i);
            if (k == 0) {
                o0 = o;
            } else if (memcmp(&o.dinf, &o0.dinf, sizeof(double)) || memcmp(&o.error, &o0.error, sizeof(double)) ||
                       o.status != o0.status || o.reuse != o0.reuse || o.final_ != o0.final_) {
                for (int j = 0; j < L; ++j) (void)hipStreamSynchronize(dev_ctx(c, j)->stream);
                return fail(DPG_ERR_INTERNAL, "devices diverged at GN iteration %d (device %d: |d| %.17g error %.17g, "
                            "device 0: %.17g %.17g)", i, k, o.dinf, o.error, o0.dinf, o0.error);
            }
            if (!o.reuse) ++nfact[(size_t)k];
            q->gn.prev_delta_inf = q->gn.last_delta_inf;
            q->gn.last_delta_inf = o.dinf;
            reuse_last[(size_t)k] = o.reuse;
        }
        if (c->hc && c->hc->failed.load()) {   // the caller's collective failed: the report is not a sum
            for (int j = 0; j < L; ++j) (void)hipStreamSynchronize(dev_ctx(c, j)->stream);
            return fail(DPG_ERR_HIP, "the caller's all-reduce of the packed system failed (GN iteration %d)", i);
        }
        if (o0.status != 0.0) {
            for (int j = 0; j < L; ++j) (void)hipStreamSynchronize(dev_ctx(c, j)->stream);
            if (o0.status == (double)DPG_GN_STATUS_DIVERGED)
                return fail(DPG_ERR_INTERNAL, "ranks diverged at GN iteration %d (different max |delta| in the vote words)", i);
            return fail(DPG_ERR_NUMERIC, "Cholesky failed (status %d)", (int)o0.status);
        }
        it = i;
        dinf = o0.dinf;
        nw = o0.error;
        if (o0.final_) break;
    }
    // the host bookkeeping the step API continues from (as after the host loop)
    for (int k = 0; k < L; ++k) {
        dpg_gn_dev* g = &dev_ctx(c, k)->gn;
        g->last_was_chord = reuse_last[(size_t)k];
        g->have_factor = 1;
        g->n_factorizations += nfact[(size_t)k];
        g->last_used_chol = 1;
    }
    S.pcg_iterations = 0;
    HIP_TRY(hipSetDevice(c->device));
    return DPG_OK;
}

static bool pipe_ok(dpg_ctx* c, const dpg_gn_params& P) {
    if (P.linear_solver != DPG_SOLVER_CHOLESKY) return false;
    for (int k = 0; k < n_dev(c); ++k) {
        const dpg_gn_dev& g = dev_ctx(c, k)->gn;
        if (!g.chol || !dpg_chol_gated_ok(g.chol)) return false;
    }
    return true;
}

// The Gauss-Newton loop on a set-up graph whose poses are set.  One device: assemble, then the
// pipelined iterations (or, for the PCG solver / a factorization that cannot run gated, the
// host-decided loop: solve + retract + re-linearize enqueued back to back, ONE read per iteration).
// Multi-device forms: the same loops with every device's share assembled into its hb_part and ONE
// all-reduce into hb_own between the assembly and the decision; every device solves the identical
// system, so the poses stay bitwise equal on all of them without a broadcast.
static int gn_loop(dpg_ctx* c, const dpg_gn_params& P, double* poses, double t0, double t1, dpg_gn_stats* st) {
    dpg_gn_stats S;
    memset(&S, 0, sizeof(S));
    const int L = n_dev(c);
    const bool multi = is_multi(c);
    int rc;
    for (int k = 0; k < L; ++k) {
        dpg_ctx* q = dev_ctx(c, k);
        HIP_TRY(hipSetDevice(q->device));
        if (multi) rc = dpg_gn_dev_assemble_part(&q->gn, nullptr, q->stream);
        else rc = dpg_gn_dev_assemble(&q->gn, q->gn.hb_own, q->stream);
        if (rc) return fail(rc, "assembly launch failed");
    }
    if (multi && (rc = coll_sum_hb(c))) return rc;
    double cur = 0.0, nw = 0.0, dinf = 0.0;
    int it = 0;
    const bool pipe = pipe_ok(c, P) && P.max_iterations > 0;
    if (!pipe) {   // (the pipelined loop takes the initial error on the device: no round trip)
        if ((rc = read_error(c, &S.initial_error))) return rc;
        cur = nw = S.initial_error;
    }
    if (pipe) {
        if ((rc = gn_loop_pipe(c, P, S, nw, dinf, it))) return rc;
    } else if (!(cur <= 0.0) && P.max_iterations > 0) {
        for (;;) {
            for (int k = 0; k < L; ++k) {
                dpg_ctx* q = dev_ctx(c, k);
                HIP_TRY(hipSetDevice(q->device));
                if ((rc = solve_retract_async_1(q, nullptr))) return rc;
                if (multi) rc = dpg_gn_dev_assemble_part(&q->gn, nullptr, q->stream);
                else rc = dpg_gn_dev_assemble(&q->gn, q->gn.hb_own, q->stream);
                if (rc) return fail(rc, "assembly launch failed");
            }
            if (multi && (rc = coll_sum_hb(c))) return rc;
            // every device reads its own scalars: its chord rule's bookkeeping (last / previous
            // max|delta|) moves with its own solves, and the devices must agree
            double sc0[3] = {0, 0, 0};
            for (int k = 0; k < L; ++k) {
                dpg_ctx* q = dev_ctx(c, k);
                double sc[3];
                HIP_TRY(hipSetDevice(q->device));
                if ((rc = fetch_1(q, nullptr, sc))) return rc;
                if (k == 0) memcpy(sc0, sc, sizeof(sc));
                else if (memcmp(sc, sc0, sizeof(sc)))
                    return fail(DPG_ERR_INTERNAL, "devices diverged at GN iteration %d (device %d)", it + 1, k);
            }
            // world > 1: decide from the all-reduced vote words (every rank's max |delta| and
            // status of this iteration, dpg_gn.hip chi2_kernel), never from the local scalars
            // alone -- ranks that disagreed would issue different numbers of all-reduces and hang
            if (multi && c->gn.n_vote > 0) {
                const int W = c->gn.world;
                std::vector<double> vw((size_t)(2 * W));
                HIP_TRY(hipSetDevice(c->device));
                HIP_TRY(hipMemcpyAsync(vw.data(), c->gn.hb_own + dpg_gn_dev_vote_offset(&c->gn), sizeof(double) * vw.size(),
                                       hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(hipStreamSynchronize(c->stream));
                for (int r = 0; r < W; ++r) {
                    if (memcmp(&vw[(size_t)r], &vw[0], sizeof(double)))
                        return fail(DPG_ERR_INTERNAL, "ranks diverged at GN iteration %d (rank %d: |d| %.17g, rank 0: %.17g)",
                                    it + 1, r, vw[(size_t)r], vw[0]);
                    sc0[2] = std::max(sc0[2], vw[(size_t)(W + r)]);
                }
                sc0[0] = vw[0];
            }
            if (sc0[2] != 0.0) return fail(DPG_ERR_NUMERIC, "Cholesky failed (status %d)", (int)sc0[2]);
            S.pcg_iterations += c->gn.last_pcg_iters;
            ++it;
            dinf = sc0[0];
            nw = sc0[1];
            if (it >= P.max_iterations) break;
            if (P.use_error_criteria) {
                if (check_conv(&P, cur, nw) || !std::isfinite(cur)) break;
            } else if (dinf < P.delta_tol) {
                break;
            }
            cur = nw;
        }
    }
    if (multi && (rc = dpg_ctx_synchronize(c))) return rc;
    if (poses && (rc = dpg_gn_get_poses(c, poses))) return rc;
    if (!poses) {
        HIP_TRY(hipSetDevice(c->device));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    const double t2 = now_ms();
    S.iterations = it;
    S.final_error = nw;
    S.last_delta_inf = dinf;
    S.ms_total = t2 - t0;
    S.ms_per_iteration = it ? (t2 - t1) / it : 0.0;
    if (st) *st = S;
    return DPG_OK;
}

// The GN loop on the graph staged by dpg_gn_setup (+ dpg_gn_take_icp_measurements) from the poses
// of dpg_gn_set_poses, with the setup's parameters: what a host loop over the step API does,
// natively (no interpreter between the launches; multi-device forms: sharded, one all-reduce per
// iteration)
int dpg_gn_run(dpg_ctx* c, double* poses_out, dpg_gn_stats* st) {
    if (!c || !c->gn_ready) return fail(DPG_ERR_STATE, "dpg_gn_run: graph not set up");
    HIP_TRY(hipSetDevice(c->device));
    const double t0 = now_ms();
    return gn_loop(c, c->gp, poses_out, t0, t0, st);
}

int dpg_optimize_graph(dpg_ctx* c, double* poses, int64_t V, const dpg_factor* F, int64_t nf, const dpg_gn_params* gp,
                       dpg_gn_stats* st) {
    const double t0 = now_ms();
    dpg_gn_params P;
    if (gp) P = *gp;
    else dpg_gn_params_default(&P);
    if (!c || !F || !poses || V <= 0 || nf < 0) return fail(DPG_ERR_ARG, "dpg_optimize_graph: bad arguments");
    int rc = dpg_gn_setup(c, V, F, nf, 0, nf, &P);
    if (rc) return rc;
    if ((rc = dpg_gn_set_poses(c, poses))) return rc;
    return gn_loop(c, P, poses, t0, now_ms(), st);
}

// ---- re-linearisation sweep (DpgSLAM::reoptimize) ----

void dpg_reopt_params_default(dpg_reopt_params* p) {
    if (!p) return;
    p->max_node_dist_within_pass = 5.0f;
    p->max_node_dist_across_passes = 2.0f;
    p->new_pass_std_dev[0] = 0.2f;
    p->new_pass_std_dev[1] = 0.2f;
    p->new_pass_std_dev[2] = 0.15f;
    for (int k = 0; k < 4; ++k) p->motion_model[k] = 0.4f;
    p->odometry_constraints = 1;
}

// candidate pairs on the GPU (dpg_reopt.hip): count per node, host prefix sum, write
static int64_t lc_candidates(dpg_ctx* c, int64_t V, const int32_t* pass, const float* est, float within,
                             float across, std::vector<int32_t>& pairs) {
    DevBuf<float> dposes;
    DevBuf<int32_t> dpass, dcount, dpairs;
    DevBuf<int64_t> doff;
    if (dposes.reserve((size_t)(3 * V)) || dpass.reserve((size_t)V) || dcount.reserve((size_t)V) ||
        doff.reserve((size_t)V))
        return fail(DPG_ERR_HIP, "allocation failed");
    int64_t K = -1;
    std::vector<int32_t> cnt((size_t)V);
    std::vector<int64_t> off((size_t)V);
    do {
        if (hipMemcpyAsync(dposes.p, est, sizeof(float) * 3 * V, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
            hipMemcpyAsync(dpass.p, pass, sizeof(int32_t) * V, hipMemcpyHostToDevice, c->stream) != hipSuccess)
            break;
        if (dpg_launch_lc_count(dposes.p, dpass.p, V, within, across, dcount.p, c->stream)) break;
        if (hipMemcpyAsync(cnt.data(), dcount.p, sizeof(int32_t) * V, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            break;
        int64_t acc = 0;
        for (int64_t i = 0; i < V; ++i) { off[(size_t)i] = acc; acc += cnt[(size_t)i]; }
        pairs.assign((size_t)(2 * acc), 0);
        if (acc > 0) {
            if (dpairs.reserve((size_t)(2 * acc))) break;
            if (hipMemcpyAsync(doff.p, off.data(), sizeof(int64_t) * V, hipMemcpyHostToDevice, c->stream) != hipSuccess)
                break;
            if (dpg_launch_lc_write(dposes.p, dpass.p, V, within, across, doff.p, dpairs.p, c->stream)) break;
            if (hipMemcpyAsync(pairs.data(), dpairs.p, sizeof(int32_t) * 2 * acc, hipMemcpyDeviceToHost, c->stream) !=
                    hipSuccess ||
                hipStreamSynchronize(c->stream) != hipSuccess)
                break;
        }
        K = acc;
    } while (false);
    dposes.release();
    dpass.release();
    dcount.release();
    dpairs.release();
    doff.release();
    if (K < 0) return fail(DPG_ERR_HIP, "loop-closure candidate search failed: %s", hipGetErrorString(hipGetLastError()));
    return K;
}

int64_t dpg_loop_closure_candidates(dpg_ctx* c, int64_t V, const int32_t* pass, const float* est, float within,
                                    float across, int32_t* pairs_out, int64_t cap) {
    if (!c || V < 0 || (V > 0 && (!pass || !est))) return fail(DPG_ERR_ARG, "bad arguments");
    std::vector<int32_t> pairs;
    const int64_t K = lc_candidates(c, V, pass, est, within, across, pairs);
    if (K < 0) return K;
    if (pairs_out && cap > 0) memcpy(pairs_out, pairs.data(), sizeof(int32_t) * 2 * (size_t)std::min(K, cap));
    return K;
}

int64_t dpg_get_map(dpg_ctx* c, const float* est, int32_t fraction, float* out, int64_t cap) {
    if (!c || !est || fraction <= 0) return fail(DPG_ERR_ARG, "bad arguments");
    const int64_t V = c->n_nodes;
    if (V <= 0 || (int64_t)c->full_off.size() != V + 1) return fail(DPG_ERR_STATE, "no scans uploaded");
    const int64_t P = c->full_off[(size_t)V];
    const int64_t K = (P + fraction - 1) / fraction;
    if (!out || cap <= 0 || K == 0) return K;
    // Rotation2Df(angle): cosf/sinf on the host, as the reference evaluates them
    std::vector<float> fr((size_t)(4 * V));
    for (int64_t v = 0; v < V; ++v) {
        fr[(size_t)(4 * v)] = est[3 * v];
        fr[(size_t)(4 * v + 1)] = est[3 * v + 1];
        fr[(size_t)(4 * v + 2)] = cosf(est[3 * v + 2]);
        fr[(size_t)(4 * v + 3)] = sinf(est[3 * v + 2]);
    }
    DevBuf<float> dfr, dout;
    DevBuf<int64_t> doff;
    int64_t ret = -1;
    do {
        if (dfr.reserve((size_t)(4 * V)) || dout.reserve((size_t)(2 * K)) || doff.reserve((size_t)(V + 1))) break;
        if (hipMemcpyAsync(dfr.p, fr.data(), sizeof(float) * 4 * V, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
            hipMemcpyAsync(doff.p, c->full_off.data(), sizeof(int64_t) * (V + 1), hipMemcpyHostToDevice, c->stream) !=
                hipSuccess)
            break;
        if (!c->map_ev[0] && (hipEventCreate(&c->map_ev[0]) != hipSuccess || hipEventCreate(&c->map_ev[1]) != hipSuccess))
            break;
        if (hipEventRecord(c->map_ev[0], c->stream) != hipSuccess) break;
        if (dpg_launch_map_points(c->full.p, doff.p, dfr.p, V, fraction, dout.p, c->stream)) break;
        if (hipEventRecord(c->map_ev[1], c->stream) != hipSuccess) break;
        if (hipMemcpyAsync(out, dout.p, sizeof(float) * 2 * std::min(K, cap), hipMemcpyDeviceToHost, c->stream) !=
                hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            break;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, c->map_ev[0], c->map_ev[1]) == hipSuccess) c->map_ms = ms;
        ret = K;
    } while (false);
    dfr.release();
    dout.release();
    doff.release();
    if (ret < 0) return fail(DPG_ERR_HIP, "map assembly failed: %s", hipGetErrorString(hipGetLastError()));
    return ret;
}

float dpg_get_map_kernel_ms(dpg_ctx* c) { return c ? c->map_ms : -1.f; }

// The sweep of DpgSLAM::reoptimize up to the alignments (dpg_slam.cc:35-107): candidates, the ICP
// edge list (successive, then candidates), the factor list (per node a pass prior or the odometry
// Between, then one Between slot per ICP edge, first at first_icp) and ONE batched ICP launched on
// the context's stream (not waited for).
static int reopt_sweep(dpg_ctx* c, int64_t V, const int32_t* pass, const float* est, const float* odom,
                       const dpg_icp_params& I, const dpg_reopt_params& R, std::vector<int32_t>& edges,
                       std::vector<dpg_factor>& F, int64_t& first_icp, int64_t& n_succ, dpg_reopt_stats& S,
                       double& t1) {
    const double t0 = now_ms();
    // 1. loop-closure candidates (dpg_slam.cc:91-98)
    std::vector<int32_t> lc;
    const int64_t K = lc_candidates(c, V, pass, est, R.max_node_dist_within_pass, R.max_node_dist_across_passes, lc);
    if (K < 0) return (int)K;
    t1 = now_ms();
    // 2. ICP edges: successive (i-1, i), then the candidates (j, i) -- {node_1 target, node_2 source}
    n_succ = V - 1;
    const int64_t E = n_succ + K;
    edges.assign((size_t)(2 * E), 0);
    for (int64_t i = 1; i < V; ++i) { edges[(size_t)(2 * (i - 1))] = (int32_t)(i - 1); edges[(size_t)(2 * (i - 1) + 1)] = (int32_t)i; }
    if (K > 0) memcpy(edges.data() + 2 * n_succ, lc.data(), sizeof(int32_t) * 2 * (size_t)K);
    // 3. factors: per node a prior (new pass) or the odometry Between (dpg_slam.cc:40-79), then one
    //    slot per ICP edge (measurements filled on device after the batch)
    F.clear();
    F.reserve((size_t)(V + E));
    int32_t cur_pass = -1;
    for (int64_t i = 0; i < V; ++i) {
        if (i == 0 || pass[i] != cur_pass) {
            dpg_factor f;
            memset(&f, 0, sizeof(f));
            f.kind = DPG_FACTOR_PRIOR;
            f.i = (int32_t)i;
            for (int k = 0; k < 3; ++k) {
                const double sd = (double)R.new_pass_std_dev[k];
                f.info[k] = 1.0 / (sd * sd);
            }
            F.push_back(f);
            cur_pass = pass[i];
        } else if (R.odometry_constraints) {
            dpg_factor f;
            const int rc = dpg_odometry_factor(odom + 3 * (i - 1), odom + 3 * i, (int32_t)(i - 1), (int32_t)i,
                                               R.motion_model[0], R.motion_model[1], R.motion_model[2],
                                               R.motion_model[3], &f);
            if (rc) return fail(rc, "odometry factor %lld has no motion (zero sigma)", (long long)i);
            F.push_back(f);
        }
    }
    first_icp = (int64_t)F.size();
    for (int64_t e = 0; e < E; ++e) {
        dpg_factor f;
        memset(&f, 0, sizeof(f));
        f.kind = DPG_FACTOR_BETWEEN;
        f.i = edges[(size_t)(2 * e)];
        f.j = edges[(size_t)(2 * e + 1)];
        F.push_back(f);
    }
    // 4. one batched ICP of every edge from the estimated poses (runIcp, dpg_slam.cc:362-446)
    int rc = dpg_icp_batch_prepare(c, edges.data(), E, est, &I);
    if (!rc) rc = dpg_icp_batch_run(c, 0, 0);
    S.n_candidates = K;
    S.n_icp_edges = E;
    S.ms_candidates = t1 - t0;
    return rc;
}

int dpg_reoptimize(dpg_ctx* c, int64_t V, const int32_t* pass, const float* est, const float* odom,
                   const dpg_icp_params* ip, const dpg_gn_params* gp, const dpg_reopt_params* rp, double* poses_out,
                   dpg_reopt_stats* st) {
    if (!c || V <= 0 || !pass || !est || !odom || !poses_out) return fail(DPG_ERR_ARG, "bad arguments");
    if (c->n_nodes != V) return fail(DPG_ERR_STATE, "scans of %lld nodes uploaded, sweep over %lld",
                                     (long long)c->n_nodes, (long long)V);
    dpg_icp_params I;
    if (ip) I = *ip;
    else dpg_icp_params_default(&I);
    dpg_gn_params P;
    if (gp) P = *gp;
    else dpg_gn_params_default(&P);
    dpg_reopt_params R;
    if (rp) R = *rp;
    else dpg_reopt_params_default(&R);
    dpg_reopt_stats S;
    memset(&S, 0, sizeof(S));
    std::vector<int32_t> edges;
    std::vector<dpg_factor> F;
    int64_t first_icp = 0, n_succ = 0;
    double t1 = 0.0;
    int rc = reopt_sweep(c, V, pass, est, odom, I, R, edges, F, first_icp, n_succ, S, t1);
    if (rc) return rc;
    const int64_t E = S.n_icp_edges;
    // the sweep's own results (the caller may fetch them again: the batch stays staged) -- the
    // alignments end here, and their outcomes give the loop-closure count
    std::vector<dpg_icp_result> res((size_t)std::max<int64_t>(E, 1));
    if ((rc = dpg_icp_batch_fetch(c, res.data(), nullptr, (int64_t)res.size()))) return rc;
    const double t2 = now_ms();
    // 5. batch Gauss-Newton from the estimated poses (optimizeGraph, dpg_slam.cc:111-119, 316-329);
    //    the ICP slots take the results where they were aligned (multi-device: on each device)
    if ((rc = dpg_gn_setup(c, V, F.data(), (int64_t)F.size(), 0, (int64_t)F.size(), &P))) return rc;
    if ((rc = dpg_gn_take_icp_measurements(c, first_icp, E, n_succ, &I))) return rc;
    {
        for (int64_t e = n_succ; e < E; ++e)
            S.n_loop_closures += (res[(size_t)e].converged && res[(size_t)e].status == DPG_ICP_OK) ? 1 : 0;
    }
    for (int64_t v = 0; v < 3 * V; ++v) poses_out[v] = (double)est[v];
    if ((rc = dpg_gn_set_poses(c, poses_out))) return rc;
    if ((rc = gn_loop(c, P, poses_out, t2, now_ms(), &S.gn))) return rc;
    const double t3 = now_ms();
    S.n_factors = (int64_t)F.size();
    S.ms_icp = t2 - t1;
    S.ms_gn = t3 - t2;
    if (st) *st = S;
    return DPG_OK;
}

int dpg_reoptimize_inc(dpg_inc* g, int64_t V, const int32_t* pass, const float* est, const float* odom,
                       const dpg_icp_params* ip, const dpg_reopt_params* rp, double* poses_out, dpg_reopt_stats* st) {
    if (!g || V <= 0 || !pass || !est || !odom || !poses_out) return fail(DPG_ERR_ARG, "dpg_reoptimize_inc: bad arguments");
    dpg_ctx* c = dpg_inc_ctx(g);
    if (c->n_nodes != V) return fail(DPG_ERR_STATE, "scans of %lld nodes uploaded, sweep over %lld",
                                     (long long)c->n_nodes, (long long)V);
    dpg_icp_params I;
    if (ip) I = *ip;
    else dpg_icp_params_default(&I);
    dpg_reopt_params R;
    if (rp) R = *rp;
    else dpg_reopt_params_default(&R);
    dpg_reopt_stats S;
    memset(&S, 0, sizeof(S));
    std::vector<int32_t> edges;
    std::vector<dpg_factor> F;
    int64_t first_icp = 0, n_succ = 0;
    double t1 = 0.0;
    int rc = reopt_sweep(c, V, pass, est, odom, I, R, edges, F, first_icp, n_succ, S, t1);
    if (rc) return rc;
    const int64_t E = S.n_icp_edges;
    std::vector<dpg_icp_result> res((size_t)std::max<int64_t>(E, 1));
    if (E > 0 && (rc = dpg_icp_batch_fetch(c, res.data(), nullptr, (int64_t)res.size()))) return rc;
    const double t2 = now_ms();
    // addObservationConstraint per aligned pair: the successive pairs always, a loop closure when
    // its alignment converged (dpg_slam.cc:85-104); the slots of dropped closures go away
    F.resize((size_t)first_icp);
    for (int64_t e = 0; e < E; ++e) {
        const dpg_icp_result& r = res[(size_t)e];
        if (r.status == DPG_ICP_INTERNAL)
            return fail(DPG_ERR_INTERNAL, "dpg_reoptimize_inc: alignment %lld failed its internal check", (long long)e);
        if (e < n_succ || (r.converged && r.status == DPG_ICP_OK)) {
            dpg_factor f;
            dpg_icp_factor(&r, edges[(size_t)(2 * e)], edges[(size_t)(2 * e + 1)], &I, &f);
            F.push_back(f);
            if (e >= n_succ) ++S.n_loop_closures;
        }
    }
    // the new ISAM2 + graph_ and its one update from the current estimates (dpg_slam.cc:36-39,111-119)
    std::vector<double> X0((size_t)(3 * V));
    for (int64_t v = 0; v < 3 * V; ++v) X0[(size_t)v] = (double)est[v];
    if ((rc = dpg_inc_reset(g))) return rc;
    dpg_inc_stats is;
    if ((rc = dpg_inc_update(g, V, X0.data(), F.data(), (int64_t)F.size(), &is))) return rc;
    if ((rc = dpg_inc_get_poses(g, poses_out, V))) return rc;
    const double t3 = now_ms();
    S.n_factors = (int64_t)F.size();
    S.ms_icp = t2 - t1;
    S.ms_gn = t3 - t2;
    S.gn.iterations = is.gn_iterations;
    S.gn.final_error = is.error;
    if (st) *st = S;
    return DPG_OK;
}

int dpg_add_node_pairs(dpg_inc* g, const float* cloud, int64_t n_pts, const float init_pose[3], const dpg_factor* extra,
                       int64_t n_extra, const int32_t* pairs, int64_t n_pairs, int32_t successive,
                       const dpg_icp_params* ip, dpg_add_node_stats* st) {
    if (!g || (!cloud && n_pts > 0) || n_pts < 0 || !init_pose || (n_extra > 0 && !extra) || n_extra < 0 ||
        n_pairs < 0 || (n_pairs > 0 && !pairs))
        return fail(DPG_ERR_ARG, "dpg_add_node_pairs: bad arguments");
    dpg_ctx* c = dpg_inc_ctx(g);
    dpg_icp_params I;
    if (ip) I = *ip;
    else dpg_icp_params_default(&I);
    dpg_add_node_stats S;
    memset(&S, 0, sizeof(S));
    const int64_t V = dpg_inc_num_nodes(g);
    if (c->n_nodes != V) return fail(DPG_ERR_STATE, "scan store holds %lld nodes, graph %lld", (long long)c->n_nodes,
                                     (long long)V);
    for (int64_t e = 0; e < n_pairs; ++e)
        if (pairs[2 * e] < 0 || pairs[2 * e + 1] < 0 || pairs[2 * e] > V || pairs[2 * e + 1] > V || pairs[2 * e] == pairs[2 * e + 1])
            return fail(DPG_ERR_ARG, "dpg_add_node_pairs: pair %lld references a missing node", (long long)e);
    // createNode: the node's cloud joins the store (node id V).  Any failure after this point
    // takes the node out of the store again (and undoes a prepared update), so the store and the
    // graph keep the same node count and the next dpg_add_node can proceed.
    const int64_t offs[2] = {0, n_pts};
    const float dummy[2] = {0.f, 0.f};
    int rc = dpg_scans_append(c, n_pts > 0 ? cloud : dummy, offs, 1, I.downsample_icp_points_ratio);
    if (rc) return rc;
    struct Undo {
        dpg_ctx* c;
        dpg_inc* g;
        int64_t V;
        bool armed = true;
        ~Undo() {
            if (!armed) return;
            dpg_inc_abort_prepare(g);
            scans_truncate(c, V);
        }
    } undo{c, g, V};
    // estimates as float (dpg_nodes_ positions), the new node's initial pose last
    std::vector<double> est((size_t)(3 * std::max<int64_t>(V, 1)));
    if (V > 0 && (rc = dpg_inc_get_poses(g, est.data(), V))) return rc;
    std::vector<float> pf((size_t)(3 * (V + 1)));
    for (int64_t q = 0; q < 3 * V; ++q) pf[(size_t)q] = (float)est[(size_t)q];
    for (int k = 0; k < 3; ++k) pf[(size_t)(3 * V + k)] = init_pose[k];
    std::vector<int32_t> edges;
    if (successive && V >= 1) { edges.push_back((int32_t)(V - 1)); edges.push_back((int32_t)V); }
    edges.insert(edges.end(), pairs, pairs + 2 * n_pairs);
    const int64_t n_succ = (successive && V >= 1) ? 1 : 0;
    const int64_t E = (int64_t)edges.size() / 2;
    std::vector<dpg_factor> F(extra, extra + n_extra);
    if (E > 0) {
        const double t0 = now_ms();
        if ((rc = dpg_icp_batch_prepare(c, edges.data(), E, pf.data(), &I))) return rc;
        // nodes below V whose index is stale (a k-d tree / grid batch overwrote the buffers, or a
        // fresh upload was not indexed) are rebuilt with the new node
        if ((rc = icp_batch_run_from(c, std::min(V, c->idx_valid)))) return rc;
        // while the GPU aligns: the update's structure on the host, with every pair a factor may
        // come from (a loop closure that does not converge stays an explicit zero block)
        {
            std::vector<int32_t> pr(edges);
            for (int64_t k = 0; k < n_extra; ++k)
                if (extra[k].kind == DPG_FACTOR_BETWEEN) { pr.push_back(extra[k].i); pr.push_back(extra[k].j); }
            if ((rc = dpg_inc_prepare(g, 1, pr.data(), (int64_t)pr.size() / 2))) return rc;
        }
        std::vector<dpg_icp_result> res((size_t)E);
        if ((rc = batch_fetch(c, res.data(), nullptr, false))) return rc;
        S.ms_icp = now_ms() - t0;
        S.n_icp_edges = E;
        for (int64_t e = 0; e < E; ++e)   // a failed kernel self-check is an error, never a factor
            if (res[(size_t)e].status == DPG_ICP_INTERNAL)
                return fail(DPG_ERR_INTERNAL, "dpg_add_node_pairs: alignment %lld failed its internal check", (long long)e);
        for (int64_t e = 0; e < E; ++e) {
            const dpg_icp_result& r = res[(size_t)e];
            const bool ok = r.converged && r.status == DPG_ICP_OK;
            if (e < n_succ || ok) {   // successive: always (dpg_slam.cc:263-267); loop closures when converged (:295-301)
                dpg_factor f;
                dpg_icp_factor(&r, edges[(size_t)(2 * e)], edges[(size_t)(2 * e + 1)], &I, &f);
                F.push_back(f);
                if (e >= n_succ) ++S.n_loop_closures;
            }
        }
    } else if (c->icp_variant == DPG_ICP_ANGULAR && n_pts > 0) {   // no alignment: only the new node's index
        rc = dpg_launch_angle_index(c->ds.p, c->ds_off_dev.p + V, 1, c->max_ds, c->tree_pts.p, c->tree_idx.p,
                                    c->buckets.p + V * (int64_t)(dpg_angle_buckets() + 1), c->kernel_variant == 2,
                                    c->stream);
        if (rc) return fail(rc, "angle index build failed");
        if (c->idx_valid == V) c->idx_valid = V + 1;
    }
    const double init[3] = {(double)init_pose[0], (double)init_pose[1], (double)init_pose[2]};
    if ((rc = dpg_inc_update(g, 1, init, F.data(), (int64_t)F.size(), &S.update))) return rc;   // rolled back itself
    undo.armed = false;
    if (st) *st = S;
    return DPG_OK;
}

int dpg_add_node(dpg_inc* g, const float* cloud, int64_t n_pts, const int32_t* pass, const float init_pose[3],
                 const dpg_factor* extra, int64_t n_extra, const dpg_icp_params* ip, const dpg_reopt_params* rp,
                 int32_t non_successive, dpg_add_node_stats* st) {
    if (!g || !pass || !init_pose) return fail(DPG_ERR_ARG, "dpg_add_node: bad arguments");
    dpg_reopt_params R;
    if (rp) R = *rp;
    else dpg_reopt_params_default(&R);
    const int64_t V = dpg_inc_num_nodes(g);
    // updatePoseGraphObsConstraints (dpg_slam.cc:273-304): loop-closure candidates (i, prev), i < V - 2,
    // by the float distance of the estimates (dpg_nodes_ positions are float), ascending i
    std::vector<int32_t> lc;
    if (non_successive && V > 1) {
        std::vector<double> est((size_t)(3 * V));
        int rc = dpg_inc_get_poses(g, est.data(), V);
        if (rc) return rc;
        const int64_t pv = V - 1;
        const float px = (float)est[(size_t)(3 * pv)], py = (float)est[(size_t)(3 * pv + 1)];
        for (int64_t i = 0; i < V - 2; ++i) {
            const float dx = (float)est[(size_t)(3 * i)] - px, dy = (float)est[(size_t)(3 * i + 1)] - py;
            const float dist = sqrtf(dx * dx + dy * dy);   // Eigen Vector2f::norm
            const float thr = pass[i] == pass[pv] ? R.max_node_dist_within_pass : R.max_node_dist_across_passes;
            if (dist <= thr) { lc.push_back((int32_t)i); lc.push_back((int32_t)pv); }
        }
    }
    return dpg_add_node_pairs(g, cloud, n_pts, init_pose, extra, n_extra, lc.data(), (int64_t)lc.size() / 2, 1, ip, st);
}

}  // extern "C"
