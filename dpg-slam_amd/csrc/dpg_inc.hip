// dpg_inc.hip -- the incremental pose-graph solver: DpgSLAM::optimizeGraph as the reference runs
// it once per new node (dpg_slam.cc:255-329, isam_->update at :320, ISAM2 built with default
// parameters at :22/:38), on a device-resident graph that grows node by node.  SURVEY 8f rank 3.
//
// Structure (kept across updates, nothing re-allocated unless it must grow):
//   * the factor list and its unique node pairs (arrival order) -- the block pattern of H;
//   * the incremental symbolic state (dpg_chol_incsym, dpg_chol_sym.cpp): the elimination order
//     is KEPT and each new node is appended at its end; a new edge adds its fill along the
//     elimination-tree path it touches.  A fresh minimum-degree order is computed only every
//     `reorder_every` nodes or when the fill has grown 1.5x past the last ordering's;
//   * the supernodal structures and device buffers of the GPU Cholesky (dpg_chol.hip), re-derived
//     from that state each update in linear time into the same buffers.
//
// Update semantics (dpg_inc_params.mode):
//   DPG_INC_ISAM2 (default) -- GTSAM ISAM2 with its default parameters: a
//     linearization point theta per variable, relinearized (theta_k <- theta_k (+) delta_k) only
//     for variables whose max |delta_k| >= relinearize_threshold (0.1), and only on updates whose
//     count, this update included, is a multiple of relinearize_skip (10): updates 10, 20, 30 --
//     GTSAM 4.0's ISAM2::update increments update_count_ first and then asks
//     UpdateImpl::relinarizationNeeded(update_count_) (update_count % relinearizeSkip == 0); every update re-linearizes every factor at theta, solves
//     H(theta) delta = -g(theta) by Cholesky and returns the estimate theta (+) delta, one
//     Gauss-Newton step from a lagging linearization point.  Deviation, documented: the solve is
//     exact (ISAM2's back-substitution stops at the wildfire threshold 0.001).
//   DPG_INC_BATCH -- Gauss-Newton to convergence from the current estimates on every update (the
//     batch optimum of the accumulated graph; what round 1's driver computed from scratch).
//   duplicate_factors = 1 reproduces SURVEY Q1: the reference passes the whole accumulated graph_
//     to every isam_->update, so a factor added u updates ago is in ISAM2 u + 1 times -- exactly
//     its information scaled by u + 1.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "dpg_chol.h"
#include "dpg_internal.h"

namespace {

constexpr int kThreads = 256;

double now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

template <typename T>
int dgrow(T** d, size_t* cap, size_t n, hipStream_t s, size_t keep) {
    n = std::max<size_t>(n, 1);
    if (*d && n <= *cap) return DPG_OK;
    const size_t nc = std::max(n, *cap + *cap / 2);
    T* p = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&p), nc * sizeof(T)) != hipSuccess) return DPG_ERR_HIP;
    if (*d && keep) {
        if (hipMemcpyAsync(p, *d, std::min(keep, *cap) * sizeof(T), hipMemcpyDeviceToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            (void)hipFree(p);
            return DPG_ERR_HIP;
        }
    }
    if (*d) (void)hipFree(*d);
    *d = p;
    *cap = nc;
    return DPG_OK;
}

// est = theta (+) x (Pose2 ChartAtOrigin retraction, as retract_kernel), x indexed by elimination
// position; maxd[v] = max |x_v|; atomicMax of the largest into maxall
__global__ void inc_estimate_kernel(const double* __restrict__ theta, const double* __restrict__ x,
                                    const int32_t* __restrict__ pos, int64_t n, double* __restrict__ est,
                                    double* __restrict__ maxd, double* __restrict__ maxall) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double m = 0.0;
    if (v < n) {
        const int64_t di = 3 * (int64_t)pos[v];
        const double c = cos(theta[3 * v + 2]), s = sin(theta[3 * v + 2]);
        const double d0 = x[di], d1 = x[di + 1], d2 = x[di + 2];
        const double cd = cos(d2), sd = sin(d2);
        est[3 * v] = theta[3 * v] + (c * d0 - s * d1);
        est[3 * v + 1] = theta[3 * v + 1] + (s * d0 + c * d1);
        est[3 * v + 2] = atan2(s * cd + c * sd, c * cd - s * sd);
        m = fmax(fabs(d0), fmax(fabs(d1), fabs(d2)));
        if (!(m == m)) m = __longlong_as_double(0x7ff0000000000000ll);
        maxd[v] = m;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
    if ((threadIdx.x & 63) == 0)
        atomicMax(reinterpret_cast<unsigned long long*>(maxall), (unsigned long long)__double_as_longlong(m));
}

// ISAM2 relinearization of the variables [0, n): theta_v <- est_v (= theta_v (+) delta_v) where
// max |delta_v| >= thr; counts them
__global__ void inc_relin_kernel(double* __restrict__ theta, const double* __restrict__ est,
                                 const double* __restrict__ maxd, int64_t n, double thr, int32_t* __restrict__ count) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n || !(maxd[v] >= thr)) return;
    theta[3 * v] = est[3 * v];
    theta[3 * v + 1] = est[3 * v + 1];
    theta[3 * v + 2] = est[3 * v + 2];
    atomicAdd(count, 1);
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }
inline uint64_t pkey(int32_t lo, int32_t hi) { return ((uint64_t)(uint32_t)lo << 32) | (uint32_t)hi; }

}  // namespace


// One helper thread of an incremental graph: runs one posted job at a time (the prepare's H-block
// buckets beside the symbolic derivation).  It sleeps on a condition variable between jobs -- a
// spinning helper slowed the calling thread's own host work by as much as it took off it
// (incsym 0.14 -> 0.16 ms, derive 0.15 -> 0.19 ms on the lease's CPU share).
struct dpg_inc_helper {
    std::mutex m;
    std::condition_variable cv;
    std::function<void()> job;
    bool has_job = false, done = true, quit = false;
    std::thread th;
    dpg_inc_helper() : th([this] { run(); }) {}
    ~dpg_inc_helper() {
        {
            std::lock_guard<std::mutex> l(m);
            quit = true;
        }
        cv.notify_all();
        th.join();
    }
    void run() {
        std::unique_lock<std::mutex> l(m);
        for (;;) {
            cv.wait(l, [this] { return quit || has_job; });
            if (quit) return;
            std::function<void()> f = std::move(job);
            has_job = false;
            l.unlock();
            f();
            l.lock();
            done = true;
            cv.notify_all();
        }
    }
    void post(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> l(m);
            job = std::move(f);
            has_job = true;
            done = false;
        }
        cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [this] { return done; });
    }
};

struct dpg_inc {
    dpg_ctx* ctx = nullptr;
    dpg_inc_params P{};
    int64_t V = 0;
    int64_t updates = 0;                       // isam_->update calls since the last reset
    std::vector<dpg_factor> F;                 // as given (base information)
    std::vector<int32_t> f_created;            // update that added each factor (Q1 multiplicity)
    std::vector<int32_t> f_pair;               // unique pair of a Between factor, -1 for a prior
    std::unordered_map<uint64_t, int32_t> pair_id;
    std::vector<int32_t> plo, phi;             // unique pairs (lo < hi) in arrival order
    dpg_chol_incsym I;
    int64_t V_at_order = 0, nnz_at_order = 0;  // size of the graph at the last full ordering
    dpg_chol_sym S;
    dpg_chol_opts opts;
    int64_t reorders = 0;
    // device
    dpg_gn_dev g{};                            // assembly buffers + the Cholesky (g.chol)
    size_t c_factors = 0, c_cptr = 0, c_clist = 0, c_hb = 0, c_partials = 0;
    double* theta = nullptr;                   // [V][3] linearization points (g.poses aliases it)
    double* est = nullptr;                     // [V][3] current estimate
    double* maxd = nullptr;                    // [V] max |delta_v| of the last update
    double* est_nxt = nullptr;                 // ISAM2 mode: the update's estimate and max |delta| are
    double* maxd_nxt = nullptr;                // written here and swapped in once the solve succeeded
    size_t c_est_nxt = 0, c_maxd_nxt = 0;
    int32_t* cnt = nullptr;                    // relinearized variables of the last update
    size_t c_theta = 0, c_est = 0, c_maxd = 0;
    std::vector<dpg_factor> h_dev_factors;     // staging (Q1 scaling)
    int64_t n_dev_f = 0;                       // leading factors already on the device as given (no Q1)
    int32_t* h_lists = nullptr;                // pinned staging of the contribution lists
    size_t c_lists = 0;
    hipEvent_t lists_ev = nullptr;             // recorded after the lists' copies
    bool lists_ev_set = false;
    bool prepared = false;                     // inc_prepare ran for the coming update (its pairs are in)
    int64_t prep_new = 0;                      // ... for this many new nodes
    int64_t prep_pairs0 = 0;                   // number of unique pairs before that prepare (rollback)
    double* theta_bak = nullptr;               // [V][3] theta before a relinearization (rollback)
    double* est_bak = nullptr;                 // [V][3] estimate before a batch update (rollback)
    size_t c_theta_bak = 0, c_est_bak = 0;
    bool prep_reordered = false;
    // the next fresh order, computed on a worker thread from a snapshot of the graph taken
    // bg_lead() nodes before it is due, then extended by the nodes and pairs that arrived since
    struct BgOrder {
        int64_t n = 0, n_pairs = 0;
        int rc = 0;
        std::vector<int32_t> perm;
        std::vector<std::vector<int32_t>> pat;
    };
    std::future<BgOrder> bg;
    const char* prep_msg = "";                 // its failure message
    double prep_ms[3] = {};                    // its incsym, derive, chol plan times
    std::unique_ptr<dpg_inc_helper> helper;    // the plan's H-block buckets beside the derivation
    std::vector<int32_t> dirty;                // the update's dirty nodes (partial refactorization)
    double prof[12] = {};                      // last update: incsym, derive, lists, chol build, chol host,
                                               // chol upload (ms); factor Mflop, largest front (blocks),
                                               // fused DAG path (1) or level path (0), supernodes, levels,
                                               // host ms of the partial refactorization's pick + launches
};

namespace {

// contribution lists (lin_gather_kernel) of every upper block, in factor order, and the device copies.
// The factor list only grows between resets (a failed update truncates it again), so without Q1
// scaling only the factors the device does not hold yet go up; the lists are rebuilt (a new factor
// lands in the middle of the CSR) straight into a pinned staging buffer and copied without a
// synchronisation -- the next rebuild comes after this update's fetch.
int inc_rebuild_lists(dpg_inc* q, hipStream_t s) {
    dpg_gn_dev& g = q->g;
    const int64_t n = q->V, nf = (int64_t)q->F.size(), P = (int64_t)q->plo.size();
    const int64_t nu = n + P;
    int64_t n_list = 0;
    for (int64_t k = 0; k < nf; ++k) n_list += q->F[(size_t)k].kind == DPG_FACTOR_BETWEEN ? 3 : 1;
    // the last rebuild's copies out of the staging buffer must be done before it is rewritten
    if (q->lists_ev_set && hipEventSynchronize(q->lists_ev) != hipSuccess) return DPG_ERR_HIP;
    const size_t need = (size_t)(nu + 1 + n_list);
    if (need > q->c_lists) {
        const size_t nc = std::max(need, q->c_lists + q->c_lists / 2) + 4096;
        if (q->h_lists) {
            (void)hipHostFree(q->h_lists);
            q->h_lists = nullptr;
            q->c_lists = 0;
        }
        if (hipHostMalloc(reinterpret_cast<void**>(&q->h_lists), nc * sizeof(int32_t)) != hipSuccess) return DPG_ERR_HIP;
        q->c_lists = nc;
    }
    int32_t* cnt = q->h_lists;
    int32_t* clist = q->h_lists + nu + 1;
    std::fill(cnt, cnt + nu + 1, 0);
    for (int64_t k = 0; k < nf; ++k) {
        const dpg_factor& f = q->F[(size_t)k];
        cnt[(size_t)f.i + 1]++;
        if (f.kind == DPG_FACTOR_BETWEEN) {
            cnt[(size_t)f.j + 1]++;
            cnt[(size_t)(n + q->f_pair[(size_t)k]) + 1]++;
        }
    }
    for (int64_t u = 0; u < nu; ++u) cnt[(size_t)u + 1] += cnt[(size_t)u];
    std::vector<int32_t> cur(cnt, cnt + nu);
    for (int64_t k = 0; k < nf; ++k) {
        const dpg_factor& f = q->F[(size_t)k];
        clist[(size_t)cur[(size_t)f.i]++] = (int32_t)(k << 2 | 0);
        if (f.kind == DPG_FACTOR_BETWEEN) {
            clist[(size_t)cur[(size_t)f.j]++] = (int32_t)(k << 2 | 1);
            clist[(size_t)cur[(size_t)(n + q->f_pair[(size_t)k])]++] = (int32_t)(k << 2 | (f.i < f.j ? 2 : 3));
        }
    }
    g.n_nodes = n;
    g.n_factors = nf;
    g.nnzb_upper = nu;
    g.shard_begin = 0;
    g.shard_end = nf;
    g.n_blocks_rows = (int32_t)nblk(n);
    const int64_t keep = q->P.duplicate_factors ? 0 : std::min(q->n_dev_f, nf);
    int rc = 0;
    rc |= dgrow(&g.factors, &q->c_factors, (size_t)nf, s, (size_t)keep);
    rc |= dgrow(&g.up_cptr, &q->c_cptr, (size_t)(nu + 1), s, 0);
    rc |= dgrow(&g.up_clist, &q->c_clist, (size_t)n_list, s, 0);
    rc |= dgrow(&g.hb_own, &q->c_hb, (size_t)(9 * nu + 3 * n + 2), s, 0);
    rc |= dgrow(&g.partials, &q->c_partials, (size_t)(6 * g.n_blocks_rows + n), s, 0);
    if (!g.scal3) {
        rc |= hipMalloc(reinterpret_cast<void**>(&g.scal3), 4 * sizeof(double)) != hipSuccess;
        if (!rc) rc |= hipHostMalloc(reinterpret_cast<void**>(&g.scal3_host), 4 * sizeof(double)) != hipSuccess;
    }
    if (rc) return DPG_ERR_HIP;
    if (q->P.duplicate_factors) {   // factors as the device sees them: Q1 multiplicity folded into the information
        q->h_dev_factors = q->F;
        for (int64_t k = 0; k < nf; ++k) {
            const double mult = (double)(q->updates - q->f_created[(size_t)k] + 1);
            for (int c = 0; c < 3; ++c) q->h_dev_factors[(size_t)k].info[c] *= mult;
        }
        if (nf && hipMemcpyAsync(g.factors, q->h_dev_factors.data(), sizeof(dpg_factor) * (size_t)nf,
                                 hipMemcpyHostToDevice, s) != hipSuccess)
            return DPG_ERR_HIP;
    } else if (nf > keep) {
        // pageable source: the copy is staged before the call returns, and q->F changes only later
        if (hipMemcpyAsync(g.factors + keep, q->F.data() + keep, sizeof(dpg_factor) * (size_t)(nf - keep),
                           hipMemcpyHostToDevice, s) != hipSuccess)
            return DPG_ERR_HIP;
    }
    q->n_dev_f = q->P.duplicate_factors ? 0 : nf;
    if (hipMemcpyAsync(g.up_cptr, cnt, sizeof(int32_t) * (size_t)(nu + 1), hipMemcpyHostToDevice, s) != hipSuccess)
        return DPG_ERR_HIP;
    if (n_list && hipMemcpyAsync(g.up_clist, clist, sizeof(int32_t) * (size_t)n_list, hipMemcpyHostToDevice, s) != hipSuccess)
        return DPG_ERR_HIP;
    if (!q->lists_ev && hipEventCreateWithFlags(&q->lists_ev, hipEventDisableTiming) != hipSuccess) return DPG_ERR_HIP;
    if (hipEventRecord(q->lists_ev, s) != hipSuccess) return DPG_ERR_HIP;
    q->lists_ev_set = true;
    return DPG_OK;
}

// the Cholesky structures planned by the prepare go up
int inc_rebuild_chol(dpg_inc* q) {
    dpg_gn_dev& g = q->g;
    const double t = now_ms();
    const int rc2 = dpg_chol_create_sym_upload(&g.chol);   // planned by inc_prepare
    q->prof[3] = now_ms() - t + q->prep_ms[2];
    if (!rc2) {
        dpg_chol_build_times(g.chol, q->prof + 4);
        double st[6];
        dpg_chol_stats(g.chol, st);
        q->prof[6] = st[3] * 1e-6;
        q->prof[7] = st[2];
        q->prof[8] = dpg_chol_fused(g.chol);
        q->prof[9] = st[0];
        q->prof[10] = st[1];
    }
    return rc2;
}

int inc_rebuild(dpg_inc* q, hipStream_t s) {
    const int rc = inc_rebuild_lists(q, s);
    return rc ? rc : inc_rebuild_chol(q);
}

int set_err(int code, const char* msg) { return dpg_set_error(code, msg); }

void bg_discard(dpg_inc* q) {
    if (q->bg.valid()) (void)q->bg.get();   // joins the worker
}

}  // namespace

extern "C" {

void dpg_inc_params_default(dpg_inc_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->mode = DPG_INC_ISAM2;
    p->relinearize_skip = 10;
    p->relinearize_threshold = 0.1;
    p->duplicate_factors = 0;
    p->reorder_every = 32;
    p->reorder_lead = 8;
    dpg_gn_params_default(&p->gn);
}

dpg_inc* dpg_inc_create(dpg_ctx* ctx, const dpg_inc_params* p) {
    if (!ctx) {
        set_err(DPG_ERR_ARG, "dpg_inc_create: ctx is NULL");
        return nullptr;
    }
    if (dpg_ctx_num_gpus(ctx) != 1 || dpg_ctx_is_multi(ctx)) {
        set_err(DPG_ERR_ARG, "dpg_inc_create: the incremental graph needs a single-device context (dpg_ctx_create)");
        return nullptr;
    }
    dpg_inc* q = new dpg_inc();
    q->ctx = ctx;
    if (p) q->P = *p;
    else dpg_inc_params_default(&q->P);
    if (q->P.relinearize_skip < 1) q->P.relinearize_skip = 1;
    if (q->P.reorder_every < 1) q->P.reorder_every = 1;
    if (q->P.reorder_lead < 0 || q->P.reorder_lead >= q->P.reorder_every) q->P.reorder_lead = 0;
    q->opts = *dpg_ctx_chol_opts(ctx);   // the context's solver options
    q->P.gn.linear_solver = DPG_SOLVER_CHOLESKY;
    dpg_ctx_adopt(ctx, q, [](void* x) { dpg_inc_destroy(static_cast<dpg_inc*>(x)); });
    return q;
}

int dpg_inc_reset(dpg_inc* q) {
    if (!q) return set_err(DPG_ERR_ARG, "dpg_inc_reset: NULL");
    bg_discard(q);
    q->V = 0;
    q->updates = 0;
    q->F.clear();
    q->n_dev_f = 0;
    q->f_created.clear();
    q->f_pair.clear();
    q->pair_id.clear();
    q->plo.clear();
    q->phi.clear();
    q->I = dpg_chol_incsym();
    q->V_at_order = q->nnz_at_order = 0;
    q->prepared = false;
    q->prep_new = 0;
    q->prep_pairs0 = 0;
    if (q->g.chol) dpg_chol_forget_factor(q->g.chol);
    return DPG_OK;
}

// Undo the structural half of an update that will not happen (its alignments failed, or its
// numeric update failed): the pairs it added leave the pattern and the symbolic state is dropped,
// so the next prepare orders the graph afresh from the pairs that remain.
int dpg_inc_abort_prepare(dpg_inc* q) {
    if (!q) return set_err(DPG_ERR_ARG, "dpg_inc_abort_prepare: NULL");
    if (!q->prepared) return DPG_OK;
    bg_discard(q);   // its snapshot may hold the pairs that leave now; the next prepare reorders anyway
    for (size_t k = (size_t)q->prep_pairs0; k < q->plo.size(); ++k) q->pair_id.erase(pkey(q->plo[k], q->phi[k]));
    q->plo.resize((size_t)q->prep_pairs0);
    q->phi.resize((size_t)q->prep_pairs0);
    q->I = dpg_chol_incsym();
    q->V_at_order = q->nnz_at_order = 0;
    q->prepared = false;
    q->prep_new = 0;
    if (q->g.chol) dpg_chol_forget_factor(q->g.chol);
    return DPG_OK;
}

void dpg_inc_destroy(dpg_inc* q) {
    if (!q) return;
    dpg_ctx_release_child(q->ctx, q);
    hipStream_t s = reinterpret_cast<hipStream_t>(dpg_ctx_stream_of(q->ctx));
    (void)hipStreamSynchronize(s);
    void* ptrs[] = {q->g.factors, q->g.up_cptr, q->g.up_clist, q->g.hb_own, q->g.partials, q->g.scal3,
                    q->theta, q->est, q->maxd, q->cnt, q->est_nxt, q->maxd_nxt, q->theta_bak, q->est_bak};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (q->g.scal3_host) (void)hipHostFree(q->g.scal3_host);
    if (q->h_lists) (void)hipHostFree(q->h_lists);
    if (q->lists_ev) (void)hipEventDestroy(q->lists_ev);
    if (q->g.chol) dpg_chol_destroy(q->g.chol);
    delete q;
}

int64_t dpg_inc_num_nodes(const dpg_inc* q) { return q ? q->V : -1; }

// diagnostics: host-time breakdown (ms) of the last update's symbolic phase -- incremental
// symbolic state, derived structures, contribution lists + factor upload, GPU solver structures
int dpg_inc_last_profile(const dpg_inc* q, double* out, int n) {
    if (!q || !out) return DPG_ERR_ARG;
    for (int k = 0; k < n && k < 12; ++k) out[k] = q->prof[k];
    return DPG_OK;
}
dpg_ctx* dpg_inc_ctx(dpg_inc* q) { return q ? q->ctx : nullptr; }

// diagnostics: the graph's unique node pairs in arrival order (lo < hi); returns their number and
// copies min(n, number) of them when lo / hi are given
int64_t dpg_inc_pairs(const dpg_inc* q, int32_t* lo, int32_t* hi, int64_t n) {
    if (!q) return -1;
    const int64_t P = (int64_t)q->plo.size();
    if (lo && hi)
        for (int64_t k = 0; k < P && k < n; ++k) { lo[k] = q->plo[(size_t)k]; hi[k] = q->phi[(size_t)k]; }
    return P;
}

// The structural half of the next update (host only, no device call): n_new nodes join, the node
// pairs (a_k, b_k) enter the pattern (a superset of the coming Between factors' pairs is fine: a
// pair without factors is an explicit zero block), the symbolic analysis is extended or redone and
// the Cholesky planned.  dpg_add_node_pairs runs it while the GPU aligns the node's edges; the
// next dpg_inc_update (for the same n_new) uploads the plan and solves.
}  // extern "C"

namespace {

// The structural half of an update, in two parts.  prep_pairs (calling thread): validation, and
// the update's new node pairs enter the pattern (pair ids in arrival order).  prep_symbolic: the
// order extended or refreshed, the derived structures and the Cholesky plan -- host only; it touches
// the symbolic state (I, S, the plan inside g.chol, the ordering bookkeeping) and nothing the
// numeric half of the update reads, so dpg_add_node_pairs runs it while the GPU aligns the node's
// edges.  It reports failures through its return code and prep_msg; the caller aborts the prepare.
int prep_pairs(dpg_inc* q, int64_t n_new, const int32_t* pairs, int64_t n_pairs,
               std::vector<std::pair<int32_t, int32_t>>& new_pairs) {
    if (!q || n_new < 0 || n_pairs < 0 || (n_pairs > 0 && !pairs)) return set_err(DPG_ERR_ARG, "dpg_inc_prepare: bad arguments");
    const int64_t V1 = q->V + n_new;
    for (int64_t e = 0; e < n_pairs; ++e)
        if (pairs[2 * e] < 0 || pairs[2 * e + 1] < 0 || pairs[2 * e] >= V1 || pairs[2 * e + 1] >= V1 ||
            pairs[2 * e] == pairs[2 * e + 1])
            return set_err(DPG_ERR_ARG, "dpg_inc_prepare: a pair references a missing node");
    if (V1 == 0) return set_err(DPG_ERR_STATE, "dpg_inc_prepare: empty graph");
    if (q->prepared) return set_err(DPG_ERR_STATE, "dpg_inc_prepare: an update is already prepared");
    q->prep_pairs0 = (int64_t)q->plo.size();
    new_pairs.clear();
    for (int64_t e = 0; e < n_pairs; ++e) {
        const int32_t lo = std::min(pairs[2 * e], pairs[2 * e + 1]), hi = std::max(pairs[2 * e], pairs[2 * e + 1]);
        if (q->pair_id.find(pkey(lo, hi)) == q->pair_id.end()) {
            q->pair_id.emplace(pkey(lo, hi), (int32_t)q->plo.size());
            q->plo.push_back(lo);
            q->phi.push_back(hi);
            new_pairs.emplace_back(lo, hi);
        }
    }
    q->prep_new = n_new;
    q->prepared = true;
    return DPG_OK;
}

int prep_symbolic(dpg_inc* q, int64_t V1, int64_t n_new, const std::vector<std::pair<int32_t, int32_t>>& new_pairs) {
    const double t1 = now_ms();
    if (q->I.n > 0) dpg_incsym_append(&q->I, n_new);
    // ordering: extended, or fresh every reorder_every nodes / after 1.5x fill growth
    // (the order due every reorder_every nodes comes from the worker thread when one was started
    // for it: the snapshot's order, the nodes since appended at its end and the pairs since added,
    // as between reorders)
    bool reordered = false, from_bg = false;
    const double expect = q->V_at_order > 0 ? (double)q->nnz_at_order * (double)V1 / (double)q->V_at_order : 0.0;
    if (q->I.n == 0 || V1 - q->V_at_order >= q->P.reorder_every) {
        reordered = true;
        from_bg = q->I.n > 0 && q->bg.valid();
    } else {
        for (auto& pr : new_pairs) dpg_incsym_add_edge(&q->I, pr.first, pr.second);
        if ((double)q->I.nnz > 1.5 * expect + 64.0) reordered = true;
    }
    if (from_bg) {
        dpg_inc::BgOrder r = q->bg.get();
        if (r.rc || r.n > V1 || r.n_pairs > (int64_t)q->plo.size()) {
            from_bg = false;
        } else {
            dpg_incsym_init(&q->I, r.n, r.perm, r.pat);
            dpg_incsym_append(&q->I, V1 - r.n);
            for (int64_t k = r.n_pairs; k < (int64_t)q->plo.size(); ++k) dpg_incsym_add_edge(&q->I, q->plo[(size_t)k], q->phi[(size_t)k]);
        }
    }
    if (reordered && !from_bg) {
        bg_discard(q);
        if (dpg_incsym_reset(&q->I, V1, q->plo.data(), q->phi.data(), (int64_t)q->plo.size(), &q->opts)) {
            q->prep_msg = "dpg_inc_prepare: symbolic analysis failed";
            return DPG_ERR_NUMERIC;
        }
    }
    if (reordered) {
        q->V_at_order = V1;
        q->nnz_at_order = q->I.nnz;
        q->reorders += 1;
    }
    if (q->P.reorder_lead > 0 && !q->bg.valid() && V1 >= 256 && V1 - q->V_at_order >= q->P.reorder_every - q->P.reorder_lead) {
        const int64_t P = (int64_t)q->plo.size();
        std::vector<int32_t> lo(q->plo), hi(q->phi);
        q->bg = std::async(std::launch::async, [V1, P, lo = std::move(lo), hi = std::move(hi), o = q->opts]() {
            dpg_inc::BgOrder r;
            r.n = V1;
            r.n_pairs = P;
            r.rc = dpg_incsym_order(V1, lo.data(), hi.data(), P, r.perm, r.pat, &o);
            return r;
        });
    }
    const double t1a = now_ms();
    // the plan's first part needs only the order (I's, which the derivation copies into S) and the
    // pairs: on the helper thread while this one derives the column patterns and supernodes
    const bool ahead = V1 >= 256;
    int hrc = DPG_OK;
    if (ahead) {
        if (!q->helper) q->helper.reset(new dpg_inc_helper());
        q->helper->post([q, V1, &hrc] {
            hrc = dpg_chol_plan_blocks(&q->g.chol, V1, q->I.pos.data(), q->I.perm.data(), q->plo.data(), q->phi.data(),
                                       (int64_t)q->plo.size());
        });
    }
    const int drc = dpg_incsym_derive(&q->I, &q->opts, &q->S);
    if (ahead) q->helper->wait();
    // buckets built for a derivation that failed (or a helper that failed) must not reach a later
    // plan of the same size: the plan then builds its own
    if (ahead && (drc || hrc)) dpg_chol_blocks_invalidate(q->g.chol);
    if (drc) {
        q->prep_msg = "dpg_inc_prepare: symbolic derivation failed";
        return DPG_ERR_NUMERIC;
    }
    const double t1b = now_ms();
    const int rc = dpg_chol_create_sym_plan(&q->g.chol, V1, q->plo.data(), q->phi.data(), (int64_t)q->plo.size(), &q->S,
                                            &q->opts);
    if (rc) {
        q->prep_msg = "dpg_inc_prepare: Cholesky plan failed";
        return rc;
    }
    q->prep_ms[0] = t1a - t1;
    q->prep_ms[1] = t1b - t1a;
    q->prep_ms[2] = now_ms() - t1b;
    q->prep_reordered = reordered;
    return DPG_OK;
}

}  // namespace

extern "C" {

int dpg_inc_prepare(dpg_inc* q, int64_t n_new, const int32_t* pairs, int64_t n_pairs) {
    std::vector<std::pair<int32_t, int32_t>> new_pairs;
    int rc = prep_pairs(q, n_new, pairs, n_pairs, new_pairs);
    if (rc) return rc;
    if ((rc = prep_symbolic(q, q->V + n_new, n_new, new_pairs))) {
        const char* msg = q->prep_msg;
        dpg_inc_abort_prepare(q);
        return set_err(rc, msg);
    }
    return DPG_OK;
}

int dpg_inc_update(dpg_inc* q, int64_t n_new, const double* init, const dpg_factor* factors, int64_t n_factors,
                   dpg_inc_stats* st) {
    if (!q || n_new < 0 || n_factors < 0 || (n_new > 0 && !init) || (n_factors > 0 && !factors))
        return set_err(DPG_ERR_ARG, "dpg_inc_update: bad arguments");
    const double t0 = now_ms();
    hipStream_t s = reinterpret_cast<hipStream_t>(dpg_ctx_stream_of(q->ctx));
    if (hipSetDevice(dpg_ctx_device_of(q->ctx)) != hipSuccess) return set_err(DPG_ERR_HIP, "hipSetDevice failed");
    const int64_t V0 = q->V, V1 = V0 + n_new;
    // validate before touching any state
    for (int64_t k = 0; k < n_factors; ++k) {
        const dpg_factor& f = factors[k];
        const bool ok = (f.kind == DPG_FACTOR_PRIOR && f.i >= 0 && f.i < V1) ||
                        (f.kind == DPG_FACTOR_BETWEEN && f.i >= 0 && f.j >= 0 && f.i < V1 && f.j < V1 && f.i != f.j);
        if (!ok) return set_err(DPG_ERR_ARG, "dpg_inc_update: a factor references a missing node");
    }
    if (V1 == 0) return set_err(DPG_ERR_STATE, "dpg_inc_update: empty graph");
    // device state for the new nodes (theta and the estimate start at the initial values)
    int rc = 0;
    rc |= dgrow(&q->theta, &q->c_theta, (size_t)(3 * V1), s, (size_t)(3 * V0));
    rc |= dgrow(&q->est, &q->c_est, (size_t)(3 * V1), s, (size_t)(3 * V0));
    rc |= dgrow(&q->maxd, &q->c_maxd, (size_t)V1, s, (size_t)V0);
    if (!q->cnt) rc |= hipMalloc(reinterpret_cast<void**>(&q->cnt), sizeof(int32_t)) != hipSuccess;
    if (rc) return set_err(DPG_ERR_HIP, "dpg_inc_update: out of device memory");
    if (n_new > 0) {
        if (hipMemcpyAsync(q->theta + 3 * V0, init, sizeof(double) * 3 * (size_t)n_new, hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipMemcpyAsync(q->est + 3 * V0, init, sizeof(double) * 3 * (size_t)n_new, hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipMemsetAsync(q->maxd + V0, 0, sizeof(double) * (size_t)n_new, s) != hipSuccess)
            return set_err(DPG_ERR_HIP, "dpg_inc_update: upload failed");
    }
    // graph + symbolic state: the pairs of this update's Between factors are in the pattern already
    // when dpg_add_node_pairs prepared it while its alignments ran, else prepare them now
    if (!q->prepared) {
        std::vector<int32_t> pr;
        pr.reserve((size_t)(2 * n_factors));
        for (int64_t k = 0; k < n_factors; ++k)
            if (factors[k].kind == DPG_FACTOR_BETWEEN) { pr.push_back(factors[k].i); pr.push_back(factors[k].j); }
        if ((rc = dpg_inc_prepare(q, n_new, pr.data(), (int64_t)pr.size() / 2))) return rc;
    } else if (q->prep_new != n_new) {
        dpg_inc_abort_prepare(q);
        return set_err(DPG_ERR_STATE, "dpg_inc_update: prepared for another number of new nodes");
    }
    // ISAM2::update counts the update first, then relinearizes when the count is a multiple of
    // relinearizeSkip (updates 10, 20, ...)
    const bool relin = q->P.mode == DPG_INC_ISAM2 && ((q->updates + 1) % q->P.relinearize_skip) == 0 && V0 > 0;
    // every pair of this update's Between factors must be in the prepared pattern
    for (int64_t k = 0; k < n_factors; ++k)
        if (factors[k].kind == DPG_FACTOR_BETWEEN &&
            q->pair_id.find(pkey(std::min(factors[k].i, factors[k].j), std::max(factors[k].i, factors[k].j))) ==
                q->pair_id.end()) {
            dpg_inc_abort_prepare(q);
            return set_err(DPG_ERR_STATE, "dpg_inc_update: a factor's pair was not prepared");
        }
    // from here the update commits; any failure below rolls the graph back to its state before the
    // call (factors, node count, update count, the pairs this update added, theta and the estimate)
    const int64_t nF0 = (int64_t)q->F.size(), upd0 = q->updates;
    q->prepared = false;
    q->updates += 1;
    q->V = V1;
    for (int64_t k = 0; k < n_factors; ++k) {
        const dpg_factor& f = factors[k];
        const int32_t pid = f.kind == DPG_FACTOR_BETWEEN ? q->pair_id[pkey(std::min(f.i, f.j), std::max(f.i, f.j))] : -1;
        q->F.push_back(f);
        q->f_created.push_back((int32_t)q->updates);
        q->f_pair.push_back(pid);
    }
    bool theta_saved = false, est_saved = false;
    auto rollback = [&](int code, const char* msg) -> int {
        (void)hipStreamSynchronize(s);
        if (q->g.chol) dpg_chol_forget_factor(q->g.chol);
        q->F.resize((size_t)nF0);
        q->n_dev_f = std::min(q->n_dev_f, nF0);
        q->f_created.resize((size_t)nF0);
        q->f_pair.resize((size_t)nF0);
        q->V = V0;
        q->updates = upd0;
        q->prepared = true;   // the pairs this update added leave the pattern
        dpg_inc_abort_prepare(q);
        if (theta_saved) (void)hipMemcpy(q->theta, q->theta_bak, sizeof(double) * 3 * (size_t)V0, hipMemcpyDeviceToDevice);
        if (est_saved) (void)hipMemcpy(q->est, q->est_bak, sizeof(double) * 3 * (size_t)V0, hipMemcpyDeviceToDevice);
        return set_err(code, msg);
    };
    // the contribution lists (and their copies on s) on the graph's helper thread while this one
    // uploads the Cholesky's plan: disjoint state (the lists and assembly buffers / g.chol)
    const double t1b = now_ms();
    int lrc = DPG_OK;
    double lists_ms = 0.0;
    if (q->helper) {
        q->helper->post([q, s, &lrc, &lists_ms] {
            const double t = now_ms();
            lrc = inc_rebuild_lists(q, s);
            lists_ms = now_ms() - t;
        });
    } else {
        lrc = inc_rebuild_lists(q, s);
        lists_ms = now_ms() - t1b;
    }
    rc = inc_rebuild_chol(q);
    if (q->helper) q->helper->wait();
    q->prof[2] = lists_ms;
    if (lrc) return rollback(lrc, "dpg_inc_update: contribution lists failed");
    if (rc) return rollback(rc, "dpg_inc_update: solver rebuild failed");
    // the solver remembers its factorization's analysis for the next update's partial refactorization
    // (ISAM2 updates without the Q1 information scaling, which changes every block every update)
    dpg_chol_track_factor(q->g.chol, q->P.mode == DPG_INC_ISAM2 && q->P.full_refactor == 0 && !q->P.duplicate_factors);
    const double t2 = now_ms();
    dpg_inc_stats S;
    memset(&S, 0, sizeof(S));
    if (q->P.mode == DPG_INC_ISAM2) {
        // 1. relinearize the variables whose delta passed the threshold (before the new factors)
        if (relin) {
            if (dgrow(&q->theta_bak, &q->c_theta_bak, (size_t)(3 * V0), s, 0) ||
                hipMemcpyAsync(q->theta_bak, q->theta, sizeof(double) * 3 * (size_t)V0, hipMemcpyDeviceToDevice, s) !=
                    hipSuccess)
                return rollback(DPG_ERR_HIP, "dpg_inc_update: theta snapshot failed");
            theta_saved = true;
            if (hipMemsetAsync(q->cnt, 0, sizeof(int32_t), s) != hipSuccess) return rollback(DPG_ERR_HIP, "memset");
            hipLaunchKernelGGL(inc_relin_kernel, dim3(nblk(V0)), dim3(kThreads), 0, s, q->theta, q->est, q->maxd, V0,
                               q->P.relinearize_threshold, q->cnt);
        }
        // 2. linearize everything at theta, factor, solve, estimate = theta (+) delta (into the
        //    spare buffers: the current estimate stays intact until the solve is known good)
        if (dgrow(&q->est_nxt, &q->c_est_nxt, (size_t)(3 * V1), s, 0) || dgrow(&q->maxd_nxt, &q->c_maxd_nxt, (size_t)V1, s, 0))
            return rollback(DPG_ERR_HIP, "dpg_inc_update: out of device memory");
        q->g.poses = q->theta;
        if ((rc = dpg_gn_dev_assemble(&q->g, q->g.hb_own, s))) return rollback(rc, "assembly failed");
        // isam_->update's partial re-elimination: between reorders and relinearizations every H
        // block is the same sum at the same theta unless a new factor or pair touches its nodes, so
        // the fronts off the new nodes' and factors' paths to the root keep their factors
        // (dpg_chol_solve_partial; bit-identical to refactoring every front)
        const bool partial = q->P.full_refactor == 0 && !relin && !q->prep_reordered && V0 > 0;
        if (partial) {
            std::vector<int32_t>& dirty = q->dirty;
            dirty.clear();
            for (int64_t v = V0; v < V1; ++v) dirty.push_back((int32_t)v);
            for (int64_t k = 0; k < n_factors; ++k) {
                dirty.push_back(factors[k].i);
                if (factors[k].kind == DPG_FACTOR_BETWEEN) dirty.push_back(factors[k].j);
            }
            for (size_t k = (size_t)q->prep_pairs0; k < q->plo.size(); ++k) {
                dirty.push_back(q->plo[k]);
                dirty.push_back(q->phi[k]);
            }
            rc = dpg_chol_solve_partial(q->g.chol, q->g.hb_own, dirty.data(), (int64_t)dirty.size(), s);
        } else {
            rc = dpg_chol_solve(q->g.chol, q->g.hb_own, s);
        }
        if (rc) return rollback(rc, "Cholesky launch failed");
        {
            int64_t pst[4];
            dpg_chol_partial_stats(q->g.chol, pst);
            S.fronts_kept = (int32_t)pst[1];
            q->prof[11] = (double)pst[3] * 1e-6;
        }
        if (hipMemsetAsync(q->g.scal3, 0, sizeof(double), s) != hipSuccess) return rollback(DPG_ERR_HIP, "memset");
        hipLaunchKernelGGL(inc_estimate_kernel, dim3(nblk(V1)), dim3(kThreads), 0, s, q->theta, dpg_chol_x_dev(q->g.chol),
                           dpg_chol_pos_dev(q->g.chol), V1, q->est_nxt, q->maxd_nxt, q->g.scal3);
        double sc[3];
        q->g.last_used_chol = 1;
        if ((rc = dpg_gn_dev_fetch(&q->g, q->g.hb_own, s, sc))) return rollback(rc, "fetch failed");
        if (sc[2] != 0.0) return rollback(DPG_ERR_NUMERIC, "dpg_inc_update: Cholesky failed (H not positive definite)");
        // every read that can fail before the commit: a failure rolls the whole update back
        int32_t nrel = 0;
        if (relin && hipMemcpy(&nrel, q->cnt, sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
            return rollback(DPG_ERR_HIP, "dpg_inc_update: relinearized-count read-back failed");
        std::swap(q->est, q->est_nxt);
        std::swap(q->c_est, q->c_est_nxt);
        std::swap(q->maxd, q->maxd_nxt);
        std::swap(q->c_maxd, q->c_maxd_nxt);
        S.relinearized = nrel;
        S.gn_iterations = 1;
        S.error = sc[1];
        S.last_delta_inf = sc[0];
    } else {
        // batch Gauss-Newton to convergence from the current estimates
        q->g.poses = q->est;
        q->g.have_factor = 0;
        q->g.last_delta_inf = 1e300;
        q->g.prev_delta_inf = 1e300;
        q->g.last_was_chord = 0;
        q->g.n_factorizations = 0;
        const dpg_gn_params& gp = q->P.gn;
        double sc[3] = {0, 0, 0};
        int it = 0;
        if (V0 > 0) {
            if (dgrow(&q->est_bak, &q->c_est_bak, (size_t)(3 * V0), s, 0) ||
                hipMemcpyAsync(q->est_bak, q->est, sizeof(double) * 3 * (size_t)V0, hipMemcpyDeviceToDevice, s) != hipSuccess)
                return rollback(DPG_ERR_HIP, "dpg_inc_update: estimate snapshot failed");
            est_saved = true;
        }
        if ((rc = dpg_gn_dev_assemble(&q->g, q->g.hb_own, s))) return rollback(rc, "assembly failed");
        for (; it < gp.max_iterations;) {
            if ((rc = dpg_gn_dev_solve_async(&q->g, q->g.hb_own, &gp, s)) ||
                (rc = dpg_gn_dev_assemble(&q->g, q->g.hb_own, s)) || (rc = dpg_gn_dev_fetch(&q->g, q->g.hb_own, s, sc)))
                return rollback(rc, "Gauss-Newton step failed");
            if (sc[2] != 0.0) return rollback(DPG_ERR_NUMERIC, "dpg_inc_update: Cholesky failed");
            ++it;
            if (sc[0] < gp.delta_tol) break;
        }
        // theta follows the estimate (a batch solve relinearizes everything)
        if (hipMemcpyAsync(q->theta, q->est, sizeof(double) * 3 * (size_t)V1, hipMemcpyDeviceToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return set_err(DPG_ERR_HIP, "copy failed");
        S.gn_iterations = it;
        S.error = sc[1];
        S.last_delta_inf = sc[0];
    }
    const double t3 = now_ms();
    S.reordered = q->prep_reordered ? 1 : 0;
    q->prof[0] = q->prep_ms[0];
    q->prof[1] = q->prep_ms[1];
    S.n_nodes = V1;
    S.n_factors = (int64_t)q->F.size();
    S.nnz_l = q->I.nnz;
    S.ms_total = t3 - t0;
    S.ms_symbolic = t2 - t1b + q->prep_ms[0] + q->prep_ms[1] + q->prep_ms[2];
    S.ms_numeric = t3 - t2;
    if (st) *st = S;
    return DPG_OK;
}

// ---- graph checkpoint (the reference's state -- dpg_nodes_ and their scans,
// graph_, isam_ (dpg_slam.h:362,367,372) -- lives only in memory) ----
// File layout (host byte order, every field fixed-width):
//   CkptHeader; dpg_factor F[n_factors]; int32 f_created[n_factors]; int32 plo[n_pairs], phi[n_pairs];
//   double theta[3 V], est[3 V], maxd[V]; int64 scan_off[n_scans + 1]; float scan_pts[scan_off[n_scans]][2]
// The pairs keep their arrival order (a non-converged loop closure's pair stays an explicit zero
// block); the scans are the full base_link clouds of the context's store.
struct CkptHeader {
    char magic[8];                   // "DPGGRAPH"
    uint32_t version, sizeof_factor, sizeof_params, pad;
    dpg_inc_params params;
    int64_t V, updates, n_factors, n_pairs, n_scans;
    int32_t ratio, pad2;
};
constexpr uint32_t kCkptVersion = 1;

int dpg_inc_save(dpg_inc* q, const char* path) {
    if (!q || !path) return set_err(DPG_ERR_ARG, "dpg_inc_save: bad arguments");
    if (q->prepared) return set_err(DPG_ERR_STATE, "dpg_inc_save: an update is prepared but not applied");
    CkptHeader h;
    memset(&h, 0, sizeof(h));
    memcpy(h.magic, "DPGGRAPH", 8);
    h.version = kCkptVersion;
    h.sizeof_factor = (uint32_t)sizeof(dpg_factor);
    h.sizeof_params = (uint32_t)sizeof(dpg_inc_params);
    h.params = q->P;
    h.V = q->V;
    h.updates = q->updates;
    h.n_factors = (int64_t)q->F.size();
    h.n_pairs = (int64_t)q->plo.size();
    int rc = dpg_scans_export(q->ctx, &h.n_scans, &h.ratio, nullptr, nullptr);
    if (rc) return rc;
    // the store belongs to the graph when it holds the graph's nodes (the dpg_add_node path); a
    // graph fed by dpg_inc_update alone is saved without scans (the context may hold any others)
    if (h.n_scans < h.V) h.n_scans = 0;
    const size_t V = (size_t)h.V;
    std::vector<double> theta(3 * V), est(3 * V), maxd(V);
    hipStream_t s = reinterpret_cast<hipStream_t>(dpg_ctx_stream_of(q->ctx));
    if (hipSetDevice(dpg_ctx_device_of(q->ctx)) != hipSuccess) return set_err(DPG_ERR_HIP, "hipSetDevice failed");
    if (V && (hipMemcpyAsync(theta.data(), q->theta, sizeof(double) * 3 * V, hipMemcpyDeviceToHost, s) != hipSuccess ||
              hipMemcpyAsync(est.data(), q->est, sizeof(double) * 3 * V, hipMemcpyDeviceToHost, s) != hipSuccess ||
              hipMemcpyAsync(maxd.data(), q->maxd, sizeof(double) * V, hipMemcpyDeviceToHost, s) != hipSuccess))
        return set_err(DPG_ERR_HIP, "dpg_inc_save: read-back failed");
    if (hipStreamSynchronize(s) != hipSuccess) return set_err(DPG_ERR_HIP, "dpg_inc_save: read-back failed");
    std::vector<int64_t> off((size_t)h.n_scans + 1, 0);
    std::vector<float> pts(2);
    if (h.n_scans > 0) {
        if ((rc = dpg_scans_export(q->ctx, &h.n_scans, &h.ratio, off.data(), nullptr))) return rc;
        pts.resize((size_t)(2 * std::max<int64_t>(off[(size_t)h.n_scans], 1)));
        if ((rc = dpg_scans_export(q->ctx, &h.n_scans, &h.ratio, off.data(), pts.data()))) return rc;
    }
    FILE* f = fopen(path, "wb");
    if (!f) return set_err(DPG_ERR_ARG, "dpg_inc_save: cannot open the file for writing");
    bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
    auto put = [&](const void* p, size_t bytes) { if (ok && bytes) ok = fwrite(p, 1, bytes, f) == bytes; };
    put(q->F.data(), sizeof(dpg_factor) * q->F.size());
    put(q->f_created.data(), sizeof(int32_t) * q->f_created.size());
    put(q->plo.data(), sizeof(int32_t) * q->plo.size());
    put(q->phi.data(), sizeof(int32_t) * q->phi.size());
    put(theta.data(), sizeof(double) * theta.size());
    put(est.data(), sizeof(double) * est.size());
    put(maxd.data(), sizeof(double) * maxd.size());
    put(off.data(), sizeof(int64_t) * off.size());
    put(pts.data(), sizeof(float) * 2 * (size_t)off[(size_t)h.n_scans]);
    ok = (fclose(f) == 0) && ok;
    return ok ? DPG_OK : set_err(DPG_ERR_HIP, "dpg_inc_save: write failed");
}

// The graph's state as host copies -- dpg_inc_save's arrays without the scans (a test's oracle
// takes over from it: tests/test_config5.py lockstep)
int64_t dpg_inc_export(dpg_inc* q, int64_t* updates, dpg_factor* F, int32_t* created, int64_t cap_factors, double* theta,
                       double* est, double* maxd) {
    if (!q || cap_factors < 0) return set_err(DPG_ERR_ARG, "dpg_inc_export: bad arguments");
    if (q->prepared) return set_err(DPG_ERR_STATE, "dpg_inc_export: an update is prepared but not applied");
    const int64_t nf = (int64_t)q->F.size();
    if (updates) *updates = q->updates;
    const size_t k = (size_t)std::min(nf, cap_factors);
    if (F && k) memcpy(F, q->F.data(), sizeof(dpg_factor) * k);
    if (created && k) memcpy(created, q->f_created.data(), sizeof(int32_t) * k);
    const size_t V = (size_t)q->V;
    hipStream_t s = reinterpret_cast<hipStream_t>(dpg_ctx_stream_of(q->ctx));
    if (V && (theta || est || maxd)) {
        if (hipSetDevice(dpg_ctx_device_of(q->ctx)) != hipSuccess) return set_err(DPG_ERR_HIP, "hipSetDevice failed");
        if ((theta && hipMemcpyAsync(theta, q->theta, sizeof(double) * 3 * V, hipMemcpyDeviceToHost, s) != hipSuccess) ||
            (est && hipMemcpyAsync(est, q->est, sizeof(double) * 3 * V, hipMemcpyDeviceToHost, s) != hipSuccess) ||
            (maxd && hipMemcpyAsync(maxd, q->maxd, sizeof(double) * V, hipMemcpyDeviceToHost, s) != hipSuccess) ||
            hipStreamSynchronize(s) != hipSuccess)
            return set_err(DPG_ERR_HIP, "dpg_inc_export: read-back failed");
    }
    return nf;
}

// A graph restored from dpg_inc_save on ctx (single device): the scan store is replaced by the
// file's (and indexed), the factors, pairs, linearization points, estimate, per-variable |delta| and
// update count are the saved ones, so the next dpg_add_node / dpg_inc_update continues the saved
// run (ISAM2's relinearization schedule included).  The elimination order is computed afresh from
// the saved pattern (what the saved graph does every reorder_every nodes), so later estimates agree
// with an uninterrupted run to rounding.  NULL on error (dpg_last_error).
dpg_inc* dpg_inc_load(dpg_ctx* ctx, const char* path) {
    if (!path) {
        set_err(DPG_ERR_ARG, "dpg_inc_load: bad arguments");
        return nullptr;
    }
    FILE* f = fopen(path, "rb");
    if (!f) {
        set_err(DPG_ERR_ARG, "dpg_inc_load: cannot open the file");
        return nullptr;
    }
    CkptHeader h;
    bool ok = fread(&h, sizeof(h), 1, f) == 1;
    if (!ok || memcmp(h.magic, "DPGGRAPH", 8) != 0 || h.version != kCkptVersion || h.sizeof_factor != sizeof(dpg_factor) ||
        h.sizeof_params != sizeof(dpg_inc_params) || h.V < 0 || h.n_factors < 0 || h.n_pairs < 0 || h.n_scans < 0 ||
        (h.n_scans != 0 && h.n_scans < h.V) ||
        h.V > ((int64_t)1 << 31) || h.n_factors > ((int64_t)1 << 31) || h.n_pairs > ((int64_t)1 << 31) ||
        h.n_scans > ((int64_t)1 << 31)) {
        fclose(f);
        set_err(DPG_ERR_ARG, "dpg_inc_load: not a graph checkpoint of this version");
        return nullptr;
    }
    const size_t V = (size_t)h.V;
    std::vector<dpg_factor> F((size_t)h.n_factors);
    std::vector<int32_t> created((size_t)h.n_factors), plo((size_t)h.n_pairs), phi((size_t)h.n_pairs);
    std::vector<double> theta(3 * V), est(3 * V), maxd(V);
    std::vector<int64_t> off((size_t)h.n_scans + 1);
    auto get = [&](void* p, size_t bytes) { if (ok && bytes) ok = fread(p, 1, bytes, f) == bytes; };
    get(F.data(), sizeof(dpg_factor) * F.size());
    get(created.data(), sizeof(int32_t) * created.size());
    get(plo.data(), sizeof(int32_t) * plo.size());
    get(phi.data(), sizeof(int32_t) * phi.size());
    get(theta.data(), sizeof(double) * theta.size());
    get(est.data(), sizeof(double) * est.size());
    get(maxd.data(), sizeof(double) * maxd.size());
    get(off.data(), sizeof(int64_t) * off.size());
    const int64_t npts = ok ? off[(size_t)h.n_scans] : 0;
    ok = ok && off[0] == 0 && npts >= 0 && npts < ((int64_t)1 << 31);
    for (size_t v = 0; ok && v < (size_t)h.n_scans; ++v) ok = off[v + 1] >= off[v];
    std::vector<float> pts((size_t)(2 * std::max<int64_t>(npts, 1)));
    get(pts.data(), sizeof(float) * 2 * (size_t)std::max<int64_t>(npts, 0));
    fclose(f);
    // the graph must reference only its own nodes and pairs
    for (int64_t k = 0; ok && k < h.n_pairs; ++k)
        ok = plo[(size_t)k] >= 0 && plo[(size_t)k] < phi[(size_t)k] && phi[(size_t)k] < h.V;
    if (!ok) {
        set_err(DPG_ERR_ARG, "dpg_inc_load: truncated or inconsistent checkpoint");
        return nullptr;
    }
    if (!ctx) {
        set_err(DPG_ERR_ARG, "dpg_inc_load: ctx is NULL");
        return nullptr;
    }
    // the graph is rebuilt and checked first; the caller's scan store is replaced only once
    // everything else has succeeded (a failed load leaves the context as it was)
    dpg_inc* q = dpg_inc_create(ctx, &h.params);
    if (!q) return nullptr;
    auto bail = [&](int code, const char* msg) -> dpg_inc* {
        dpg_inc_destroy(q);
        set_err(code, msg);
        return nullptr;
    };
    auto take_scans = [&]() -> dpg_inc* {
        if (h.n_scans > 0 && (dpg_scans_upload(ctx, pts.data(), off.data(), h.n_scans, h.ratio) || dpg_scans_index_all(ctx))) {
            dpg_inc_destroy(q);
            return nullptr;   // dpg_last_error is the store's
        }
        return q;
    };
    for (int64_t k = 0; k < h.n_pairs; ++k) {
        if (!q->pair_id.emplace(pkey(plo[(size_t)k], phi[(size_t)k]), (int32_t)k).second)
            return bail(DPG_ERR_ARG, "dpg_inc_load: a node pair is listed twice");
    }
    q->plo = plo;
    q->phi = phi;
    for (int64_t k = 0; k < h.n_factors; ++k) {
        const dpg_factor& fk = F[(size_t)k];
        int32_t pid = -1;
        if (fk.kind == DPG_FACTOR_BETWEEN) {
            const auto it = q->pair_id.find(pkey(std::min(fk.i, fk.j), std::max(fk.i, fk.j)));
            if (fk.i < 0 || fk.j < 0 || fk.i >= h.V || fk.j >= h.V || it == q->pair_id.end())
                return bail(DPG_ERR_ARG, "dpg_inc_load: a factor's pair is missing");
            pid = it->second;
        } else if (fk.kind != DPG_FACTOR_PRIOR || fk.i < 0 || fk.i >= h.V) {
            return bail(DPG_ERR_ARG, "dpg_inc_load: a factor references a missing node");
        }
        q->f_pair.push_back(pid);
    }
    if (h.V == 0) return take_scans();
    // the structure: a fresh order of the saved pattern (dpg_inc_prepare from an empty symbolic state)
    if (dpg_inc_prepare(q, h.V, nullptr, 0)) return bail(DPG_ERR_NUMERIC, "dpg_inc_load: symbolic analysis failed");
    q->prepared = false;
    q->V = h.V;
    q->updates = h.updates;
    q->F = F;
    q->n_dev_f = 0;
    q->f_created = created;
    hipStream_t s = reinterpret_cast<hipStream_t>(dpg_ctx_stream_of(ctx));
    if (hipSetDevice(dpg_ctx_device_of(ctx)) != hipSuccess) return bail(DPG_ERR_HIP, "hipSetDevice failed");
    int rc = 0;
    rc |= dgrow(&q->theta, &q->c_theta, 3 * V, s, 0);
    rc |= dgrow(&q->est, &q->c_est, 3 * V, s, 0);
    rc |= dgrow(&q->maxd, &q->c_maxd, V, s, 0);
    if (!q->cnt) rc |= hipMalloc(reinterpret_cast<void**>(&q->cnt), sizeof(int32_t)) != hipSuccess;
    if (rc) return bail(DPG_ERR_HIP, "dpg_inc_load: out of device memory");
    if (hipMemcpyAsync(q->theta, theta.data(), sizeof(double) * 3 * V, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(q->est, est.data(), sizeof(double) * 3 * V, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(q->maxd, maxd.data(), sizeof(double) * V, hipMemcpyHostToDevice, s) != hipSuccess)
        return bail(DPG_ERR_HIP, "dpg_inc_load: upload failed");
    if ((rc = inc_rebuild(q, s))) return bail(rc, "dpg_inc_load: solver rebuild failed");
    if (hipStreamSynchronize(s) != hipSuccess) return bail(DPG_ERR_HIP, "dpg_inc_load: upload failed");
    return take_scans();
}

int dpg_inc_get_poses(dpg_inc* q, double* poses, int64_t n) {
    if (!q || !poses || n < 0 || n > q->V) return set_err(DPG_ERR_ARG, "dpg_inc_get_poses: bad arguments");
    if (n == 0) return DPG_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(dpg_ctx_stream_of(q->ctx));
    if (hipMemcpyAsync(poses, q->est, sizeof(double) * 3 * (size_t)n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return set_err(DPG_ERR_HIP, "dpg_inc_get_poses: copy failed");
    return DPG_OK;
}

}  // extern "C"
