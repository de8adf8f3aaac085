// dpg_icp_kd.hip -- ICP scan matching, k-d tree variant (the default batched ICP kernel).
//
// Same semantics and bit-exact results as the grid kernel in dpg_icp.hip (PCL
// IterativeClosestPoint + reciprocal KdTreeFLANN correspondences, dpg_slam.cc:387-416), but the
// nearest-neighbour machinery is built for the strongly non-uniform density of laser scans:
//
//  * kdtree_build_kernel: every node's downsampled cloud gets a left-balanced k-d tree (point
//    per tree node, x/y alternating by level), built in LDS by one workgroup with Wald's
//    tag-and-sort construction (one bitonic sort of (tag, coordinate) keys per level).  A cloud
//    is the ICP target of some edges and the source of others: one tree serves both roles.
//  * icp_kd_kernel (one workgroup per edge, resident for all its iterations):
//      forward 1-NN: stack-free traversal of the target tree, seeded with the previous
//        iteration's match, pruning a subtree when fl(plane^2) > best (ties -> lowest index);
//      reciprocal test: PCL rebuilds a tree on the moved source every iteration; here the
//        source tree stays in the source node's own frame.  The moved points are (up to float
//        drift, bounded by delta_k) F_k applied to their originals, so "is any source k closer
//        to target j than the matched i" is a radius query of sqrt(d_ij) + delta_k around
//        F_k^-1 t_j in that static tree, with every candidate re-checked in exact float on its
//        CURRENT coordinates;
//      rigid fit + convergence exactly as dpg_icp.hip (fp64 512-lane tree of dpg_icp_tree.h, shared with the oracle).
// Built with -ffp-contract=off.

#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "dpg_atan2f.h"
#include "dpg_internal.h"
#include "dpg_icp_tree.h"

namespace {

constexpr int kT = 256;
constexpr int kW = kT / 64;
constexpr int kSums = dpg_tree::kSums;

__device__ __forceinline__ int level_of(int i) { return 31 - __clz(i + 1); }

// number of nodes in the subtree rooted at t of a complete (left-balanced) tree with N nodes
__device__ __forceinline__ int subtree_size(int t, int N) {
    int size = 0;
    long long lo = t, hi = t;
    while (lo < N) {
        size += (int)(min(hi, (long long)N - 1) - lo + 1);
        lo = 2 * lo + 1;
        hi = 2 * hi + 2;
    }
    return size;
}

// array position of the first element of level-L subtree t after sorting by tag
__device__ __forceinline__ int first_pos(int t, int L, int N) {
    const long long firstL = (1ll << L) - 1;
    long long pos = firstL;
    const long long before = t - firstL;   // level-L subtrees to the left of t
    for (int d = 0; ((1ll << (L + d)) - 1) < N; ++d) {
        const long long first_ld = (1ll << (L + d)) - 1;
        const long long cnt = min((long long)N - first_ld, before << d);
        if (cnt > 0) pos += cnt;
    }
    return (int)pos;
}

__device__ __forceinline__ uint32_t orderable(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// one workgroup per node: left-balanced k-d tree of its downsampled cloud
__global__ __launch_bounds__(kT) void kdtree_build_kernel(const float2* __restrict__ ds_pts,
                                                          const int64_t* __restrict__ ds_off,
                                                          float2* __restrict__ tree_pts,
                                                          uint16_t* __restrict__ tree_idx, int pow2cap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int v = blockIdx.x, tid = threadIdx.x;
    const int64_t off = ds_off[v];
    const int N = (int)(ds_off[v + 1] - off);
    if (N <= 0) return;
    int P = 1;
    while (P < N) P <<= 1;
    uint64_t* key = reinterpret_cast<uint64_t*>(smem);            // [pow2cap]
    uint16_t* val = reinterpret_cast<uint16_t*>(key + pow2cap);   // [pow2cap]
    float2* pts = reinterpret_cast<float2*>(smem + ((size_t)pow2cap * 10 + 15) / 16 * 16);  // [N]
    for (int i = tid; i < N; i += kT) pts[i] = ds_pts[off + i];
    for (int s = tid; s < P; s += kT) {
        val[s] = (uint16_t)(s < N ? s : 0);
        key[s] = s < N ? 0ull : ~0ull;    // tag 0 everywhere
    }
    __syncthreads();
    const int depth = level_of(N - 1) + 1;
    for (int L = 0; L < depth; ++L) {
        const int dim = L & 1;
        for (int s = tid; s < N; s += kT) {
            const uint32_t tag = (uint32_t)(key[s] >> 32);
            const float2 p = pts[val[s]];
            key[s] = ((uint64_t)tag << 32) | orderable(dim ? p.y : p.x);
        }
        __syncthreads();
        // bitonic sort of (key, val), ascending
        for (int k = 2; k <= P; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int q = tid; q < P / 2; q += kT) {
                    const int i = 2 * q - (q & (j - 1));   // lower index of the pair
                    const int l = i + j;
                    const bool up = (i & k) == 0;
                    const uint64_t a = key[i], b = key[l];
                    if ((a > b) == up) {
                        key[i] = b; key[l] = a;
                        const uint16_t t = val[i]; val[i] = val[l]; val[l] = t;
                    }
                }
                __syncthreads();
            }
        }
        // new tags
        for (int s = tid; s < N; s += kT) {
            const int t = (int)(key[s] >> 32);
            if (level_of(t) < L) continue;   // already placed
            const int pivot = first_pos(t, L, N) + subtree_size(2 * t + 1, N);
            const int nt = s < pivot ? 2 * t + 1 : (s > pivot ? 2 * t + 2 : t);
            key[s] = ((uint64_t)(uint32_t)nt << 32) | (key[s] & 0xffffffffull);
        }
        __syncthreads();
    }
    // after the last level the array is in tag (= node index) order
    for (int s = tid; s < N; s += kT) {
        tree_pts[off + s] = pts[val[s]];
        tree_idx[off + s] = val[s];
    }
}

struct Lds {
    float2* tp;       // target tree points (node order)
    float2* sp;       // source tree points (node order, source node frame)
    float2* sc;       // current (moved) source points, original order
    uint16_t* ti;     // target tree -> original index
    uint16_t* si;     // source tree -> original index
    double* wpart;    // [2 * kW][kSums + 2] (tree waves)
};

__device__ __forceinline__ size_t a16(size_t x) { return (x + 15) & ~size_t(15); }

__device__ Lds carve(unsigned char* base, int cap) {
    Lds L;
    size_t o = 0;
    L.tp = reinterpret_cast<float2*>(base + o);   o = a16(o + 8 * (size_t)cap);
    L.sp = reinterpret_cast<float2*>(base + o);   o = a16(o + 8 * (size_t)cap);
    L.sc = reinterpret_cast<float2*>(base + o);   o = a16(o + 8 * (size_t)cap);
    L.ti = reinterpret_cast<uint16_t*>(base + o); o = a16(o + 2 * (size_t)cap);
    L.si = reinterpret_cast<uint16_t*>(base + o); o = a16(o + 2 * (size_t)cap);
    L.wpart = reinterpret_cast<double*>(base + o);
    return L;
}

__device__ __forceinline__ float sqd(float ax, float ay, float bx, float by) {
    const float dx = ax - bx, dy = ay - by;
    return dx * dx + dy * dy;
}

template <int PPT>
__global__ __launch_bounds__(kT) void icp_kd_kernel(const float2* __restrict__ ds_pts,
                                                    const float2* __restrict__ tree_pts,
                                                    const uint16_t* __restrict__ tree_idx,
                                                    const dpg_icp_edge* __restrict__ edges,
                                                    dpg_icp_kparams kp, dpg_icp_result* __restrict__ results,
                                                    int32_t* __restrict__ trace) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const dpg_icp_edge E = edges[blockIdx.x];   // dispatch order (dpg_icp_batch_prepare)
    const int e = E.pad[0];                     // the edge's index in the caller's list
    const int N = E.n_src_ds, M = E.n_tgt_ds;
    Lds L = carve(smem, kp.lds_tgt);
    for (int i = t; i < M; i += kT) {
        L.tp[i] = tree_pts[E.tgt_ds_off + i];
        L.ti[i] = tree_idx[E.tgt_ds_off + i];
    }
    for (int i = t; i < N; i += kT) {
        L.sp[i] = tree_pts[E.src_ds_off + i];
        L.si[i] = tree_idx[E.src_ds_off + i];
    }
    float F[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) F[q] = E.guess[q];
    float sx[PPT], sy[PPT];
    int seed[PPT];
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int i = t + kT * m;
        seed[m] = -1;
        sx[m] = 0.f;
        sy[m] = 0.f;
        if (i < N) {
            const float2 p = ds_pts[E.src_ds_off + i];
            sx[m] = (F[0] * p.x + F[1] * p.y) + F[2];
            sy[m] = (F[3] * p.x + F[4] * p.y) + F[5];
            L.sc[i] = make_float2(sx[m], sy[m]);
        }
    }
    __syncthreads();

    const float r2f = kp.r2_f;
    double prev_mse = DBL_MAX, last_mse = 0.0;
    int k = 0, converged = 0, status = DPG_ICP_OK, last_cnt = 0;
    for (;;) {
        // inverse of the cumulative transform (maps a target point into the source node frame)
        const double det = (double)F[0] * (double)F[4] - (double)F[1] * (double)F[3];
        const double i00 = (double)F[4] / det, i01 = -(double)F[1] / det;
        const double i10 = -(double)F[3] / det, i11 = (double)F[0] / det;
        const float drift = 1e-4f + 5e-5f * (float)(k + 1);
        double acc[2][kSums];   // point i = t + 256 m -> tree lane t + 256 (m & 1)
#pragma unroll
        for (int q = 0; q < kSums; ++q) acc[0][q] = acc[1][q] = 0.0;
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int i = t + kT * m;
            if (i >= N) continue;
            const float qx = sx[m], qy = sy[m];
            // ---- forward 1-NN in the target tree, seeded ----
            float bd = r2f;
            int bi = 0x7fffffff, bp = -1;
            if (seed[m] >= 0) {
                const float2 s0 = L.tp[seed[m]];
                const float d = sqd(qx, qy, s0.x, s0.y);
                if (d <= r2f) { bd = d; bi = L.ti[seed[m]]; bp = seed[m]; }
            }
            if (M > 0) {
                int prev = -1, curr = 0;
                for (;;) {
                    const int parent = ((curr + 1) >> 1) - 1;
                    if (curr >= M) { prev = curr; curr = parent; continue; }
                    const float2 tp = L.tp[curr];
                    if (prev < curr) {   // first visit
                        const float d = sqd(qx, qy, tp.x, tp.y);
                        const int j = L.ti[curr];
                        if (d < bd || (d == bd && j < bi)) { bd = d; bi = j; bp = curr; }
                    }
                    const int dim = level_of(curr) & 1;
                    const float diff = dim ? (qy - tp.y) : (qx - tp.x);
                    const int close = 2 * curr + 1 + (diff > 0.f ? 1 : 0);
                    const int far = 2 * curr + 2 - (diff > 0.f ? 1 : 0);
                    int next;
                    if (prev < curr) next = close;
                    else if (prev == close) next = (diff * diff <= bd) ? far : parent;
                    else next = parent;
                    if (next < 0) break;
                    prev = curr;
                    curr = next;
                }
            }
            seed[m] = bp;
            bool ok = bp >= 0;   // a target with d <= r^2 exists
            // ---- reciprocal test: any source closer to t_j than i? ----
            if (ok && kp.reciprocal) {
                const float2 tj = L.tp[bp];
                const double ux = (double)tj.x - (double)F[2], uy = (double)tj.y - (double)F[5];
                const float px = (float)(i00 * ux + i01 * uy), py = (float)(i10 * ux + i11 * uy);
                const float rho = sqrtf(bd) * 1.0001f + drift;
                int prev = -1, curr = 0;
                for (;;) {
                    const int parent = ((curr + 1) >> 1) - 1;
                    if (curr >= N) { prev = curr; curr = parent; continue; }
                    const float2 sp = L.sp[curr];
                    if (prev < curr) {
                        const int kk = L.si[curr];
                        if (kk != i) {
                            const float2 c = L.sc[kk];
                            const float d = sqd(c.x, c.y, tj.x, tj.y);
                            if (d < bd || (d == bd && kk < i)) { ok = false; break; }
                        }
                    }
                    const int dim = level_of(curr) & 1;
                    const float diff = dim ? (py - sp.y) : (px - sp.x);
                    const int close = 2 * curr + 1 + (diff > 0.f ? 1 : 0);
                    const int far = 2 * curr + 2 - (diff > 0.f ? 1 : 0);
                    int next;
                    if (prev < curr) next = close;
                    else if (prev == close) next = (fabsf(diff) <= rho) ? far : parent;
                    else next = parent;
                    if (next < 0) break;
                    prev = curr;
                    curr = next;
                }
            }
            if (trace && k < kp.trace_iters) trace[((size_t)e * kp.trace_iters + k) * kp.trace_stride + i] = ok ? bi : -1;
            if (ok) {
                const float2 tq = L.tp[bp];
                dpg_tree::add_pair(acc[m & 1], qx, qy, tq.x, tq.y, bd);
            }
        }
        dpg_tree::wave_fold(acc[0]);
        dpg_tree::wave_fold(acc[1]);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < kSums; ++q) {
                L.wpart[wave * (kSums + 2) + q] = acc[0][q];
                L.wpart[(wave + kW) * (kSums + 2) + q] = acc[1][q];
            }
        }
        __syncthreads();
        double S[kSums];
#pragma unroll
        for (int q = 0; q < kSums; ++q) S[q] = dpg_tree::combine(L.wpart, kSums + 2, q);
        const int cnt = (int)S[0];
        last_cnt = cnt;
        if (cnt < kp.min_corr) { converged = 0; status = DPG_ICP_TOO_FEW_CORR; break; }
        const double n = S[0];
        double a, b;
        dpg_tree::fit_ab(S, a, b);
        const double hh = sqrt(a * a + b * b);
        double c = 1.0, s = 0.0;
        if (hh > 0.0) { c = a / hh; s = b / hh; }
        const double mpx = S[2] / n, mpy = S[3] / n, mqx = S[4] / n, mqy = S[5] / n;
        const double txd = mqx - (c * mpx - s * mpy);
        const double tyd = mqy - (s * mpx + c * mpy);
        const float cf = (float)c, sf = (float)s, txf = (float)txd, tyf = (float)tyd;
        const float nsf = -sf;
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int i = t + kT * m;
            const float x = sx[m], y = sy[m];
            sx[m] = (cf * x + nsf * y) + txf;
            sy[m] = (sf * x + cf * y) + tyf;
            if (i < N) L.sc[i] = make_float2(sx[m], sy[m]);
        }
        float Nf[6];
        Nf[0] = cf * F[0] + nsf * F[3];
        Nf[1] = cf * F[1] + nsf * F[4];
        Nf[2] = (cf * F[2] + nsf * F[5]) + txf;
        Nf[3] = sf * F[0] + cf * F[3];
        Nf[4] = sf * F[1] + cf * F[4];
        Nf[5] = (sf * F[2] + cf * F[5]) + tyf;
#pragma unroll
        for (int q = 0; q < 6; ++q) F[q] = Nf[q];
        ++k;
        const double mse = S[1] / S[0];
        last_mse = mse;
        __syncthreads();   // moved source points visible before the next reciprocal tests
        if (k >= kp.max_iter) { converged = 1; break; }
        const float tr = ((cf + cf) + 1.0f) - 1.0f;
        const double cos_angle = 0.5 * (double)tr;
        const double tsq = (double)(txf * txf + tyf * tyf);
        if (cos_angle >= kp.rot_thr && tsq <= kp.eps) { converged = 1; break; }
        if (fabs(mse - prev_mse) < kp.mse_abs) { converged = 1; break; }
        prev_mse = mse;
    }
    if (t == 0) {
        dpg_icp_result R;
#pragma unroll
        for (int q = 0; q < 6; ++q) R.T[q] = F[q];
        R.z[0] = F[2];
        R.z[1] = F[5];
        R.z[2] = dpg_atan2f(F[3], F[0]);   // Rotation2Df::fromRotationMatrix -> std::atan2(float, float)
        R.converged = converged;
        R.iterations = k;
        R.n_corr = last_cnt;
        R.status = status;
        R.pad = 0;
        R.fitness = last_mse;
        results[e] = R;
    }
}

}  // namespace

extern "C" size_t dpg_icp_kd_lds_bytes(int32_t cap) {
    auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
    size_t o = 0;
    o = al(o + 8 * (size_t)cap);
    o = al(o + 8 * (size_t)cap);
    o = al(o + 8 * (size_t)cap);
    o = al(o + 2 * (size_t)cap);
    o = al(o + 2 * (size_t)cap);
    o += sizeof(double) * 2 * kW * (kSums + 2);
    return al(o);
}

extern "C" int dpg_launch_kdtree_build(const float* ds_pts_dev, const int64_t* ds_off_dev, int64_t n_nodes,
                                       int32_t max_points, float* tree_pts_dev, uint16_t* tree_idx_dev, void* stream) {
    if (n_nodes <= 0) return DPG_OK;
    int cap = 1;
    while (cap < max_points) cap <<= 1;
    if (cap > 4096) return DPG_ERR_SIZE;
    const size_t lds = ((size_t)cap * 10 + 15) / 16 * 16 + 8 * (size_t)max_points;
    hipLaunchKernelGGL(kdtree_build_kernel, dim3((unsigned)n_nodes), dim3(kT), lds, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const float2*>(ds_pts_dev), ds_off_dev, reinterpret_cast<float2*>(tree_pts_dev),
                       tree_idx_dev, cap);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_launch_icp_kd(const float* ds_pts_dev, const float* tree_pts_dev, const uint16_t* tree_idx_dev,
                                 const dpg_icp_edge* edges_dev, int64_t n_edges, const dpg_icp_kparams* kp,
                                 int32_t max_points, dpg_icp_result* results_dev, int32_t* trace_dev, void* stream) {
    if (n_edges <= 0) return DPG_OK;
    if (max_points > kp->lds_tgt || kp->lds_tgt > 4096) return DPG_ERR_SIZE;
    const size_t lds = dpg_icp_kd_lds_bytes(kp->lds_tgt);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)n_edges), block(kT);
    const float2* ds = reinterpret_cast<const float2*>(ds_pts_dev);
    const float2* tp = reinterpret_cast<const float2*>(tree_pts_dev);
    const int ppt = (max_points + kT - 1) / kT;
#define DPG_KD_LAUNCH(P) \
    hipLaunchKernelGGL(icp_kd_kernel<P>, grid, block, lds, s, ds, tp, tree_idx_dev, edges_dev, *kp, results_dev, trace_dev)
    if (ppt <= 1) DPG_KD_LAUNCH(1);
    else if (ppt <= 2) DPG_KD_LAUNCH(2);
    else if (ppt <= 4) DPG_KD_LAUNCH(4);
    else if (ppt <= 8) DPG_KD_LAUNCH(8);
    else if (ppt <= 16) DPG_KD_LAUNCH(16);
    else return DPG_ERR_SIZE;
#undef DPG_KD_LAUNCH
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}
