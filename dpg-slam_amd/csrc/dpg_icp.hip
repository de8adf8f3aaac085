// dpg_icp.hip -- batched ICP scan matching and the ICP covariance block on gfx950 (MI355X).
//
// Replaces, for a whole batch of edges at once:
//   pcl::IterativeClosestPoint<PointXYZ,PointXYZ>::align  (called at src/dpg_slam/dpg_slam.cc:415)
//     = CorrespondenceEstimation::determineReciprocalCorrespondences over KdTreeFLANN 1-NN (R4)
//     + TransformationEstimationSVD / umeyama (R5, planar closed form)
//     + in-place transformCloud + DefaultConvergenceCriteria (R6)
//   calculate_ICP_COV (src/icp_cov/cov_func_point_to_point.h:24-31,45-283,572-575) (R7)
//   runIcp epilogue (dpg_slam.cc:416-445) (R8)
//
// Design (one 256-thread workgroup = 4 waves per edge, resident for ALL of that edge's ICP
// iterations):
//   * the target cloud (static across iterations) is counting-sorted into a uniform LDS grid
//     once; cells >= 1.05 r, so the 3x3 cell block around a query holds every point that can
//     pass the r^2 test -> the argmin over that block (ties -> lowest index) IS the exact 1-NN
//     whenever it matters;
//   * the source cloud lives in registers (PPT points per lane: i = lane + 256 m) and is
//     transformed in place each iteration exactly as pcl::transformCloud (float, no FMA);
//   * reciprocal check without a second tree: while scanning the candidates of source i, every
//     pair with d <= r^2 does an LDS 64-bit atomicMin of (bits(d) << 32 | i) on the target's
//     key -- afterwards key[j] is the (distance, lowest index) argmin over the sources near j,
//     i.e. the reverse 1-NN, and (i, j) is reciprocal iff key[j] == (bits(d_ij) << 32 | i);
//   * the rigid-fit sums are fp64 in the FIXED 512-lane tree of dpg_icp_tree.h (a 256-thread
//     workgroup carries lanes t and t + 256) that the CPU oracle replays, so transforms -- and therefore all
//     later correspondences -- are bit-identical to the oracle;
//   * every lane redundantly combines the 4 wave partials and evaluates the closed-form fit and
//     the convergence rule, so one iteration costs two workgroup barriers.
// Built with -ffp-contract=off: every float/double expression is one rounding per operation.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <float.h>
#include <stdint.h>

#include "dpg_atan2f.h"
#include "dpg_internal.h"
#include "dpg_icp_tree.h"

namespace {

constexpr int kThreads = 256;  // DPG_ICP_LANES / 2: thread t carries tree lanes t and t + 256
constexpr int kWaves = kThreads / 64;
constexpr int kSums = dpg_tree::kSums;

__device__ __forceinline__ double shfl_down_d(double v, int off) { return __shfl_down(v, off, 64); }
__device__ __forceinline__ float shfl_xor_f(float v, int off) { return __shfl_xor(v, off, 64); }

struct Lds {
    float2* tp;        // [lds_tgt] targets sorted by cell
    uint64_t* key0;    // [lds_tgt] reverse-NN keys, even iterations
    uint64_t* key1;    // [lds_tgt] odd iterations
    uint32_t* cells;   // [cells_max + 1] counts -> exclusive starts
    uint16_t* tidx;    // [lds_tgt] original target index of tp[k]
    double* wpart;     // [2 * kWaves][kSums + 2] (tree waves)
    float* fctl;       // [16]
};

__device__ __forceinline__ size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

__device__ Lds carve(unsigned char* base, int lds_tgt, int cells_max) {
    Lds L;
    size_t o = 0;
    L.tp = reinterpret_cast<float2*>(base + o);       o = align16(o + sizeof(float2) * lds_tgt);
    L.key0 = reinterpret_cast<uint64_t*>(base + o);   o = align16(o + sizeof(uint64_t) * lds_tgt);
    L.key1 = reinterpret_cast<uint64_t*>(base + o);   o = align16(o + sizeof(uint64_t) * lds_tgt);
    L.cells = reinterpret_cast<uint32_t*>(base + o);  o = align16(o + sizeof(uint32_t) * (cells_max + 1));
    L.tidx = reinterpret_cast<uint16_t*>(base + o);   o = align16(o + sizeof(uint16_t) * lds_tgt);
    L.wpart = reinterpret_cast<double*>(base + o);    o = align16(o + sizeof(double) * 2 * kWaves * (kSums + 2));
    L.fctl = reinterpret_cast<float*>(base + o);
    return L;
}

// (double)d <= r2 for a float d, evaluated as a float compare against r2_f (exact equivalence)
__device__ __forceinline__ uint64_t rev_key(float d, int i) {
    return (static_cast<uint64_t>(__float_as_uint(d)) << 32) | static_cast<uint32_t>(i);
}

template <int PPT>
__global__ __launch_bounds__(kThreads) void icp_edges_kernel(const float2* __restrict__ ds_pts,
                                                             const dpg_icp_edge* __restrict__ edges,
                                                             dpg_icp_kparams kp,
                                                             dpg_icp_result* __restrict__ results,
                                                             int32_t* __restrict__ trace) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const dpg_icp_edge E = edges[blockIdx.x];   // dispatch order (dpg_icp_batch_prepare)
    const int e = E.pad[0];                     // the edge's index in the caller's list
    const int N = E.n_src_ds;
    const int M = E.n_tgt_ds;
    Lds L = carve(smem, kp.lds_tgt, kp.cells_max);

    // ---------------- targets: load, bbox, grid, counting sort (once per edge) ----------------
    float tx[PPT], ty[PPT];
    float mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int j = t + kThreads * m;
        if (j < M) {
            const float2 q = ds_pts[E.tgt_ds_off + j];
            tx[m] = q.x;
            ty[m] = q.y;
            mnx = fminf(mnx, q.x); mxx = fmaxf(mxx, q.x);
            mny = fminf(mny, q.y); mxy = fmaxf(mxy, q.y);
            L.key0[j] = ~0ull;
            L.key1[j] = ~0ull;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        mnx = fminf(mnx, shfl_xor_f(mnx, off)); mxx = fmaxf(mxx, shfl_xor_f(mxx, off));
        mny = fminf(mny, shfl_xor_f(mny, off)); mxy = fmaxf(mxy, shfl_xor_f(mxy, off));
    }
    if (lane == 0) {
        L.fctl[4 * wave + 0] = mnx; L.fctl[4 * wave + 1] = mxx;
        L.fctl[4 * wave + 2] = mny; L.fctl[4 * wave + 3] = mxy;
    }
    __syncthreads();
    mnx = fminf(fminf(L.fctl[0], L.fctl[4]), fminf(L.fctl[8], L.fctl[12]));
    mxx = fmaxf(fmaxf(L.fctl[1], L.fctl[5]), fmaxf(L.fctl[9], L.fctl[13]));
    mny = fminf(fminf(L.fctl[2], L.fctl[6]), fminf(L.fctl[10], L.fctl[14]));
    mxy = fmaxf(fmaxf(L.fctl[3], L.fctl[7]), fmaxf(L.fctl[11], L.fctl[15]));
    if (M == 0) { mnx = mny = mxx = mxy = 0.f; }
    // grid geometry: cell >= h_min, at most cells_max cells (any valid grid gives the same NN)
    const float ex = mxx - mnx, ey = mxy - mny;
    float h = kp.h_min;
    {
        const float area_h = sqrtf((ex + h) * (ey + h) / (float)kp.cells_max) * 1.02f;
        if (area_h > h) h = area_h;
    }
    int gx = (int)(ex / h) + 1, gy = (int)(ey / h) + 1;
    while (gx * gy > kp.cells_max) {  // uniform across the block: same inputs everywhere
        h *= 1.05f;
        gx = (int)(ex / h) + 1;
        gy = (int)(ey / h) + 1;
    }
    const float inv_h = 1.0f / h;
    const int ncell = gx * gy;
    for (int c = t; c <= ncell; c += kThreads) L.cells[c] = 0u;
    __syncthreads();
    int tcell[PPT];
    uint32_t trank[PPT];
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int j = t + kThreads * m;
        if (j < M) {
            int cx = (int)floorf((tx[m] - mnx) * inv_h);
            int cy = (int)floorf((ty[m] - mny) * inv_h);
            cx = min(max(cx, 0), gx - 1);
            cy = min(max(cy, 0), gy - 1);
            tcell[m] = cy * gx + cx;
            trank[m] = atomicAdd(&L.cells[tcell[m]], 1u);
        }
    }
    __syncthreads();
    {   // exclusive scan of cells[0, ncell)
        const int chunk = (ncell + kThreads - 1) / kThreads;
        const int c0 = min(t * chunk, ncell), c1 = min(c0 + chunk, ncell);
        uint32_t local = 0;
        for (int c = c0; c < c1; ++c) local += L.cells[c];
        uint32_t incl = local;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t v = __shfl_up(incl, off, 64);
            if (lane >= off) incl += v;
        }
        if (lane == 63) reinterpret_cast<uint32_t*>(L.wpart)[wave] = incl;
        __syncthreads();
        uint32_t base = incl - local;
        for (int w = 0; w < wave; ++w) base += reinterpret_cast<uint32_t*>(L.wpart)[w];
        for (int c = c0; c < c1; ++c) {
            const uint32_t v = L.cells[c];
            L.cells[c] = base;
            base += v;
        }
        if (t == 0) L.cells[ncell] = (uint32_t)M;
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int j = t + kThreads * m;
        if (j < M) {
            const uint32_t pos = L.cells[tcell[m]] + trank[m];
            L.tp[pos] = make_float2(tx[m], ty[m]);
            L.tidx[pos] = (uint16_t)j;
        }
    }

    // ---------------- sources: registers, initial guess transform ----------------
    float F[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) F[q] = E.guess[q];
    float sx[PPT], sy[PPT];
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int i = t + kThreads * m;
        if (i < N) {
            const float2 p = ds_pts[E.src_ds_off + i];
            sx[m] = (F[0] * p.x + F[1] * p.y) + F[2];
            sy[m] = (F[3] * p.x + F[4] * p.y) + F[5];
        } else {
            sx[m] = 0.f;
            sy[m] = 0.f;
        }
    }
    __syncthreads();

    const float r2f = kp.r2_f;
    double prev_mse = DBL_MAX;
    double last_mse = 0.0;
    int k = 0, converged = 0, status = DPG_ICP_OK, last_cnt = 0;
    for (;;) {
        uint64_t* key = (k & 1) ? L.key1 : L.key0;
        // ---- R4 forward 1-NN over the 3x3 cell block + reverse keys ----
        float bd[PPT], bx[PPT], by[PPT];
        int bi[PPT];
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int i = t + kThreads * m;
            bd[m] = INFINITY;
            bi[m] = 0x7fffffff;
            bx[m] = 0.f;
            by[m] = 0.f;
            if (i >= N) continue;
            const float qx = sx[m], qy = sy[m];
            const float fx = floorf((qx - mnx) * inv_h), fy = floorf((qy - mny) * inv_h);
            if (!(fx >= -1.f && fy >= -1.f && fx <= (float)gx && fy <= (float)gy)) continue;
            const int cx = (int)fx, cy = (int)fy;
            const int c0 = max(cx - 1, 0), c1 = min(cx + 1, gx - 1);
            if (c0 > c1) continue;
            for (int yy = max(cy - 1, 0); yy <= min(cy + 1, gy - 1); ++yy) {
                const uint32_t s0 = L.cells[yy * gx + c0], s1 = L.cells[yy * gx + c1 + 1];
                for (uint32_t s = s0; s < s1; ++s) {
                    const float2 tq = L.tp[s];
                    const float dx = qx - tq.x, dy = qy - tq.y;
                    const float d = dx * dx + dy * dy;
                    const int j = L.tidx[s];
                    if (d < bd[m] || (d == bd[m] && j < bi[m])) {
                        bd[m] = d; bi[m] = j; bx[m] = tq.x; by[m] = tq.y;
                    }
                    if (kp.reciprocal && d <= r2f) atomicMin(reinterpret_cast<unsigned long long*>(&key[j]),
                                                             (unsigned long long)rev_key(d, i));
                }
            }
        }
        __syncthreads();
        // ---- acceptance + fp64 lane sums: point i = t + 256 m goes to tree lane t + 256 (m & 1) ----
        double acc[2][kSums];
#pragma unroll
        for (int q = 0; q < kSums; ++q) acc[0][q] = acc[1][q] = 0.0;
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int i = t + kThreads * m;
            bool ok = (i < N) && (bd[m] <= r2f);
            if (ok && kp.reciprocal) ok = (key[bi[m]] == rev_key(bd[m], i));
            if (trace && k < kp.trace_iters && i < N)
                trace[((size_t)e * kp.trace_iters + k) * kp.trace_stride + i] = ok ? bi[m] : -1;
            if (ok) dpg_tree::add_pair(acc[m & 1], sx[m], sy[m], bx[m], by[m], bd[m]);
        }
        dpg_tree::wave_fold(acc[0]);
        dpg_tree::wave_fold(acc[1]);
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < kSums; ++q) {
                L.wpart[wave * (kSums + 2) + q] = acc[0][q];
                L.wpart[(wave + kWaves) * (kSums + 2) + q] = acc[1][q];
            }
        }
        __syncthreads();
        // ---- every lane: combine the eight tree waves, fit, converge (uniform control flow) ----
        double S[kSums];
#pragma unroll
        for (int q = 0; q < kSums; ++q) S[q] = dpg_tree::combine(L.wpart, kSums + 2, q);
        // this iteration's key buffer is free again: reset the entries this lane owns
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int j = t + kThreads * m;
            if (j < M) key[j] = ~0ull;
        }
        const int cnt = (int)S[0];
        last_cnt = cnt;
        if (cnt < kp.min_corr) { converged = 0; status = DPG_ICP_TOO_FEW_CORR; break; }
        // R5 planar closed form (see oracle rigid_from_sums)
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
            const float x = sx[m], y = sy[m];
            sx[m] = (cf * x + nsf * y) + txf;
            sy[m] = (sf * x + cf * y) + tyf;
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
        // R6 DefaultConvergenceCriteria
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

// R7: [x, y, yaw] block of d2J_dX2 over index-paired full clouds (s < min(n_data, n_model)).
// A grid smaller than the edge count leaves the rest of the GPU to the pose graph that runs beside
// it (dpg_ctx_set_cov_workgroups); every edge's sums are the same either way.
__global__ __launch_bounds__(kThreads) void cov_block_kernel(const float2* __restrict__ full_pts,
                                                             const dpg_icp_edge* __restrict__ edges, int64_t n_edges,
                                                             const dpg_icp_result* __restrict__ results,
                                                             double* __restrict__ hess) {
    __shared__ double red[kWaves][3];
    const int t = threadIdx.x;
    for (int64_t b = blockIdx.x; b < n_edges; b += gridDim.x) {   // edges strided over the grid
    const dpg_icp_edge E = edges[b];
    const int e = E.pad[0];   // results / hess by the caller's edge index
    const float* T = results[e].T;
    const double a = (double)dpg_atan2f(T[3], T[0]);   // yaw = atan2f(T10, T00) (cov :31)
    const double x = T[2], y = T[5];
    const double ca = cos(a), sa = sin(a);
    const int n = min(E.n_src_full, E.n_tgt_full);
    double h02 = 0.0, h12 = 0.0, h22 = 0.0;
    for (int s = t; s < n; s += kThreads) {
        const float2 p = full_pts[E.src_full_off + s];
        const float2 q = full_pts[E.tgt_full_off + s];
        const double px = p.x, py = p.y, qx = q.x, qy = q.y;
        const double ux = ca * px - sa * py, uy = sa * px + ca * py;
        const double rx = (x - qx) + ux, ry = (y - qy) + uy;
        h02 += -2.0 * uy;
        h12 += 2.0 * ux;
        h22 += 2.0 * (ux * ux + uy * uy) - 2.0 * (ux * rx + uy * ry);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        h02 += shfl_down_d(h02, off);
        h12 += shfl_down_d(h12, off);
        h22 += shfl_down_d(h22, off);
    }
    if ((t & 63) == 0) { red[t >> 6][0] = h02; red[t >> 6][1] = h12; red[t >> 6][2] = h22; }
    __syncthreads();
    if (t == 0) {
        const double H02 = (red[0][0] + red[1][0]) + (red[2][0] + red[3][0]);
        const double H12 = (red[0][1] + red[1][1]) + (red[2][1] + red[3][1]);
        const double H22 = (red[0][2] + red[1][2]) + (red[2][2] + red[3][2]);
        const double h00 = 2.0 * (double)n;
        double* o = hess + 9 * (size_t)e;
        o[0] = h00; o[1] = 0.0; o[2] = H02;
        o[3] = 0.0; o[4] = h00; o[5] = H12;
        o[6] = H02; o[7] = H12; o[8] = H22;
    }
    __syncthreads();   // red is reused by the next edge
    }
}

// The 6x6 ICP covariance the reference computes and discards (cov :553-566, commented out): the
// sums that d2J_dX2 (over s < n_h) and d2J_dZdX cov_z d2J_dZdX^T (over k < n_b) reduce to at
// b = c = z = 0 (T20 = T21 = 0, T22 = 1), with a = atan2f(T10, T00), u = R(a) p, d = t - q,
// w = d . (cos a, sin a), v = d . (sin a, -cos a) -- derived independently (tools/cov6_derive.py)
// and checked against the reference's own expressions (tests/golden/cov6_expr.npz):
//   d2J_dX2 per pair:   xx = yy = zz = 2, xa = -2 u_y, ya = 2 u_x, zb = -2 p_x, zc = 2 p_y,
//                       aa = -2 u.d, bb = -2 p_x w, bc = 2 p_y w, cc = 2 p_y v (all others 0)
//   B_k B_k^T per pair: xx = yy = zz = 8, xa = 4(-v cos a + w sin a - u_y),
//                       ya = 4(-v sin a - w cos a + u_x), zb = 4(w - p_x), zc = 4(v + p_y),
//                       aa = 4(v^2 + w^2 + |u|^2), bb = 4(w^2 + p_x^2), bc = 4(w v - p_x p_y),
//                       cc = 4(v^2 + p_y^2)
// out[0..7]: the d2J_dX2 sums xa ya aa zb zc bb bc cc; out[8..15] the same entries of sum B B^T.
// One workgroup; fixed reduction order (strided per thread, wave shuffles, waves in order).
__global__ __launch_bounds__(kThreads) void cov6_kernel(const float2* __restrict__ pts, int n_data, int n_model,
                                                       const float* __restrict__ T6, double* __restrict__ out) {
    __shared__ double red[kWaves][16];
    const int t = threadIdx.x;
    const double a = (double)dpg_atan2f(T6[3], T6[0]);   // yaw = atan2f(T10, T00) (cov :31)
    const double x = T6[2], y = T6[5];
    const double ca = cos(a), sa = sin(a);
    const int nh = min(n_data, n_model), nb = min(nh, 200);
    double acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.0;
    for (int s = t; s < nh; s += kThreads) {
        const float2 p = pts[s];
        const float2 q = pts[n_data + s];
        const double px = p.x, py = p.y, qx = q.x, qy = q.y;
        const double ux = ca * px - sa * py, uy = sa * px + ca * py;
        const double dx = x - qx, dy = y - qy;
        const double w = dx * ca + dy * sa, v = dx * sa - dy * ca;
        acc[0] += -2.0 * uy;
        acc[1] += 2.0 * ux;
        acc[2] += -2.0 * (ux * dx + uy * dy);
        acc[3] += -2.0 * px;
        acc[4] += 2.0 * py;
        acc[5] += -2.0 * px * w;
        acc[6] += 2.0 * py * w;
        acc[7] += 2.0 * py * v;
        if (s < nb) {
            acc[8] += 4.0 * ((-v * ca + w * sa) - uy);
            acc[9] += 4.0 * ((-v * sa - w * ca) + ux);
            acc[10] += 4.0 * ((v * v + w * w) + (ux * ux + uy * uy));
            acc[11] += 4.0 * (w - px);
            acc[12] += 4.0 * (v + py);
            acc[13] += 4.0 * (w * w + px * px);
            acc[14] += 4.0 * (w * v - px * py);
            acc[15] += 4.0 * (v * v + py * py);
        }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) acc[q] += shfl_down_d(acc[q], off);
    if ((t & 63) == 0)
#pragma unroll
        for (int q = 0; q < 16; ++q) red[t >> 6][q] = acc[q];
    __syncthreads();
    if (t < 16) out[t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

}  // namespace

extern "C" size_t dpg_icp_lds_bytes(int32_t lds_tgt, int32_t cells_max) {
    size_t o = 0;
    auto a16 = [](size_t x) { return (x + 15) & ~size_t(15); };
    o = a16(o + sizeof(float2) * lds_tgt);
    o = a16(o + sizeof(uint64_t) * lds_tgt);
    o = a16(o + sizeof(uint64_t) * lds_tgt);
    o = a16(o + sizeof(uint32_t) * (cells_max + 1));
    o = a16(o + sizeof(uint16_t) * lds_tgt);
    o = a16(o + sizeof(double) * 2 * kWaves * (kSums + 2));
    o += sizeof(float) * 16;
    return a16(o);
}

extern "C" int dpg_launch_icp(const float* ds_pts_dev, const dpg_icp_edge* edges_dev, int64_t n_edges,
                              const dpg_icp_kparams* kp, int32_t max_points, dpg_icp_result* results_dev,
                              int32_t* trace_dev, void* stream) {
    if (n_edges <= 0) return DPG_OK;
    if (max_points > kp->lds_tgt || kp->lds_tgt > 65535) return DPG_ERR_SIZE;
    const size_t lds = dpg_icp_lds_bytes(kp->lds_tgt, kp->cells_max);
    if (lds > 160 * 1024) return DPG_ERR_SIZE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)n_edges), block(kThreads);
    const float2* pts = reinterpret_cast<const float2*>(ds_pts_dev);
    const int ppt = (max_points + kThreads - 1) / kThreads;
    if (ppt <= 1)
        hipLaunchKernelGGL(icp_edges_kernel<1>, grid, block, lds, s, pts, edges_dev, *kp, results_dev, trace_dev);
    else if (ppt <= 2)
        hipLaunchKernelGGL(icp_edges_kernel<2>, grid, block, lds, s, pts, edges_dev, *kp, results_dev, trace_dev);
    else if (ppt <= 4)
        hipLaunchKernelGGL(icp_edges_kernel<4>, grid, block, lds, s, pts, edges_dev, *kp, results_dev, trace_dev);
    else if (ppt <= 8)
        hipLaunchKernelGGL(icp_edges_kernel<8>, grid, block, lds, s, pts, edges_dev, *kp, results_dev, trace_dev);
    else if (ppt <= 16)
        hipLaunchKernelGGL(icp_edges_kernel<16>, grid, block, lds, s, pts, edges_dev, *kp, results_dev, trace_dev);
    else
        return DPG_ERR_SIZE;
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_launch_cov(const float* full_pts_dev, const dpg_icp_edge* edges_dev, int64_t n_edges,
                              const dpg_icp_result* results_dev, double* hess_dev, int32_t max_workgroups, void* stream) {
    if (n_edges <= 0) return DPG_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t grid = max_workgroups > 0 ? std::min<int64_t>(n_edges, max_workgroups) : n_edges;
    hipLaunchKernelGGL(cov_block_kernel, dim3((unsigned)grid), dim3(kThreads), 0, s,
                       reinterpret_cast<const float2*>(full_pts_dev), edges_dev, n_edges, results_dev, hess_dev);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_launch_cov6(const float* pts_dev, int32_t n_data, int32_t n_model, const float* T6_dev, double* out_dev,
                               void* stream) {
    hipLaunchKernelGGL(cov6_kernel, dim3(1), dim3(kThreads), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const float2*>(pts_dev), n_data, n_model, T6_dev, out_dev);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}
