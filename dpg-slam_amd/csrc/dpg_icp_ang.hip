// dpg_icp_ang.hip -- ICP scan matching, angular-index variant (the default batched ICP kernel).
//
// Same semantics and bit-exact results as the grid / k-d kernels (PCL IterativeClosestPoint with
// reciprocal KdTreeFLANN correspondences, dpg_slam.cc:387-416), with a neighbour index built for
// laser scans: a scan is uniform in ANGLE, not in space (near the sensor its points are a few mm
// apart, far away tens of cm), so every cloud is indexed by the angle of its points around the
// node origin:
//   angle_index_kernel: per node, points sorted by pseudo-angle (an octant polynomial of
//     atan2 in [0, 2 pi): one reciprocal, slope within [0.98, 1.06] of the true angle's) by a
//     bitonic sort in LDS, plus a table of the first sorted position of each of B uniform buckets.
//   exactness: every point p with |p - q| <= rho lies within the angle asin(s) <= s / sqrt(1 - s^2)
//     of q (s = rho/|q| < 1), so its pseudo-angle lies within 1.07 s / sqrt(1 - s^2) (+ a margin
//     far above float error) of q's; the bucket map is the same float function at build and query
//     time; queries with s >= 0.7 scan everything.  tests/test_window_bound.py checks the bound
//     numerically in float32 arithmetic.
//   icp_ang_kernel (one workgroup per edge, all iterations resident in LDS):
//     forward 1-NN: radius = distance to the previous iteration's match (r when unseeded), the
//       window scan keeps the exact (distance, lowest index) argmin;
//     reciprocal test: radius query in the SOURCE index (source node frame, static) around
//       F_k^-1 t_j with radius sqrt(d_ij) + drift_k, candidates re-checked in exact float on their
//       CURRENT coordinates (see dpg_icp_kd.hip for the drift argument);
//     rigid fit + convergence exactly as the other variants (fp64 256-lane fixed tree).
// Built with -ffp-contract=off.

#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "dpg_internal.h"

#ifdef DPG_ICP_STATS
// diagnostics build only: [0] point-iterations, [1] forward candidates, [2] forward wave trips,
// [3] reciprocal candidates, [4] reciprocal wave trips, [5] correspondences, [6] no forward match,
// [7] full-scan forward windows
__device__ unsigned long long g_icp_stats[8];
#define ICP_STAT(k, v) atomicAdd(&g_icp_stats[k], (unsigned long long)(v))
#endif

namespace {

constexpr int kT = 256;
constexpr int kW = kT / 64;
constexpr int kSums = 10;
constexpr int kB = 1024;                        // pseudo-angle buckets per cloud (~1 point each)
constexpr float kTwoPi = 6.28318530717958647692f;
constexpr float kBucketScale = (float)kB / kTwoPi;
constexpr float kPaSlope = 1.07f;               // bound on d(pseudo-angle)/d(angle) (max 1.0584)
constexpr float kPaMargin = 2e-5f;              // absolute pseudo-angle margin (float error ~1e-6)

// pseudo-angle in [0, 2 pi): atan2 approximated per octant by f(t) = t (pi/4 + 0.273 (1 - t)),
// t = min(|x|,|y|) / max(|x|,|y|) (max error 1.5e-3 rad, slope ratio to atan in [0.98, 1.0584]);
// 0 at the origin.
__device__ __forceinline__ float pseudo_angle(float x, float y) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    if (!(mx > 0.0f)) return 0.0f;
    const float t = mn * __builtin_amdgcn_rcpf(mx);
    const float f = t * (1.0584f - 0.273f * t);
    float phi = ay > ax ? 1.5707963f - f : f;
    if (x < 0.0f) phi = 3.14159265f - phi;
    if (y < 0.0f) phi = kTwoPi - phi;
    return phi;
}

__device__ __forceinline__ int bucket_of(float pa) {
    int b = (int)floorf(pa * kBucketScale);
    return min(max(b, 0), kB - 1);
}

__device__ __forceinline__ uint32_t orderable(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// one workgroup per node: points sorted by angle + bucket starts
__global__ __launch_bounds__(kT) void angle_index_kernel(const float2* __restrict__ ds_pts,
                                                         const int64_t* __restrict__ ds_off,
                                                         float2* __restrict__ idx_pts,
                                                         uint16_t* __restrict__ idx_orig,
                                                         uint16_t* __restrict__ buckets /* [V][kB+1] */) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int v = blockIdx.x, tid = threadIdx.x;
    const int64_t off = ds_off[v];
    const int N = (int)(ds_off[v + 1] - off);
    uint16_t* bk = buckets + (size_t)v * (kB + 1);
    if (N <= 0) {
        for (int b = tid; b <= kB; b += kT) bk[b] = 0;
        return;
    }
    int P = 1;
    while (P < N) P <<= 1;
    uint64_t* key = reinterpret_cast<uint64_t*>(smem);   // [P]: orderable(angle) << 32 | index
    for (int s = tid; s < P; s += kT) {
        if (s < N) {
            const float2 p = ds_pts[off + s];
            key[s] = ((uint64_t)orderable(pseudo_angle(p.x, p.y)) << 32) | (uint32_t)s;
        } else {
            key[s] = ~0ull;
        }
    }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int q = tid; q < P / 2; q += kT) {
                const int i = 2 * q - (q & (j - 1));
                const int l = i + j;
                const bool up = (i & k) == 0;
                const uint64_t a = key[i], b = key[l];
                if ((a > b) == up) { key[i] = b; key[l] = a; }
            }
            __syncthreads();
        }
    }
    for (int s = tid; s < N; s += kT) {
        const int o = (int)(key[s] & 0xffffffffu);
        const float2 p = ds_pts[off + o];
        idx_pts[off + s] = p;
        idx_orig[off + s] = (uint16_t)o;
        const int b = bucket_of(pseudo_angle(p.x, p.y));
        int bp = -1;
        if (s > 0) {
            const float2 pp = ds_pts[off + (int)(key[s - 1] & 0xffffffffu)];
            bp = bucket_of(pseudo_angle(pp.x, pp.y));
        }
        for (int bb = bp + 1; bb <= b; ++bb) bk[bb] = (uint16_t)s;   // first sorted position >= bucket
        if (s == N - 1)
            for (int bb = b + 1; bb <= kB; ++bb) bk[bb] = (uint16_t)N;
    }
}

// A point as the search sees it (16 B, one LDS load): coordinates + key = original index << 16 |
// sorted position.  The exact PCL/FLANN order "(float distance, lowest original index)" is then
// the unsigned order of the 64-bit word (bits(d) << 32 | key): d >= 0, so its bits order as it does.
struct Rec {
    float x, y;
    uint32_t key, pad;
};

// one ds_read_b128 per record: the pad word is kept live (an empty asm), otherwise the compiler
// narrows the load to ds_read_b96, which costs twice the LDS cycles per wave (8 vs 4)
__device__ __forceinline__ Rec ld_rec(const Rec* p) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    asm volatile("" : "+v"(v.w));
    return Rec{__uint_as_float(v.x), __uint_as_float(v.y), v.z, v.w};
}

__device__ __forceinline__ uint64_t dkey(float d, uint32_t key) {
    return ((uint64_t)__float_as_uint(d) << 32) | key;
}

struct Lds {
    Rec* tp;          // target points in angle order
    Rec* scs;         // current (moved) source points in the source's angle order
    uint16_t* spos;   // source original index -> sorted position
    uint16_t* tb;     // target bucket starts [kB+1]
    uint16_t* sb;     // source bucket starts [kB+1]
    double* wpart;    // [kW][kSums + 2]
};

__device__ __forceinline__ size_t a16(size_t x) { return (x + 15) & ~size_t(15); }

__device__ Lds carve(unsigned char* base, int cap) {
    Lds L;
    size_t o = 0;
    L.tp = reinterpret_cast<Rec*>(base + o);      o = a16(o + 16 * (size_t)cap);
    L.scs = reinterpret_cast<Rec*>(base + o);     o = a16(o + 16 * (size_t)cap);
    L.spos = reinterpret_cast<uint16_t*>(base + o); o = a16(o + 2 * (size_t)cap);
    L.tb = reinterpret_cast<uint16_t*>(base + o); o = a16(o + 2 * (size_t)(kB + 1));
    L.sb = reinterpret_cast<uint16_t*>(base + o); o = a16(o + 2 * (size_t)(kB + 1));
    L.wpart = reinterpret_cast<double*>(base + o);
    return L;
}

__device__ __forceinline__ float sqd(float ax, float ay, float bx, float by) {
    const float dx = ax - bx, dy = ay - by;
    return dx * dx + dy * dy;
}

// The sorted positions of the points that can lie within `rad` of q (angle window), as ONE
// wrapped range: positions start, start+1, ... (mod n), `count` of them (the whole cloud when
// the window would span too wide an angle).
__device__ __forceinline__ int window(const uint16_t* bk, int n, float qx, float qy, float rad, int& start) {
    const float sn = rad * __builtin_amdgcn_rsqf(qx * qx + qy * qy) * 1.0001f + 1e-6f;   // sin of the half-angle
    if (!(sn < 0.7f)) {
        start = 0;
        return n;
    }
    const float half = kPaSlope * sn * __builtin_amdgcn_rsqf(1.0f - sn * sn) * 1.0001f + kPaMargin;
    const float pq = pseudo_angle(qx, qy);
    float lo = pq - half, hi = pq + half;
    if (lo < 0.0f) lo += kTwoPi;
    if (hi >= kTwoPi) hi -= kTwoPi;
    start = bk[bucket_of(lo)];
    const int end = bk[bucket_of(hi) + 1];
    return lo <= hi ? end - start : (n - start) + end;   // else: straddles pseudo-angle 0
}

template <int PPT>
__global__ __launch_bounds__(kT) void icp_ang_kernel(const float2* __restrict__ ds_pts,
                                                     const float2* __restrict__ idx_pts,
                                                     const uint16_t* __restrict__ idx_orig,
                                                     const uint16_t* __restrict__ buckets,
                                                     const dpg_icp_edge* __restrict__ edges,
                                                     dpg_icp_kparams kp, dpg_icp_result* __restrict__ results,
                                                     int32_t* __restrict__ trace) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int e = blockIdx.x;
    const dpg_icp_edge E = edges[e];
    const int N = E.n_src_ds, M = E.n_tgt_ds;
    const int vt = E.tgt_node, vs = E.src_node;
    const int cap = kp.lds_tgt, mask = cap - 1;   // cap: a power of two >= every cloud
    Lds L = carve(smem, cap);
    // sorted clouds, padded to cap with far-away dummies: a window [start, start + count) then
    // runs modulo cap (one AND per candidate); the dummies in the wrap gap never win
    for (int i = t; i < cap; i += kT) {
        if (i < M) {
            const float2 p = idx_pts[E.tgt_ds_off + i];
            L.tp[i] = Rec{p.x, p.y, ((uint32_t)idx_orig[E.tgt_ds_off + i] << 16) | (uint32_t)i, 0u};
        } else {
            L.tp[i] = Rec{1e18f, 1e18f, 0xffffffffu, 0u};
        }
    }
    for (int s = t; s < cap; s += kT) {
        if (s < N) {
            const uint16_t o = idx_orig[E.src_ds_off + s];
            L.scs[s].key = ((uint32_t)o << 16) | (uint32_t)s;
            L.spos[o] = (uint16_t)s;
        } else {
            L.scs[s] = Rec{1e18f, 1e18f, 0xffffffffu, 0u};
        }
    }
    for (int b = t; b <= kB; b += kT) {
        L.tb[b] = buckets[(size_t)vt * (kB + 1) + b];
        L.sb[b] = buckets[(size_t)vs * (kB + 1) + b];
    }
    float F[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) F[q] = E.guess[q];
    __syncthreads();
    float sx[PPT], sy[PPT];
    int seed[PPT], sp[PPT];
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int i = t + kT * m;
        seed[m] = -1;
        sp[m] = 0;
        sx[m] = 0.f;
        sy[m] = 0.f;
        if (i < N) {
            const float2 p = ds_pts[E.src_ds_off + i];
            sx[m] = (F[0] * p.x + F[1] * p.y) + F[2];
            sy[m] = (F[3] * p.x + F[4] * p.y) + F[5];
            sp[m] = L.spos[i];
            L.scs[sp[m]].x = sx[m];
            L.scs[sp[m]].y = sy[m];
        }
    }
    __syncthreads();

    const float r2f = kp.r2_f;
    const float rmax = sqrtf(r2f) * 1.0001f + 1e-5f;
    double prev_mse = DBL_MAX, last_mse = 0.0;
    int k = 0, converged = 0, status = DPG_ICP_OK, last_cnt = 0;
    for (;;) {
        const double det = (double)F[0] * (double)F[4] - (double)F[1] * (double)F[3];
        const double i00 = (double)F[4] / det, i01 = -(double)F[1] / det;
        const double i10 = -(double)F[3] / det, i11 = (double)F[0] / det;
        const float drift = 1e-4f + 5e-5f * (float)(k + 1);
        double acc[kSums];
#pragma unroll
        for (int q = 0; q < kSums; ++q) acc[q] = 0.0;
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            // every lane runs every step (dead lanes predicated off): the candidate loops below
            // are wave-uniform (exit on __any), with straight-line predicated bodies
            const int i = t + kT * m;
            const bool live = i < N;
            const float qx = sx[m], qy = sy[m];
            // ---- forward 1-NN (target index), seeded radius ----
            uint64_t best = dkey(r2f, 0xffffffffu);   // "none": every candidate with d <= r beats it
            float rad = rmax;
            if (live && seed[m] >= 0) {
                const Rec r = L.tp[seed[m]];
                const float d = sqd(qx, qy, r.x, r.y);
                if (d <= r2f) {
                    best = dkey(d, r.key);
                    rad = sqrtf(d) * 1.0001f + 1e-6f;
                }
            }
            {
                int s = 0;
                int fc = live ? window(L.tb, M, qx, qy, rad, s) : 0;
                s = s >= M ? s - M : s;
                if (s + fc > M) fc += cap - M;   // wraps: step over the padding gap
#ifdef DPG_ICP_STATS
                {
                    int trips = 0;
                    for (int c = 0; __any(c < fc); c += 2) ++trips;
                    if (live) { ICP_STAT(0, 1); ICP_STAT(1, fc); if (fc >= M) ICP_STAT(7, 1); }
                    if (lane == 0) ICP_STAT(2, trips);
                }
#endif
                for (int c = 0; __any(c < fc); c += 2) {   // exact (d, original index) argmin
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const Rec r = ld_rec(L.tp + s);
                        const uint64_t kd = dkey(sqd(qx, qy, r.x, r.y), r.key);
                        best = (c + u < fc && kd < best) ? kd : best;
                        s = (s + 1) & mask;
                    }
                }
            }
            const uint32_t bkey = (uint32_t)best;
            const float bd = __uint_as_float((uint32_t)(best >> 32));
            const int bp = bkey == 0xffffffffu ? -1 : (int)(bkey & 0xffffu);
            const int bi = (int)(bkey >> 16);
            seed[m] = live ? bp : seed[m];
            bool ok = live && bp >= 0;
            // ---- reciprocal test in the static source index ----
            if (kp.reciprocal) {
                float2 tj = make_float2(0.f, 0.f);
                int s = 0, rc = 0;
                if (ok) {
                    const Rec r = L.tp[bp];
                    tj = make_float2(r.x, r.y);
                    const double ux = (double)tj.x - (double)F[2], uy = (double)tj.y - (double)F[5];
                    const float px = (float)(i00 * ux + i01 * uy), py = (float)(i10 * ux + i11 * uy);
                    rc = window(L.sb, N, px, py, sqrtf(bd) * 1.0001f + drift, s);
                    s = s >= N ? s - N : s;
                    if (s + rc > N) rc += cap - N;
                }
                // i's own word: any other current source with a smaller (d, original index) word
                // is closer to t_j (or tied with a lower index) and breaks reciprocity
                const uint64_t mine = dkey(bd, ((uint32_t)i << 16) | (uint32_t)sp[m]);
#ifdef DPG_ICP_STATS
                {
                    int trips = 0;
                    for (int c = 0; __any(ok & (c < rc)); c += 2) ++trips;
                    if (ok) ICP_STAT(3, rc);
                    if (live && !ok) ICP_STAT(6, 1);
                    if (lane == 0) ICP_STAT(4, trips);
                }
#endif
                for (int c = 0; __any(ok & (c < rc)); c += 2) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const Rec r = ld_rec(L.scs + s);
                        const uint64_t kd = dkey(sqd(r.x, r.y, tj.x, tj.y), r.key);
                        ok = ok & !((c + u < rc) & (kd < mine));
                        s = (s + 1) & mask;
                    }
                }
            }
#ifdef DPG_ICP_STATS
            if (ok) ICP_STAT(5, 1);
#endif
            if (live && trace && k < kp.trace_iters)
                trace[((size_t)e * kp.trace_iters + k) * kp.trace_stride + i] = ok ? bi : -1;
            if (ok) {
                const Rec tq = L.tp[bp];
                const double px = qx, py = qy, tx = tq.x, ty = tq.y;
                acc[0] = acc[0] + 1.0;
                acc[1] = acc[1] + (double)bd;
                acc[2] = acc[2] + px;
                acc[3] = acc[3] + py;
                acc[4] = acc[4] + tx;
                acc[5] = acc[5] + ty;
                acc[6] = acc[6] + px * tx;
                acc[7] = acc[7] + px * ty;
                acc[8] = acc[8] + py * tx;
                acc[9] = acc[9] + py * ty;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
            for (int q = 0; q < kSums; ++q) acc[q] = acc[q] + __shfl_down(acc[q], off, 64);
        }
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < kSums; ++q) L.wpart[wave * (kSums + 2) + q] = acc[q];
        }
        __syncthreads();
        double S[kSums];
#pragma unroll
        for (int q = 0; q < kSums; ++q)
            S[q] = (L.wpart[0 * (kSums + 2) + q] + L.wpart[1 * (kSums + 2) + q]) +
                   (L.wpart[2 * (kSums + 2) + q] + L.wpart[3 * (kSums + 2) + q]);
        const int cnt = (int)S[0];
        last_cnt = cnt;
        if (cnt < kp.min_corr) { converged = 0; status = DPG_ICP_TOO_FEW_CORR; break; }
        const double n = S[0];
        const double a = (S[6] + S[9]) - (S[2] * S[4] + S[3] * S[5]) / n;
        const double b = (S[7] - S[8]) - (S[2] * S[5] - S[3] * S[4]) / n;
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
            if (i < N) {
                L.scs[sp[m]].x = sx[m];
                L.scs[sp[m]].y = sy[m];
            }
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
        __syncthreads();
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
        R.z[2] = (float)atan2((double)F[3], (double)F[0]);
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

extern "C" int32_t dpg_angle_buckets(void) { return kB; }

#ifdef DPG_ICP_STATS
extern "C" int dpg_icp_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_icp_stats), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_icp_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

extern "C" size_t dpg_icp_ang_lds_bytes(int32_t cap) {
    auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
    size_t o = 0;
    o = al(o + 16 * (size_t)cap);
    o = al(o + 16 * (size_t)cap);
    o = al(o + 2 * (size_t)cap);
    o = al(o + 2 * (size_t)(kB + 1));
    o = al(o + 2 * (size_t)(kB + 1));
    o += sizeof(double) * kW * (kSums + 2);
    return al(o);
}

extern "C" int dpg_launch_angle_index(const float* ds_pts_dev, const int64_t* ds_off_dev, int64_t n_nodes,
                                      int32_t max_points, float* idx_pts_dev, uint16_t* idx_orig_dev,
                                      uint16_t* buckets_dev, void* stream) {
    if (n_nodes <= 0) return DPG_OK;
    int cap = 1;
    while (cap < max_points) cap <<= 1;
    if (cap > 4096) return DPG_ERR_SIZE;
    hipLaunchKernelGGL(angle_index_kernel, dim3((unsigned)n_nodes), dim3(kT), 8 * (size_t)cap,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float2*>(ds_pts_dev), ds_off_dev,
                       reinterpret_cast<float2*>(idx_pts_dev), idx_orig_dev, buckets_dev);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_launch_icp_ang(const float* ds_pts_dev, const float* idx_pts_dev, const uint16_t* idx_orig_dev,
                                  const uint16_t* buckets_dev, const dpg_icp_edge* edges_dev, int64_t n_edges, const dpg_icp_kparams* kp,
                                  int32_t max_points, dpg_icp_result* results_dev, int32_t* trace_dev, void* stream) {
    if (n_edges <= 0) return DPG_OK;
    if (max_points > kp->lds_tgt || kp->lds_tgt > 4096 || (kp->lds_tgt & (kp->lds_tgt - 1))) return DPG_ERR_SIZE;
    const size_t lds = dpg_icp_ang_lds_bytes(kp->lds_tgt);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)n_edges), block(kT);
    const float2* ds = reinterpret_cast<const float2*>(ds_pts_dev);
    const float2* ip = reinterpret_cast<const float2*>(idx_pts_dev);
    const int ppt = (max_points + kT - 1) / kT;
#define DPG_ANG_LAUNCH(P)                                                                                     \
    hipLaunchKernelGGL(icp_ang_kernel<P>, grid, block, lds, s, ds, ip, idx_orig_dev, buckets_dev, edges_dev, \
                       *kp, results_dev, trace_dev)
    if (ppt <= 1) DPG_ANG_LAUNCH(1);
    else if (ppt <= 2) DPG_ANG_LAUNCH(2);
    else if (ppt <= 4) DPG_ANG_LAUNCH(4);
    else if (ppt <= 8) DPG_ANG_LAUNCH(8);
    else if (ppt <= 16) DPG_ANG_LAUNCH(16);
    else return DPG_ERR_SIZE;
#undef DPG_ANG_LAUNCH
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}
