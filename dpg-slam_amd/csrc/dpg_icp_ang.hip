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
//     rigid fit + convergence exactly as the other variants (fp64 512-lane fixed tree).
// Built with -ffp-contract=off.

#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "dpg_atan2f.h"
#include "dpg_internal.h"
#include "dpg_icp_tree.h"

#if defined(DPG_ICP_STATS) || defined(DPG_ICP_TIMING)
// diagnostics builds only.  DPG_ICP_STATS (counters): [0] point-iterations, [1] forward
// candidates, [2] forward wave trips, [3] reciprocal candidates, [4] reciprocal wave trips,
// [5] correspondences, [6] no forward match, [7] full-scan forward windows, [13] full-scan
// reciprocal windows, [14] sum over workgroup-iterations of the slowest wave's trips, [15] sum
// of all waves' trips (imbalance = 8 [14] / [15]).  DPG_ICP_TIMING
// (per-wave s_memtime cycles summed over waves and iterations, last iteration excluded):
// [8] search, [9] sums + fold, [10] arrival + fit + publish barrier, [11] move + barrier,
// [12] wave-iterations, [45] queue phase (barrier, cooperative scans, barrier, finalize), [40]
// set-up ticks, [41] / [42] shader / 100 MHz ticks from entry to the end of the loop, [43] waves,
// DPG_ICP_SETUPCLK (no other diagnostics): wave 0 of every workgroup records its set-up steps in
// g_icp_setup[dispatch slot][10]: shader ticks at entry, after the target records, source keys,
// bucket tables, barrier, source transform, barrier, at the end; 100 MHz ticks at entry and end.
// DPG_ICP_STATS also: [40] queued forward windows, [41] their candidates, [42] cooperative
// reciprocal scans, [43] their candidates, [44] workgroup-iterations with a non-empty queue,
// [46] float bits of max |moved - (F p + t)| over every moved source point (m, the incremental
// move's accumulated float drift against the exact image of the static point under the current
// float transform), [47] float bits of the max of that drift over the window margin the next
// reciprocal test adds for it, 1e-4 + 5e-5 (k + 1) m (must stay below 1)
#define DPG_ICP_DIAG 1
__device__ unsigned long long g_icp_stats[64];
#define ICP_STAT_ADD(k, v) atomicAdd(&g_icp_stats[k], (unsigned long long)(v))
#endif
#ifdef DPG_ICP_SETUPCLK
constexpr int kSetupSlots = 65536;
__device__ unsigned long long g_icp_setup[kSetupSlots * 10];
#endif
#ifdef DPG_ICP_STATS
#define ICP_STAT(k, v) ICP_STAT_ADD(k, v)
// [16..27] forward / [28..39] reciprocal wave trips of a slot, summed per bin of trips per slot:
// 0, 1, 2, 3, 4, 5-8, 9-16, 17-32, 33-64, 65-128, 129-256, >256
__device__ __forceinline__ int trip_bin(int t) {
    return t <= 4 ? t : t <= 8 ? 5 : t <= 16 ? 6 : t <= 32 ? 7 : t <= 64 ? 8 : t <= 128 ? 9 : t <= 256 ? 10 : 11;
}
#endif
#ifdef DPG_ICP_TIMING
#define ICP_STAMP(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#else
#define ICP_STAMP(var)
#endif

namespace {

constexpr int kT = 512;                         // ICP workgroup (8 waves)
constexpr int kTI = 256;                        // index-build workgroup
constexpr int kSums = dpg_tree::kSums;
constexpr int kB = 1024;                        // pseudo-angle buckets per cloud (~1 point each)
constexpr float kTwoPi = 6.28318530717958647692f;
constexpr float kBucketScale = (float)kB / kTwoPi;
constexpr float kPaSlope = 1.07f;               // bound on d(pseudo-angle)/d(angle) (max 1.0584)
constexpr float kPaMargin = 2e-5f;              // absolute pseudo-angle margin (float error ~1e-6)
// variant 5's window constants (window_pa): the chord bound's coefficient, the slope and the margin
// in bucket units, each rounded up past the float error of the folded expression
constexpr float kWinQuad = 0.8172f * 1.001f;
constexpr float kWinSlope = kPaSlope * 1.0003f * kBucketScale;
constexpr float kWinMargin = (kPaMargin + 2e-6f) * kBucketScale;

// pseudo-angle in [0, 2 pi): atan2 approximated per octant by f(t) = t (pi/4 + 0.273 (1 - t)),
// t = min(|x|,|y|) / max(|x|,|y|) (max error 1.5e-3 rad, slope ratio to atan in [0.98, 1.0584]);
// 0 at the origin.
template <bool kAbsMinMax = false>
__device__ __forceinline__ float pseudo_angle(float x, float y) {
    const float ax = fabsf(x), ay = fabsf(y);
    float mx, mn;
    if constexpr (kAbsMinMax) {   // max / min of the magnitudes straight from x, y (abs operand
        // modifiers, no separate canonicalizing max per magnitude; the same values: no NaN here)
        asm("v_max_f32_e64 %0, |%1|, |%2|" : "=v"(mx) : "v"(x), "v"(y));
        asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(mn) : "v"(x), "v"(y));
    } else {
        mx = fmaxf(ax, ay);
        mn = fminf(ax, ay);
    }
    if (!(mx > 0.0f)) return 0.0f;
    const float t = mn * __builtin_amdgcn_rcpf(mx);
    const float f = t * (1.0584f - 0.273f * t);
    float phi = ay > ax ? 1.5707963f - f : f;
    if (x < 0.0f) phi = 3.14159265f - phi;
    if (y < 0.0f) phi = kTwoPi - phi;
    return phi;
}

// variant 5: the same pseudo-angle in bucket units (pseudo_angle<true> * kBucketScale with the scale
// folded into the constants): the query side only -- within a few ulp of the build side's
// pa * scale, far inside the windows' margin of kPaMargin * scale buckets
constexpr float kPaA = 1.0584f * kBucketScale, kPaB = 0.273f * kBucketScale;
constexpr float kPaQ1 = 1.5707963f * kBucketScale, kPaQ2 = 3.14159265f * kBucketScale, kPaQ4 = kTwoPi * kBucketScale;
__device__ __forceinline__ float pseudo_angle_b(float x, float y) {
    float mx, mn;
    asm("v_max_f32_e64 %0, |%1|, |%2|" : "=v"(mx) : "v"(x), "v"(y));
    asm("v_min_f32_e64 %0, |%1|, |%2|" : "=v"(mn) : "v"(x), "v"(y));
    if (!(mx > 0.0f)) return 0.0f;
    const float t = mn * __builtin_amdgcn_rcpf(mx);
    const float f = t * (kPaA - kPaB * t);
    float phi = fabsf(y) > fabsf(x) ? kPaQ1 - f : f;
    if (x < 0.0f) phi = kPaQ2 - phi;
    if (y < 0.0f) phi = kPaQ4 - phi;
    return phi;
}
// the query's pseudo-angle as the variant's window takes it (radians; bucket units from variant 5)
template <int VAR>
__device__ __forceinline__ float query_angle(float x, float y) {
    if constexpr (VAR >= 5) return pseudo_angle_b(x, y);
    else return pseudo_angle<(VAR >= 4)>(x, y);
}

__device__ __forceinline__ int bucket_of(float pa) {
    int b = (int)floorf(pa * kBucketScale);
    return min(max(b, 0), kB - 1);
}
// the same bucket with the floor and the conversion in one instruction (v_cvt_flr_i32_f32 is
// (int)floorf for the finite pa * scale)
__device__ __forceinline__ int bucket_of_flr(float pa) {
    int b;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(b) : "v"(pa * kBucketScale));
    return min(max(b, 0), kB - 1);
}
template <int VAR>
__device__ __forceinline__ int bucket_q(float pa) {
    if constexpr (VAR >= 5) {   // pa in bucket units already
        int b;
        asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(b) : "v"(pa));
        return min(max(b, 0), kB - 1);
    }
    if constexpr (VAR >= 2) return bucket_of_flr(pa);
    else return bucket_of(pa);
}

__device__ __forceinline__ uint32_t orderable(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// one workgroup per node: the points sorted by (pseudo-angle, original index) and the bucket
// starts.  A counting sort by bucket -- the bucket is monotone in the pseudo-angle, so the bucket
// order refines to the key order -- then each bucket (~1 point at kB = 1024) sorted by its full
// 64-bit key by one thread; a cloud with a bucket of more than kIdxSmall points (a narrow cone)
// sorts the whole array by a bitonic network instead (so does `bitonic`, the A/B reference: the
// round-1..4 build).  The keys are unique, so every path gives the same order; bucket b starts at
// the number of points in buckets < b.  ~8 barriers per cloud instead of the network's 55.
constexpr int kIdxSmall = 16;
static_assert(kB == 4 * kTI, "the bucket scan takes four buckets per thread");
__global__ __launch_bounds__(kTI) void angle_index_kernel(const float2* __restrict__ ds_pts,
                                                         const int64_t* __restrict__ ds_off,
                                                         float2* __restrict__ idx_pts,
                                                         uint16_t* __restrict__ idx_orig,
                                                         uint16_t* __restrict__ buckets /* [V][kB+1] */,
                                                         int32_t bitonic) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int cnt[kB];          // bucket sizes, then the scatter cursors
    __shared__ int bstart[kB + 1];   // first sorted position of each bucket
    __shared__ int wsum[kTI / 64];
    __shared__ int big;
    const int v = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t off = ds_off[v];
    const int N = (int)(ds_off[v + 1] - off);
    uint16_t* bk = buckets + (size_t)v * (kB + 1);
    if (N <= 0) {
        for (int b = tid; b <= kB; b += kTI) bk[b] = 0;
        return;
    }
    uint64_t* key = reinterpret_cast<uint64_t*>(smem);   // [P]: orderable(angle) << 32 | index
    for (int b = tid; b < kB; b += kTI) cnt[b] = 0;
    if (tid == 0) big = bitonic;
    __syncthreads();
    for (int s = tid; s < N; s += kTI) {
        const float2 p = ds_pts[off + s];
        atomicAdd(&cnt[bucket_of(pseudo_angle(p.x, p.y))], 1);
    }
    __syncthreads();
    {   // exclusive scan: thread t owns buckets 4t .. 4t + 3
        int c[4], run = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            c[j] = cnt[4 * tid + j];
            run += c[j];
        }
        int inc = run;   // inclusive scan of the per-thread sums inside the wave
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int u = __shfl_up(inc, d, 64);
            if (lane >= d) inc += u;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        int base = inc - run;
        for (int w = 0; w < wave; ++w) base += wsum[w];
        int mx = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bstart[4 * tid + j] = base;
            base += c[j];
            mx = max(mx, c[j]);
            cnt[4 * tid + j] = 0;   // only this thread reads these four
        }
        if (tid == 0) bstart[kB] = N;
        if (mx > kIdxSmall) big = 1;
    }
    __syncthreads();
    if (!big) {
        for (int s = tid; s < N; s += kTI) {
            const float2 p = ds_pts[off + s];
            const float pa = pseudo_angle(p.x, p.y);
            const int b = bucket_of(pa);
            key[bstart[b] + atomicAdd(&cnt[b], 1)] = ((uint64_t)orderable(pa) << 32) | (uint32_t)s;
        }
        __syncthreads();
        for (int b = tid; b < kB; b += kTI) {   // insertion sort of one bucket by its full keys
            const int lo = bstart[b], hi = bstart[b + 1];
            for (int i = lo + 1; i < hi; ++i) {
                const uint64_t k = key[i];
                int j = i - 1;
                while (j >= lo && key[j] > k) {
                    key[j + 1] = key[j];
                    --j;
                }
                key[j + 1] = k;
            }
        }
        __syncthreads();
    } else {
        int P = 1;
        while (P < N) P <<= 1;
        for (int s = tid; s < P; s += kTI) {
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
                for (int q = tid; q < P / 2; q += kTI) {
                    const int i = 2 * q - (q & (j - 1));
                    const int l = i + j;
                    const bool up = (i & k) == 0;
                    const uint64_t a = key[i], b = key[l];
                    if ((a > b) == up) { key[i] = b; key[l] = a; }
                }
                __syncthreads();
            }
        }
    }
    for (int s = tid; s < N; s += kTI) {
        const int o = (int)(key[s] & 0xffffffffu);
        idx_pts[off + s] = ds_pts[off + o];
        idx_orig[off + s] = (uint16_t)o;
    }
    for (int b = tid; b <= kB; b += kTI) bk[b] = (uint16_t)bstart[b];
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

// Workgroup shape: kT = 512 threads (8 waves; 4 workgroups = 32 waves per CU at <= 64 VGPRs and
// ~38 KB of LDS each), thread t owns the source points i = t + kT m and is lane t of the fp64
// reduction tree (dpg_icp_tree.h, DPG_ICP_LANES = 512).  Per iteration:
//   1. search: each thread runs the forward and reciprocal windows of its points in its own lane;
//      a window of more than kp.defer_cap candidates goes to the workgroup's cooperative queue
//      instead (a point near the sensor origin can span the whole cloud, and one such lane used to
//      hold its wave -- and the other seven at the fit -- for a full scan);
//   2. barrier; the waves drain the queue, one item per wave at a time, 64 candidates per trip,
//      wave-wide argmin / any (same exact result as the lane's own scan); barrier (only when the
//      queue was not empty);
//   3. each thread finalizes its points, sums its accepted pairs (tree lane t), the wave folds by
//      DPP/swizzle, and the LAST wave to arrive (LDS counter) combines the eight partials, fits
//      and decides convergence; one barrier publishes the result; the source moves; barrier.
//
// In-lane candidate loops (R4) visit kU records per trip, wave-uniformly, with no per-candidate
// bounds test: a lane whose own window is exhausted keeps evaluating the records that follow it.
// That is exact -- every record visited is a real point of the cloud, so the forward argmin over a
// superset of the window that contains the true nearest neighbour is the same (distance, lowest
// original index) minimum, and any extra source record that beats i at t_j is a genuine
// reciprocity violation.  Records [n, n + kU) repeat [0, kU) mod n so that a trip never wraps
// inside itself; the trip start advances by kU mod n.  The cooperative scan visits the window
// exactly.
constexpr int kWaves = kT / 64;
static_assert(kT == dpg_tree::kLanes, "one tree lane per thread");
#ifndef DPG_ANG_KU
#define DPG_ANG_KU 4
#endif
#ifndef DPG_ANG_WPE
#define DPG_ANG_WPE 8
#endif
constexpr int kU = DPG_ANG_KU;   // candidates per trip
// an unmatched point searches kClear beyond r once; while the distance it has moved since stays
// below the margin found, it provably has no target within r and skips its forward search
constexpr float kClear = 0.1f;
constexpr int kQCap = 64;        // cooperative queue items per iteration (a full queue: in-lane scan)

// One queued window (16 B), as indices only: the wave that takes it recomputes the window from
// LDS, with the same float expressions the owner would have used.  w0 = i | sp << 16 (source
// original index, sorted position); w1 = kind (0 forward, 1 reciprocal) | v << 1 with v = the
// point's seed + 1 (forward) or its forward match position (reciprocal); w2, w3 = result: the
// best key of a forward item (lo, hi) and, in bit 0 of w1 after the scan, whether the point has a
// (reciprocal) correspondence.
struct QItem {
    uint32_t w[4];
};

// what the fitting wave hands every wave after the fit of an iteration
struct Bcast {
    double inv[4];   // inverse of the new 2x2 rotation block (reciprocal windows), fp64
    double mse;
    double prev_mse; // wave 0's convergence state
    float F[6];      // final transform so far
    float r[4];      // this iteration's (cos, sin, tx, ty)
    int code;        // 0 continue, 1 converged (stop), 2 too few correspondences (stop)
    int cnt;
    int qtail;       // cooperative queue: items pushed this iteration (may exceed kQCap)
    int qhead;       // unused
    int iter;        // iterations fitted so far (every wave checks it after the publish barrier)
    float finv[4];   // the inverse rounded to float, as the reciprocal windows use it (variant 3)
    float drift;     // the next reciprocal tests' drift margin 1e-4 + 5e-5 (k + 1) m (variant 3)
};

// fp64 inverse of the 2x2 block of a 2x3 float transform (same expressions every time)
__device__ __forceinline__ void inverse2(const float F[6], double inv[4]) {
    const double det = (double)F[0] * (double)F[4] - (double)F[1] * (double)F[3];
    inv[0] = (double)F[4] / det;
    inv[1] = -(double)F[1] / det;
    inv[2] = -(double)F[3] / det;
    inv[3] = (double)F[0] / det;
}

struct Lds {
    Rec* tp;          // target points in angle order, [cap + kU]
    Rec* scs;         // current (moved) source points in the source's angle order, [cap + kU]
    uint16_t* spos;   // source original index -> sorted position (setup only)
    QItem* q;         // cooperative queue [kQCap] (aliases spos after the setup)
    uint16_t* tb;     // target bucket starts [kB+1]
    uint16_t* sb;     // source bucket starts [kB+1]
    double* wpart;    // [kWaves][kSums + 2] wave partials of the tree
    int* arrive;      // waves done with this iteration's sums
    Bcast* bc;        // wave 0's fit, read by every wave
};

// Record placement by cloud size (MODE): 0 -- target and source records in LDS (clouds up to 4096
// points); 1 -- the source records in a global scratch slice of the edge, the target in LDS (up to
// 8192); 2 -- both in global scratch (up to 16384).  The scratch slice of workgroup b is
// [2 (cap + kU)] records at gscr + 2 (cap + kU) b: target, then source.
constexpr int kModeMaxPts[3] = {4096, 8192, 16384};

__host__ __device__ inline size_t ang_lds_layout(int cap, size_t* off /* [7] or null */, int mode = 0) {
    size_t o = 0, p[7];
    const size_t spos_q = 2 * (size_t)cap > sizeof(QItem) * kQCap ? 2 * (size_t)cap : sizeof(QItem) * kQCap;
    p[0] = o; o = (o + (mode == 2 ? 0 : 16 * (size_t)(cap + kU)) + 15) & ~size_t(15);
    p[1] = o; o = (o + (mode >= 1 ? 0 : 16 * (size_t)(cap + kU)) + 15) & ~size_t(15);
    p[2] = o; o = (o + spos_q + 15) & ~size_t(15);
    p[3] = o; o = (o + 2 * (size_t)(kB + 1) + 15) & ~size_t(15);
    p[4] = o; o = (o + 2 * (size_t)(kB + 1) + 15) & ~size_t(15);
    p[5] = o; o = (o + sizeof(double) * kWaves * (kSums + 2) + 15) & ~size_t(15);
    p[6] = o; o = (o + sizeof(Bcast) + 16 + 15) & ~size_t(15);
    if (off)
        for (int q = 0; q < 7; ++q) off[q] = p[q];
    return o;
}

template <int MODE>
__device__ Lds carve(unsigned char* base, int cap, Rec* gscr) {
    size_t p[7];
    ang_lds_layout(cap, p, MODE);
    Lds L;
    Rec* g = gscr + (size_t)blockIdx.x * 2 * (size_t)(cap + kU);
    L.tp = MODE == 2 ? g : reinterpret_cast<Rec*>(base + p[0]);
    L.scs = MODE >= 1 ? g + (cap + kU) : reinterpret_cast<Rec*>(base + p[1]);
    L.spos = reinterpret_cast<uint16_t*>(base + p[2]);
    L.q = reinterpret_cast<QItem*>(base + p[2]);
    L.tb = reinterpret_cast<uint16_t*>(base + p[3]);
    L.sb = reinterpret_cast<uint16_t*>(base + p[4]);
    L.wpart = reinterpret_cast<double*>(base + p[5]);
    L.bc = reinterpret_cast<Bcast*>(base + p[6]);
    L.arrive = reinterpret_cast<int*>(base + p[6] + ((sizeof(Bcast) + 15) & ~size_t(15)));
    return L;
}

typedef float f2v __attribute__((ext_vector_type(2)));

// kU consecutive records with four ds_read_b128 issued back to back and ONE wait (the compiler,
// left alone, narrows an unused pad word to ds_read_b96 -- 8 LDS cycles instead of 4 -- or
// serialises the loads behind per-load waits under the 64-VGPR budget)
template <bool kLds, int KN = kU>
__device__ __forceinline__ void ld_recs(const Rec* p, uint4 (&r)[KN]) {
    static_assert(KN == 2 || KN == 4 || KN == 8, "ld_recs issues two, four or eight loads");
    if constexpr (!kLds) {   // records in global scratch (large clouds): plain 16-byte loads
        const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
        for (int u = 0; u < KN; ++u) r[u] = q[u];
        return;
    }
    const uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>(p);   // LDS byte offset
    if constexpr (KN == 2) {
        asm volatile(
            "ds_read_b128 %0, %2\n\t"
            "ds_read_b128 %1, %2 offset:16\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(r[0]), "=&v"(r[1])
            : "v"(a)
            : "memory");
    } else if constexpr (KN == 4) {
        asm volatile(
            "ds_read_b128 %0, %4\n\t"
            "ds_read_b128 %1, %4 offset:16\n\t"
            "ds_read_b128 %2, %4 offset:32\n\t"
            "ds_read_b128 %3, %4 offset:48\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
            : "v"(a)
            : "memory");
    } else {
        asm volatile(
            "ds_read_b128 %0, %8\n\t"
            "ds_read_b128 %1, %8 offset:16\n\t"
            "ds_read_b128 %2, %8 offset:32\n\t"
            "ds_read_b128 %3, %8 offset:48\n\t"
            "ds_read_b128 %4, %8 offset:64\n\t"
            "ds_read_b128 %5, %8 offset:80\n\t"
            "ds_read_b128 %6, %8 offset:96\n\t"
            "ds_read_b128 %7, %8 offset:112\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7])
            : "v"(a)
            : "memory");
    }
}

// workgroup-uniform values (the transform, the reduced sums) kept in SGPRs: frees VGPRs for the
// candidate loops (8 waves per SIMD need <= 64)
__device__ __forceinline__ float uni(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ double uni(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane(x); }

// squared distance, (ax - bx)^2 + (ay - by)^2 in float: packed subtract / multiply (v_pk_*_f32,
// the same IEEE operations lane by lane), then one add -- bit-identical to the scalar form.
__device__ __forceinline__ float sqd(float ax, float ay, float bx, float by) {
    f2v d = (f2v){ax, ay} - (f2v){bx, by};
    d = d * d;
    return d.x + d.y;
}

// one candidate record r against (qx, qy): the 64-bit order word (bits(d) << 32 | key) with d
// computed straight into the record's pad register (the hi half of the word: no register move),
// d = (qx - rx)^2 + (qy - ry)^2 in float as sqd (packed subtract / multiply, one add)
__device__ __forceinline__ uint64_t cand_key(const uint4& r, float qx, float qy) {
    f2v d = (f2v){qx, qy} - (f2v){__uint_as_float(r.x), __uint_as_float(r.y)};
    d = d * d;
    uint32_t w = r.w;
    asm volatile("v_add_f32 %0, %1, %2" : "+v"(w) : "v"(d.x), "v"(d.y));
    return ((uint64_t)w << 32) | r.z;
}

// hardware square root (<= 1 ulp): only ever used for window radii and clearances that carry a
// relative margin of >= 1e-5, so the windows stay supersets (exact) without the correctly
// rounded sequence
__device__ __forceinline__ float hw_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
template <int VAR>
__device__ __forceinline__ float bsqrt(float x) {
    if constexpr (VAR >= 1) return hw_sqrt(x);
    else return sqrtf(x);
}

// (s + step) mod n for s in [0, n), step = kU mod n < n: one add and an unsigned min
__device__ __forceinline__ int advance(int s, int step, int n) {
    const uint32_t a = (uint32_t)(s + step);
    return (int)min(a, a - (uint32_t)n);
}

// The sorted positions of the points that can lie within `rad` of q (angle window), as ONE
// wrapped range: start in [0, n), `count` positions (the whole cloud when the window would span
// too wide an angle).
template <int VAR = 1>
__device__ __forceinline__ int window_pa(const uint16_t* bk, int n, float qx, float qy, float pq, float rad, int& start);
template <int VAR = 1>
__device__ __forceinline__ int window(const uint16_t* bk, int n, float qx, float qy, float rad, int& start) {
    return window_pa<VAR>(bk, n, qx, qy, query_angle<VAR>(qx, qy), rad, start);
}
// the same with q's pseudo-angle pq already computed (the forward search computes it once for the
// unseeded probe and the window)
template <int VAR>
__device__ __forceinline__ int window_pa(const uint16_t* bk, int n, float qx, float qy, float pq, float rad, int& start) {
    if constexpr (VAR >= 5) {
        // variant 5: the same bound with its margins folded into three constants, in bucket units.
        // s0 = rad / |q| is within 4e-7 of the sine; hs >= kPaSlope sn (1 + 0.8172 sn^2) scale +
        // the absolute margins of the form below (its 1.0001 factors and the 1e-6 on the sine are
        // inside the 1.0003 and the 2e-6), so the window is a superset of the form below's ideal
        // one; s0 < 0.6999 keeps sn < 0.7, the chord bound's domain
        const float s0 = rad * __builtin_amdgcn_rsqf(qx * qx + qy * qy);
        if (!(s0 < 0.6999f)) {
            start = 0;
            return n;
        }
        const float hs = fmaf(s0 * fmaf(s0 * s0, kWinQuad, 1.0f), kWinSlope, kWinMargin);
        const float ps = pq;   // bucket units (query_angle)
        int blo, bhi;
        asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(blo) : "v"(ps - hs));
        asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(bhi) : "v"(ps + hs));
        const bool wrap = blo < 0 || bhi >= kB;
        const int s = bk[blo & (kB - 1)];
        const int end = bk[(bhi & (kB - 1)) + 1];
        const int cnt = wrap ? (n - s) + end : end - s;
        start = s >= n ? s - n : s;
        return min(cnt, n);
    }
    const float sn = rad * __builtin_amdgcn_rsqf(qx * qx + qy * qy) * 1.0001f + 1e-6f;   // sin of the half-angle
    if (!(sn < 0.7f)) {
        start = 0;
        return n;
    }
    // 1 / sqrt(1 - x) is convex on x = sn^2 in [0, 0.49]: below its chord 1 + 0.8172 x (the value
    // 1/sqrt(0.51) = 1.40028 at the end), so the half-angle bound needs no reciprocal square root
    // (the window only widens: a superset, exact as above)
    const float half = kPaSlope * sn * fmaf(sn * sn, 0.8172f, 1.0f) * 1.0001f + kPaMargin;
    if constexpr (VAR >= 3) {
        // the wrap at pseudo-angle 0 in bucket space: floor((pq -+ half) * scale) taken modulo kB
        // (a power of two) -- the same buckets as wrapping the angle first, up to a few ulp of the
        // bucket coordinate, far inside the kPaMargin the half-angle carries; a window that rounds
        // to more than the cloud is the whole cloud
        static_assert((kB & (kB - 1)) == 0, "bucket count is a power of two");
        int blo, bhi;
        asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(blo) : "v"((pq - half) * kBucketScale));
        asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(bhi) : "v"((pq + half) * kBucketScale));
        const bool wrap = blo < 0 || bhi >= kB;   // straddles pseudo-angle 0
        const int s = bk[blo & (kB - 1)];
        const int end = bk[(bhi & (kB - 1)) + 1];
        const int cnt = wrap ? (n - s) + end : end - s;
        start = s >= n ? s - n : s;
        return min(cnt, n);
    }
    float lo = pq - half, hi = pq + half;
    if (lo < 0.0f) lo += kTwoPi;
    if (hi >= kTwoPi) hi -= kTwoPi;
    int s = bk[bucket_q<VAR>(lo)];
    const int end = bk[bucket_q<VAR>(hi) + 1];
    const int cnt = lo <= hi ? end - s : (n - s) + end;   // else: straddles pseudo-angle 0
    start = s >= n ? s - n : s;
    return cnt;
}

// Wave-level reservation of queue slots for the lanes that want one: one LDS atomic per wave.
// Returns the lane's slot, or -1 (no request, or the queue is full: the lane scans in-lane).
// Called by all 64 lanes.
__device__ __forceinline__ int queue_push(bool want, int* tail) {
    const uint64_t mask = __ballot(want);
    if (mask == 0) return -1;
    int base = 0;
    if ((threadIdx.x & 63) == 0) base = atomicAdd(tail, __popcll(mask));
    base = __builtin_amdgcn_readfirstlane(base);
    const int idx = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    return (want && idx < kQCap) ? idx : -1;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, off, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), off, 64);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ double rdlane(double x, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// The forward search's starting point for a point at q (R4 seeding): seed >= 0 is the last
// match (its distance bounds the radius), -1 means no knowledge (search r + kClear, probing the
// target at q's own bearing first).  Returns the initial best key and sets the radius.  Used by
// the owner lane and by the cooperative scan with identical arithmetic.
template <int VAR>
__device__ __forceinline__ uint64_t forward_init(const Lds& L, int M, int sd, float qx, float qy, float pq, float r2f, float rmax,
                                                 float rext, float r2ext, float& rad) {
    uint64_t best = dkey(r2f, 0xffffffffu);   // "none": every candidate with d <= r beats it
    rad = rmax;
    if (sd == -1) {
        rad = rext;
        best = dkey(r2ext, 0xffffffffu);
        int p0 = L.tb[bucket_q<VAR>(VAR >= 2 ? pq : pseudo_angle(qx, qy))];
        p0 = p0 >= M ? 0 : p0;
        if (M > 0) {
            const Rec r = L.tp[p0];
            const float d = sqd(qx, qy, r.x, r.y);
            if (d <= r2ext) {
                best = dkey(d, r.key);
                rad = bsqrt<VAR>(d) * 1.0001f + 1e-6f;
            }
        }
    } else {
        const Rec r = L.tp[sd];
        const float d = sqd(qx, qy, r.x, r.y);
        if (d <= r2f) {
            best = dkey(d, r.key);
            rad = bsqrt<VAR>(d) * 1.0001f + 1e-6f;
        }
    }
    return best;
}

// per-point state, one register: sorted position << 16 | seed (int16: >= 0 last match, -1 no
// knowledge, < -1 clearance in 1e-4 m)
__device__ __forceinline__ int st_seed(uint32_t st) { return (int)(int16_t)(uint16_t)(st & 0xffffu); }
__device__ __forceinline__ int st_sp(uint32_t st) { return (int)(st >> 16); }
__device__ __forceinline__ uint32_t st_with_seed(uint32_t st, int seed) { return (st & 0xffff0000u) | (uint32_t)(uint16_t)(int16_t)seed; }

// waves per SIMD: 8 for clouds up to 1024 points (<= 64 VGPRs); wider forms hold more points per
// lane in registers and are limited by LDS anyway (2 workgroups per CU at 2048 points, 1 above):
// 4 (<= 128 VGPRs) at 4 points per lane, 2 (<= 256) beyond
constexpr int ang_wpe(int ppt, int mode) { return mode == 0 && ppt <= 2 ? DPG_ANG_WPE : mode == 0 && ppt == 4 ? 4 : 2; }

template <int PPT, int MODE, int VAR>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(ang_wpe(PPT, MODE), ang_wpe(PPT, MODE)))) void icp_ang_kernel(const float2* __restrict__ ds_pts,
                                                     const float2* __restrict__ idx_pts,
                                                     const uint16_t* __restrict__ idx_orig,
                                                     const uint16_t* __restrict__ buckets,
                                                     const dpg_icp_edge* __restrict__ edges,
                                                     dpg_icp_kparams kp, dpg_icp_result* __restrict__ results,
                                                     int32_t* __restrict__ trace, Rec* __restrict__ gscr) {
    constexpr bool kTpL = MODE != 2, kScsL = MODE == 0;   // records in LDS?
    // issue priority for the synchronised phases (variant 1): 2 from the search barrier to the
    // next search, 3 for the fit -- the other seven waves of the workgroup wait on them, while the
    // searches of the CU's other workgroups fill the SIMDs (config 4: kernel -1.5 %, A/B in one
    // process, profiles/r03/v6_icp_variant_ab.txt)
    constexpr bool kPrio = VAR >= 1;
    // queue slots: PPT <= 4 packs them into okq / qhi (7 bits each), wider forms keep a byte per point
    constexpr bool kWideQ = PPT >= 8;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const dpg_icp_edge E = edges[blockIdx.x];   // dispatch order (dpg_icp_batch_prepare)
    const int e = E.pad[0];                     // the edge's index in the caller's list
    const int N = E.n_src_ds, M = E.n_tgt_ds;
    const int vt = E.tgt_node, vs = E.src_node;
    const int cap = kp.lds_tgt;
    const int dcap = kp.defer_cap > 0 ? kp.defer_cap : 0x7fffffff;   // windows above it are queued
#ifdef DPG_ICP_TIMING
    // per wave: shader-clock ticks and constant 100 MHz ticks over the whole workgroup (their ratio is
    // the shader clock the edge ran at), and the set-up's shader ticks (records into LDS)
    const unsigned long long c_in = __builtin_amdgcn_s_memtime(), r_in = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef DPG_ICP_STATS
    __shared__ unsigned st_wmax;
    if (t == 0) st_wmax = 0;
#endif
    constexpr int kTrip = kU;   // candidates per trip
    const int stepM = M > 0 ? kTrip % M : 0, stepN = N > 0 ? kTrip % N : 0;
    Lds L = carve<MODE>(smem, cap, gscr);
#ifdef DPG_ICP_SETUPCLK
    const unsigned long long su0 = __builtin_amdgcn_s_memtime(), sr0 = __builtin_amdgcn_s_memrealtime();
#endif
    // sorted target + the kU repeated records after it
    for (int i = t; i < M + kU && M > 0; i += kT) {
        const int p = i < M ? i : (i - M) % M;
        const float2 q = idx_pts[E.tgt_ds_off + p];
        L.tp[i] = Rec{q.x, q.y, ((uint32_t)idx_orig[E.tgt_ds_off + p] << 16) | (uint32_t)p, 0u};
    }
#ifdef DPG_ICP_SETUPCLK
    const unsigned long long su1 = __builtin_amdgcn_s_memtime();
#endif
    for (int s = t; s < N + kU && N > 0; s += kT) {
        const int p = s < N ? s : (s - N) % N;
        const uint16_t o = idx_orig[E.src_ds_off + p];
        L.scs[s].key = ((uint32_t)o << 16) | (uint32_t)p;
        L.scs[s].pad = 0u;
        if (s < N) L.spos[o] = (uint16_t)s;
    }
#ifdef DPG_ICP_SETUPCLK
    const unsigned long long su2 = __builtin_amdgcn_s_memtime();
#endif
    for (int b = t; b <= kB; b += kT) {
        L.tb[b] = buckets[(size_t)vt * (kB + 1) + b];
        L.sb[b] = buckets[(size_t)vs * (kB + 1) + b];
    }
#ifdef DPG_ICP_SETUPCLK
    const unsigned long long su3 = __builtin_amdgcn_s_memtime();
#endif
    float F[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) F[q] = uni(E.guess[q]);
    if (t == 0) {   // loop state lives in LDS (SGPR budget of 8 waves per SIMD)
        Bcast B;
        inverse2(F, B.inv);
        B.mse = 0.0;
        B.prev_mse = DBL_MAX;
#pragma unroll
        for (int q = 0; q < 6; ++q) B.F[q] = F[q];
        B.r[0] = B.r[1] = B.r[2] = B.r[3] = 0.f;
        B.code = 0;
        B.cnt = 0;
        B.qtail = 0;
        B.qhead = 0;
        B.iter = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) B.finv[q] = (float)B.inv[q];
        B.drift = 1e-4f + 5e-5f * (float)1;
        *L.bc = B;
        *L.arrive = 0;
    }
    __syncthreads();
#ifdef DPG_ICP_SETUPCLK
    const unsigned long long su4 = __builtin_amdgcn_s_memtime();
#endif
    float sx[PPT], sy[PPT];
    uint32_t st[PPT];
    // store the moved source point at its sorted position (and its repeat past n)
    auto put = [&](int m) {
        const int sp = st_sp(st[m]);
        L.scs[sp].x = sx[m];
        L.scs[sp].y = sy[m];
        if (sp < kU)
            for (int r = N + sp; r < N + kU; r += N) {
                L.scs[r].x = sx[m];
                L.scs[r].y = sy[m];
            }
    };
#pragma unroll
    for (int m = 0; m < PPT; ++m) {
        const int i = t + kT * m;
        st[m] = st_with_seed(0u, -1);
        sx[m] = 0.f;
        sy[m] = 0.f;
        if (i < N) {
            const float2 p = ds_pts[E.src_ds_off + i];
            sx[m] = (F[0] * p.x + F[1] * p.y) + F[2];
            sy[m] = (F[3] * p.x + F[4] * p.y) + F[5];
            st[m] = ((uint32_t)L.spos[i] << 16) | (st[m] & 0xffffu);
            put(m);
        }
    }
#ifdef DPG_ICP_SETUPCLK
    const unsigned long long su5 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();   // spos is dead from here on: its LDS holds the queue
#ifdef DPG_ICP_SETUPCLK
    const unsigned long long su6 = __builtin_amdgcn_s_memtime();
#endif

    const float r2f = kp.r2_f;
    const float rmax = sqrtf(r2f) * 1.0001f + 1e-5f;
    const float rmax_hi = sqrtf(r2f) * 1.00001f + 1e-6f;   // every target beyond it has float d > r^2
    const float rext = rmax + kClear, r2ext = rext * rext;
    int k = 0, converged = 0, status = DPG_ICP_OK;
#ifdef DPG_ICP_TIMING
    unsigned long long ph[5] = {0, 0, 0, 0, 0}, nit = 0;
    const unsigned long long c_setup = __builtin_amdgcn_s_memtime() - c_in;
#endif
    // the forward result of a point (best key) -> its match position (-1: none) and next seed
    auto forward_done = [&](int m, uint64_t best, bool ext) -> int {
        const uint32_t bkey = (uint32_t)best;
        const float bd = __uint_as_float((uint32_t)(best >> 32));
        const int bp = (bkey == 0xffffffffu || bd > r2f) ? -1 : (int)(bkey & 0xffffu);   // R4: d > r^2 rejected
        int nsd = bp;
        if (bp < 0 && ext) {   // nothing within r: the nearest target is >= min(sqrt(bd), rext) away
            const float clr = fminf(bsqrt<VAR>(bd), rext) * 0.99999f - rmax_hi;
            const int q = clr > 0.f ? (int)(clr * 1e4f) : 0;   // units of 1e-4 m, rounded down
            nsd = -1 - q;
        }
        st[m] = st_with_seed(st[m], nsd);
        return bp;
    };
    for (;;) {
        ICP_STAMP(c0);
        if constexpr (kPrio) __builtin_amdgcn_s_setprio(0);
        // variant 3: the inverse and the drift margin arrive as floats (no per-slot conversions)
        const float i00 = uni(VAR >= 3 ? L.bc->finv[0] : (float)L.bc->inv[0]), i01 = uni(VAR >= 3 ? L.bc->finv[1] : (float)L.bc->inv[1]);
        const float i10 = uni(VAR >= 3 ? L.bc->finv[2] : (float)L.bc->inv[2]), i11 = uni(VAR >= 3 ? L.bc->finv[3] : (float)L.bc->inv[3]);
        const float ftx = uni(L.bc->F[2]), fty = uni(L.bc->F[5]);
        const float drift = VAR >= 3 ? uni(L.bc->drift) : 1e-4f + 5e-5f * (float)(k + 1);
        // bit m: point t + 512 m has a (reciprocal) correspondence; bits 8 + 7 m ..: queue slot + 1
        uint32_t okq = 0;
        static_assert(PPT <= 32, "one ok bit per point");
        uint32_t qhi = 0;   // PPT == 4: the slot of point 3 (7 bits)
        uint32_t qsl[kWideQ ? PPT / 4 : 1];   // PPT >= 8: slot + 1 of point m in byte m of qsl
#pragma unroll
        for (int q = 0; q < (kWideQ ? PPT / 4 : 1); ++q) qsl[q] = 0;
#ifdef DPG_ICP_STATS
        unsigned wtrips = 0;
#endif
        auto set_slot = [&](int m, int slot) {
            if constexpr (kWideQ) qsl[m >> 2] |= (uint32_t)(slot + 1) << (8 * (m & 3));
            else if (m < 3) okq |= (uint32_t)(slot + 1) << (8 + 7 * m);
            else qhi |= (uint32_t)(slot + 1) << (7 * (m - 3));
        };
        auto get_slot = [&](int m) -> int {
            if constexpr (kWideQ) return (int)((qsl[m >> 2] >> (8 * (m & 3))) & 0xffu) - 1;
            else return (int)(m < 3 ? (okq >> (8 + 7 * m)) & 0x7fu : (qhi >> (7 * (m - 3))) & 0x7fu) - 1;
        };
        {
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            // every lane runs every trip (dead lanes included): the candidate loops are
            // wave-uniform (exit on __any) with straight-line bodies
            const int i = t + kT * m;
            const bool live = i < N;
            const float qx = sx[m], qy = sy[m];
            const int sd = st_seed(st[m]);
            // ---- forward 1-NN (target index), seeded radius ----
            const bool search = live && sd >= -1;   // < -1: clearance, provably no target within r
            float rad;
            const float pq = VAR >= 2 ? query_angle<VAR>(qx, qy) : 0.f;   // once for the probe and the window
            uint64_t best = forward_init<VAR>(L, M, search ? sd : 0, qx, qy, pq, r2f, rmax, rext, r2ext, rad);
            bool pend;   // this point's forward window went to the queue
            {
                int s = 0;
                int fc = search ? (VAR >= 2 ? window_pa<VAR>(L.tb, M, qx, qy, pq, rad, s) : window(L.tb, M, qx, qy, rad, s)) : 0;
                const int slot = queue_push(fc > dcap, &L.bc->qtail);
                pend = slot >= 0;
                if (pend) {
                    *reinterpret_cast<uint2*>(&L.q[slot].w[0]) =
                        make_uint2((uint32_t)i | ((uint32_t)st_sp(st[m]) << 16), (uint32_t)(sd + 1) << 1);
                    set_slot(m, slot);
                    fc = 0;
                }
#ifdef DPG_ICP_STATS
                {
                    int trips = 0;
                    for (int c = 0; __any(c < fc); c += kTrip) ++trips;
                    if (live) { ICP_STAT(0, 1); ICP_STAT(1, fc); if (fc >= M) ICP_STAT(7, 1); }
                    if (lane == 0) { ICP_STAT(2, trips); ICP_STAT(16 + trip_bin(trips), trips); }
                    wtrips += trips;
                }
#endif
                auto ftrip = [&]() {
                    uint4 r[kTrip];
                    ld_recs<kTpL, kTrip>(L.tp + s, r);
#pragma unroll
                    for (int u = 0; u < kTrip; ++u) {
                        uint64_t kd;
                        if constexpr (VAR >= 1) kd = cand_key(r[u], qx, qy);
                        else kd = dkey(sqd(qx, qy, __uint_as_float(r[u].x), __uint_as_float(r[u].y)), r[u].z);
                        best = kd < best ? kd : best;
                    }
                    s = advance(s, stepM, M);
                };
                if constexpr (VAR >= 2) {   // exact (d, original index) argmin
                    if (__any(0 < fc)) {
                        int c = 0;
                        do { ftrip(); c += kTrip; } while (__any(c < fc));
                    }
                } else {
                    for (int c = 0; __any(c < fc); c += kTrip) ftrip();
                }

            }
            int bp = -1;
            if (search && !pend) bp = forward_done(m, best, sd == -1);
            bool ok = live && bp >= 0;
#ifdef DPG_ICP_STATS
            int rtrips = 0;   // the reciprocal trips made (the loop ends once every lane is beaten)
#endif
            // ---- reciprocal test in the static source index ----
            if (kp.reciprocal) {
                const float bd = __uint_as_float((uint32_t)(best >> 32));
                float2 tj = make_float2(0.f, 0.f);
                int s = 0, rc = 0;
                if (ok) {
                    const Rec r = L.tp[bp];
                    tj = make_float2(r.x, r.y);
                    // t_j in the source node frame; float error ~1e-6 m, far inside the window margin
                    const float ux = tj.x - ftx, uy = tj.y - fty;
                    const float px = i00 * ux + i01 * uy, py = i10 * ux + i11 * uy;
                    rc = window<VAR>(L.sb, N, px, py, bsqrt<VAR>(bd) * 1.0001f + drift, s);
                }
                const int slot = queue_push(ok && rc > dcap, &L.bc->qtail);
                if (slot >= 0) {
                    *reinterpret_cast<uint2*>(&L.q[slot].w[0]) =
                        make_uint2((uint32_t)i | ((uint32_t)st_sp(st[m]) << 16), 1u | ((uint32_t)bp << 1));
                    set_slot(m, slot);
                    ok = false;
                    rc = 0;
                }
                // i's own word: any other current source with a smaller (d, original index) word
                // is closer to t_j (or tied with a lower index) and breaks reciprocity
                const uint64_t mine = dkey(bd, ((uint32_t)i << 16) | (uint32_t)st_sp(st[m]));
#ifdef DPG_ICP_STATS
                if (ok) { ICP_STAT(3, rc); if (rc >= N) ICP_STAT(13, 1); }
                if (live && !ok && !pend && slot < 0) ICP_STAT(6, 1);
#endif
                if constexpr (VAR >= 1) {
                    // the wave's still-reciprocal lanes as a mask: the beat tests are ballots
                    // folded by scalar ors, the loop condition one scalar and
                    uint64_t okm = __ballot(ok);
                    auto rtrip = [&]() {
                        uint4 r[kTrip];
                        ld_recs<kScsL, kTrip>(L.scs + s, r);
                        uint64_t beat = 0;
#pragma unroll
                        for (int u = 0; u < kTrip; ++u) beat |= __ballot(cand_key(r[u], tj.x, tj.y) < mine);
                        okm &= ~beat;
                        s = advance(s, stepN, N);
                    };
                    int c = 0;
                    for (; (okm & __ballot(c < rc)) != 0; c += kTrip) {
                        rtrip();
#ifdef DPG_ICP_STATS
                        ++rtrips;
#endif
                    }
                    ok = ok && ((okm >> lane) & 1u);
                } else {
                for (int c = 0; __any(ok & (c < rc)); c += kU) {
                    uint4 r[kU];
                    ld_recs<kScsL>(L.scs + s, r);
                    bool beat = false;
#pragma unroll
                    for (int u = 0; u < kU; ++u) {
                        const uint64_t kd = dkey(sqd(__uint_as_float(r[u].x), __uint_as_float(r[u].y), tj.x, tj.y), r[u].z);
                        beat = beat | (kd < mine);
                    }
                    ok = ok & !beat;
                    s = advance(s, stepN, N);
                }
                }
            }
#ifdef DPG_ICP_STATS
            if (kp.reciprocal && lane == 0) { ICP_STAT(4, rtrips); ICP_STAT(28 + trip_bin(rtrips), rtrips); }
            if (kp.reciprocal) wtrips += rtrips;
            if (ok) ICP_STAT(5, 1);
#endif
            okq |= (ok ? 1u : 0u) << m;
        }
        }
        ICP_STAMP(c1);
        // ---- the cooperative queue: windows too wide for one lane, 64 candidates per trip ----
        __syncthreads();
        if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);
        const int nq = min((int)uni((uint32_t)L.bc->qtail), kQCap);
        if (nq > 0) {   // nq is the same in every wave (read after the barrier)
            const int w0q = __builtin_amdgcn_readfirstlane(wave);
            for (int h = w0q; h < nq; h += kWaves) {   // items dealt round-robin to the waves
                QItem* it = L.q + h;
                const uint32_t w0 = uni(it->w[0]), w1 = uni(it->w[1]);
                const int i = (int)(w0 & 0xffffu), ps = (int)(w0 >> 16);
                const float qx = uni(L.scs[ps].x), qy = uni(L.scs[ps].y);   // the point as the owner saw it
                bool okw = true;
                int bp, s = 0, cnt = 0;
                uint64_t best = 0;
                if ((w1 & 1u) == 0u) {   // forward argmin over the window, then the reciprocal test
                    float rad;
                    const uint64_t b0 = forward_init<VAR>(L, M, (int)(w1 >> 1) - 1, qx, qy, query_angle<VAR>(qx, qy), r2f, rmax, rext, r2ext, rad);
                    const int fc = window(L.tb, M, qx, qy, rad, s);
                    best = lane == 0 ? b0 : ~0ull;
                    for (int c = lane; c < fc; c += 64) {
                        const int p = s + c >= M ? s + c - M : s + c;
                        const Rec r = ld_rec(L.tp + p);
                        const uint64_t kd = dkey(sqd(qx, qy, r.x, r.y), r.key);
                        best = kd < best ? kd : best;
                    }
                    best = wave_min_u64(best);
#ifdef DPG_ICP_STATS
                    if (lane == 0) { ICP_STAT(40, 1); ICP_STAT(41, fc); }
#endif
                    const uint32_t bkey = (uint32_t)best;
                    const float bd = __uint_as_float((uint32_t)(best >> 32));
                    bp = (bkey == 0xffffffffu || bd > r2f) ? -1 : (int)(bkey & 0xffffu);
                    okw = bp >= 0;
                } else {
                    bp = (int)(w1 >> 1);
                }
                if (okw && kp.reciprocal) {   // does any current source point beat i at t_j?
                    const Rec r = L.tp[bp];
                    const float tjx = r.x, tjy = r.y;
                    const float bd = sqd(qx, qy, tjx, tjy);   // the same float the forward search kept
                    const float ux = tjx - ftx, uy = tjy - fty;
                    const float px = i00 * ux + i01 * uy, py = i10 * ux + i11 * uy;
                    cnt = window(L.sb, N, px, py, bsqrt<VAR>(bd) * 1.0001f + drift, s);
                    const uint64_t mine = dkey(bd, ((uint32_t)i << 16) | (uint32_t)ps);
                    bool beat = false;
                    for (int c = lane; c < cnt; c += 64) {
                        const int p = s + c >= N ? s + c - N : s + c;
                        const Rec q = ld_rec(L.scs + p);
                        beat = beat | (dkey(sqd(q.x, q.y, tjx, tjy), q.key) < mine);
                    }
                    okw = !__any(beat);
                }
#ifdef DPG_ICP_STATS
                if (lane == 0) { ICP_STAT(42, 1); ICP_STAT(43, cnt); }
#endif
                if (lane == 0) *reinterpret_cast<uint4*>(it) = make_uint4(w0, (w1 & ~1u) | (okw ? 1u : 0u) | ((w1 & 1u) << 31),
                                                                            (uint32_t)best, (uint32_t)(best >> 32));
            }
#ifdef DPG_ICP_STATS
            if (t == 0) ICP_STAT(44, 1);
#endif
            __syncthreads();
        }
        // finalize the points whose windows were queued
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int slot = get_slot(m);
            if (slot >= 0) {
                const uint4 it = *reinterpret_cast<const uint4*>(L.q + slot);
                if ((it.y >> 31) == 0u)   // forward item: its best key -> match, next seed
                    (void)forward_done(m, ((uint64_t)it.w << 32) | it.z, st_seed(st[m]) == -1);
                okq |= (it.y & 1u) << m;
            }
            const int i = t + kT * m;
            if (i < N && trace && k < kp.trace_iters)
                trace[((size_t)e * kp.trace_iters + k) * kp.trace_stride + i] =
                    ((okq >> m) & 1u) ? (int)(L.tp[st_seed(st[m])].key >> 16) : -1;
        }
        ICP_STAMP(c2);
        // ---- R5 sums: this thread is tree lane t (points t + 512 m, m ascending) ----
        {
            double acc[kSums];
#pragma unroll
            for (int q = 0; q < kSums; ++q) acc[q] = 0.0;
#pragma unroll
            for (int m = 0; m < PPT; ++m) {
                if ((okq >> m) & 1u) {
                    const Rec tq = ld_rec(L.tp + st_seed(st[m]));
                    dpg_tree::add_pair(acc, sx[m], sy[m], tq.x, tq.y, sqd(sx[m], sy[m], tq.x, tq.y));
                }
            }
            acc[0] = 0.0;   // the count is an integer: ballots instead
            const double wf = dpg_tree::wave_fold_t(acc);
            int cnt = 0;
#pragma unroll
            for (int m = 0; m < PPT; ++m) cnt += __popcll(__ballot((okq >> m) & 1u));
            if ((lane & 7) == 0) {
                const int q = dpg_tree::fold_sum(lane >> 3);
                L.wpart[wave * (kSums + 2) + q] = q == 0 ? (double)cnt : wf;
            }
        }
        ICP_STAMP(c3);
        // ---- the last wave to arrive combines the partials, fits (R5) and decides (R6) ----
        int last = 0;
#ifdef DPG_ICP_STATS
        if (lane == 0) { atomicMax(&st_wmax, wtrips); ICP_STAT(15, wtrips); }
#endif
        if (lane == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            last = atomicAdd(L.arrive, 1) == kWaves - 1;
            if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        if (__builtin_amdgcn_readlane(last, 0)) {
            if constexpr (kPrio) __builtin_amdgcn_s_setprio(3);
            double S[kSums];
            if constexpr (VAR >= 1) {   // lane q combines sum q (the same fixed tree), then broadcast
                const double sq = lane < kSums ? dpg_tree::combine(L.wpart, kSums + 2, lane) : 0.0;
#pragma unroll
                for (int q = 0; q < kSums; ++q) S[q] = rdlane(sq, q);
            } else {
#pragma unroll
                for (int q = 0; q < kSums; ++q) S[q] = uni(dpg_tree::combine(L.wpart, kSums + 2, q));
            }
            Bcast B = *L.bc;
            float F[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) F[q] = uni(B.F[q]);
            const double prev_mse = uni(B.prev_mse);
            B.cnt = (int)S[0];
            B.qtail = 0;   // every wave is past the queue of this iteration
            B.qhead = 0;
            B.iter = k + 1;
            if (B.cnt < kp.min_corr) {
                B.code = 2;   // stop, "Not enough correspondences found" (transform unchanged)
            } else if constexpr (VAR >= 1) {
                // the same IEEE operations as below, the seven independent divisions by the count
                // (and S1 / S0) in ONE vector division across lanes 0-6, then the two by |(a, b)|
                // in another: two division latencies on the fit's path instead of nine
                const double n = S[0];
                double num = 0.0, den = 1.0;
                switch (lane) {
                    case 0: num = S[2] * S[4] + S[3] * S[5]; den = n; break;
                    case 1: num = S[2] * S[5] - S[3] * S[4]; den = n; break;
                    case 2: num = S[2]; den = n; break;
                    case 3: num = S[3]; den = n; break;
                    case 4: num = S[4]; den = n; break;
                    case 5: num = S[5]; den = n; break;
                    case 6: num = S[1]; den = S[0]; break;
                    default: break;
                }
                const double qv = num / den;
                const double a = S[6] - rdlane(qv, 0), b = S[7] - rdlane(qv, 1);
                const double mpx = rdlane(qv, 2), mpy = rdlane(qv, 3), mqx = rdlane(qv, 4), mqy = rdlane(qv, 5);
                const double mse = rdlane(qv, 6);
                const double hh = sqrt(a * a + b * b);
                double c = 1.0, sn = 0.0;
                if (hh > 0.0) {
                    const double cs = (lane == 0 ? a : b) / hh;
                    c = rdlane(cs, 0);
                    sn = rdlane(cs, 1);
                }
                const double txd = mqx - (c * mpx - sn * mpy);
                const double tyd = mqy - (sn * mpx + c * mpy);
                const float cf = (float)c, sf = (float)sn, txf = (float)txd, tyf = (float)tyd;
                const float nsf = -sf;
                B.r[0] = cf; B.r[1] = sf; B.r[2] = txf; B.r[3] = tyf;
                float Nf[6];
                Nf[0] = cf * F[0] + nsf * F[3];
                Nf[1] = cf * F[1] + nsf * F[4];
                Nf[2] = (cf * F[2] + nsf * F[5]) + txf;
                Nf[3] = sf * F[0] + cf * F[3];
                Nf[4] = sf * F[1] + cf * F[4];
                Nf[5] = (sf * F[2] + cf * F[5]) + tyf;
#pragma unroll
                for (int q = 0; q < 6; ++q) B.F[q] = Nf[q];
                B.mse = mse;
                const float tr = ((cf + cf) + 1.0f) - 1.0f;
                const double cos_angle = 0.5 * (double)tr;
                const double tsq = (double)(txf * txf + tyf * tyf);
                B.code = (k + 1 >= kp.max_iter || (cos_angle >= kp.rot_thr && tsq <= kp.eps) ||
                          fabs(mse - prev_mse) < kp.mse_abs) ? 1 : 0;
                B.prev_mse = mse;
                B.drift = 1e-4f + 5e-5f * (float)(k + 2);
            } else {
                const double n = S[0];
                double a, b;
                dpg_tree::fit_ab(S, a, b);
                const double hh = sqrt(a * a + b * b);
                double c = 1.0, sn = 0.0;
                if (hh > 0.0) { c = a / hh; sn = b / hh; }
                const double mpx = S[2] / n, mpy = S[3] / n, mqx = S[4] / n, mqy = S[5] / n;
                const double txd = mqx - (c * mpx - sn * mpy);
                const double tyd = mqy - (sn * mpx + c * mpy);
                const float cf = (float)c, sf = (float)sn, txf = (float)txd, tyf = (float)tyd;
                const float nsf = -sf;
                B.r[0] = cf; B.r[1] = sf; B.r[2] = txf; B.r[3] = tyf;
                float Nf[6];
                Nf[0] = cf * F[0] + nsf * F[3];
                Nf[1] = cf * F[1] + nsf * F[4];
                Nf[2] = (cf * F[2] + nsf * F[5]) + txf;
                Nf[3] = sf * F[0] + cf * F[3];
                Nf[4] = sf * F[1] + cf * F[4];
                Nf[5] = (sf * F[2] + cf * F[5]) + tyf;
#pragma unroll
                for (int q = 0; q < 6; ++q) B.F[q] = Nf[q];
                const double mse = S[1] / S[0];
                B.mse = mse;
                const float tr = ((cf + cf) + 1.0f) - 1.0f;
                const double cos_angle = 0.5 * (double)tr;
                const double tsq = (double)(txf * txf + tyf * tyf);
                B.code = (k + 1 >= kp.max_iter || (cos_angle >= kp.rot_thr && tsq <= kp.eps) ||
                          fabs(mse - prev_mse) < kp.mse_abs) ? 1 : 0;
                B.prev_mse = mse;
            }
            if (lane == 0) {
                *L.bc = B;
                *L.arrive = 0;
#ifdef DPG_ICP_STATS
                ICP_STAT(14, st_wmax);
                st_wmax = 0;
#endif
            }
            if constexpr (kPrio) __builtin_amdgcn_s_setprio(2);
        }
        __syncthreads();
        ICP_STAMP(c4);
        const int code = __builtin_amdgcn_readfirstlane(L.bc->code);
        if (__builtin_amdgcn_readfirstlane(L.bc->iter) != k + 1) {   // no fit this iteration: internal error
            converged = 0; status = DPG_ICP_INTERNAL; break;
        }
        if (code == 2) { converged = 0; status = DPG_ICP_TOO_FEW_CORR; break; }
        const float cf = uni(L.bc->r[0]), sf = uni(L.bc->r[1]), txf = uni(L.bc->r[2]), tyf = uni(L.bc->r[3]);
        const float nsf = -sf;
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int i = t + kT * m;
            const float x = sx[m], y = sy[m];
            sx[m] = (cf * x + nsf * y) + txf;
            sy[m] = (sf * x + cf * y) + tyf;
            if (i < N) put(m);
#ifdef DPG_ICP_STATS
            if (i < N) {   // drift of the moved point against F_{k+1} p, and the margin it gets
                const float2 p0 = ds_pts[E.src_ds_off + i];
                const double fx = ((double)L.bc->F[0] * p0.x + (double)L.bc->F[1] * p0.y) + (double)L.bc->F[2];
                const double fy = ((double)L.bc->F[3] * p0.x + (double)L.bc->F[4] * p0.y) + (double)L.bc->F[5];
                const double dv = sqrt(((double)sx[m] - fx) * ((double)sx[m] - fx) + ((double)sy[m] - fy) * ((double)sy[m] - fy));
                const double ratio = dv / (1e-4 + 5e-5 * (double)(k + 2));
                atomicMax(&g_icp_stats[46], (unsigned long long)__float_as_uint((float)dv));
                atomicMax(&g_icp_stats[47], (unsigned long long)__float_as_uint((float)ratio));
            }
#endif
            const int sd = st_seed(st[m]);
            if (sd < -1) {   // the clearance shrinks by the distance the point just moved
                const float dx = sx[m] - x, dy = sy[m] - y;
                const float mv = bsqrt<VAR>(dx * dx + dy * dy) * 1.0001f + 1e-6f;
                const int q = (-1 - sd) - (int)ceilf(mv * 1e4f);
                st[m] = st_with_seed(st[m], q > 0 ? -1 - q : -1);
            }
        }
        ++k;
        if (code == 1) { converged = 1; break; }
        if (k >= kp.max_iter) { converged = 0; status = DPG_ICP_INTERNAL; break; }   // unreachable (the fit stops it)
        if (__builtin_amdgcn_readlane(last, 0)) {   // off the publish path: the next reciprocal
            double inv[4];                          // tests' inverse, while the others move points
            float Fn[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) Fn[q] = uni(L.bc->F[q]);
            if constexpr (VAR >= 1) {   // inverse2's four divisions by the determinant, lanes 0-3
                const double det = (double)Fn[0] * (double)Fn[4] - (double)Fn[1] * (double)Fn[3];
                const double num = lane == 0 ? (double)Fn[4] : lane == 1 ? -(double)Fn[1] : lane == 2 ? -(double)Fn[3] : (double)Fn[0];
                const double q = num / det;
                if (lane < 4) {
                    L.bc->inv[lane] = q;
                    L.bc->finv[lane] = (float)q;
                }
            } else {
                inverse2(Fn, inv);
                if (lane == 0)
#pragma unroll
                    for (int q = 0; q < 4; ++q) L.bc->inv[q] = inv[q];
            }
        }
        __syncthreads();   // moved source complete before the next reciprocal tests
#ifdef DPG_ICP_TIMING
        {
            ICP_STAMP(c5);
            ph[0] += c1 - c0; ph[1] += c3 - c2; ph[2] += c4 - c3; ph[3] += c5 - c4; ph[4] += c2 - c1; ++nit;
        }
#endif
    }
#ifdef DPG_ICP_TIMING
    if (lane == 0) {
        ICP_STAT_ADD(8, ph[0]); ICP_STAT_ADD(9, ph[1]); ICP_STAT_ADD(10, ph[2]); ICP_STAT_ADD(11, ph[3]);
        ICP_STAT_ADD(12, nit); ICP_STAT_ADD(45, ph[4]);
        ICP_STAT_ADD(40, c_setup);
        ICP_STAT_ADD(41, __builtin_amdgcn_s_memtime() - c_in);
        ICP_STAT_ADD(42, __builtin_amdgcn_s_memrealtime() - r_in);
        ICP_STAT_ADD(43, 1);
    }
#endif
#ifdef DPG_ICP_SETUPCLK
    if (t == 0 && blockIdx.x < kSetupSlots) {
        unsigned long long* g = g_icp_setup + (size_t)blockIdx.x * 10;
        g[0] = su0; g[1] = su1; g[2] = su2; g[3] = su3; g[4] = su4; g[5] = su5; g[6] = su6;
        g[7] = __builtin_amdgcn_s_memtime(); g[8] = sr0; g[9] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if (t == 0) {
        const Bcast B = *L.bc;   // on a too-few stop: the transform, MSE of the last fitted iteration
        for (int q = 0; q < 6; ++q) F[q] = B.F[q];
        const int last_cnt = B.cnt;
        const double last_mse = B.mse;
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

extern "C" int32_t dpg_angle_buckets(void) { return kB; }

#ifdef DPG_ICP_SETUPCLK
// diagnostics build: the per-workgroup set-up stamps of the last launch (n <= kSetupSlots records)
extern "C" int dpg_icp_setup_clock(unsigned long long* out, int64_t n) {
    if (n < 0 || n > kSetupSlots) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_icp_setup), (size_t)n * 10 * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef DPG_ICP_DIAG
extern "C" int dpg_icp_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_icp_stats), 64 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[64] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_icp_stats), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

extern "C" size_t dpg_icp_ang_lds_bytes(int32_t cap) { return ang_lds_layout(cap, nullptr, cap <= 4096 ? 0 : cap <= 8192 ? 1 : 2); }
extern "C" size_t dpg_icp_ang_scratch_per_edge(int32_t cap) {
    return cap <= kModeMaxPts[0] ? 0 : 2 * (size_t)(cap + kU) * sizeof(Rec);
}

extern "C" int dpg_launch_angle_index(const float* ds_pts_dev, const int64_t* ds_off_dev, int64_t n_nodes,
                                      int32_t max_points, float* idx_pts_dev, uint16_t* idx_orig_dev,
                                      uint16_t* buckets_dev, int32_t bitonic, void* stream) {
    if (n_nodes <= 0) return DPG_OK;
    int cap = 1;
    while (cap < max_points) cap <<= 1;
    if (cap > kModeMaxPts[2]) return DPG_ERR_SIZE;
    hipLaunchKernelGGL(angle_index_kernel, dim3((unsigned)n_nodes), dim3(kTI), 8 * (size_t)cap,
                       reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float2*>(ds_pts_dev), ds_off_dev,
                       reinterpret_cast<float2*>(idx_pts_dev), idx_orig_dev, buckets_dev, bitonic);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_launch_icp_ang(const float* ds_pts_dev, const float* idx_pts_dev, const uint16_t* idx_orig_dev,
                                  const uint16_t* buckets_dev, const dpg_icp_edge* edges_dev, int64_t n_edges, const dpg_icp_kparams* kp,
                                  int32_t max_points, dpg_icp_result* results_dev, int32_t* trace_dev, void* scratch,
                                  size_t scratch_bytes, void* stream) {
    if (n_edges <= 0) return DPG_OK;
    const int mode = max_points <= kModeMaxPts[0] ? 0 : max_points <= kModeMaxPts[1] ? 1 : 2;
    if (max_points > kp->lds_tgt || max_points > kModeMaxPts[2] || kp->lds_tgt > kModeMaxPts[mode]) return DPG_ERR_SIZE;
    // diagnostic forms 6 / 7: the same kernel with an LDS allocation that leaves room for only two /
    // three workgroups per CU (the occupancy A/B of small shards, tools/icp_lpt_probe.py)
    const int var0 = kp->kernel_variant;
    const size_t lds = std::max(ang_lds_layout(kp->lds_tgt, nullptr, mode),
                                var0 == 6 ? (size_t)80 * 1024 : var0 == 7 ? (size_t)54 * 1024 : (size_t)0);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const float2* ds = reinterpret_cast<const float2*>(ds_pts_dev);
    const float2* ip = reinterpret_cast<const float2*>(idx_pts_dev);
    const int ppt = (max_points + kT - 1) / kT;
    // the large-cloud forms run in chunks of edges that fit the scratch (one slice per workgroup)
    const size_t per_edge = mode ? 2 * (size_t)(kp->lds_tgt + kU) * sizeof(Rec) : 0;
    const int64_t chunk = mode ? (int64_t)(scratch && per_edge ? scratch_bytes / per_edge : 0) : n_edges;
    if (chunk <= 0) return DPG_ERR_SIZE;
    Rec* g = reinterpret_cast<Rec*>(scratch);
    const int var = kp->kernel_variant;   // A/B of kernel forms (tools/icp_var_ab.py); 0 = the default
    for (int64_t e0 = 0; e0 < n_edges; e0 += chunk) {
        const dim3 grid((unsigned)std::min<int64_t>(chunk, n_edges - e0)), block(kT);
        const dpg_icp_edge* ed = edges_dev + e0;
// variant 5 (default): variant 4 with the window bound's margins folded into three constants and the
// query pseudo-angles in bucket units (-1.6 % at config 4, byte-identical);
// variant 1 of the diagnostic switch = variant 4, the A/B reference; variant 2 = the default kernel
// after the angle index built by the bitonic network (dpg_launch_angle_index's A/B reference).
// variant 4 (the kernel's VAR >= 1..4 steps): hardware square roots in the
// window bounds, the candidate distance computed into the record's pad register, reciprocal beats
// as ballots, the fit's divisions as lane-parallel vector divisions, issue priority for the
// synchronised phases (1); the forward pseudo-angle once per point, fused floor+convert, do-while
// forward trips (2); float inverse + drift from the fitting wave, bucket-space wrap (3); abs-modifier
// magnitudes in the query pseudo-angles (4).  Variant 0: round 2's form of the same arithmetic
// (A/B reference, DPG_ICP_VARIANT=0).  Both give byte-identical results.
#define DPG_ANG_K(P, M, V) hipLaunchKernelGGL((icp_ang_kernel<P, M, V>), grid, block, lds, s, ds, ip, idx_orig_dev, buckets_dev, ed, *kp, \
                           results_dev, trace_dev, g)
#define DPG_ANG_LAUNCH(P, M)                                                                                     \
        if (var == 1) DPG_ANG_K(P, M, 4);                                                                       \
        else DPG_ANG_K(P, M, 5)
#define DPG_ANG_LAUNCH0(P) DPG_ANG_LAUNCH(P, 0)
        if (mode == 0) {
            if (ppt <= 1) DPG_ANG_LAUNCH0(1);
            else if (ppt <= 2) DPG_ANG_LAUNCH0(2);
            else if (ppt <= 4) DPG_ANG_LAUNCH0(4);
            else DPG_ANG_LAUNCH0(8);
        } else if (mode == 1) {
            DPG_ANG_LAUNCH(16, 1);
        } else {
            DPG_ANG_LAUNCH(32, 2);
        }
        if (hipGetLastError() != hipSuccess) return DPG_ERR_HIP;
    }
#undef DPG_ANG_LAUNCH
#undef DPG_ANG_LAUNCH0
#undef DPG_ANG_K
    return DPG_OK;
}
