// dpg_chol.hip -- supernodal multifrontal Cholesky of the pose-graph normal equations on gfx950.
//
// The CHOLESKY solve that GTSAM runs inside GaussNewtonOptimizer / ISAM2 as a
// level-scheduled GPU factorization: the symbolic analysis (dpg_chol_sym.cpp) and the per-level
// task lists run once per sparsity pattern; each GN iteration then runs, per elimination-tree
// level, task-list kernels over all fronts of the level (dense fronts are column-major in HBM):
//   assemble: one workgroup per (front, 32-column tile), built in LDS: zero, scatter the
//             original 3x3 blocks of H, add the children's update matrices child by child
//             (deterministic order, no atomics), store once;
//   then per 48-column panel step:
//     panel:  one workgroup per front, one panel row per thread in registers, right-looking
//             by 3x3 block columns;
//     update: one workgroup per 32x32 tile of every front's trailing lower triangle (SYRK),
//             so a large front's Schur complement is spread over many CUs;
//   forward:  L y = -g, ONE launch: fronts as a DAG (children's pending row updates gathered,
//             diagonal blocks solved by one wave from LDS, L21 y handed to the parent);
//   backward: L^T x = y, ONE launch, top-down (ancestors' x gathered by row position).
// fp64 throughout, explicit fma in the inner products (this file is held to a tolerance, not to
// bit-exactness; the build keeps -ffp-contract=off for the ICP kernels); the fronts of one
// factorization stay resident in HBM (tens of MB).

#include <hip/hip_runtime.h>
#include <time.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "dpg_chol.h"
#include "dpg_internal.h"
#include "dpg_gn_pipe.h"

namespace {

constexpr int kT = 256;     // threads per front workgroup
constexpr int kNB = 48;     // factorization panel width (scalar columns, 16 3x3 blocks)
constexpr int kSB = 64;     // triangular-solve diagonal block
constexpr int kCT = 32;     // assembly column tile
constexpr int kUT = 32;     // trailing-update tile (rows and columns)

// Phase timestamps (timing builds of tools/chol_bench only): workgroup 0 of launch `pid` writes
// wall_clock64() (100 MHz) into slot [pid][k].
#ifdef DPG_CHOL_TIMING
constexpr int kProfSlots = 40;
__device__ unsigned long long g_prof[4096 * kProfSlots];
constexpr int kProfL = 512, kProfW = 2048;
__device__ unsigned long long g_span[kProfL * kProfW * 2];   // per launch, per workgroup: start, end
#define PROF_MARK(pid, k)                                                                       \
    do {                                                                                        \
        if (blockIdx.x == 0 && threadIdx.x == 0 && (pid) < 4096) g_prof[(pid) * kProfSlots + (k)] = wall_clock64(); \
    } while (0)
#define PROF_BEGIN(pid) do { if (threadIdx.x == 0 && (pid) < kProfL && blockIdx.x < kProfW) g_span[((size_t)(pid) * kProfW + blockIdx.x) * 2] = wall_clock64(); } while (0)
#define PROF_END(pid) do { if (threadIdx.x == 0 && (pid) < kProfL && blockIdx.x < kProfW) g_span[((size_t)(pid) * kProfW + blockIdx.x) * 2 + 1] = wall_clock64(); } while (0)
// per-front phase stamps of the fused kernel: [front][0 claim, 1 children ready, 2 assembled,
// 3 factored, 4 done]
__device__ unsigned long long g_front[16384 * 8];
#define FT_MARK(s, k) do { if (threadIdx.x == 0 && (s) < 16384) g_front[(s) * 8 + (k)] = wall_clock64(); } while (0)
// per-panel stamps of large fronts: [front][panel][0 wake, 1 loaded, 2 tile updated, 3 factored, 4 published]
__device__ unsigned long long g_panel[16384 * 16 * 8];
__device__ unsigned long long g_steps[16384 * 16 * 8];
#define ST_MARK(s, p, k) do { if (threadIdx.x == 0 && (s) < 16384 && (p) < 16 && (k) < 8) g_steps[((s) * 16 + (p)) * 8 + (k)] = wall_clock64(); } while (0)
#define PN_MARK(s, p, k) do { if (threadIdx.x == 0 && (s) < 16384 && (p) < 16) g_panel[((s) * 16 + (p)) * 8 + (k)] = wall_clock64(); } while (0)
// per-front stamps of the backward solve: [front][0 claim, 1 parent ready, 2 z updated, 3 solved, 4 done]
__device__ unsigned long long g_bwd[16384 * 8];
#define BW_MARK(s, k) do { if (threadIdx.x == 0 && (s) < 16384) g_bwd[(s) * 8 + (k)] = wall_clock64(); } while (0)
#else
#define BW_MARK(s, k) do { } while (0)
#define FT_MARK(s, k) do { } while (0)
#define PN_MARK(s, p, k) do { } while (0)
#define ST_MARK(s, p, k) do { } while (0)
#define PROF_MARK(pid, k) do { } while (0)
#define PROF_BEGIN(pid) do { } while (0)
#define PROF_END(pid) do { } while (0)
#endif

struct SnDev {
    int32_t c0, k, r, nchild;   // k, r in 3x3 blocks
    int64_t front_off;          // doubles
    int64_t rows_off;           // into rows / relmap
    int64_t child_off;          // into child_list
    int64_t omap_off;
    int64_t acc_off;            // doubles (3r pending row updates of the forward solve)
    int32_t omap_n, parent;     // parent supernode, -1 at a root
    int32_t G, need;            // fused factorization: team size, sum of the children's team sizes
    int32_t ftask;              // large fronts: first tile task
    int32_t inv;                // L11^-1 of the front at linv + inv (k3 x k3, column-major), -1: none
    int32_t seg_off, seg_n;     // backward solve: the row segments by owning supernode (SolveSeg)
};

// A front's rows (ascending positions) fall into segments owned by its ancestors, the parent's
// first: the backward solve takes each segment's x as soon as its owner has published it.
struct SolveSeg { int32_t sn, t0, t1, pad; };   // rows [t0, t1) (blocks) owned by supernode sn

struct OEnt {                   // one upper 3x3 block of H -> its front position
    int32_t u;                  // block index in the packed hb buffer
    int16_t a, b;               // local block row / column in the front
    int32_t tr, pad;            // 1: the front wants H(lo,hi)^T
};

// ---- numeric factorization: three task-list kernels per elimination-tree level ----
// (task lists are built once per sparsity pattern in dpg_chol_create)

// assembly: one workgroup per (front, kCT-column tile), built in LDS: zeroed, the original H
// blocks scattered in, then each child's update-matrix entries that land in the tile's columns
// (contiguous child columns [ja, jb), precomputed) added child by child -- within a child the
// map is injective, so all its entries are in flight at once; an LDS barrier between children
// fixes the summation order.  The finished tile is stored once, coalesced.
struct AsmTask {
    int32_t s, c0;              // front, first column of the tile
    int32_t om_b, om_e;         // omap entries whose block column meets the tile
    int32_t ch_off, ch_cnt;     // into AsmChild: the children with columns in the tile
};
struct AsmChild { int32_t c, ja, jb, pad; };

__global__ __launch_bounds__(kT) void chol_assemble(const AsmTask* __restrict__ tasks,
                                                    const AsmChild* __restrict__ tchild,
                                                    const SnDev* __restrict__ sns,
                                                    const OEnt* __restrict__ omap, const double* __restrict__ hb,
                                                    const int32_t* __restrict__ relmap, double* __restrict__ fronts,
                                                    int pid) {
    extern __shared__ __attribute__((aligned(16))) double T[];   // [kCT][m3], column-major
    const int tid = threadIdx.x;
    PROF_BEGIN(pid);
    PROF_MARK(pid, 0);
    const AsmTask tk = tasks[blockIdx.x];
    const SnDev S = sns[tk.s];
    const int m3 = 3 * (S.k + S.r);
    const int c0 = tk.c0, nc = min(c0 + kCT, m3) - c0;
    for (int e = tid; e < nc * m3; e += kT) T[e] = 0.0;
    __syncthreads();
    PROF_MARK(pid, 1);
    for (int q = tid; q < (tk.om_e - tk.om_b) * 9; q += kT) {
        const OEnt o = omap[tk.om_b + q / 9];
        const int ii = (q % 9) / 3, jj = q % 3;
        const int row = 3 * o.a + ii, col = 3 * o.b + jj;
        if (col < c0 || col >= c0 + nc || row < col) continue;
        const double* B = hb + 9 * (int64_t)o.u;
        T[(col - c0) * m3 + row] = o.tr ? B[3 * jj + ii] : B[3 * ii + jj];
    }
    PROF_MARK(pid, 2);
    for (int q = 0; q < tk.ch_cnt; ++q) {
        __syncthreads();
        const AsmChild ch = tchild[tk.ch_off + q];
        const SnDev C = sns[ch.c];
        const int r3c = 3 * C.r, k3c = 3 * C.k, m3c = 3 * (C.k + C.r);
        const int32_t* rm = relmap + C.rows_off;
        const double* Fc = fronts + C.front_off + (int64_t)k3c * m3c + k3c;
        const int nj = ch.jb - ch.ja;
        for (int e = tid; e < nj * r3c; e += kT) {
            const int jl = e / r3c, i = e - jl * r3c, j = ch.ja + jl;
            if (i < j) continue;
            const int pj = 3 * rm[j / 3] + j % 3, pi = 3 * rm[i / 3] + i % 3;
            T[(pj - c0) * m3 + pi] += Fc[(int64_t)j * m3c + i];
        }
    }
    __syncthreads();
    PROF_MARK(pid, 3);
    double* F = fronts + S.front_off + (int64_t)c0 * m3;
    for (int e = tid; e < nc * m3; e += kT) {
        const int jl = e / m3, row = e - jl * m3;
        if (row >= c0 + jl) F[e] = T[e];
    }
    PROF_MARK(pid, 4);
    __syncthreads();
    PROF_END(pid);
}

// 1/sqrt(d) from the hardware estimate (relative error ~5e-8) and ONE third-order correction:
// with e = 1 - d y^2, 1/sqrt(d) = y (1 - e)^(-1/2) = y (1 + e/2 + 3e^2/8 + O(e^3)), the O(e^3) term
// ~1e-22 -- full fp64 precision in 4 dependent operations (two Newton steps take 6).
__device__ __forceinline__ double rsqrt_nr(double d) {
    const double y = __builtin_amdgcn_rsq(d);
    const double e = fma(-(d * y), y, 1.0);
    return fma(y * e, fma(e, 0.375, 0.5), y);
}

// Cholesky factor of a 3x3 SPD block and the inverse of that factor, from the block's leading
// minors (d00, M2, det): the three reciprocal square roots are independent, so the dependent chain
// is about a third of the column-by-column one (a wave64 fp64 op is ~32 cycles of latency).
// Branch-free: a non-positive minor only raises `bad` (the solve then reports failure).
struct Chol3 { double l00, l10, l11, l20, l21, l22, m00, m10, m11, m20, m21, m22; };
__device__ __forceinline__ Chol3 chol3(double d00, double d10, double d11, double d20, double d21, double d22,
                                       bool& bad) {
    const double M2 = fma(d00, d11, -d10 * d10);
    const double c0 = fma(d11, d22, -d21 * d21), c1 = fma(d10, d22, -d21 * d20), c2 = fma(d10, d21, -d11 * d20);
    const double det = fma(d00, c0, fma(-d10, c1, d20 * c2));
    bad |= !(d00 > 0.0 && M2 > 0.0 && det > 0.0);
    const double r0 = rsqrt_nr(d00), r1 = rsqrt_nr(M2), r2 = rsqrt_nr(det);
    Chol3 L;
    L.l00 = d00 * r0;                  // sqrt(d00)
    const double s2 = M2 * r1;         // sqrt(M2)
    L.l11 = s2 * r0;                   // sqrt(M2 / d00)
    L.l22 = (det * r2) * r1;           // sqrt(det / M2)
    L.m00 = r0;
    L.m11 = L.l00 * r1;                // sqrt(d00 / M2)
    L.m22 = s2 * r2;                   // sqrt(M2 / det)
    L.l10 = d10 * r0;
    L.l20 = d20 * r0;
    L.l21 = fma(-L.l20, L.l10, d21) * L.m11;
    L.m10 = -L.l10 * (L.m00 * L.m11);
    L.m21 = -L.l21 * (L.m11 * L.m22);
    L.m20 = fma(L.l10, L.l21, -L.l20 * L.l11) * (L.m00 * L.m11 * L.m22);
    return L;
}

// panel: one workgroup per front, one panel row per thread in registers (NT >= rows), right-
// looking by 3x3 BLOCK columns (the system is 3x3-blocked, so panels are too): every thread
// factors the 3x3 diagonal block itself, solves its own row's three entries, and the panel's block
// rows are broadcast through LDS -- two barriers per three columns.  The block loop stays rolled
// (compact code: these launches run on cold instruction caches): each step shifts the register
// row by three so the current block is always p[0..2], and finished entries go straight to HBM.
// The trailing matrix is left to chol_update.
template <int NT>
__global__ __launch_bounds__(NT) void chol_panel(const int2* __restrict__ tasks, const SnDev* __restrict__ sns,
                                                 double* __restrict__ fronts, int32_t* __restrict__ status, int pid) {
    __shared__ double s_d[6];          // the current diagonal block (lower: 00 10 11 20 21 22)
    __shared__ double4 s_l[kNB];       // L(c, 3b .. 3b+2) of the panel's own rows (w unused)
    const int i = threadIdx.x;
    const int2 tk = tasks[blockIdx.x];
    const SnDev S = sns[tk.x];
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k;
    const int j0 = tk.y, w = min(kNB, k3 - j0), R = m3 - j0;
    double* F = fronts + S.front_off + (int64_t)j0 * m3 + j0;
    PROF_BEGIN(pid);
    PROF_MARK(pid, 0);
    double p[kNB];
#pragma unroll
    for (int c = 0; c < kNB; ++c) p[c] = (i < R && c < w && c <= i) ? F[(int64_t)c * m3 + i] : 0.0;
    PROF_MARK(pid, 1);
    bool bad = false;
#pragma unroll 1
    for (int c0 = 0; c0 < w; c0 += 3) {
        PROF_MARK(pid, 2 + c0 / 3);
        if (i == c0) s_d[0] = p[0];
        if (i == c0 + 1) { s_d[1] = p[0]; s_d[2] = p[1]; }
        if (i == c0 + 2) { s_d[3] = p[0]; s_d[4] = p[1]; s_d[5] = p[2]; }
        __syncthreads();
        if (c0 == 3) PROF_MARK(pid, 22);
        double d00 = s_d[0], d10 = s_d[1], d11 = s_d[2], d20 = s_d[3], d21 = s_d[4], d22 = s_d[5];
        if (!(d00 > 0.0)) { bad = true; d00 = 1.0; }
        const double i00 = rsqrt_nr(d00), l00 = d00 * i00;
        const double l10 = d10 * i00, l20 = d20 * i00;
        double e11 = d11 - l10 * l10;
        if (!(e11 > 0.0)) { bad = true; e11 = 1.0; }
        const double i11 = rsqrt_nr(e11), l11 = e11 * i11;
        const double l21 = (d21 - l20 * l10) * i11;
        double e22 = d22 - l20 * l20 - l21 * l21;
        if (!(e22 > 0.0)) { bad = true; e22 = 1.0; }
        const double i22 = rsqrt_nr(e22), l22 = e22 * i22;
        double x0 = 0.0, x1 = 0.0, x2 = 0.0;
        if (i == c0) { x0 = l00; }
        else if (i == c0 + 1) { x0 = l10; x1 = l11; }
        else if (i == c0 + 2) { x0 = l20; x1 = l21; x2 = l22; }
        else if (i > c0 + 2 && i < R) {
            x0 = p[0] * i00;
            x1 = (p[1] - x0 * l10) * i11;
            x2 = (p[2] - x0 * l20 - x1 * l21) * i22;
        }
        if (i >= c0 && i < R) {
            F[(int64_t)c0 * m3 + i] = x0;
            if (i >= c0 + 1) F[(int64_t)(c0 + 1) * m3 + i] = x1;
            if (i >= c0 + 2) F[(int64_t)(c0 + 2) * m3 + i] = x2;
        }
        if (c0 == 3) PROF_MARK(pid, 23);
        if (i > c0 + 2 && i < w) s_l[i] = make_double4(x0, x1, x2, 0.0);
        __syncthreads();
        if (c0 == 3) PROF_MARK(pid, 24);
        const bool upd = i > c0 + 2 && i < R;
#pragma unroll
        for (int c = 3; c < kNB; ++c) {
            const int cc = c0 + c;
            double v = p[c];
            if (upd && cc < w && cc <= i) {
                const double4 l = s_l[cc];
                v = fma(-x0, l.x, v);
                v = fma(-x1, l.y, v);
                v = fma(-x2, l.z, v);
            }
            p[c - 3] = v;
        }
        p[kNB - 3] = p[kNB - 2] = p[kNB - 1] = 0.0;
        if (c0 == 3) PROF_MARK(pid, 25);
    }
    if (bad && i == 0) atomicExch(status, 1);
    PROF_MARK(pid, 20);
    __syncthreads();
    PROF_END(pid);
}

// update: one workgroup per 32x32 tile (rows i0.., cols l0..) of a front's trailing lower
// triangle: F(i, l) -= sum_c L(i, j0 + c) L(l, j0 + c) over the panel's w columns.
__global__ __launch_bounds__(kT) void chol_update(const int4* __restrict__ tasks, const SnDev* __restrict__ sns,
                                                  double* __restrict__ fronts, int pid) {
    PROF_BEGIN(pid);
    PROF_MARK(pid, 0);
    __shared__ double A[kNB][33], B[kNB][33];
    const int tid = threadIdx.x;
    const int4 tk = tasks[blockIdx.x];
    const SnDev S = sns[tk.x];
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k;
    const int j0 = tk.y, w = min(kNB, k3 - j0), i0 = tk.z, l0 = tk.w;
    double* F = fronts + S.front_off;
    for (int e = tid; e < kNB * 32; e += kT) {
        const int c = e >> 5, rr = e & 31;
        A[c][rr] = (c < w && i0 + rr < m3) ? F[(int64_t)(j0 + c) * m3 + i0 + rr] : 0.0;
        B[c][rr] = (c < w && l0 + rr < m3) ? F[(int64_t)(j0 + c) * m3 + l0 + rr] : 0.0;
    }
    __syncthreads();
    const int tx = tid & 31, ty = tid >> 5;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int c = 0; c < w; ++c) {
        const double a = A[c][tx];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = fma(a, B[c][4 * ty + q], acc[q]);
    }
    const int i = i0 + tx;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int l = l0 + 4 * ty + q;
        if (i < m3 && l < m3 && i >= l) F[(int64_t)l * m3 + i] -= acc[q];
    }
#ifdef DPG_CHOL_TIMING
    __syncthreads();
    PROF_END(pid);
#endif
}

// ---- triangular solves: ONE launch each, fronts as a dependency DAG ----
// Workgroups claim fronts through an atomic ticket in topological order (forward: leaves first;
// backward: root first), so a workgroup only ever waits on fronts already claimed by running
// workgroups.  Hand-off (cdna_hip_programming.md Guideline 16): the payload is written with
// agent-scope (sc1, write-through) stores, drained (s_waitcnt vmcnt(0)) and the workgroup
// synchronised before ONE lane signals with an agent-scope atomic; the consumer polls relaxed,
// then one agent-scope acquire, then agent-scope loads.  Every spin is bounded: on timeout the
// status word gets 2 and the solve reports failure instead of hanging.
using u64 = unsigned long long;

__device__ __forceinline__ void st_agent(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<u64*>(p), (u64)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(double* p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load(reinterpret_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// 16-B write-through (sc1) accesses of a front: a buffer descriptor over the whole front (front
// offsets are even, so its base is 16-B aligned) and element pairs (e, e + 1), e even.  An 8-B sc1
// access moves 0.54-0.70x the bytes of a 16-B one per instruction, an 8-B sc1 store ~1/2.7
// (MI355X_MICROARCH.md, inter-workgroup visibility).  A column segment of a front is covered by the
// aligned pairs that overlap it; the element a pair holds outside the segment is the row above it
// in the same column or row 0 of the next column (both above the diagonal: never read as data) or
// the front's padding.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t front_rsrc(const double* F, int m3) {
    const uint64_t p = reinterpret_cast<uint64_t>(F);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane(((m3 * m3 + 1) & ~1) * 8);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}
__device__ __forceinline__ double2 ld2_sc1(__amdgpu_buffer_rsrc_t r, uint32_t e) {
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, e * 8u, 0, 16));
}
__device__ __forceinline__ void st2_sc1(__amdgpu_buffer_rsrc_t r, uint32_t e, double x, double y) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(x, y)), r, e * 8u, 0, 16);
}

// Poll without the agent acquire: every handed-off byte the waiting workgroup reads is stored sc1
// by its producer and loaded sc1 (ld_agent) here, so the L1 is never consulted for it (Guideline
// 16, the sc1-load form); the wavefront fence only keeps the compiler from hoisting those loads.
__device__ __forceinline__ void wait_geq_sc1(int32_t* w, int32_t target, int32_t* status) {
    unsigned spins = 0;
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 25)) {
            atomicExch(status, 2);
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// A pipelined Gauss-Newton loop (dpg_gn_pipe.h) enqueues both solve paths of an iteration before
// the previous one is read: gate[0] = the iteration runs, gate[1] = it reuses the factor.  mode 0
// runs when active, 1 when active and refactoring, 2 when active and reusing; no gate: always.
__device__ __forceinline__ bool gate_off(const int32_t* gate, int mode) {
    if (!gate) return false;
    const int32_t a = gate[0], r = gate[1];   // written by an earlier launch
    return !a || (mode == 1 && r) || (mode == 2 && !r);
}

__device__ __forceinline__ int claim_lds(const int32_t* order, int32_t* ticket, int* slot) {
    if (threadIdx.x == 0) *slot = order[atomicAdd(ticket, 1)];
    __syncthreads();
    return *slot;
}

// 16-lane groups: sum of a partial over the group (xor butterfly: every lane gets the total)
__device__ __forceinline__ double group16_sum(double a) {
    a += __shfl_xor(a, 8, 16);
    a += __shfl_xor(a, 4, 16);
    a += __shfl_xor(a, 2, 16);
    a += __shfl_xor(a, 1, 16);
    return a;
}

// ---- L11^-1 of the large fronts (opts.solve_inv_cols) ----
// The triangular solves spend their critical path in the top fronts' diagonal parts: a chain of
// dependent substitution steps per 64-column block, each waiting on its block's loads (profiles/r05
// chol timing: 59 of the backward's 122 us).  After each factorization this kernel inverts L11 of
// every front with at least solve_inv_cols pivot columns; the solves then apply it as ONE product
// (all loads in flight at once).  Task (s, j0): columns [j0, j0 + kInvCols) of X = L11^-1 by
// column-parallel forward substitution, ascending i (a fixed summation order).
// One WAVE per column j of X = L11^-1 (four per workgroup): lane l owns rows j + l + 64 q (q < 3:
// fronts up to 192 pivot columns); step i broadcasts x_i from its owner (one readlane) and every lane
// adds L(r, i) x_i to its rows r > i.  L's columns come straight from the fronts (L2), 16 steps'
// worth loaded ahead into registers; no LDS, so many columns run per compute unit.
constexpr int kInvCols = 4;              // columns (waves) per workgroup
constexpr int kInvThreads = 64 * kInvCols;
constexpr int kInvMaxQ = 3;              // rows per lane
constexpr int kInvAhead = 16;            // steps of L loaded ahead
__device__ __forceinline__ double rdlane_(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}
__global__ __launch_bounds__(kInvThreads) void chol_inv_l11(const int2* __restrict__ tasks, const SnDev* __restrict__ sns,
                                                            const double* __restrict__ fronts, double* __restrict__ linv,
                                                            const int32_t* gate) {
    if (gate_off(gate, 1)) return;
    const int2 tk = tasks[blockIdx.x];
    const SnDev S = sns[tk.x];
    const int lane = threadIdx.x & 63;
    const int j = tk.y + (int)(threadIdx.x >> 6);      // this wave's column
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k;
    if (j >= k3) return;                                // whole wave
    const int nr = k3 - j;                              // rows j .. k3 - 1
    const double* F = fronts + S.front_off;
    double* Li = linv + S.inv;
    double sacc[kInvMaxQ], xo[kInvMaxQ], rd[kInvMaxQ];
#pragma unroll
    for (int q = 0; q < kInvMaxQ; ++q) {
        const int b = lane + 64 * q;
        sacc[q] = xo[q] = 0.0;
        rd[q] = b < nr ? 1.0 / F[(int64_t)(j + b) * m3 + j + b] : 0.0;
    }
    // L(j + b, j + a) of this lane's rows b = lane + 64 q, 0 where b <= a or past the front
    auto ld = [&](int a, int q) -> double {
        const int b = lane + 64 * q;
        const bool in = b > a && b < nr && a < nr;
        const double t = F[(int64_t)(j + (a < nr ? a : 0)) * m3 + j + (in ? b : 0)];
        return in ? t : 0.0;
    };
    double cur[kInvAhead][kInvMaxQ], nxt[kInvAhead][kInvMaxQ];
#pragma unroll
    for (int u = 0; u < kInvAhead; ++u)
#pragma unroll
        for (int q = 0; q < kInvMaxQ; ++q) cur[u][q] = ld(u, q);
    for (int a0 = 0; a0 < nr; a0 += kInvAhead) {
#pragma unroll
        for (int u = 0; u < kInvAhead; ++u)   // the next 16 steps' columns, in flight during these 16
#pragma unroll
            for (int q = 0; q < kInvMaxQ; ++q) nxt[u][q] = ld(a0 + kInvAhead + u, q);
#pragma unroll
        for (int u = 0; u < kInvAhead; ++u) {
            const int a = a0 + u;                       // step: row j + a
            if (a >= nr) break;                         // (uniform)
            const int own = a & 63, qa = a >> 6;
            double s_own = sacc[0], r_own = rd[0];
#pragma unroll
            for (int q = 1; q < kInvMaxQ; ++q)
                if (qa == q) { s_own = sacc[q]; r_own = rd[q]; }
            const double v = a == 0 ? r_own : -s_own * r_own;   // meaningful on lane own
#pragma unroll
            for (int q = 0; q < kInvMaxQ; ++q)
                if (qa == q && lane == own) xo[q] = v;
            const double x = rdlane_(v, own);
#pragma unroll
            for (int q = 0; q < kInvMaxQ; ++q) sacc[q] = fma(cur[u][q], x, sacc[q]);   // (0 above the rows)
        }
#pragma unroll
        for (int u = 0; u < kInvAhead; ++u)
#pragma unroll
            for (int q = 0; q < kInvMaxQ; ++q) cur[u][q] = nxt[u][q];
    }
#pragma unroll
    for (int q = 0; q < kInvMaxQ; ++q) {
        const int b = lane + 64 * q;
        if (b < nr) Li[(int64_t)j * k3 + j + b] = xo[q];
    }
}

// y[0, k3) <- L11^-1 y (tmp: k3 doubles of LDS): one thread per output row, the columns in
// ascending order over four accumulators; the loads of a column are contiguous across the rows
__device__ __forceinline__ void inv_apply_lower(const double* __restrict__ Li, int k3, double* y, double* tmp) {
    const int tid = threadIdx.x;
    for (int t = tid; t < k3; t += kT) tmp[t] = y[t];
    __syncthreads();
    for (int i = tid; i < k3; i += kT) {
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        int k = 0;
#pragma unroll 2
        for (; k + 3 <= i; k += 4) {
            a0 = fma(Li[(int64_t)k * k3 + i], tmp[k], a0);
            a1 = fma(Li[(int64_t)(k + 1) * k3 + i], tmp[k + 1], a1);
            a2 = fma(Li[(int64_t)(k + 2) * k3 + i], tmp[k + 2], a2);
            a3 = fma(Li[(int64_t)(k + 3) * k3 + i], tmp[k + 3], a3);
        }
        for (; k <= i; ++k) a0 = fma(Li[(int64_t)k * k3 + i], tmp[k], a0);
        y[i] = (a0 + a1) + (a2 + a3);
    }
    __syncthreads();
}
// z[0, k3) <- L11^-T z (tmp: k3 doubles of LDS): 16 lanes per output k, the dot down column k of
// L11^-1 (rows k .. k3, contiguous)
__device__ __forceinline__ void inv_apply_upper(const double* __restrict__ Li, int k3, double* z, double* tmp) {
    const int tid = threadIdx.x, g = tid >> 4, gl = tid & 15;
    for (int t = tid; t < k3; t += kT) tmp[t] = z[t];
    __syncthreads();
    for (int k0 = 0; k0 < k3; k0 += kT / 16) {
        const int k = k0 + g;
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        if (k < k3) {
            const double* cl = Li + (int64_t)k * k3;
            int i = k + gl;
#pragma unroll 2
            for (; i + 48 < k3; i += 64) {
                a0 = fma(cl[i], tmp[i], a0);
                a1 = fma(cl[i + 16], tmp[i + 16], a1);
                a2 = fma(cl[i + 32], tmp[i + 32], a2);
                a3 = fma(cl[i + 48], tmp[i + 48], a3);
            }
            for (; i < k3; i += 16) a0 = fma(cl[i], tmp[i], a0);
        }
        const double a = group16_sum((a0 + a1) + (a2 + a3));
        if (k < k3 && gl == 0) z[k] = a;
    }
    __syncthreads();
}

// forward: L y = -g.  A front gathers its children's pending row updates (child order: fixed
// summation order), solves its diagonal blocks (one wave, LDS), then hands L21 y to its parent.
__device__ __forceinline__ double rdlane(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// The diagonal block at (jb, jb) of a front (bw x bw) into LDS (leading dimension kSB), padded
// to nb = chain_len(bw): its STRICT lower triangle (zero elsewhere and past bw), and the
// reciprocals of its diagonal (0 past bw).
__device__ __forceinline__ int chain_len(int bw) { return bw <= 8 ? 8 : bw <= 16 ? 16 : bw <= 32 ? 32 : 64; }
__device__ __forceinline__ void load_diag(double* D, double* rd, const double* F, int m3, int jb, int bw) {
    const int nb = chain_len(bw);
    constexpr int kPer = kSB * kSB / kT;   // every load of the block in flight at once (8 per thread)
    double v[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int e = threadIdx.x + kT * q, i = e % nb, j = e / nb;
        v[q] = (e < nb * nb && i < bw && j < bw && i >= j) ? F[(int64_t)(jb + j) * m3 + jb + i] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int e = threadIdx.x + kT * q, i = e % nb, j = e / nb;
        if (e < nb * nb) {
            D[j * kSB + i] = i > j ? v[q] : 0.0;
            if (i == j) rd[j] = j < bw ? 1.0 / v[q] : 0.0;
        }
    }
}

// One wave solves the padded unit-scaled triangle by a readlane -> fma chain; lane = row, the
// lane's scaled entries in registers (lanes >= N compute garbage nobody reads).
// forward (L y = b):  yl_i -= L(i, j) / L(j, j) * yl_j, j ascending; y = yl / L_ii afterwards
// rl: this lane's reciprocal of the block's diagonal (0 past bw), broadcast per column by readlane
// (scalar operands: the 64-step chains fit two waves per SIMD)
template <int N>
__device__ __forceinline__ double fwd_chain(const double* D, double rl, double yl, int lane) {
    double dr[N];
#pragma unroll
    for (int j = 0; j < N; ++j) dr[j] = D[j * kSB + lane] * rdlane(rl, j);
#pragma unroll
    for (int j = 0; j < N; ++j) yl = fma(-dr[j], rdlane(yl, j), yl);
    return yl;
}
// backward (L^T x = z): zl_i -= L(j, i) / L(j, j) * zl_j, j descending; x = zl / L_ii afterwards
template <int N>
__device__ __forceinline__ double bwd_chain(const double* D, double rl, double zl, int lane) {
    double dr[N];
#pragma unroll
    for (int j = 0; j < N; ++j) dr[j] = D[lane * kSB + j] * rdlane(rl, j);
#pragma unroll
    for (int j = N - 1; j >= 0; --j) zl = fma(-dr[j], rdlane(zl, j), zl);
    return zl;
}
template <bool kFwd>
__device__ __forceinline__ double run_chain(const double* D, double rl, double v, int lane, int bw) {
    const int nb = chain_len(bw);
    if constexpr (kFwd)
        return nb == 8 ? fwd_chain<8>(D, rl, v, lane) : nb == 16 ? fwd_chain<16>(D, rl, v, lane)
             : nb == 32 ? fwd_chain<32>(D, rl, v, lane) : fwd_chain<64>(D, rl, v, lane);
    else
        return nb == 8 ? bwd_chain<8>(D, rl, v, lane) : nb == 16 ? bwd_chain<16>(D, rl, v, lane)
             : nb == 32 ? bwd_chain<32>(D, rl, v, lane) : bwd_chain<64>(D, rl, v, lane);
}

// ---- inverted diagonal blocks (once per factorization) ----
// The solves' diagonal blocks were triangular substitutions: a chain of up to 64 dependent steps
// (readlane -> fp64 fma) on one wave, ~1 us per block, on the critical path of every forward and
// backward solve -- and a Gauss-Newton step runs the solves 13 times per factorization... once.
// chol_inv_diag inverts every 64-column diagonal block after the factorization (one wave per
// block: lane c computes column c of inv(B) by column-oriented forward substitution, the block's
// entries read as wave-uniform scalar loads, 64 accumulators in registers); the solves then apply
// inv(B) (forward) or inv(B)^T (backward) as a mat-vec: independent products, 4 partial sums.
// Layout: dinv[(3 c0 + jb + col) * kSB + row] = inv(B)[row][col] for row, col < bw, B = the front's
// diagonal block at (jb, jb) (bw = min(kSB, k3 - jb)); one kSB-double column per pivot column.
constexpr int kDL = kSB + 1;   // leading dimension of D in the inverse path (transposed stores conflict-free)

// 8 consecutive doubles of LDS (16-B aligned, OFF bytes past base) into registers: four
// ds_read_b128 and one wait as inline asm with immediate offsets; `dep` is a fake operand that
// orders the loads after the arithmetic producing it.  (Left to itself the compiler issued all
// 2016 loads of a block up front and spilled 4000 registers.)
template <int OFF>
__device__ __forceinline__ void lds_ld8(uint32_t base, double (&v)[8], double& dep) {
    uint4 r0, r1, r2, r3;
    asm volatile(
        "ds_read_b128 %0, %5 offset:%6\n\t"
        "ds_read_b128 %1, %5 offset:%7\n\t"
        "ds_read_b128 %2, %5 offset:%8\n\t"
        "ds_read_b128 %3, %5 offset:%9\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "+v"(dep)
        : "v"(base), "i"(OFF), "i"(OFF + 16), "i"(OFF + 32), "i"(OFF + 48)
        : "memory");
    v[0] = __hiloint2double((int)r0.y, (int)r0.x); v[1] = __hiloint2double((int)r0.w, (int)r0.z);
    v[2] = __hiloint2double((int)r1.y, (int)r1.x); v[3] = __hiloint2double((int)r1.w, (int)r1.z);
    v[4] = __hiloint2double((int)r2.y, (int)r2.x); v[5] = __hiloint2double((int)r2.w, (int)r2.z);
    v[6] = __hiloint2double((int)r3.y, (int)r3.x); v[7] = __hiloint2double((int)r3.w, (int)r3.z);
}

// inv(B) by column-oriented forward substitution, B (column-major kSB x kSB, identity past bw) in
// LDS, lane c = column c of the inverse in registers (acc): x_J = acc_J / B_JJ, then
// acc_i -= B_iJ x_J below it, 8 rows per LDS round (entries read as broadcasts: every lane the
// same address).  Template recursion keeps every offset an immediate.
template <int J, int Q>
struct InvRows {
    static __device__ __forceinline__ void run(uint32_t base, double (&acc)[kSB], double xj) {
        if constexpr (Q < kSB / 8) {
            double v[8];
            // issued once the rows two rounds up have taken this column: two rounds in flight
            lds_ld8<(J * kSB + 8 * Q) * 8>(base, v, acc[Q >= (J >> 3) + 3 ? 8 * (Q - 2) + 7 : J]);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[8 * Q + u] = fma(-v[u], xj, acc[8 * Q + u]);
            InvRows<J, Q + 1>::run(base, acc, xj);
        }
    }
};
template <int J>
struct InvCol {
    static __device__ __forceinline__ void run(uint32_t base, double (&acc)[kSB]) {
        if constexpr (J < kSB) {
            double v[8];
            lds_ld8<(J * kSB + (J & ~7)) * 8>(base, v, acc[J > 0 ? J - 1 : 0]);   // after x_{J-1}
            const double xj = acc[J] / v[J & 7];
            acc[J] = xj;
#pragma unroll
            for (int u = (J & 7) + 1; u < 8; ++u) acc[(J & ~7) + u] = fma(-v[u], xj, acc[(J & ~7) + u]);
            InvRows<J, (J >> 3) + 1>::run(base, acc, xj);
            InvCol<J + 1>::run(base, acc);
        }
    }
};

// one wave per diagonal block; every block padded to 64 columns (one code path)
__global__ __launch_bounds__(64) void chol_inv_diag(const int2* __restrict__ blocks, const SnDev* __restrict__ sns,
                                                    const double* __restrict__ fronts, double* __restrict__ dinv) {
    __shared__ __attribute__((aligned(16))) double B[kSB * kSB];
    const int2 b = blocks[blockIdx.x];   // (front, jb)
    const SnDev S = sns[b.x];
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k, jb = b.y, bw = min(kSB, k3 - jb);
    const int lane = threadIdx.x;
    const double* F = fronts + S.front_off;
    for (int j = 0; j < kSB; ++j)   // lane = row: column j of the block, padded with the identity
        B[j * kSB + lane] = (j < bw && lane < bw) ? (lane >= j ? F[(int64_t)(jb + j) * m3 + jb + lane] : 0.0)
                                                  : (lane == j ? 1.0 : 0.0);
    __syncthreads();
    double acc[kSB];
#pragma unroll
    for (int i = 0; i < kSB; ++i) acc[i] = i == lane ? 1.0 : 0.0;
    InvCol<0>::run((uint32_t)reinterpret_cast<uintptr_t>(B), acc);
    double* out = dinv + (3 * (int64_t)S.c0 + jb) * kSB;
    if (lane < bw)
#pragma unroll
        for (int i = 0; i < kSB; ++i)
            if (i < bw) out[(int64_t)lane * kSB + i] = acc[i];
}

// the inverted block at (jb, jb) into D (ld kDL), zero past bw: as stored (forward: D(i, j) =
// inv(B)[i][j] at D[j kDL + i]) or transposed (backward: D[j kDL + i] = inv(B)[j][i])
template <bool kT_>
__device__ __forceinline__ void load_dinv(double* D, const double* dinv_front, int jb, int bw) {
    const double* src = dinv_front + (int64_t)jb * kSB;
    constexpr int kPer = kSB * kSB / kT;
    double v[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int e = threadIdx.x + kT * q, r = e % kSB, cc = e / kSB;   // src[cc * kSB + r] = inv(B)[r][cc]
        v[q] = (r < bw && cc < bw) ? src[e] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int e = threadIdx.x + kT * q, r = e % kSB, cc = e / kSB;
        if constexpr (kT_) D[r * kDL + cc] = v[q];
        else D[cc * kDL + r] = v[q];
    }
}

// one wave: v[jb + lane] <- sum_j D[j kDL + lane] v[jb + j], lane < bw (reads before the write)
__device__ __forceinline__ void apply_dinv(const double* D, double* v, int jb, int bw, int lane) {
    const int nb = chain_len(bw);
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    for (int j = 0; j < nb; j += 4) {
        const double v0 = j < bw ? v[jb + j] : 0.0, v1 = j + 1 < bw ? v[jb + j + 1] : 0.0;
        const double v2 = j + 2 < bw ? v[jb + j + 2] : 0.0, v3 = j + 3 < bw ? v[jb + j + 3] : 0.0;
        a0 = fma(D[j * kDL + lane], v0, a0);
        a1 = fma(D[(j + 1) * kDL + lane], v1, a1);
        a2 = fma(D[(j + 2) * kDL + lane], v2, a2);
        a3 = fma(D[(j + 3) * kDL + lane], v3, a3);
    }
    if (lane < bw) v[jb + lane] = (a0 + a1) + (a2 + a3);
}

// Staging of a front's L in LDS while the solve waits for its children (forward) or its parent
// (backward): every load the front's own arithmetic needs is issued before the wait, so after it
// only the handed-off values (pending row updates / the ancestors' x) travel.  The region holds
// R doubles (a launch parameter), beside the kSB x kSB diagonal-block buffer D:
//   full:  the front's pivot columns, [k3][m3] column-major exactly as in HBM (ld m3), when
//          m3 k3 <= R (its diagonal blocks are copied LDS -> D);
//   else:  the first C columns of L21 (rows k3..m3, ld r3), C a multiple of 4 (the dot products
//          keep their 4-accumulator order whichever memory a column comes from); the diagonal
//          blocks come from HBM (the first one needed is loaded before the wait).
struct Stage {
    bool full;
    int C;
};
__device__ __forceinline__ Stage stage_plan(int m3, int k3, int R) {
    if ((int64_t)m3 * k3 <= (int64_t)R) return Stage{true, k3};
    const int r3 = m3 - k3;
    const int C = r3 > 0 ? min(k3, R / r3) & ~3 : 0;
    return Stage{false, C};
}
// n doubles src -> dst, 8 loads in flight per thread
__device__ __forceinline__ void stage_copy(double* dst, const double* src, int n) {
    for (int e0 = 0; e0 < n; e0 += 8 * kT) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = e0 + threadIdx.x + kT * q;
            v[q] = e < n ? src[e] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = e0 + threadIdx.x + kT * q;
            if (e < n) dst[e] = v[q];
        }
    }
}
// L2 warm-up of the solves' unstaged reads: one load per 128-B line of every part of the front's
// L a solve reads from global memory after its wait (everything but a fully staged front and L21's
// first C columns), issued BEFORE the staging loads and retired with them -- so the front's lines
// are in this XCD's L2 when the (often tens of us long) wait ends and the diagonal blocks' and the
// column dots' loads, each a dependent round trip, hit there instead of the fabric.  The front was
// written by an earlier launch (plain loads are coherent).  Rows j, j + 16, ... of column j, and
// its last row (a 16-double step never skips a line).
constexpr int kWarm = 16;
__device__ __forceinline__ void warm_issue(const double* F, int m3, int k3, int C, double (&v)[kWarm]) {
    const int per = ((m3 + 15) >> 4) + 1, n = k3 * per;
#pragma unroll
    for (int q = 0; q < kWarm; ++q) {
        const int e = threadIdx.x + kT * q;
        v[q] = 0.0;
        if (e < n) {
            const int j = e / per;
            const int r = min(j + 16 * (e - j * per), m3 - 1);
            if (!(j < C && r >= k3)) v[q] = F[(int64_t)j * m3 + r];
        }
    }
}
// the touches retire here (an empty asm using each value: the loads cannot be dropped)
__device__ __forceinline__ void warm_retire(const double (&v)[kWarm]) {
#pragma unroll
    for (int q = 0; q < kWarm; ++q) asm volatile("" ::"v"(v[q]));
}

// the first C columns of L21 (rows k3..m3 of the front at F) -> dst [C][r3]
__device__ __forceinline__ void stage_l21(double* dst, const double* F, int m3, int k3, int C) {
    const int r3 = m3 - k3, n = C * r3;
    for (int e0 = 0; e0 < n; e0 += 8 * kT) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = e0 + threadIdx.x + kT * q;
            v[q] = e < n ? F[(int64_t)(e / r3) * m3 + k3 + e % r3] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = e0 + threadIdx.x + kT * q;
            if (e < n) dst[e] = v[q];
        }
    }
}


// z[j] -= sum_t A[j * lda + t] x[t] for j < nj, t < nt (A column-major, the dot runs down a
// column: contiguous): 16 lanes per j, so a long dot is 1/16 of the serial chain.
// Dots of at most 64 terms (a lane holds at most 4 of them: the triangular blocks' row panels,
// short L21s) are straight-line: four columns per 16-lane group in flight at once (16 loads per
// lane instead of one dependent round trip per column pass), the same fma order as the loop below.
__device__ __forceinline__ void sub_coldots(double* z, const double* A, int64_t lda, const double* x, int nj, int nt) {
    const int g = threadIdx.x >> 4, gl = threadIdx.x & 15;
    if (nt <= 64) {
        constexpr int kU = 4;
        for (int j0 = 0; j0 < nj; j0 += kU * (kT / 16)) {
            double v[kU][4];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int j = j0 + u * (kT / 16) + g;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int t = gl + 16 * q;
                    v[u][q] = (j < nj && t < nt) ? A[(int64_t)j * lda + t] : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int j = j0 + u * (kT / 16) + g;
                double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
                if (gl + 48 < nt) {   // the loop's one 4-wide trip
                    a0 = fma(v[u][0], x[gl], a0);
                    a1 = fma(v[u][1], x[gl + 16], a1);
                    a2 = fma(v[u][2], x[gl + 32], a2);
                    a3 = fma(v[u][3], x[gl + 48], a3);
                } else {              // its tail
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        if (gl + 16 * q < nt) a0 = fma(v[u][q], x[gl + 16 * q], a0);
                }
                const double a = group16_sum((a0 + a1) + (a2 + a3));
                if (j < nj && gl == 0) z[j] -= a;
            }
        }
        return;
    }
    for (int j0 = 0; j0 < nj; j0 += kT / 16) {
        const int j = j0 + g;
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        if (j < nj) {
            const double* Aj = A + (int64_t)j * lda;
            int t = gl;
            // 8 loads in flight per lane (the fronts come from L2/MALL: latency, not bandwidth)
#pragma unroll 2
            for (; t + 48 < nt; t += 64) {
                const double v0 = Aj[t], v1 = Aj[t + 16], v2 = Aj[t + 32], v3 = Aj[t + 48];
                a0 = fma(v0, x[t], a0);
                a1 = fma(v1, x[t + 16], a1);
                a2 = fma(v2, x[t + 32], a2);
                a3 = fma(v3, x[t + 48], a3);
            }
            for (; t < nt; t += 16) a0 = fma(Aj[t], x[t], a0);
        }
        const double a = group16_sum((a0 + a1) + (a2 + a3));
        if (j < nj && gl == 0) z[j] -= a;
    }
}

// The front's own arithmetic of the forward solve after its children's pending row updates are in:
// diagonal blocks by one wave, the rows below each block, then the pending update L21 y for the
// parent.  kFull: the front is staged in LDS at Rg (ld m3); else D holds the current diagonal block
// (the first one prestaged) and L21s the first C columns of L21.
template <bool kFull>
__device__ __forceinline__ void fwd_front(const SnDev& S, const double* F, double* Rg, double* D, const double* L21s,
                                          int C, double* rd, double* y, double* aR, double* acc, const double* dinv_f,
                                          const double* Li) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k, r3 = 3 * S.r;
    const double* A = kFull ? Rg : F;   // the front's columns, ld m3
    if (Li) inv_apply_lower(Li, k3, y, D);   // y_p <- L11^-1 y_p: the whole diagonal part as one product
    for (int jb = 0; jb < (Li ? 0 : k3); jb += kSB) {
        const int bw = min(kSB, k3 - jb);
        if (jb > 0) {   // the first block was loaded before the wait
            if (dinv_f) load_dinv<false>(D, dinv_f, jb, bw);
            else if constexpr (kFull) load_diag(D, rd, Rg, m3, jb, bw);
            else load_diag(D, rd, F, m3, jb, bw);
            __syncthreads();
        }
        if (wave == 0) {
            if (dinv_f) {   // y_blk <- inv(B) y_blk
                apply_dinv(D, y, jb, bw, lane);
            } else {        // lane = row; y_j broadcast by v_readlane (uniform j)
                double yl = lane < bw ? y[jb + lane] : 0.0;
                const double rl = lane < bw ? rd[lane] : 0.0;
                yl = run_chain<true>(D, rl, yl, lane, bw);
                if (lane < bw) y[jb + lane] = yl * rl;
            }
        }
        __syncthreads();
        for (int i = jb + bw + tid; i < k3; i += kT) {
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
            int j = 0;
#pragma unroll 2
            for (; j + 3 < bw; j += 4) {   // loads batched: a front not staged comes from L2/MALL
                const double v0 = A[(jb + j) * m3 + i], v1 = A[(jb + j + 1) * m3 + i];
                const double v2 = A[(jb + j + 2) * m3 + i], v3 = A[(jb + j + 3) * m3 + i];
                a0 = fma(v0, y[jb + j], a0);
                a1 = fma(v1, y[jb + j + 1], a1);
                a2 = fma(v2, y[jb + j + 2], a2);
                a3 = fma(v3, y[jb + j + 3], a3);
            }
            for (; j < bw; ++j) a0 = fma(A[(jb + j) * m3 + i], y[jb + j], a0);
            y[i] -= (a0 + a1) + (a2 + a3);
        }
        __syncthreads();
    }
    for (int t = tid; t < r3; t += kT) {
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        int j = 0;
        if constexpr (kFull) {
#pragma unroll 2
            for (; j + 3 < k3; j += 4) {
                a0 = fma(Rg[j * m3 + k3 + t], y[j], a0);
                a1 = fma(Rg[(j + 1) * m3 + k3 + t], y[j + 1], a1);
                a2 = fma(Rg[(j + 2) * m3 + k3 + t], y[j + 2], a2);
                a3 = fma(Rg[(j + 3) * m3 + k3 + t], y[j + 3], a3);
            }
            for (; j < k3; ++j) a0 = fma(Rg[j * m3 + k3 + t], y[j], a0);
        } else {
            for (; j < C; j += 4) {   // C is a multiple of 4: the same accumulator order as below
                a0 = fma(L21s[j * r3 + t], y[j], a0);
                a1 = fma(L21s[(j + 1) * r3 + t], y[j + 1], a1);
                a2 = fma(L21s[(j + 2) * r3 + t], y[j + 2], a2);
                a3 = fma(L21s[(j + 3) * r3 + t], y[j + 3], a3);
            }
#pragma unroll 2
            for (; j + 3 < k3; j += 4) {
                a0 = fma(F[j * m3 + k3 + t], y[j], a0);
                a1 = fma(F[(j + 1) * m3 + k3 + t], y[j + 1], a1);
                a2 = fma(F[(j + 2) * m3 + k3 + t], y[j + 2], a2);
                a3 = fma(F[(j + 3) * m3 + k3 + t], y[j + 3], a3);
            }
            for (; j < k3; ++j) a0 = fma(F[j * m3 + k3 + t], y[j], a0);
        }
        st_agent(acc + S.acc_off + t, aR[t] + ((a0 + a1) + (a2 + a3)));
    }
}

__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(2))) void chol_forward_dag(const int32_t* __restrict__ order, int32_t* sync,
                                                       int32_t* status, const SnDev* __restrict__ sns,
                                                       const int32_t* __restrict__ child_list,
                                                       const int32_t* __restrict__ relmap,
                                                       const double* __restrict__ fronts,
                                                       const double* __restrict__ g,
                                                       const int32_t* __restrict__ perm,
                                                       double* __restrict__ ysol, double* acc, int R,
                                                       const double* __restrict__ dinv, const int32_t* gate,
                                                       const double* __restrict__ linv) {
    extern __shared__ __attribute__((aligned(16))) double smem_fw[];
    double* sm = smem_fw + 2;   // smem_fw[0]: the claimed front (no static LDS)
    const int tid = threadIdx.x;
    if (gate_off(gate, 2)) return;
    __builtin_amdgcn_s_setprio(2);   // as chol_factor_dag
    const int s = claim_lds(order, sync, reinterpret_cast<int*>(smem_fw));
    const SnDev S = sns[s];
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k, r3 = 3 * S.r;
    const double* F = fronts + S.front_off;
    const double* dinv_f = dinv ? dinv + 3 * (int64_t)S.c0 * kSB : nullptr;   // inverted diagonal blocks
    const double* Li = (linv && S.inv >= 0) ? linv + S.inv : nullptr;          // L11^-1
    double* D = sm;                  // kSB x kDL diagonal block (with Li: k3 doubles of scratch)
    double* Rg = D + kSB * kDL;      // staging region, R doubles (Stage)
    double* L21s = Rg;               // (not full) first C columns of L21
    double* rd = Rg + R;             // kSB reciprocals of the diagonal block's diagonal
    double* y = rd + kSB;            // k3
    double* aR = y + k3;             // r3
    const Stage P = stage_plan(m3, k3, R);
    // before the wait: the right-hand side and the front's L (earlier launches)
    for (int t = tid; t < k3; t += kT) {
        const int node = perm[S.c0 + t / 3];
        y[t] = -g[3 * node + t % 3];
    }
    for (int t = tid; t < r3; t += kT) aR[t] = 0.0;
    if (Li) {
    } else if (dinv_f) load_dinv<false>(D, dinv_f, 0, min(kSB, k3));
    else load_diag(D, rd, F, m3, 0, min(kSB, k3));
    if (P.full) {
        stage_copy(Rg, F, m3 * k3);
    } else {
        double wv[kWarm];
        if (!Li) warm_issue(F, m3, k3, P.C, wv);
        stage_l21(L21s, F, m3, k3, P.C);
        if (!Li) warm_retire(wv);
    }
    if (S.nchild > 0) {
        if (tid == 0) wait_geq_sc1(sync + 1 + s, S.nchild, status);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int ci = 0; ci < S.nchild; ++ci) {
        const int c = child_list[S.child_off + ci];
        const SnDev C = sns[c];
        const int32_t* rm = relmap + C.rows_off;
        for (int t = tid; t < 3 * C.r; t += kT) {
            const int li = 3 * rm[t / 3] + t % 3;
            const double v = ld_agent(acc + C.acc_off + t);
            if (li < k3) y[li] -= v;
            else aR[li - k3] += v;
        }
        __syncthreads();
    }
    if (P.full) fwd_front<true>(S, F, Rg, D, L21s, P.C, rd, y, aR, acc, dinv_f, Li);
    else fwd_front<false>(S, F, Rg, D, L21s, P.C, rd, y, aR, acc, dinv_f, Li);
    for (int t = tid; t < k3; t += kT) ysol[3 * (int64_t)S.c0 + t] = y[t];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0 && S.parent >= 0)
        __hip_atomic_fetch_add(sync + 1 + S.parent, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// backward: L^T x = y.  A front gathers x at its row positions and subtracts L21^T x_r from y,
// segment by segment as the rows' owners publish (the highest ancestor's rows first, the parent's
// last: after the parent's signal only its own rows remain), then solves its diagonal blocks and
// publishes its own x.  Its L is staged in LDS before any wait (Stage).
constexpr int kMaxSeg = 32;   // row segments held in LDS (a front with more waits for its parent, then takes every row)

// z -= L21[rows r0..r1)^T x_r[r0..r1) (scalar rows of the L21 block)
template <bool kFull>
__device__ __forceinline__ void bwd_z(const double* F, const double* Rg, const double* L21s, int C, int m3, int k3,
                                      double* z, const double* xr, int r0, int r1) {
    const int r3 = m3 - k3;
    if constexpr (kFull) {
        sub_coldots(z, Rg + k3 + r0, m3, xr + r0, k3, r1 - r0);
    } else {
        sub_coldots(z, L21s + r0, r3, xr + r0, C, r1 - r0);
        sub_coldots(z + C, F + (int64_t)C * m3 + k3 + r0, m3, xr + r0, k3 - C, r1 - r0);
    }
}

template <bool kFull>
__device__ __forceinline__ void bwd_diag(const double* F, const double* Rg, double* D, double* rd, int m3, int k3,
                                         double* z, const double* dinv_f, int s) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nblk = (k3 + kSB - 1) / kSB;
    for (int b = nblk - 1; b >= 0; --b) {
        const int jb = b * kSB, bw = min(kSB, k3 - jb);
        ST_MARK(s, 8 + b, 0);   // timing builds: per block, load / chain / column dots
        if (b != nblk - 1) {   // the last block was loaded before the wait
            if (dinv_f) load_dinv<true>(D, dinv_f, jb, bw);
            else if constexpr (kFull) load_diag(D, rd, Rg, m3, jb, bw);
            else load_diag(D, rd, F, m3, jb, bw);
            __syncthreads();
        }
        ST_MARK(s, 8 + b, 1);
        if (wave == 0) {
            if (dinv_f) {   // z_blk <- inv(B)^T z_blk
                apply_dinv(D, z, jb, bw, lane);
            } else {        // lane = row; x_j broadcast by v_readlane (uniform j): ~3 dependent ops per step
                double zl = lane < bw ? z[jb + lane] : 0.0;
                const double rl = lane < bw ? rd[lane] : 0.0;
                zl = run_chain<false>(D, rl, zl, lane, bw);
                if (lane < bw) z[jb + lane] = zl * rl;
            }
        }
        __syncthreads();
        ST_MARK(s, 8 + b, 2);
        sub_coldots(z, (kFull ? Rg : F) + jb, m3, z + jb, jb, bw);
        __syncthreads();
        ST_MARK(s, 8 + b, 3);
    }
}

template <bool kFull>
__device__ __forceinline__ void bwd_front(int s, const SnDev& S, int nseg, const SolveSeg* sg, const int32_t* rp,
                                          int32_t* sync, int32_t* status, double* xsol, const double* F, double* Rg,
                                          double* D, const double* L21s, int C, double* rd, double* z, double* xr,
                                          const double* dinv_f, const double* Li) {
    const int tid = threadIdx.x;
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k, r3 = 3 * S.r;
    if (nseg == 0) {   // the root (no rows), or too many segments: wait for the parent, take every row
        if (S.parent >= 0) {
            if (tid == 0) wait_geq_sc1(sync + 1 + S.parent, 1, status);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        BW_MARK(s, 1);
        for (int t = tid; t < r3; t += kT) xr[t] = ld_agent(xsol + 3 * (int64_t)rp[t / 3] + t % 3);
        __syncthreads();
        bwd_z<kFull>(F, Rg, L21s, C, m3, k3, z, xr, 0, r3);
    } else {
        for (int q = nseg - 1; q >= 0; --q) {
            const SolveSeg g = sg[q];
            if (tid == 0) wait_geq_sc1(sync + 1 + g.sn, 1, status);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (q == 0) BW_MARK(s, 1);
            for (int t = 3 * g.t0 + tid; t < 3 * g.t1; t += kT) xr[t] = ld_agent(xsol + 3 * (int64_t)rp[t / 3] + t % 3);
            __syncthreads();
            bwd_z<kFull>(F, Rg, L21s, C, m3, k3, z, xr, 3 * g.t0, 3 * g.t1);
        }
    }
    __syncthreads();
    BW_MARK(s, 2);
    if (Li) inv_apply_upper(Li, k3, z, D);   // x_p <- L11^-T z_p: one product
    else bwd_diag<kFull>(F, Rg, D, rd, m3, k3, z, dinv_f, s);
}

__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(2))) void chol_backward_dag(const int32_t* __restrict__ order, int32_t* sync,
                                                        int32_t* status, const SnDev* __restrict__ sns,
                                                        const int32_t* __restrict__ rows,
                                                        const SolveSeg* __restrict__ segs,
                                                        const double* __restrict__ fronts,
                                                        const double* __restrict__ ysol, double* xsol, int R,
                                                        int max_seg, const double* __restrict__ dinv,
                                                        const int32_t* gate, const int32_t* __restrict__ perm,
                                                        double* __restrict__ X, double* max_out,
                                                        const double* __restrict__ linv) {
    extern __shared__ __attribute__((aligned(16))) double smem_b[];
    double* sm = smem_b + 2;   // smem_b[0]: the claimed front (no static LDS)
    const int tid = threadIdx.x;
    if (gate_off(gate, 0)) return;
    __builtin_amdgcn_s_setprio(2);   // as chol_factor_dag
    const int s = claim_lds(order, sync, reinterpret_cast<int*>(smem_b));
    const SnDev S = sns[s];
    BW_MARK(s, 0);
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k, r3 = 3 * S.r;
    const double* F = fronts + S.front_off;
    const double* dinv_f = dinv ? dinv + 3 * (int64_t)S.c0 * kSB : nullptr;   // inverted diagonal blocks
    // the inverse is valid on the gated loop's chord iterations (a refactoring iteration's is being
    // computed beside this solve) and whenever the caller passes it ungated
    const double* Li = (linv && S.inv >= 0 && (!gate || gate[1])) ? linv + S.inv : nullptr;   // L11^-1
    double* D = sm;                  // kSB x kDL diagonal block (with Li: k3 doubles of scratch)
    double* Rg = D + kSB * kDL;      // staging region, R doubles (Stage)
    double* L21s = Rg;               // (not full) first C columns of L21
    double* rd = Rg + R;             // kSB reciprocals of the diagonal block's diagonal
    double* z = rd + kSB;            // k3
    double* xr = z + k3;             // r3
    int32_t* rp = reinterpret_cast<int32_t*>(xr + r3);   // r3 / 3 row positions
    SolveSeg* sg = reinterpret_cast<SolveSeg*>(xr + r3 + ((S.r + 3) / 4) * 2);   // [kMaxSeg], 16-B aligned
    const int nseg = S.seg_n <= max_seg ? S.seg_n : 0;   // max_seg <= kMaxSeg
    const Stage P = stage_plan(m3, k3, R);
    // before any wait: y, the row positions, the segments, the front's L (all from earlier launches)
    for (int j = tid; j < k3; j += kT) z[j] = ysol[3 * (int64_t)S.c0 + j];
    for (int t = tid; t < S.r; t += kT) rp[t] = rows[S.rows_off + t];
    for (int q = tid; q < nseg; q += kT) sg[q] = segs[S.seg_off + q];
    if (!Li) {
        const int jb = ((k3 + kSB - 1) / kSB - 1) * kSB;
        if (dinv_f) load_dinv<true>(D, dinv_f, jb, k3 - jb);
        else load_diag(D, rd, F, m3, jb, k3 - jb);
    }
    if (P.full) {
        stage_copy(Rg, F, m3 * k3);
    } else {
        double wv[kWarm];
        if (!Li) warm_issue(F, m3, k3, P.C, wv);
        stage_l21(L21s, F, m3, k3, P.C);
        if (!Li) warm_retire(wv);
    }
    __syncthreads();
    if (P.full) bwd_front<true>(s, S, nseg, sg, rp, sync, status, xsol, F, Rg, D, L21s, P.C, rd, z, xr, dinv_f, Li);
    else bwd_front<false>(s, S, nseg, sg, rp, sync, status, xsol, F, Rg, D, L21s, P.C, rd, z, xr, dinv_f, Li);
    BW_MARK(s, 3);
    for (int j = tid; j < k3; j += kT) st_agent(xsol + 3 * (int64_t)S.c0 + j, z[j]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(sync + 1 + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    BW_MARK(s, 4);
    if (X) {   // the Gauss-Newton retraction of this front's nodes (retract_kernel's work), max |x|
        double m = 0.0;
        for (int j = tid; j < S.k; j += kT)
            m = fmax(m, pose_retract(X + 3 * (int64_t)perm[S.c0 + j], z[3 * j], z[3 * j + 1], z[3 * j + 2]));
        if (tid < ((S.k + 63) & ~63)) {   // the waves that own nodes
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
            if ((tid & 63) == 0)
                atomicMax(reinterpret_cast<unsigned long long*>(max_out), (unsigned long long)__double_as_longlong(m));
        }
    }
}

// ---- fused factorization + forward solve: ONE launch, fronts as a DAG ----
// One 512-thread workgroup per front, claimed in topological order (as the solves above).  A
// front waits for its children, then
//   assembles itself column tile by column tile in LDS (H blocks + children's update matrices,
//     child by child: fixed summation order),
//   factors its k3 pivot columns right-looking by kFNB-column panels: the panel is staged in LDS,
//     wave 0 factors its top w x w block with the rows in registers (rsq + Newton, 3x3-block steps,
//     wave-synchronous, no workgroup barrier), every other row solves against it independently
//     (one row per thread, L_top broadcast from LDS), then the whole workgroup applies the rank-w
//     update to the trailing lower triangle in 64x64 tiles (4x4 register tile per thread),
//   runs its part of the forward solve L y = -g while its L is hot (children's pending row updates
//     gathered in child order, diagonal blocks by one wave, L21 y handed to the parent),
//   and signals its parent.
// Hand-off (Guideline 16, R1): everything another workgroup reads -- the update matrix (columns
// >= k3) and the pending row updates -- is stored write-through (sc1, agent-scope relaxed stores)
// and read back with sc1 loads; every storing wave drains, the workgroup synchronises, ONE lane
// adds to the parent's counter; the consumer polls relaxed, then one agent-scope acquire.
constexpr int kFT = 512;    // threads per front workgroup
constexpr int kFNB = 24;    // panel width (scalar columns = 8 3x3 blocks)
constexpr int kSmall = 96;  // fronts up to this many rows are assembled + factored entirely in LDS
constexpr int kMaxCh = 8;   // ... if they have at most this many children
constexpr int kPF = (kSmall * (kSmall + 1) / 2 + kFT - 1) / kFT;   // per-thread prefetch slots per child
constexpr int kPFL = 4;      // large fronts: entries in flight per thread in the extend-add / publish rounds
constexpr int kGmax = 32;    // largest team (workgroups per front)

struct ChMeta { int64_t front_off, acc_off, rows_off; int32_t k, r; };




// LDS carve of the factorization phase (doubles): panel [kFNB][Rp] with row offset `off` so that
// trailing rows start 32-B aligned, L_top column-major [kFNB][kFNB], 1/diag, step scratch.
__host__ __device__ inline int fused_rp(int R, int off) { return (R + off + 3) & ~3; }
constexpr int kFScr = kFNB * kFNB + 8 * (kFNB / 3) + 384;   // L_top, 3x3 inverses, POTRF exchange
__host__ __device__ inline size_t fused_lds_doubles(int m3, int k3, bool db) {
    // right-hand side | scratch | one or two panel buffers (the first also holds the assembly tile)
    const size_t large = ((m3 + 1) & ~1) + kFScr + (db ? 2 : 1) * (size_t)kFNB * fused_rp(m3, 3);
    (void)k3;
    const size_t small = m3 <= kSmall ? (size_t)m3 * m3 + m3 + (kMaxCh * sizeof(ChMeta) + kMaxCh * (kSmall / 3) * 4 + 7) / 8 : 0;
    return 2 + std::max(small, large);
}

// packed lower triangle of an n x n matrix, column-major: entry e -> (row i, column j), i >= j
__device__ __forceinline__ void tri_ij(int e, int n, int& i, int& j) {
    const float b = 2.0f * (float)n + 1.0f;
    int jj = (int)((b - sqrtf(b * b - 8.0f * (float)e)) * 0.5f);
    jj = max(0, min(jj, n - 1));
    while (jj > 0 && jj * n - jj * (jj - 1) / 2 > e) --jj;
    while (jj + 1 < n && (jj + 1) * n - (jj + 1) * jj / 2 <= e) ++jj;
    j = jj;
    i = jj + e - (jj * n - jj * (jj - 1) / 2);
}

// A front of at most kSmall rows, entirely in LDS: H blocks and the right-hand side are scattered
// while the children are still running; after the wait the children's update matrices and pending
// row updates arrive through ONE pipelined round of sc1 loads (child c + 1 in flight while child c
// is added; child order fixes the summation order); the factorization runs by 3x3 block columns
// with the right-hand side as an extra column (so the forward solve is folded in); the finished
// L columns, y, the update matrix (sc1) and the pending row updates (sc1) go out once.
__device__ __forceinline__ void small_front(int s, const SnDev& S, int32_t* sync, int32_t* status, const SnDev* __restrict__ sns,
                            const OEnt* __restrict__ omap, const int32_t* __restrict__ relmap,
                            const int32_t* __restrict__ child_list, const double* __restrict__ hb,
                            const double* __restrict__ g, const int32_t* __restrict__ perm, double* fronts,
                            double* __restrict__ ysol, double* acc, double* sm) {
    const int tid = threadIdx.x;
    const int k3 = 3 * S.k, r3 = 3 * S.r, m3 = k3 + r3;
    double* F = fronts + S.front_off;
    double* A = sm;                                           // [m3][m3] column-major
    double* bv = A + m3 * m3;                                 // [m3] right-hand side column
    ChMeta* chm = reinterpret_cast<ChMeta*>(bv + m3);   // m3 (m3 + 1) doubles: 16-B aligned
    int32_t* crm = reinterpret_cast<int32_t*>(chm + kMaxCh);  // [kMaxCh][kSmall / 3] child relmaps
    const int nch = S.nchild;
    // ---- before the wait: everything that does not come from the children
    for (int e = tid; e < m3 * m3; e += kFT) A[e] = 0.0;
    for (int t = tid; t < m3; t += kFT) bv[t] = t < k3 ? -g[3 * perm[S.c0 + t / 3] + t % 3] : 0.0;
    if (tid < nch) {
        const SnDev C = sns[child_list[S.child_off + tid]];
        chm[tid] = ChMeta{C.front_off, C.acc_off, C.rows_off, C.k, C.r};
        for (int q = 0; q < C.r; ++q) crm[tid * (kSmall / 3) + q] = relmap[C.rows_off + q];
    }
    __syncthreads();
    for (int q = tid; q < S.omap_n * 9; q += kFT) {
        const OEnt o = omap[S.omap_off + q / 9];
        const int ii = (q % 9) / 3, jj = q % 3;
        const int row = 3 * o.a + ii, col = 3 * o.b + jj;
        if (row < col) continue;
        const double* B = hb + 9 * (int64_t)o.u;
        A[col * m3 + row] = o.tr ? B[3 * jj + ii] : B[3 * ii + jj];
    }
    if (nch > 0) {
        if (tid == 0) wait_geq_sc1(sync + s, S.need, status);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    FT_MARK(s, 1);
    // ---- children: update matrices (packed lower triangles) + pending row updates
    auto load_child = [&](int ci, double (&v)[kPF], double& va) {
        const ChMeta C = chm[ci];
        const int n = 3 * C.r, tri = n * (n + 1) / 2, m3c = 3 * (C.k + C.r), k3c = 3 * C.k;
        double* Fc = fronts + C.front_off + (int64_t)k3c * m3c + k3c;
#pragma unroll
        for (int q = 0; q < kPF; ++q) {
            const int e = tid + kFT * q;
            v[q] = 0.0;
            if (e < tri) {
                int i, j;
                tri_ij(e, n, i, j);
                v[q] = ld_agent(Fc + (int64_t)j * m3c + i);
            }
        }
        va = tid < n ? ld_agent(acc + C.acc_off + tid) : 0.0;
    };
    auto add_child = [&](int ci, const double (&v)[kPF], double va) {
        const ChMeta C = chm[ci];
        const int n = 3 * C.r, tri = n * (n + 1) / 2;
        const int32_t* rm = crm + ci * (kSmall / 3);
#pragma unroll
        for (int q = 0; q < kPF; ++q) {
            const int e = tid + kFT * q;
            if (e < tri) {
                int i, j;
                tri_ij(e, n, i, j);
                const int pj = 3 * rm[j / 3] + j % 3, pi = 3 * rm[i / 3] + i % 3;
                A[pj * m3 + pi] += v[q];
            }
        }
        if (tid < n) bv[3 * rm[tid / 3] + tid % 3] -= va;
    };
    if (nch > 0) {
        double va_[kPF], vb_[kPF], aa = 0.0, ab = 0.0;
        load_child(0, va_, aa);
        for (int ci = 0; ci < nch; ci += 2) {
            if (ci + 1 < nch) load_child(ci + 1, vb_, ab);
            add_child(ci, va_, aa);
            __syncthreads();
            if (ci + 1 < nch) {
                if (ci + 2 < nch) load_child(ci + 2, va_, aa);
                add_child(ci + 1, vb_, ab);
                __syncthreads();
            }
        }
    }
    FT_MARK(s, 2);
    // ---- factorization by 3x3 block columns, right-hand side as column m3
    bool bad = false;
    for (int c0 = 0; c0 < k3; c0 += 3) {
        const double* C0 = A + c0 * m3;
        const double* C1 = C0 + m3;
        const double* C2 = C1 + m3;
        double d00 = C0[c0], d10 = C0[c0 + 1], d20 = C0[c0 + 2], d11 = C1[c0 + 1], d21 = C1[c0 + 2], d22 = C2[c0 + 2];
        if (!(d00 > 0.0)) { bad = true; d00 = 1.0; }
        const double i00 = rsqrt_nr(d00), l00 = d00 * i00;
        const double l10 = d10 * i00, l20 = d20 * i00;
        double e11 = d11 - l10 * l10;
        if (!(e11 > 0.0)) { bad = true; e11 = 1.0; }
        const double i11 = rsqrt_nr(e11), l11 = e11 * i11;
        const double l21 = (d21 - l20 * l10) * i11;
        double e22 = d22 - l20 * l20 - l21 * l21;
        if (!(e22 > 0.0)) { bad = true; e22 = 1.0; }
        const double i22 = rsqrt_nr(e22), l22 = e22 * i22;
        const double y0 = bv[c0] * i00;
        const double y1 = (bv[c0 + 1] - l10 * y0) * i11;
        const double y2 = (bv[c0 + 2] - l20 * y0 - l21 * y1) * i22;
        for (int i = c0 + 3 + tid; i < m3; i += kFT) {
            const double x0 = C0[i] * i00;
            const double x1 = (C1[i] - x0 * l10) * i11;
            const double x2 = (C2[i] - x0 * l20 - x1 * l21) * i22;
            A[c0 * m3 + i] = x0;
            A[(c0 + 1) * m3 + i] = x1;
            A[(c0 + 2) * m3 + i] = x2;
            bv[i] -= x0 * y0 + x1 * y1 + x2 * y2;
        }
        __syncthreads();
        if (tid == 0) {
            A[c0 * m3 + c0] = l00; A[c0 * m3 + c0 + 1] = l10; A[c0 * m3 + c0 + 2] = l20;
            A[(c0 + 1) * m3 + c0 + 1] = l11; A[(c0 + 1) * m3 + c0 + 2] = l21; A[(c0 + 2) * m3 + c0 + 2] = l22;
            bv[c0] = y0; bv[c0 + 1] = y1; bv[c0 + 2] = y2;
        }
        const int b0 = c0 + 3, nr = m3 - b0;
        for (int e = tid; e < nr * nr; e += kFT) {
            const int l = b0 + e / nr, i = b0 + e % nr;
            if (i < l) continue;
            double v = A[l * m3 + i];
            v = fma(-C0[i], C0[l], v);
            v = fma(-C1[i], C1[l], v);
            v = fma(-C2[i], C2[l], v);
            A[l * m3 + i] = v;
        }
        __syncthreads();
    }
    if (bad && tid == 0) atomicExch(status, 1);
    FT_MARK(s, 3);
    // ---- out: L columns + y (read by the backward solve, next launch), update matrix + pending (sc1)
    for (int e = tid; e < k3 * m3; e += kFT) {
        const int j = e / m3, i = e - j * m3;
        if (i >= j) F[(int64_t)j * m3 + i] = A[e];
    }
    for (int t = tid; t < k3; t += kFT) ysol[3 * (int64_t)S.c0 + t] = bv[t];
    if (S.parent >= 0) {   // the update matrix: 16-B sc1 stores of the aligned pairs over its columns
        const auto rs = front_rsrc(F, m3);
        const int npc = (r3 + 2) >> 1;
        for (int e = tid; e < r3 * npc; e += kFT) {
            const int jj = e / npc, k = e - jj * npc, j = k3 + jj;
            const uint32_t a = (uint32_t)(j * m3 + k3);
            const int i0 = 2 * k - (int)(a & 1u);   // rows k3 + i0, k3 + i0 + 1
            if (i0 + 1 < jj || i0 >= r3) continue;
            const double* Aj = A + j * m3 + k3;
            st2_sc1(rs, (a & ~1u) + 2u * k, i0 >= jj ? Aj[i0] : 0.0, i0 + 1 < r3 ? Aj[i0 + 1] : 0.0);
        }
        for (int t = tid; t < r3; t += kFT) st_agent(acc + S.acc_off + t, -bv[k3 + t]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    FT_MARK(s, 4);
    if (tid == 0 && S.parent >= 0)
        __hip_atomic_fetch_add(sync + S.parent, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A front of more than kSmall rows is factored by a TEAM of G workgroups (G consecutive tickets).
// Its columns are cut into tiles of kFNB: pivot tiles [kFNB t, min(kFNB t + kFNB, k3)), then update
// tiles from k3; tile t belongs to member t mod G, and only its owner ever writes it (plain stores).
// Per pivot panel p the owner -- who has already applied panels 0..p-1 to its tile -- factors it
// (POTRF of the top block by one wave, TRSM of the rows below, one row per thread), publishes it
// write-through (sc1) and raises the front's panel flag; every member with tiles right of p loads
// the panel (sc1) into LDS and applies the rank-w update to its own tiles (4x4 register tiles).
// Member 0 also carries the right-hand side (forward solve folded in, as in small_front).  The
// children's update matrices are added into the owners' columns in child order; at the end every
// member republishes its update tiles write-through and adds 1 to the parent's counter (which
// waits for the sum of its children's team sizes).
struct Tiles {
    int k3, m3, np, nt;
    __device__ int c0(int t) const { return t < np ? kFNB * t : k3 + kFNB * (t - np); }
    __device__ int c1(int t) const { return t < np ? min(kFNB * t + kFNB, k3) : min(k3 + kFNB * (t - np + 1), m3); }
};

// per (large front, tile): the H blocks and the children's column ranges that land in the tile
struct FTask { int32_t om_b, om_e, ch_off, ch_cnt; };
struct FChild { int32_t ja, jb, k, r; int64_t front_off, rows_off; };

// Panel q of a large front, in LDS (P, the panel frame: column c of the tile at P[c * Rp + off + i],
// rows i >= c valid, zeros above): POTRF of the top w x w block, TRSM of the rows below, L_top
// copied back.  `scr` holds L_top, the 3x3 inverses and the POTRF column exchange.
__device__ void factor_lds(int q, int s, const Tiles& T, double* P, double* scr, bool& bad) {
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int k3 = T.k3, m3 = T.m3;
    const int j0 = kFNB * q, w = min(kFNB, k3 - j0), R = m3 - j0;
    const int off = (4 - (w & 3)) & 3, Rp = fused_rp(R, off);
    double* Lt = scr;
    double* rdg = Lt + kFNB * kFNB;
    int* flg = reinterpret_cast<int*>(rdg + 8 * (kFNB / 3));   // [kFNB / 3] step epochs (zeroed by the chain's start)
    PN_MARK(s, q, 5);
    // POTRF of the top w x w block, pipelined over the waves: wave v owns the 3x3 block column
    // 3v..3v+2 (lane = row, its three columns in registers).  It applies each earlier step's
    // update as soon as that step's columns are posted (L_top in LDS + an LDS epoch flag: a
    // wave-to-wave hand-off, no workgroup barrier per step), then factors its own 3x3 block,
    // posts its columns and raises its flag -- the chain per step is flag -> three fma ->
    // chol3 -> post.  Same arithmetic and order as a step-by-step POTRF.
    {
        const int i = lane, cv = 3 * wave, ep = q + 1;
        if (cv < w) {   // wave-uniform
            double col[3];
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const int c = cv + r;
                col[r] = (i < w && i >= c) ? P[c * Rp + off + i] : 0.0;
            }
            for (int st = 0; st < wave; ++st) {
                while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(flg + st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < ep)
                    __builtin_amdgcn_s_sleep(0);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const int c0 = 3 * st;
                const int ii = i < kFNB ? i : 0;
                const double x0 = Lt[c0 * kFNB + ii], x1 = Lt[(c0 + 1) * kFNB + ii], x2 = Lt[(c0 + 2) * kFNB + ii];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int c = cv + r;
                    const double y0 = Lt[c0 * kFNB + c], y1 = Lt[(c0 + 1) * kFNB + c], y2 = Lt[(c0 + 2) * kFNB + c];
                    const double v = fma(-x2, y2, fma(-x1, y1, fma(-x0, y0, col[r])));
                    col[r] = (i >= c && i < w) ? v : col[r];
                }
            }
            ST_MARK(s, q, wave);
            const double d00 = rdlane(col[0], cv), d10 = rdlane(col[0], cv + 1), d20 = rdlane(col[0], cv + 2);
            const double d11 = rdlane(col[1], cv + 1), d21 = rdlane(col[1], cv + 2), d22 = rdlane(col[2], cv + 2);
            const Chol3 L = chol3(d00, d10, d11, d20, d21, d22, bad);
            double x0 = col[0] * L.m00;
            double x1 = fma(col[0], L.m10, col[1] * L.m11);
            double x2 = fma(col[0], L.m20, fma(col[1], L.m21, col[2] * L.m22));
            if (i == cv) { x0 = L.l00; x1 = 0.0; x2 = 0.0; }
            else if (i == cv + 1) { x0 = L.l10; x1 = L.l11; x2 = 0.0; }
            else if (i == cv + 2) { x0 = L.l20; x1 = L.l21; x2 = L.l22; }
            if (i < kFNB) {
                Lt[cv * kFNB + i] = (i >= cv && i < w) ? x0 : 0.0;
                Lt[(cv + 1) * kFNB + i] = (i >= cv + 1 && i < w) ? x1 : 0.0;
                Lt[(cv + 2) * kFNB + i] = (i >= cv + 2 && i < w) ? x2 : 0.0;
            }
            if (i == 0) {
                double* mi = rdg + 2 * cv;   // 8 doubles per 3x3 block
                mi[0] = L.m00; mi[1] = L.m10; mi[2] = L.m11; mi[3] = L.m20; mi[4] = L.m21; mi[5] = L.m22;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (i == 0) __hip_atomic_store(flg + wave, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (cv < kFNB) {   // a short last panel: this wave's columns are past w
            for (int r = 0; r < 3; ++r)
                if (i < kFNB) Lt[(cv + r) * kFNB + i] = 0.0;
        }
    }
    __syncthreads();
    PN_MARK(s, q, 6);
    // rows below: a L_top^T = row, one row per thread, by 3x3 blocks (x_b = a_b Minv_b^T, then the
    // later blocks of the row are updated -- all their products independent)
    for (int i = w + tid; i < R; i += kFT) {
        double a[kFNB];
#pragma unroll
        for (int c = 0; c < kFNB; ++c) a[c] = c < w ? P[c * Rp + off + i] : 0.0;
#pragma unroll
        for (int b = 0; b < kFNB; b += 3) {
            if (b < w) {
                const double* mi = rdg + 2 * b;
                const double x0 = a[b] * mi[0];
                const double x1 = fma(a[b], mi[1], a[b + 1] * mi[2]);
                const double x2 = fma(a[b], mi[3], fma(a[b + 1], mi[4], a[b + 2] * mi[5]));
                a[b] = x0; a[b + 1] = x1; a[b + 2] = x2;
#pragma unroll
                for (int cc = b + 3; cc < kFNB; ++cc)
                    a[cc] = fma(-x2, Lt[(b + 2) * kFNB + cc], fma(-x1, Lt[(b + 1) * kFNB + cc], fma(-x0, Lt[b * kFNB + cc], a[cc])));
            }
        }
#pragma unroll
        for (int c = 0; c < kFNB; ++c)
            if (c < w) P[c * Rp + off + i] = a[c];
    }
    __syncthreads();
    PN_MARK(s, q, 7);
    for (int e = tid; e < w * w; e += kFT) {
        const int c = e / w, r = e - c * w;
        if (r >= c) P[c * Rp + off + r] = Lt[c * kFNB + r];
    }
    __syncthreads();
    PN_MARK(s, q, 3);
}

// the factored panel q (LDS) -> its front columns, write-through, then the panel flag
__device__ void publish_panel(int q, int s, const Tiles& T, double* F, const double* P, int32_t* pflag) {
    const int tid = threadIdx.x;
    const int j0 = kFNB * q, w = min(kFNB, T.k3 - j0), R = T.m3 - j0;
    const int off = (4 - (w & 3)) & 3, Rp = fused_rp(R, off);
    const auto rs = front_rsrc(F, T.m3);
    const int npc = (R + 2) >> 1;   // aligned pairs per column segment (rows j0 .. m3)
    for (int e = tid; e < w * npc; e += kFT) {
        const int c = e / npc, k = e - c * npc;
        const uint32_t a = (uint32_t)((j0 + c) * T.m3 + j0);
        const int i0 = 2 * k - (int)(a & 1u);   // the pair's first row (segment frame)
        if (i0 + 1 < c || i0 >= R) continue;   // wholly above the diagonal, or past the column
        const double* pc = P + c * Rp + off;
        st2_sc1(rs, (a & ~1u) + 2u * k, i0 >= c ? pc[i0] : 0.0, i0 + 1 < R ? pc[i0 + 1] : 0.0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(pflag + s, q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    PN_MARK(s, q, 4);
}

// the pivot columns of tile p (= panel p's columns) -> LDS in the panel frame, zeros above the
// diagonal; SC1: the columns were handed off by another workgroup (sc1 loads), else plain
template <bool SC1>
__device__ void load_panel(int p, const Tiles& T, double* F, double* P) {
    const int tid = threadIdx.x;
    const int j0 = kFNB * p, w = min(kFNB, T.k3 - j0), R = T.m3 - j0;
    const int off = (4 - (w & 3)) & 3, Rp = fused_rp(R, off);
    if (SC1) {   // 16-B sc1 loads of the aligned pairs (publish_panel's cover of each column segment)
        const auto rs = front_rsrc(F, T.m3);
        const int npc = (R + 2) >> 1, tot = w * npc;
        constexpr int kB2 = 8;
        for (int e0 = 0; e0 < tot; e0 += kFT * kB2) {
            double2 v[kB2];
#pragma unroll
            for (int q = 0; q < kB2; ++q) {
                const int e = e0 + tid + kFT * q;
                const int c = e / npc, k = e - c * npc;
                const uint32_t a = (uint32_t)((j0 + c) * T.m3 + j0);
                const int i0 = 2 * k - (int)(a & 1u);
                v[q] = make_double2(0.0, 0.0);
                if (e < tot && i0 < R && i0 + 1 >= c) v[q] = ld2_sc1(rs, (a & ~1u) + 2u * k);
            }
#pragma unroll
            for (int q = 0; q < kB2; ++q) {
                const int e = e0 + tid + kFT * q;
                const int c = e / npc, k = e - c * npc;
                const uint32_t a = (uint32_t)((j0 + c) * T.m3 + j0);
                const int i0 = 2 * k - (int)(a & 1u);
                if (e < tot) {
                    double* pc = P + c * Rp + off;
                    if (i0 >= 0 && i0 < R) pc[i0] = i0 >= c ? v[q].x : 0.0;
                    if (i0 + 1 < R) pc[i0 + 1] = i0 + 1 >= c ? v[q].y : 0.0;
                }
            }
        }
        return;
    }
    constexpr int kB = 16;
    for (int e0 = 0; e0 < w * R; e0 += kFT * kB) {
        double v[kB];
#pragma unroll
        for (int q = 0; q < kB; ++q) {
            const int e = e0 + tid + kFT * q;
            const int c = e / R, i = e - c * R;
            double* a = F + (uint32_t)((j0 + c) * T.m3 + j0 + i);
            v[q] = (e < w * R && i >= c) ? (SC1 ? ld_agent(a) : *a) : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kB; ++q) {
            const int e = e0 + tid + kFT * q;
            const int c = e / R, i = e - c * R;
            if (e < w * R) P[c * Rp + off + i] = v[q];
        }
    }
}

// rank-w update of tile t with panel p (in LDS), 4x4 register tiles, RMW of the owner's columns
// (WT: the results are stored write-through, the tile is handed off next; SC1: the tile was handed
// off to this workgroup, read it sc1)
template <bool WT, bool SC1 = false>
__device__ void update_tile(int t, int p, const Tiles& T, double* F, const double* P) {
    const int tid = threadIdx.x;
    const int m3 = T.m3, j0 = kFNB * p, w = min(kFNB, T.k3 - j0), R = m3 - j0;
    const int off = (4 - (w & 3)) & 3, Rp = fused_rp(R, off);
    const int l0 = T.c0(t) - j0, l1 = T.c1(t) - j0;   // the tile's columns, panel frame
    const int g0 = ((l0 + off) & ~3) - off;            // 4-aligned group start (<= l0)
    const int ncg = (l1 - g0 + 3) >> 2, nrg = (R - g0 + 3) >> 2;
    for (int q = tid; q < nrg * ncg; q += kFT) {
        const int ib = g0 + 4 * (q % nrg), lb = g0 + 4 * (q / nrg);
        if (ib + 3 < lb) continue;
        double ac[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) ac[a][b] = 0.0;
#pragma unroll 1
        for (int c = 0; c < w; ++c) {
            const double2* pc = reinterpret_cast<const double2*>(P + c * Rp);
            const double2 i01 = pc[(off + ib) >> 1], i23 = pc[((off + ib) >> 1) + 1];
            const double2 l01 = pc[(off + lb) >> 1], l23 = pc[((off + lb) >> 1) + 1];
            const double vi[4] = {i01.x, i01.y, i23.x, i23.y};
            const double vl[4] = {l01.x, l01.y, l23.x, l23.y};
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) ac[a][b] = fma(vi[a], vl[b], ac[a][b]);
        }
        // the tile's current values (clamped addresses: all 16 loads issue before any store)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t o = (uint32_t)((j0 + min(max(lb + b, l0), l1 - 1)) * m3 + j0);
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                double* src = F + o + (uint32_t)min(ib + a, R - 1);
                ac[a][b] = (SC1 ? ld_agent(src) : *src) - ac[a][b];
            }
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int l = lb + b;
            const uint32_t o = (uint32_t)((j0 + l) * m3 + j0);
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const int i = ib + a;
                if (l >= l0 && l < l1 && i < R && i >= l) {
                    if (WT) st_agent(F + o + (uint32_t)i, ac[a][b]);
                    else F[o + (uint32_t)i] = ac[a][b];
                }
            }
        }
    }
}

// the chain's own step: pivot tile p + 1 (loaded into Pn, its panel frame) -= panel p (Pc, full
// width) restricted to the tile; LDS to LDS, 4x4 register tiles
__device__ void update_next_lds(int p, const Tiles& T, const double* Pc, double* Pn) {
    const int tid = threadIdx.x;
    const int j0 = kFNB * p, R = T.m3 - j0, Rp = fused_rp(R, 0);   // panel p is full: off 0
    const int j1 = j0 + kFNB, w1 = min(kFNB, T.k3 - j1), R1 = R - kFNB;
    const int off1 = (4 - (w1 & 3)) & 3, Rp1 = fused_rp(R1, off1);
    const int ncg = (w1 + 3) >> 2, nrg = (R1 + 3) >> 2;
    for (int q = tid; q < nrg * ncg; q += kFT) {
        const int ib = 4 * (q % nrg), lb = 4 * (q / nrg);
        if (ib + 3 < lb) continue;
        double ac[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) ac[a][b] = 0.0;
#pragma unroll 2
        for (int c = 0; c < kFNB; ++c) {
            const double2* pc = reinterpret_cast<const double2*>(Pc + c * Rp + kFNB);
            const double2 i01 = pc[ib >> 1], i23 = pc[(ib >> 1) + 1];
            const double2 l01 = pc[lb >> 1], l23 = pc[(lb >> 1) + 1];
            const double vi[4] = {i01.x, i01.y, i23.x, i23.y};
            const double vl[4] = {l01.x, l01.y, l23.x, l23.y};
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) ac[a][b] = fma(vi[a], vl[b], ac[a][b]);
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int l = lb + b;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const int i = ib + a;
                if (l < w1 && i < R1 && i >= l) Pn[l * Rp1 + off1 + i] -= ac[a][b];
            }
        }
    }
}

// forward solve folded in: y of panel p's rows (one wave), then the rows below (bv, LDS)
__device__ void rhs_panel(int p, const Tiles& T, const double* P, double* bv) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int j0 = kFNB * p, w = min(kFNB, T.k3 - j0), R = T.m3 - j0;
    const int off = (4 - (w & 3)) & 3, Rp = fused_rp(R, off);
    if (wave == 0) {
        double bl = lane < w ? bv[j0 + lane] : 0.0;
        for (int c = 0; c < w; ++c) {
            const double yc = __shfl(bl, c, 64) / P[c * Rp + off + c];
            if (lane == c) bl = yc;
            else if (lane > c && lane < w) bl = fma(-P[c * Rp + off + lane], yc, bl);
        }
        if (lane < w) bv[j0 + lane] = bl;
    }
    __syncthreads();
    for (int i = w + tid; i < R; i += kFT) {
        double sacc = 0.0;
        for (int c = 0; c < w; ++c) sacc = fma(P[c * Rp + off + i], bv[j0 + c], sacc);
        bv[j0 + i] -= sacc;
    }
    __syncthreads();
}

// A front of more than kSmall rows is factored by a TEAM of G workgroups (G consecutive tickets).
// Its columns are cut into tiles of kFNB: pivot tiles [kFNB t, min(kFNB t + kFNB, k3)), then update
// tiles from k3.  Member 0 runs the panel CHAIN and owns tile 0; tile t >= 1 belongs to helper
// 1 + (t - 1) mod (G - 1), which alone assembles it and applies the panels to it, except that the
// last panel before a pivot tile's own (panel t - 1) is applied by member 0:
//   assembly, per own tile, in LDS: H's blocks, then the children's update-matrix columns that land
//     in the tile (host-precomputed ranges), child by child, kFT * kPFL sc1 loads in flight;
//   chain (member 0): panel p is in LDS; it loads pivot tile p + 1 (handed off write-through by its
//     helper once panels 0..p-1 are in: flag tready[t]), applies panel p to it LDS to LDS, factors and
//     publishes it (write-through + panel flag) -- the chain never waits on a panel load or a flag it
//     could not have had a step earlier; with one LDS panel buffer (db == 0, very tall fronts) the
//     step goes through the front instead;
//   helpers: for p = 0, 1, ..: wait for panel p, load it, first bring pivot tile p + 2 up to date and
//     hand it off, then apply panel p to their other tiles;
//   the owner of the last tile (a helper that loads every panel) carries the right-hand side
//   (forward solve folded in, as in small_front);
//   at the end every member republishes its update tiles write-through and adds 1 to the parent's
//   counter (which waits for the sum of its children's team sizes).
__device__ __forceinline__ int tile_owner(int t, int G) { return t == 0 || G == 1 ? 0 : 1 + (t - 1) % (G - 1); }

__device__ __forceinline__ void large_front(int s, int mem, const SnDev& S, int32_t* sync, int32_t* pflag,
                            int32_t* tready, int32_t* status,
                            const SnDev* __restrict__ sns, const OEnt* __restrict__ omap,
                            const int32_t* __restrict__ relmap, const int32_t* __restrict__ child_list,
                            const FTask* __restrict__ ftasks, const FChild* __restrict__ fchild,
                            const double* __restrict__ hb, const double* __restrict__ g,
                            const int32_t* __restrict__ perm, double* fronts, double* __restrict__ ysol,
                            double* acc, double* sm, int db) {
    const int tid = threadIdx.x;
    const int k3 = 3 * S.k, r3 = 3 * S.r, m3 = k3 + r3, G = S.G;
    double* F = fronts + S.front_off;
    Tiles T{k3, m3, (k3 + kFNB - 1) / kFNB, 0};
    T.nt = T.np + (r3 + kFNB - 1) / kFNB;
    int32_t* trdy = tready + S.ftask;
    const bool has_b = mem == tile_owner(T.nt - 1, G);   // the right-hand side: a helper that sees every panel
    const int t_first = mem, t_step = mem == 0 ? T.nt : G - 1;   // own tiles: t_first, += t_step
    double* bv = sm;                               // [m3] right-hand side (member 0)
    double* scr = bv + ((m3 + 1) & ~1);            // POTRF / TRSM scratch
    double* PA = scr + kFScr;                      // tile under assembly / panel buffers
    double* PB = db ? PA + (size_t)kFNB * fused_rp(m3, 3) : PA;
    if (has_b)
        for (int t = tid; t < m3; t += kFT) bv[t] = t < k3 ? -g[3 * perm[S.c0 + t / 3] + t % 3] : 0.0;
    // ---- assembly of the own tiles in LDS (the first one's H blocks before the wait)
    bool waited = S.need == 0;
    for (int t = t_first; t < T.nt; t += t_step) {
        const FTask tk = ftasks[S.ftask + t];
        const int cs = T.c0(t), nc = T.c1(t) - cs;
        double* Tl = PA;                           // [nc][m3] column-major
        for (int e = tid; e < nc * m3; e += kFT) Tl[e] = 0.0;
        __syncthreads();
        for (int q = tid; q < (tk.om_e - tk.om_b) * 9; q += kFT) {
            const OEnt o = omap[tk.om_b + q / 9];
            const int ii = (q % 9) / 3, jj = q % 3;
            const int row = 3 * o.a + ii, col = 3 * o.b + jj;
            if (col < cs || col >= cs + nc || row < col) continue;
            const double* B = hb + 9 * (int64_t)o.u;
            Tl[(col - cs) * m3 + row] = o.tr ? B[3 * jj + ii] : B[3 * ii + jj];
        }
        if (!waited) {
            if (tid == 0) wait_geq_sc1(sync + s, S.need, status);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            waited = true;
            FT_MARK(s, 1);
        }
        for (int cq = 0; cq < tk.ch_cnt; ++cq) {
            __syncthreads();
            const FChild C = fchild[tk.ch_off + cq];
            const int n = 3 * C.r, m3c = 3 * (C.k + C.r), k3c = 3 * C.k, nj = C.jb - C.ja;
            // the child's update matrix: column j of it, rows i >= j, is front element
            // (k3c + j) m3c + k3c + i -- 16-B sc1 loads of the aligned pairs over each column
            const auto rs = front_rsrc(fronts + C.front_off, m3c);
            const int32_t* rm = relmap + C.rows_off;
            const int npc = (n + 2) >> 1, tot = nj * npc;
            for (int e0 = 0; e0 < tot; e0 += kFT * kPFL) {
                double2 v[kPFL];
                int d0[kPFL], d1[kPFL];
#pragma unroll
                for (int q = 0; q < kPFL; ++q) {
                    const int e = e0 + tid + kFT * q;
                    const int jj = e / npc, k = e - jj * npc, j = C.ja + jj;
                    const uint32_t a = (uint32_t)((k3c + j) * m3c + k3c);
                    const int i0 = 2 * k - (int)(a & 1u);
                    d0[q] = -1;
                    d1[q] = -1;
                    v[q] = make_double2(0.0, 0.0);
                    if (e < tot && i0 + 1 >= j && i0 < n) {
                        v[q] = ld2_sc1(rs, (a & ~1u) + 2u * k);
                        const int cj = (3 * rm[j / 3] + j % 3 - cs) * m3;
                        if (i0 >= j) d0[q] = cj + 3 * rm[i0 / 3] + i0 % 3;
                        if (i0 + 1 < n) d1[q] = cj + 3 * rm[(i0 + 1) / 3] + (i0 + 1) % 3;
                    }
                }
#pragma unroll
                for (int q = 0; q < kPFL; ++q) {
                    if (d0[q] >= 0) Tl[d0[q]] += v[q].x;
                    if (d1[q] >= 0) Tl[d1[q]] += v[q].y;
                }
            }
        }
        __syncthreads();
        if (t == 0 && mem == 0 && db) {
            // the chain's first panel straight from the assembled tile: LDS to LDS into the panel
            // frame of PB (zeros above the diagonal, as load_panel), no round trip through the front
            const int off = (4 - (nc & 3)) & 3, Rp = fused_rp(m3, off);
            for (int e = tid; e < nc * m3; e += kFT) {
                const int c = e / m3, i = e - c * m3;
                PB[c * Rp + off + i] = i >= c ? Tl[e] : 0.0;
            }
            __syncthreads();
            continue;
        }
        const bool handoff = t == 1 && mem != 0;   // pivot tile 1 goes to the chain as assembled
        for (int e = tid; e < nc * m3; e += kFT) {
            const int col = cs + e / m3, row = e % m3;
            if (row >= col) {
                if (handoff) st_agent(F + (uint32_t)(col * m3 + row), Tl[e]);
                else F[(uint32_t)(col * m3 + row)] = Tl[e];
            }
        }
        if (handoff) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (handoff && tid == 0) __hip_atomic_store(trdy + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!waited) {   // a helper without tiles (G > nt cannot happen; kept for safety)
        if (tid == 0) wait_geq_sc1(sync + s, S.need, status);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (has_b) {   // the children's pending row updates, child order
        for (int ci = 0; ci < S.nchild; ++ci) {
            const SnDev C = sns[child_list[S.child_off + ci]];
            const int32_t* rm = relmap + C.rows_off;
            for (int t = tid; t < 3 * C.r; t += kFT) bv[3 * rm[t / 3] + t % 3] -= ld_agent(acc + C.acc_off + t);
            __syncthreads();
        }
    }
    FT_MARK(s, 2);

    bool bad = false;
    if (mem == 0) {
        // ---- the panel chain
        double* cur = db ? PB : PA;   // db: panel 0 is in PB already (the assembly's relayout)
        if (tid < kFNB / 3) reinterpret_cast<int*>(scr + kFNB * kFNB + 8 * (kFNB / 3))[tid] = 0;   // POTRF step epochs
        if (!db) load_panel<false>(0, T, F, cur);   // tile 0: assembled by this workgroup
        __syncthreads();
        factor_lds(0, s, T, cur, scr, bad);
        publish_panel(0, s, T, F, cur, pflag);
        for (int p = 0; p < T.np; ++p) {
            double* nxt = cur == PA ? PB : PA;
            if (has_b && !db) rhs_panel(p, T, cur, bv);
            if (p + 1 < T.np) {
                const int t = p + 1;
                PN_MARK(s, t, 0);
                if (tile_owner(t, G) != 0) {
                    if (tid == 0) wait_geq_sc1(trdy + t, 1, status);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                }
                if (db) {
                    load_panel<true>(t, T, F, nxt);
                    __syncthreads();
                    PN_MARK(s, t, 1);
                    update_next_lds(p, T, cur, nxt);
                } else {   // through the front: sc1 reads of the handed-off tile, then reload
                    PN_MARK(s, t, 1);
                    update_tile<true, true>(t, p, T, F, cur);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                    load_panel<true>(t, T, F, nxt);
                }
                __syncthreads();
                PN_MARK(s, t, 2);
                factor_lds(t, s, T, nxt, scr, bad);
                publish_panel(t, s, T, F, nxt, pflag);
            }
            if (has_b && db) rhs_panel(p, T, cur, bv);
            cur = nxt;
        }
    } else {
        // ---- helpers: apply each panel to the own tiles right of it (pivot tile p + 1 excepted)
        double* P = PA;
        for (int p = 0; p < T.np; ++p) {
            bool need = false;
            for (int t = t_first; t < T.nt; t += t_step) need |= t > p && !(t == p + 1 && t < T.np);
            if (!need && !has_b) break;
            if (tid == 0) wait_geq_sc1(pflag + s, p + 1, status);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            load_panel<true>(p, T, F, P);
            __syncthreads();
            const int tc = p + 2;   // the chain's next-but-one tile first, handed off when done
            const bool mine = tc < T.np && tile_owner(tc, G) == mem;
            if (mine) {
                update_tile<true>(tc, p, T, F, P);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) __hip_atomic_store(trdy + tc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // the last panel's update of an update tile is its final value: stored write-through for
            // the parent (no republishing pass after the chain)
            const bool fin = p == T.np - 1 && S.parent >= 0;
            for (int t = t_first; t < T.nt; t += t_step)
                if (t > p && !(t == p + 1 && t < T.np) && !(mine && t == tc)) {
                    if (fin) update_tile<true>(t, p, T, F, P);
                    else update_tile<false>(t, p, T, F, P);
                }
            __syncthreads();
            if (has_b) rhs_panel(p, T, P, bv);
        }
    }
    if (bad && (tid & 63) == 0) atomicExch(status, 1);
    // ---- out: member 0 (or the right-hand side's owner): y and the pending updates
    if (has_b) {
        for (int t = tid; t < k3; t += kFT) ysol[3 * (int64_t)S.c0 + t] = bv[t];
        if (S.parent >= 0)
            for (int t = tid; t < r3; t += kFT) st_agent(acc + S.acc_off + t, -bv[k3 + t]);
    }
    FT_MARK(s, 3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (mem == 0) FT_MARK(s, 4);
    if (tid == 0 && S.parent >= 0)
        __hip_atomic_fetch_add(sync + S.parent, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kFT, 2) void chol_factor_dag(const int32_t* __restrict__ order, int32_t* sync,
                                                       int32_t* status, const SnDev* __restrict__ sns,
                                                       const OEnt* __restrict__ omap,
                                                       const int32_t* __restrict__ relmap,
                                                       const int32_t* __restrict__ child_list,
                                                       const FTask* __restrict__ ftasks,
                                                       const FChild* __restrict__ fchild,
                                                       const double* __restrict__ hb, const double* __restrict__ g,
                                                       const int32_t* __restrict__ perm, double* fronts,
                                                       double* __restrict__ ysol, double* acc, int ns, int db,
                                                       const int32_t* gate, const uint8_t* __restrict__ keep) {
    extern __shared__ __attribute__((aligned(16))) double smem_f[];
    double* sm = smem_f + 2;   // smem_f[0]: the claimed ticket (no static LDS: keeps the base 16-B aligned)
    if (gate_off(gate, 1)) return;
    // issue priority over co-resident waves of other kernels (the batch covariance runs beside the
    // first factorization of a step, dpg_icp_batch_run): this kernel is a chain of dependent steps
    __builtin_amdgcn_s_setprio(2);
    const int code = claim_lds(order, sync, reinterpret_cast<int*>(smem_f));
    const int s = code >> 6, mem = code & 63;
    const SnDev S = sns[s];
    if (keep && keep[s]) {   // partial refactorization: the front keeps its factored values (and its
                             // update matrix, which the parent reads as from a finished member)
        if (threadIdx.x == 0 && S.parent >= 0)
            __hip_atomic_fetch_add(sync + 1 + S.parent, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (mem == 0) FT_MARK(s, 0);
    if (S.G == 1 && 3 * (S.k + S.r) <= kSmall && S.nchild <= kMaxCh)
        small_front(s, S, sync + 1, status, sns, omap, relmap, child_list, hb, g, perm, fronts, ysol, acc, sm);
    else
        large_front(s, mem, S, sync + 1, sync + 1 + ns, sync + 2 + 3 * ns, status, sns, omap, relmap, child_list,
                    ftasks, fchild, hb, g, perm, fronts, ysol, acc, sm, db);
}

// partial refactorization: the kept fronts (and their pending forward-solve updates) the new layout
// moved, as runs {src, dst, doubles, buffer} (one run per blockIdx.y; buffer 0: fronts, 1: the
// pending updates), through a scratch buffer (gather, then scatter: old and new places overlap)
__global__ __launch_bounds__(256) void chol_copy_runs(const double* __restrict__ src0, const double* __restrict__ src1,
                                                      double* __restrict__ dst0, double* __restrict__ dst1,
                                                      const int64_t* __restrict__ runs) {
    const int64_t* r = runs + 4 * blockIdx.y;
    const int64_t s0 = r[0], d0 = r[1], n = r[2];
    const double* src = r[3] ? src1 : src0;
    double* dst = r[3] ? dst1 : dst0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[d0 + i] = src[s0 + i];
}

// device buffers are kept between rebuilds of the same solver (an incremental graph re-derives its
// structures every update): a buffer is re-allocated only when it must grow (by 1.5x at least)
template <typename T>
int dreserve(T** d, size_t* cap, size_t n) {
    n = std::max<size_t>(n, 1);
    if (*d && n <= *cap) return DPG_OK;
    if (*d) (void)hipFree(*d);
    *d = nullptr;
    const size_t nc = std::max(n, *cap + *cap / 2);
    *cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(d), nc * sizeof(T)) != hipSuccess) return DPG_ERR_HIP;
    *cap = nc;
    return DPG_OK;
}

struct CholDev {
    dpg_chol_opts opts;   // the context's solver options at creation
    dpg_chol_sym sym;
    int64_t n = 0;
    SnDev* sns = nullptr;
    OEnt* omap = nullptr;
    int32_t* child_list = nullptr;
    int32_t* relmap = nullptr;
    int32_t* rows = nullptr;
    int32_t* perm = nullptr;
    int32_t* pos = nullptr;
    double* fronts = nullptr;
    double* acc = nullptr;
    double* ysol = nullptr;
    double* xsol = nullptr;
    int32_t* status = nullptr;
    double* dinv = nullptr;            // inverted diagonal blocks of the solves ([3n][kSB])
    double* linv = nullptr;            // L11^-1 of the large fronts (SnDev.inv offsets)
    int2* inv_tasks = nullptr;         // chol_inv_l11: (front, first column) per workgroup
    int64_t n_inv_tasks = 0, linv_total = 0;
    size_t lds_inv = 0, c_linv = 0;
    int2* dblocks = nullptr;           // (front, jb) of every diagonal block
    int64_t n_dblocks = 0;
    bool use_dinv = false;             // DPG_SOLVE_DINV=1: inverted diagonal blocks (measured slower)
    std::vector<int32_t> level_ptr;
    std::vector<size_t> lds_solve;   // per level
    int64_t nnzb_upper = 0;
    // factorization task lists (device) and the per-level launch plan (host)
    int32_t* order_fwd = nullptr;      // fronts bottom-up (level order) / top-down
    int32_t* order_fac = nullptr;      // fused factorization tickets (front * 64 + member)
    FTask* ftasks = nullptr;           // large fronts: per-tile assembly lists
    FChild* fchild = nullptr;
    int64_t n_tickets = 0;
    int32_t* order_bwd = nullptr;
    SolveSeg* segs = nullptr;
    int32_t* sync = nullptr;           // [ticket_f, cnt_f[ns], ticket_b, done_b[ns]], zeroed per solve
    size_t sync_bytes = 0;
    size_t lds_solve_max = 0;
    int32_t solve_stage = 0;   // R: LDS staging region of the solves, doubles (Stage)
    int32_t solve_maxseg = 0;  // backward: fronts with more row segments wait for the parent (<= kMaxSeg)
    AsmTask* asm_tasks = nullptr;
    AsmChild* asm_child = nullptr;
    int2* panel_tasks = nullptr;
    int4* upd_tasks = nullptr;
    struct Step { int32_t panel_off, panel_cnt, rpt /* panel rows / kT, rounded up */, max_rows, upd_off, upd_cnt; };
    struct Level { int32_t asm_off, asm_cnt; size_t lds_asm; std::vector<Step> steps; };
    std::vector<Level> plan;
    int64_t n_launches = 0;
    // fused DAG factorization + forward solve (used when every front fits its LDS budget)
    bool fused = false;
    size_t lds_fused = 0;
    bool fused_db = true;
    // L11^-1 (chol_inv_l11): valid for the last factorization (inv_valid: computed by an ungated
    // solve); the gated loop computes it on `aux` beside each refactoring iteration's backward solve
    // and its chord iterations wait for it (ev_inv of the previous iteration)
    bool inv_valid = false;
    bool keep_inv = false;   // ungated solves compute L11^-1 after their backward solve (for dpg_chol_resolve)
    hipStream_t aux = nullptr;
    hipEvent_t ev_fac = nullptr, ev_inv[2] = {nullptr, nullptr};
    int inv_par = 0;
    // capacities (elements) of the device buffers above, for rebuilds
    size_t c_fronts = 0, c_acc = 0, c_ysol = 0, c_xsol = 0, c_status = 0, c_sync = 0, c_dinv = 0;
    double t_build[2] = {0, 0};   // last chol_build: host structures, uploads (ms)
    char* stage = nullptr;        // pinned staging buffer of the uploads
    size_t c_stage = 0;
    char* arena = nullptr;        // device: every structure array above (sns .. upd_tasks), one copy
    size_t c_arena = 0;
    // partial refactorization (dpg_chol_track_factor): `fac_sym` is the analysis the values in
    // `fronts` were factored under (valid while fac_valid and fronts == fac_ptr), fac_G its team
    // sizes; sym_is_fac: the current analysis is that one (it moves to fac_sym with the next plan)
    bool track = false, fac_valid = false, sym_is_fac = false, fac_db = false;
    double* fac_ptr = nullptr;         // fronts, y and the pending updates of that factorization
    double* fac_ysol = nullptr;
    double* fac_acc = nullptr;
    dpg_chol_sym fac_sym;
    std::vector<int32_t> cur_G, fac_G;
    std::vector<uint8_t> h_keep;
    std::vector<int32_t> h_old;
    std::vector<int64_t> h_runs;
    double* scratch = nullptr;    // the moved fronts between the gather and the scatter
    size_t c_scratch = 0;
    char* pstage = nullptr;       // pinned: keep flags + runs, one copy up
    size_t c_pstage = 0;
    char* dpart = nullptr;
    size_t c_dpart = 0;
    hipEvent_t pev = nullptr;     // after that copy (the staging buffer's next rewrite waits for it)
    bool pev_set = false;
    int64_t pstats[4] = {0, 0, 0, 0};   // last solve: fronts refactored, kept, doubles moved, host ns of the pick
    void* host = nullptr;         // CholHost of the build in progress (a plan and its upload may run
                                  // on different threads, one after the other)
};

void free_host(void* p);

// a new analysis in; *S gets back one whose buffers the caller reuses.  With tracking, the analysis
// of the last factorization moves to fac_sym instead (the partial refactorization compares with it)
void take_sym(CholDev* c, dpg_chol_sym* S) {
    if (c->track && c->sym_is_fac) {
        std::swap(c->fac_sym, c->sym);
        c->fac_G.swap(c->cur_G);
        c->sym_is_fac = false;
    }
    std::swap(c->sym, *S);
}

}  // namespace

extern "C" void dpg_chol_destroy(void* h) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    if (!c) return;
    // (the structure arrays live in c->arena)
    if (c->aux) (void)hipStreamSynchronize(c->aux);
    void* ptrs[] = {c->arena, c->fronts, c->acc, c->ysol, c->xsol, c->status, c->sync, c->dinv, c->linv, c->scratch, c->dpart};
    if (c->pev) (void)hipEventDestroy(c->pev);
    if (c->pstage) (void)hipHostFree(c->pstage);
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (c->stage) (void)hipHostFree(c->stage);
    if (c->ev_fac) (void)hipEventDestroy(c->ev_fac);
    for (hipEvent_t e : c->ev_inv)
        if (e) (void)hipEventDestroy(e);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    free_host(c->host);
    delete c;
}

namespace {
// Device structures of the factorization for the symbolic analysis in c->sym (reusing c's buffers).
int chol_build(CholDev* c, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs);
}  // namespace

extern "C" int dpg_chol_create(void** out, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi,
                               int64_t n_pairs, const dpg_chol_opts* opts) {
    *out = nullptr;
    CholDev* c = new CholDev();
    if (opts) c->opts = *opts;
    if (dpg_chol_symbolic(n, pair_lo, pair_hi, n_pairs, &c->opts, &c->sym)) {
        delete c;
        return DPG_ERR_NUMERIC;
    }
    const int rc = chol_build(c, n, pair_lo, pair_hi, n_pairs);
    if (rc) { dpg_chol_destroy(c); return rc; }
    *out = c;
    return DPG_OK;
}

// The same from a given symbolic analysis; *h is reused (its buffers grow when needed) or created.
int dpg_chol_create_sym(void** h, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                        dpg_chol_sym* S, const dpg_chol_opts* opts) {
    CholDev* c = *h ? reinterpret_cast<CholDev*>(*h) : new CholDev();
    if (opts) c->opts = *opts;
    take_sym(c, S);   // *S gets an earlier analysis (its buffers are reused by the next derive)
    const int rc = chol_build(c, n, pair_lo, pair_hi, n_pairs);
    if (rc) { dpg_chol_destroy(c); *h = nullptr; return rc; }
    *h = c;
    return DPG_OK;
}

namespace {
double wall_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

// host-side structures of one build (kept between builds: the incremental graph rebuilds per update)
struct CholHost {
    struct Blk { int32_t row, u, tr; };   // an upper block of H in its column's bucket
    struct Blk4 { int32_t row, col, u, tr; };
    std::vector<int64_t> colptr;
    std::vector<Blk> ent;
    std::vector<Blk4> byrow;
    std::vector<int32_t> lidx, lstamp;
    std::vector<int64_t> om_ptr, om_cur;
    std::vector<OEnt> omap;
    std::vector<SnDev> sns;
    std::vector<FTask> ftasks;
    std::vector<FChild> fchild;
    std::vector<double> prio, hgt;
    std::vector<int32_t> hcnt;
    std::vector<SolveSeg> segs;
    std::vector<std::pair<double, int32_t>> key;
    std::vector<int32_t> fo, bwd, order_fac, cuts;
    std::vector<AsmTask> asm_t;
    std::vector<AsmChild> asm_c;
    std::vector<int2> panel_t;
    std::vector<int4> upd_t;
    std::vector<int2> dblocks;
    std::vector<int2> inv_t;            // chol_inv_l11 tasks (front, first column)
    std::vector<int32_t> tcnt, tfill;   // per-tile child counts / fill cursors of one large front
    std::vector<char> tused;
    int64_t acc_total = 0;
    // colptr / ent built ahead by dpg_chol_plan_blocks (the incremental prepare runs it beside the
    // symbolic derivation) for a graph of blocks_n nodes and blocks_np pairs; the next plan takes them
    bool blocks_ready = false;
    int64_t blocks_n = -1, blocks_np = -1;
};

#ifdef DPG_PLAN_TIMING
double g_plan_t[8];
#define PLAN_T(k) g_plan_t[k] += wall_ms()
#else
#define PLAN_T(k) do { } while (0)
#endif

// A child's update rows j = 0 .. 3r-1 land in parent front row 3 rm[j / 3] + j % 3, increasing in
// j: the first j landing at or after parent row c.
inline int32_t first_at_or_after(const int32_t* rm, int32_t r, int32_t c) {
    int32_t lo = 0, hi = 3 * r;
    while (lo < hi) {
        const int32_t mid = (lo + hi) / 2;
        if (3 * rm[mid / 3] + mid % 3 < c) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// H's upper blocks bucketed by column position, each bucket in ascending row order (the plan's
// first part; pos / perm: the ordering -- the symbolic analysis's, or the incremental state's it
// will copy)
void plan_blocks(CholHost& H, int64_t n, const int32_t* pos, const int32_t* perm, const int32_t* pair_lo,
                 const int32_t* pair_hi, int64_t n_pairs) {
    std::vector<int64_t>& colptr = H.colptr;
    colptr.assign((size_t)n + 1, 0);
    for (int64_t p = 0; p < n; ++p) colptr[(size_t)p + 1] = 1;   // the diagonal block
    for (int64_t q = 0; q < n_pairs; ++q)
        colptr[(size_t)std::min(pos[(size_t)pair_lo[q]], pos[(size_t)pair_hi[q]]) + 1]++;
    for (int64_t p = 0; p < n; ++p) colptr[(size_t)p + 1] += colptr[(size_t)p];
    std::vector<CholHost::Blk>& ent = H.ent;
    ent.resize((size_t)colptr[(size_t)n]);
    {
        // two counting sorts: the blocks by row (the pairs' later position; the diagonal block is
        // its column's first row), then stably into their column buckets -- each bucket comes out
        // in ascending row order without a per-bucket sort
        std::vector<int64_t>& rptr = H.om_cur;
        rptr.assign((size_t)n + 1, 0);
        for (int64_t p = 0; p < n; ++p) rptr[(size_t)p + 1] = 1;
        for (int64_t q = 0; q < n_pairs; ++q)
            rptr[(size_t)std::max(pos[(size_t)pair_lo[q]], pos[(size_t)pair_hi[q]]) + 1]++;
        for (int64_t p = 0; p < n; ++p) rptr[(size_t)p + 1] += rptr[(size_t)p];
        std::vector<CholHost::Blk4>& byrow = H.byrow;
        byrow.resize(ent.size());
        for (int64_t p = 0; p < n; ++p) byrow[(size_t)rptr[(size_t)p]++] = CholHost::Blk4{(int32_t)p, (int32_t)p, perm[(size_t)p], 0};
        for (int64_t q = 0; q < n_pairs; ++q) {
            const int32_t plo = pos[(size_t)pair_lo[q]], phi = pos[(size_t)pair_hi[q]];
            // front wants A(later, earlier) = H(later_node, earlier_node); hb holds H(lo, hi)
            const int32_t r = std::max(plo, phi);
            byrow[(size_t)rptr[(size_t)r]++] = CholHost::Blk4{r, std::min(plo, phi), (int32_t)(n + q), plo > phi ? 0 : 1};
        }
        rptr.assign(colptr.begin(), colptr.end() - 1);   // column cursors
        for (const CholHost::Blk4& b : byrow) ent[(size_t)rptr[(size_t)b.col]++] = CholHost::Blk{b.row, b.u, b.tr};
    }
    H.blocks_n = n;
    H.blocks_np = n_pairs;
}

// Host half of chol_build: every device structure, in H; the plan fields of c.
int chol_plan(CholDev* c, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs, CholHost& H) {
    const dpg_chol_sym& S = c->sym;
    c->lds_fused = 0;
    c->n_launches = 0;
    c->n = n;
    c->nnzb_upper = n + n_pairs;
    PLAN_T(0);
    // omap: every upper block of H -> (front, local block row, local block col, transpose), grouped
    // by front, each front's entries by (column, row): the blocks are bucketed by column position
    // (counting sort), each bucket sorted by row, and the fronts walked column by column
    const bool pre = H.blocks_ready && H.blocks_n == n && H.blocks_np == n_pairs;
    H.blocks_ready = false;
#ifdef DPG_PLAN_VERIFY
    if (pre) {   // the prebuilt buckets must equal this plan's own
        const std::vector<int64_t> cp0 = H.colptr;
        const std::vector<CholHost::Blk> e0 = H.ent;
        plan_blocks(H, n, S.pos.data(), S.perm.data(), pair_lo, pair_hi, n_pairs);
        bool same = cp0 == H.colptr && e0.size() == H.ent.size();
        for (size_t k = 0; same && k < e0.size(); ++k)
            same = e0[k].row == H.ent[k].row && e0[k].u == H.ent[k].u && e0[k].tr == H.ent[k].tr;
        if (!same) { fprintf(stderr, "DPG_PLAN_VERIFY: prebuilt H-block buckets differ\n"); abort(); }
    }
#endif
    if (!pre) plan_blocks(H, n, S.pos.data(), S.perm.data(), pair_lo, pair_hi, n_pairs);
    const std::vector<int64_t>& colptr = H.colptr;
    const std::vector<CholHost::Blk>& ent = H.ent;
    PLAN_T(1);
    std::vector<int64_t>& om_ptr = H.om_ptr;
    om_ptr.assign((size_t)S.ns + 1, 0);
    std::vector<OEnt>& omap = H.omap;
    omap.resize(ent.size());
    {
        std::vector<int32_t>& lidx = H.lidx;
        std::vector<int32_t>& lst = H.lstamp;
        lidx.resize((size_t)n);
        lst.assign((size_t)n, -1);
        size_t o = 0;
        for (int32_t s = 0; s < S.ns; ++s) {
            const int32_t c0 = S.sn_c0[(size_t)s], c1 = S.sn_c0[(size_t)s + 1], k = c1 - c0;
            for (int64_t t = S.sn_rows_ptr[(size_t)s]; t < S.sn_rows_ptr[(size_t)s + 1]; ++t) {
                lidx[(size_t)S.sn_rows[(size_t)t]] = k + (int32_t)(t - S.sn_rows_ptr[(size_t)s]);
                lst[(size_t)S.sn_rows[(size_t)t]] = s;
            }
            om_ptr[(size_t)s] = (int64_t)o;
            for (int32_t cpos = c0; cpos < c1; ++cpos)
                for (int64_t e = colptr[(size_t)cpos]; e < colptr[(size_t)cpos + 1]; ++e) {
                    const CholHost::Blk& b = ent[(size_t)e];
                    int32_t a;
                    if (b.row < c1) a = b.row - c0;
                    else if (lst[(size_t)b.row] == s) a = lidx[(size_t)b.row];
                    else return DPG_ERR_NUMERIC;   // the block is outside its front: bad analysis
                    omap[o++] = OEnt{b.u, (int16_t)a, (int16_t)(cpos - c0), b.tr, 0};
                }
        }
        om_ptr[(size_t)S.ns] = (int64_t)o;
    }
#ifdef DPG_PLAN_VERIFY
    {   // the straightforward construction (binary search per block, per-front sort) must agree
        std::vector<OEnt> ref;
        for (int32_t s = 0; s < S.ns; ++s) {
            const int32_t c0 = S.sn_c0[(size_t)s], k = S.sn_c0[(size_t)s + 1] - c0;
            auto li = [&](int32_t p) -> int32_t {
                if (p >= c0 && p < c0 + k) return p - c0;
                const int32_t* b = S.sn_rows.data() + S.sn_rows_ptr[(size_t)s];
                const int32_t* e = S.sn_rows.data() + S.sn_rows_ptr[(size_t)s + 1];
                const int32_t* it = std::lower_bound(b, e, p);
                return (it == e || *it != p) ? -1 : k + (int32_t)(it - b);
            };
            const size_t r0 = ref.size();
            for (int64_t v = 0; v < n; ++v)
                if (S.sn_of[(size_t)S.pos[(size_t)v]] == s) {
                    const int32_t l = li(S.pos[(size_t)v]);
                    ref.push_back(OEnt{(int32_t)v, (int16_t)l, (int16_t)l, 0, 0});
                }
            for (int64_t q = 0; q < n_pairs; ++q) {
                const int32_t plo = S.pos[(size_t)pair_lo[q]], phi = S.pos[(size_t)pair_hi[q]];
                if (S.sn_of[(size_t)std::min(plo, phi)] != s) continue;
                ref.push_back(OEnt{(int32_t)(n + q), (int16_t)li(std::max(plo, phi)), (int16_t)li(std::min(plo, phi)),
                                   plo > phi ? 0 : 1, 0});
            }
            std::sort(ref.begin() + r0, ref.end(), [](const OEnt& x, const OEnt& y) { return x.b != y.b ? x.b < y.b : x.a < y.a; });
            if ((int64_t)r0 != om_ptr[(size_t)s]) { fprintf(stderr, "omap ptr mismatch at front %d\n", s); abort(); }
        }
        for (size_t i = 0; i < ref.size(); ++i)
            if (ref[i].u != omap[i].u || ref[i].a != omap[i].a || ref[i].b != omap[i].b || ref[i].tr != omap[i].tr) {
                fprintf(stderr, "omap mismatch at %zu\n", i);
                abort();
            }
    }
#endif
    PLAN_T(2);
    std::vector<SnDev>& sns = H.sns;
    sns.resize((size_t)S.ns);
    int64_t& acc_total = H.acc_total;
    acc_total = 0;
    for (int32_t s = 0; s < S.ns; ++s) {
        SnDev& d = sns[(size_t)s];
        d.c0 = S.sn_c0[(size_t)s];
        d.k = S.sn_c0[(size_t)s + 1] - d.c0;
        d.r = (int32_t)(S.sn_rows_ptr[(size_t)s + 1] - S.sn_rows_ptr[(size_t)s]);
        d.nchild = (int32_t)(S.child_ptr[(size_t)s + 1] - S.child_ptr[(size_t)s]);
        d.front_off = S.front_off[(size_t)s];
        d.rows_off = S.sn_rows_ptr[(size_t)s];
        d.child_off = S.child_ptr[(size_t)s];
        d.omap_off = om_ptr[(size_t)s];
        d.omap_n = (int32_t)(om_ptr[(size_t)s + 1] - om_ptr[(size_t)s]);
        d.acc_off = acc_total;
        d.parent = S.sn_parent[(size_t)s];
        const int32_t m3 = 3 * (d.k + d.r);
        d.G = (m3 <= kSmall && d.nchild <= kMaxCh)
                  ? 1
                  : std::min(kGmax, (3 * d.k + kFNB - 1) / kFNB + (3 * d.r + kFNB - 1) / kFNB);
        d.need = 0;
        acc_total += 3 * d.r;
    }
    for (int32_t s = 0; s < S.ns; ++s)
        if (sns[(size_t)s].parent >= 0) sns[(size_t)sns[(size_t)s].parent].need += sns[(size_t)s].G;
    if (c->track) {
        c->cur_G.resize((size_t)S.ns);
        for (int32_t s = 0; s < S.ns; ++s) c->cur_G[(size_t)s] = sns[(size_t)s].G;
    }
    // L11^-1 of the fronts with at least solve_inv_cols pivot columns (and at most 64 kInvMaxQ = 192)
    H.inv_t.clear();
    c->linv_total = 0;
    c->lds_inv = 0;
    for (int32_t s = 0; s < S.ns; ++s) {
        SnDev& d = sns[(size_t)s];
        const int32_t k3 = 3 * d.k;
        d.inv = -1;
        if (c->opts.solve_inv_cols <= 0 || k3 < c->opts.solve_inv_cols || k3 > 64 * kInvMaxQ ||
            c->linv_total + (int64_t)k3 * k3 > INT32_MAX)
            continue;
        d.inv = (int32_t)c->linv_total;
        c->linv_total += (int64_t)k3 * k3;
        for (int32_t j0 = 0; j0 < k3; j0 += kInvCols) H.inv_t.push_back(make_int2(s, j0));
    }
    c->n_inv_tasks = (int64_t)H.inv_t.size();
    std::vector<SolveSeg>& segs = H.segs;
    segs.clear();
    for (int32_t s = 0; s < S.ns; ++s) {
        SnDev& d = sns[(size_t)s];
        d.seg_off = (int32_t)segs.size();
        const int32_t* rw = S.sn_rows.data() + d.rows_off;
        for (int32_t t = 0; t < d.r;) {
            const int32_t a = S.sn_of[(size_t)rw[t]];
            int32_t t1 = t + 1;
            while (t1 < d.r && S.sn_of[(size_t)rw[t1]] == a) ++t1;
            segs.push_back(SolveSeg{a, t, t1, 0});
            t = t1;
        }
        d.seg_n = (int32_t)segs.size() - d.seg_off;
    }
    // large fronts: per tile, the H blocks (omap range) and the children's column ranges
    PLAN_T(3);
    std::vector<FTask>& ftasks = H.ftasks;
    std::vector<FChild>& fchild = H.fchild;
    ftasks.clear();
    fchild.clear();
    for (int32_t s = 0; s < S.ns; ++s) {
        SnDev& d = sns[(size_t)s];
        d.ftask = (int32_t)ftasks.size();
        const int32_t k3 = 3 * d.k, m3 = 3 * (d.k + d.r);
        if (d.G == 1 && m3 <= kSmall && d.nchild <= kMaxCh) continue;
        const OEnt* ob = omap.data() + d.omap_off;
        std::vector<int32_t>& cuts = H.cuts;
        cuts.clear();
        for (int32_t c = 0; c < k3; c += kFNB) cuts.push_back(c);
        for (int32_t c = k3; c < m3; c += kFNB) cuts.push_back(c);
        cuts.push_back(m3);
        // the children's column ranges per tile, tile-major and child order within a tile: each
        // child visits only the tiles its rows reach (its rows map to increasing front rows, so
        // the tiles' boundaries fall at increasing j), counted, then placed
        const int32_t nt = (int32_t)cuts.size() - 1;
        std::vector<int32_t>& tcnt = H.tcnt;
        tcnt.assign((size_t)nt + 1, 0);
        const int64_t ch0 = S.child_ptr[(size_t)s], ch1 = S.child_ptr[(size_t)s + 1];
        // the tile holding front row c: [0, k3) in kFNB steps, then [k3, m3) in kFNB steps
        const int32_t nt_k = (k3 + kFNB - 1) / kFNB;
        auto tile_of = [&](int32_t c) { return c < k3 ? c / kFNB : nt_k + (c - k3) / kFNB; };
        for (int64_t ci = ch0; ci < ch1; ++ci) {
            const SnDev& cd = sns[(size_t)S.child_list[(size_t)ci]];
            if (cd.r == 0) continue;
            const int32_t* rm = S.relmap.data() + cd.rows_off;
            const int32_t ta = tile_of(3 * rm[0]), tb = tile_of(3 * rm[cd.r - 1] + 2);
            for (int32_t t = ta; t <= tb; ++t) tcnt[(size_t)t + 1]++;   // an upper bound: empty ranges drop below
        }
        const size_t base = fchild.size();
        for (int32_t t = 0; t < nt; ++t) tcnt[(size_t)t + 1] += tcnt[(size_t)t];
        fchild.resize(base + (size_t)tcnt[(size_t)nt]);
        std::vector<int32_t>& tfill = H.tfill;
        tfill.assign(tcnt.begin(), tcnt.end() - 1);
        std::vector<char>& used = H.tused;
        used.assign(fchild.size() - base, 0);
        for (int64_t ci = ch0; ci < ch1; ++ci) {
            const SnDev& cd = sns[(size_t)S.child_list[(size_t)ci]];
            if (cd.r == 0) continue;
            const int32_t* rm = S.relmap.data() + cd.rows_off;
            const int32_t ta = tile_of(3 * rm[0]), tb = tile_of(3 * rm[cd.r - 1] + 2);
            int32_t ja = first_at_or_after(rm, cd.r, cuts[(size_t)ta]);
            for (int32_t t = ta; t <= tb; ++t) {
                const int32_t jb = first_at_or_after(rm, cd.r, cuts[(size_t)t + 1]);
                const size_t at = (size_t)tfill[(size_t)t]++;
                if (jb > ja) {
                    fchild[base + at] = FChild{ja, jb, cd.k, cd.r, cd.front_off, cd.rows_off};
                    used[at] = 1;
                }
                ja = jb;
            }
        }
        // compact (a child whose rows skip a whole tile left an unused slot there)
        size_t w = base;
        for (int32_t t = 0; t < nt; ++t) {
            const int32_t c0 = cuts[(size_t)t], c1 = cuts[(size_t)t + 1];
            FTask ft{0, 0, (int32_t)w, 0};
            ft.om_b = (int32_t)d.omap_off + (int32_t)(std::lower_bound(ob, ob + d.omap_n, c0 / 3,
                          [](const OEnt& o, int32_t v) { return o.b < v; }) - ob);
            ft.om_e = (int32_t)d.omap_off + (int32_t)(std::upper_bound(ob, ob + d.omap_n, (c1 - 1) / 3,
                          [](int32_t v, const OEnt& o) { return v < o.b; }) - ob);
            for (int32_t a = tcnt[(size_t)t]; a < tcnt[(size_t)t + 1]; ++a)
                if (used[(size_t)a]) fchild[w++] = fchild[base + (size_t)a];
            ft.ch_cnt = (int32_t)w - ft.ch_off;
            ftasks.push_back(ft);
        }
        fchild.resize(w);
    }
    // fused tickets (front * 64 + team member) in critical-path order: a front's priority is its
    // estimated time plus its parent's priority (the longest remaining path to the root), so
    // sorting by descending priority is topological (children first) and starts the long chains
    // before the bulk of the leaves
#ifdef DPG_PLAN_VERIFY
    {   // the child column ranges by a linear scan must agree
        size_t fi = 0;
        for (int32_t s = 0; s < S.ns; ++s) {
            const SnDev& d = sns[(size_t)s];
            const int32_t k3 = 3 * d.k, m3 = 3 * (d.k + d.r);
            if (d.G == 1 && m3 <= kSmall && d.nchild <= kMaxCh) continue;
            std::vector<int32_t> cu;
            for (int32_t c = 0; c < k3; c += kFNB) cu.push_back(c);
            for (int32_t c = k3; c < m3; c += kFNB) cu.push_back(c);
            cu.push_back(m3);
            for (size_t t = 0; t + 1 < cu.size(); ++t)
                for (int64_t ci = S.child_ptr[(size_t)s]; ci < S.child_ptr[(size_t)s + 1]; ++ci) {
                    const SnDev& cd = sns[(size_t)S.child_list[(size_t)ci]];
                    const int32_t* rm = S.relmap.data() + cd.rows_off;
                    int32_t ja = 3 * cd.r, jb = 0;
                    for (int32_t j = 0; j < 3 * cd.r; ++j) {
                        const int32_t pj = 3 * rm[j / 3] + j % 3;
                        if (pj >= cu[t] && pj < cu[t + 1]) { ja = std::min(ja, j); jb = j + 1; }
                    }
                    if (jb > ja) {
                        if (fi >= fchild.size() || fchild[fi].ja != ja || fchild[fi].jb != jb) {
                            fprintf(stderr, "fchild mismatch at %zu\n", fi);
                            abort();
                        }
                        ++fi;
                    }
                }
        }
        if (fi != fchild.size()) { fprintf(stderr, "fchild count mismatch\n"); abort(); }
    }
#endif
    PLAN_T(4);
    std::vector<double>& prio = H.prio;
    prio.assign((size_t)S.ns, 0.0);
    for (int32_t s = S.ns - 1; s >= 0; --s) {
        const SnDev& d = sns[(size_t)s];
        const int32_t m3 = 3 * (d.k + d.r);
        // (us, fitted to tools/chol_bench_t's per-front log: a small front's time grows with its
        // columns -- ~0.9 us each for the in-LDS factorization -- as well as its rows)
        const double est = d.G == 1 ? 4.0 + 0.06 * m3 + 0.9 * (3 * d.k) : 10.0 + 20.0 * ((3 * d.k + kFNB - 1) / kFNB);
        prio[(size_t)s] = est + (d.parent >= 0 ? prio[(size_t)d.parent] : 0.0);
    }
    // (descending priority, ties in level-list order)
    std::vector<std::pair<double, int32_t>>& key = H.key;
    key.resize((size_t)S.ns);
    for (int32_t i = 0; i < S.ns; ++i) key[(size_t)i] = {-prio[(size_t)S.level_list[(size_t)i]], i};
    std::sort(key.begin(), key.end());
    std::vector<int32_t>& fo = H.fo;
    fo.resize((size_t)S.ns);
    for (int32_t i = 0; i < S.ns; ++i) fo[(size_t)i] = S.level_list[(size_t)key[(size_t)i].second];
#ifdef DPG_PLAN_VERIFY
    {
        std::vector<int32_t> ref(S.level_list.begin(), S.level_list.end());
        std::stable_sort(ref.begin(), ref.end(), [&](int32_t a, int32_t b) { return prio[(size_t)a] > prio[(size_t)b]; });
        if (ref != fo) { fprintf(stderr, "front order mismatch\n"); abort(); }
    }
#endif
    std::vector<int32_t>& order_fac = H.order_fac;
    order_fac.clear();
    for (int32_t s : fo)
        for (int32_t m = 0; m < sns[(size_t)s].G; ++m) order_fac.push_back(s * 64 + m);
    c->n_tickets = (int64_t)order_fac.size();
    PLAN_T(5);
    c->level_ptr = S.level_ptr;
    // assembly tiles of front s, `ct` columns each: the omap range and the children (with their
    // contiguous column range) that land in the tile
    auto build_tiles = [&](int32_t s, int32_t ct, std::vector<AsmTask>& tl, std::vector<AsmChild>& cl) {
        const SnDev& d = sns[(size_t)s];
        const int32_t m3 = 3 * (d.k + d.r);
        const OEnt* ob = omap.data() + d.omap_off;
        for (int32_t c0 = 0; c0 < m3; c0 += ct) {
            const int32_t c1 = std::min(c0 + ct, m3);
            AsmTask t{s, c0, 0, 0, (int32_t)cl.size(), 0};
            // omap entries with block column in [c0 / 3, (c1 - 1) / 3]
            t.om_b = (int32_t)d.omap_off + (int32_t)(std::lower_bound(ob, ob + d.omap_n, c0 / 3,
                         [](const OEnt& o, int32_t v) { return o.b < v; }) - ob);
            t.om_e = (int32_t)d.omap_off + (int32_t)(std::upper_bound(ob, ob + d.omap_n, (c1 - 1) / 3,
                         [](int32_t v, const OEnt& o) { return v < o.b; }) - ob);
            for (int64_t ci = S.child_ptr[(size_t)s]; ci < S.child_ptr[(size_t)s + 1]; ++ci) {
                const int32_t ch = S.child_list[(size_t)ci];
                const SnDev& cd = sns[(size_t)ch];
                const int32_t ja = first_at_or_after(S.relmap.data() + cd.rows_off, cd.r, c0);
                const int32_t jb = first_at_or_after(S.relmap.data() + cd.rows_off, cd.r, c1);
                if (jb > ja) cl.push_back(AsmChild{ch, ja, jb, 0});
            }
            t.ch_cnt = (int32_t)cl.size() - t.ch_off;
            tl.push_back(t);
        }
    };
    // fused path: LDS budget of the largest front
    for (int32_t s = 0; s < S.ns; ++s) {
        const SnDev& d = sns[(size_t)s];
        c->lds_fused = std::max(c->lds_fused, 8 * fused_lds_doubles(3 * (d.k + d.r), 3 * d.k, true));
    }
    // two panel buffers for the chain when every front fits, else one (the chain step goes through HBM)
    c->fused_db = c->lds_fused <= 160 * 1024;
    if (!c->fused_db) {
        c->lds_fused = 0;
        for (int32_t s = 0; s < S.ns; ++s) {
            const SnDev& d = sns[(size_t)s];
            c->lds_fused = std::max(c->lds_fused, 8 * fused_lds_doubles(3 * (d.k + d.r), 3 * d.k, false));
        }
    }
    c->fused = c->lds_fused <= 160 * 1024 && c->opts.fused;
    // LDS of the DAG solves: the largest front
    // the solves' LDS: diagonal block D + staging region R + reciprocals + right-hand side / gathered
    // x + row positions.  Their VGPR budget (the 64-step chains) already holds them to two
    // workgroups per CU, so R defaults to what fills 80 KB; opts.solve_stage overrides it (doubles,
    // 0 = no staging)
    size_t lds_rest = 0;
    for (int32_t s = 0; s < S.ns; ++s) {
        const int32_t m3 = 3 * (sns[(size_t)s].k + sns[(size_t)s].r);
        lds_rest = std::max(lds_rest, (size_t)(kSB * kDL + kSB + m3 + 2 + m3 / 6 + 2 + 2 * kMaxSeg) * sizeof(double));
    }
    {
        const long room = (long)(80 * 1024) - (long)lds_rest;
        const long want = c->opts.solve_stage >= 0 ? (long)c->opts.solve_stage : room / (long)sizeof(double);
        const long cap = ((long)(160 * 1024) - (long)lds_rest) / (long)sizeof(double);
        c->solve_stage = (int32_t)std::max<long>(0, std::min<long>(want, cap)) & ~1;
        // tests: 0 = every front takes the parent path
        c->solve_maxseg = c->opts.solve_maxseg >= 0 ? std::min(c->opts.solve_maxseg, kMaxSeg) : kMaxSeg;
    }
    c->lds_solve_max = (size_t)c->solve_stage * sizeof(double) + lds_rest;
    if (c->lds_solve_max > 160 * 1024) return DPG_ERR_SIZE;
    std::vector<AsmTask>& asm_t = H.asm_t;
    std::vector<AsmChild>& asm_c = H.asm_c;
    std::vector<int2>& panel_t = H.panel_t;
    std::vector<int4>& upd_t = H.upd_t;
    asm_t.clear();
    asm_c.clear();
    panel_t.clear();
    upd_t.clear();
    c->plan.clear();
    if (!c->fused) {
        // level-synchronous path: per level, assembly tiles, then panel + update steps
        c->plan.assign((size_t)S.n_levels, CholDev::Level{});
        for (int32_t l = 0; l < S.n_levels; ++l) {
            int32_t maxk3 = 0;
            CholDev::Level& L = c->plan[(size_t)l];
            L.asm_off = (int32_t)asm_t.size();
            L.lds_asm = 0;
            for (int32_t q = S.level_ptr[(size_t)l]; q < S.level_ptr[(size_t)l + 1]; ++q) {
                const int32_t s = S.level_list[(size_t)q];
                const SnDev& d = sns[(size_t)s];
                const int32_t m3 = 3 * (d.k + d.r);
                L.lds_asm = std::max(L.lds_asm, (size_t)kCT * m3 * sizeof(double));
                maxk3 = std::max(maxk3, 3 * d.k);
                build_tiles(s, kCT, asm_t, asm_c);
            }
            L.asm_cnt = (int32_t)asm_t.size() - L.asm_off;
            c->n_launches += 1;
            for (int32_t j0 = 0; j0 < maxk3; j0 += kNB) {
                CholDev::Step st{(int32_t)panel_t.size(), 0, 1, 0, (int32_t)upd_t.size(), 0};
                int32_t maxR = 0;
                for (int32_t q = S.level_ptr[(size_t)l]; q < S.level_ptr[(size_t)l + 1]; ++q) {
                    const int32_t s = S.level_list[(size_t)q];
                    const SnDev& d = sns[(size_t)s];
                    const int32_t m3 = 3 * (d.k + d.r), k3 = 3 * d.k;
                    if (k3 <= j0) continue;
                    panel_t.push_back(make_int2(s, j0));
                    maxR = std::max(maxR, m3 - j0);
                    const int32_t base = j0 + std::min(kNB, k3 - j0), nt = (m3 - base + kUT - 1) / kUT;
                    for (int32_t ti = 0; ti < nt; ++ti)
                        for (int32_t tl = 0; tl <= ti; ++tl) upd_t.push_back(make_int4(s, j0, base + kUT * ti, base + kUT * tl));
                }
                st.panel_cnt = (int32_t)panel_t.size() - st.panel_off;
                st.upd_cnt = (int32_t)upd_t.size() - st.upd_off;
                st.max_rows = maxR;
                st.rpt = maxR <= kT ? 1 : maxR <= 2 * kT ? 2 : maxR <= 4 * kT ? 4 : 0;
                if (st.rpt == 0) return DPG_ERR_SIZE;
                L.steps.push_back(st);
                c->n_launches += 1 + (st.upd_cnt > 0);
            }
            if (L.lds_asm > 160 * 1024) return DPG_ERR_SIZE;
        }
    }
    // solves: the forward solve runs in the factorization's critical-path order (children first);
    // the backward solve by descending height -- the estimated time of the longest path from a
    // front DOWN to a leaf, which exceeds every child's, so the order is topological (parents
    // first) and the deepest chain is claimed first (the reverse of the forward order claimed the
    // fronts near the root first, whatever hangs below them: a chain front could be claimed
    // microseconds after its parent finished)
    PLAN_T(6);
    {
        std::vector<double>& hgt = H.hgt;
        hgt.assign((size_t)S.ns, 0.0);
        for (int32_t s = 0; s < S.ns; ++s) {   // children precede parents in supernode order
            const SnDev& d = sns[(size_t)s];
            hgt[(size_t)s] += 2.0 + 0.01 * (3 * (d.k + d.r)) + 0.05 * (3 * d.k);   // us, tools/chol_bench_t
            if (d.parent >= 0) hgt[(size_t)d.parent] = std::max(hgt[(size_t)d.parent], hgt[(size_t)s]);
        }
        // counting sort by height in 0.25 us buckets, descending; inside a bucket by descending
        // supernode index, so a parent (higher index, greater height) still precedes its children
        std::vector<int32_t>& cnt = H.hcnt;
        double hmax = 0.0;
        for (int32_t s = 0; s < S.ns; ++s) hmax = std::max(hmax, hgt[(size_t)s]);
        const int32_t nb = (int32_t)(hmax * 4.0) + 2;
        cnt.assign((size_t)nb + 1, 0);
        for (int32_t s = 0; s < S.ns; ++s) ++cnt[(size_t)(nb - 1 - (int32_t)(hgt[(size_t)s] * 4.0)) + 1];
        for (int32_t b = 0; b < nb; ++b) cnt[(size_t)b + 1] += cnt[(size_t)b];
        H.bwd.resize((size_t)S.ns);
        for (int32_t s = S.ns - 1; s >= 0; --s)
            H.bwd[(size_t)cnt[(size_t)(nb - 1 - (int32_t)(hgt[(size_t)s] * 4.0))]++] = s;
    }
    // [ticket | children-done counters [ns] | panel flags [ns] | backward: ticket | done [ns] |
    //  pivot-tile hand-off flags [per large-front tile]]
    c->sync_bytes = ((size_t)(2 + 3 * S.ns + ftasks.size()) * sizeof(int32_t) + 15) & ~size_t(15);
    H.dblocks.clear();
    for (int32_t s = 0; s < S.ns; ++s)
        for (int32_t jb = 0; jb < 3 * sns[(size_t)s].k; jb += kSB) H.dblocks.push_back(make_int2(s, jb));
    c->n_dblocks = (int64_t)H.dblocks.size();
    // measured (tools/r3_gn_job.sh, profiles/r03): the inversion launch (~55 us at config 4) costs
    // more than the chains it removes from the solves (re-solve 0.250 -> 0.241 ms), so the chains
    // stay the default; opts.solve_dinv selects the inverted blocks
    c->use_dinv = c->opts.solve_dinv != 0;
    PLAN_T(7);
    return DPG_OK;
}

// The structure arrays are packed into one pinned staging buffer and go up in ONE asynchronous
// copy into one device arena (the pointers of c point into it); one synchronisation at the end.
int chol_upload(CholDev* c, int64_t n, const CholHost& H) {
    const dpg_chol_sym& S = c->sym;
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    struct Piece { void** d; const void* h; size_t bytes; };
    Piece pieces[24];
    int np = 0;
    auto add = [&](auto** d, const auto& h) {
        using T = typename std::remove_reference<decltype(h)>::type::value_type;
        pieces[np++] = Piece{reinterpret_cast<void**>(d), h.data(), h.size() * sizeof(T)};
    };
    add(&c->sns, H.sns);
    add(&c->omap, H.omap);
    add(&c->child_list, S.child_list);
    add(&c->relmap, S.relmap);
    add(&c->rows, S.sn_rows);
    add(&c->perm, S.perm);
    add(&c->pos, S.pos);
    add(&c->order_fwd, H.fo);
    add(&c->order_fac, H.order_fac);
    add(&c->ftasks, H.ftasks);
    add(&c->fchild, H.fchild);
    add(&c->order_bwd, H.bwd);
    add(&c->segs, H.segs);
    add(&c->dblocks, H.dblocks);
    add(&c->inv_tasks, H.inv_t);
    if (!c->fused) {
        add(&c->asm_tasks, H.asm_t);
        add(&c->asm_child, H.asm_c);
        add(&c->panel_tasks, H.panel_t);
        add(&c->upd_tasks, H.upd_t);
    }
    size_t total = 0;
    for (int i = 0; i < np; ++i) total += al(std::max<size_t>(pieces[i].bytes, 1));
    if (total > c->c_stage) {
        if (c->stage) (void)hipHostFree(c->stage);
        c->stage = nullptr;
        const size_t want = std::max(total, c->c_stage + c->c_stage / 2);
        c->c_stage = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&c->stage), want) != hipSuccess) return DPG_ERR_HIP;
        c->c_stage = want;
    }
    if (total > c->c_arena) {
        if (c->arena) (void)hipFree(c->arena);
        c->arena = nullptr;
        const size_t want = std::max(total, c->c_arena + c->c_arena / 2);
        c->c_arena = 0;
        if (hipMalloc(reinterpret_cast<void**>(&c->arena), want) != hipSuccess) return DPG_ERR_HIP;
        c->c_arena = want;
    }
    size_t off = 0;
    for (int i = 0; i < np; ++i) {
        if (pieces[i].bytes) memcpy(c->stage + off, pieces[i].h, pieces[i].bytes);
        *pieces[i].d = c->arena + off;
        off += al(std::max<size_t>(pieces[i].bytes, 1));
    }
    int rc = hipMemcpyAsync(c->arena, c->stage, total, hipMemcpyHostToDevice, nullptr) != hipSuccess;
    // a re-allocated front, y or pending-update buffer has lost the tracked factorization (a new
    // allocation may come back at the old address: the capacities tell)
    const size_t cap0[3] = {c->c_fronts, c->c_acc, c->c_ysol};
    rc |= dreserve(&c->sync, &c->c_sync, c->sync_bytes / sizeof(int32_t));
    rc |= dreserve(&c->fronts, &c->c_fronts, (size_t)S.front_off[(size_t)S.ns]);
    rc |= dreserve(&c->acc, &c->c_acc, (size_t)H.acc_total);
    rc |= dreserve(&c->ysol, &c->c_ysol, (size_t)(3 * n));
    if (rc || cap0[0] != c->c_fronts || cap0[1] != c->c_acc || cap0[2] != c->c_ysol) c->fac_valid = false;
    rc |= dreserve(&c->xsol, &c->c_xsol, (size_t)(3 * n));
    rc |= dreserve(&c->status, &c->c_status, 1);
    rc |= dreserve(&c->dinv, &c->c_dinv, (size_t)(3 * n) * kSB);
    rc |= dreserve(&c->linv, &c->c_linv, (size_t)std::max<int64_t>(c->linv_total, 1));
    if (!rc) rc |= hipMemsetAsync(c->status, 0, sizeof(int32_t), nullptr) != hipSuccess;
    // the staging buffer is reused by the next build: wait for the copy (always, even after an error)
    rc |= hipStreamSynchronize(nullptr) != hipSuccess;
    return rc ? DPG_ERR_HIP : DPG_OK;
}

// the host structures of c's build in progress (a plan and its upload may be split:
// dpg_chol_create_sym_plan / _upload, possibly on two threads one after the other)
CholHost& build_host(CholDev* c) {
    if (!c->host) c->host = new CholHost();
    return *static_cast<CholHost*>(c->host);
}
void free_host(void* p) { delete static_cast<CholHost*>(p); }
int chol_build_plan(CholDev* c, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs) {
    const double t_b0 = wall_ms();
    const int rc = chol_plan(c, n, pair_lo, pair_hi, n_pairs, build_host(c));
    c->t_build[0] = wall_ms() - t_b0;
    return rc;
}
int chol_build_upload(CholDev* c) {
    const double t_b1 = wall_ms();
    const int rc = chol_upload(c, c->n, build_host(c));
    c->t_build[1] = wall_ms() - t_b1;
    return rc;
}
int chol_build(CholDev* c, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs) {
    const int rc = chol_build_plan(c, n, pair_lo, pair_hi, n_pairs);
    return rc ? rc : chol_build_upload(c);
}
}  // namespace

// dpg_chol_create_sym in two halves: the plan (host only: no device call, so it may run while the
// caller's stream still works, on any thread) and the upload of what it planned (nothing between)
int dpg_chol_create_sym_plan(void** h, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                             dpg_chol_sym* S, const dpg_chol_opts* opts) {
    CholDev* c = *h ? reinterpret_cast<CholDev*>(*h) : new CholDev();
    if (opts) c->opts = *opts;
    take_sym(c, S);
    const int rc = chol_build_plan(c, n, pair_lo, pair_hi, n_pairs);
    if (rc) { dpg_chol_destroy(c); *h = nullptr; return rc; }
    *h = c;
    return DPG_OK;
}
// chol_plan's first part ahead of the plan (pos / perm: the ordering the plan's analysis will
// carry); creates the solver object when *h is NULL.  Host only; not concurrently with a plan or an
// upload of the same object.
int dpg_chol_plan_blocks(void** h, int64_t n, const int32_t* pos, const int32_t* perm, const int32_t* pair_lo,
                         const int32_t* pair_hi, int64_t n_pairs) {
    if (!h || n <= 0 || !pos || !perm || n_pairs < 0 || (n_pairs > 0 && (!pair_lo || !pair_hi))) return DPG_ERR_ARG;
    CholDev* c = *h ? reinterpret_cast<CholDev*>(*h) : new CholDev();
    *h = c;
    CholHost& H = build_host(c);
    H.blocks_ready = false;
    plan_blocks(H, n, pos, perm, pair_lo, pair_hi, n_pairs);
    H.blocks_ready = true;
    return DPG_OK;
}
// drop prebuilt H-block buckets (their ordering was not the one the next plan will carry: the
// derivation they were built beside failed)
void dpg_chol_blocks_invalidate(void* h) {
    if (h) build_host(reinterpret_cast<CholDev*>(h)).blocks_ready = false;
}
int dpg_chol_create_sym_upload(void** h) {
    CholDev* c = reinterpret_cast<CholDev*>(*h);
    if (!c) return DPG_ERR_STATE;
    const int rc = chol_build_upload(c);
    if (rc) { dpg_chol_destroy(c); *h = nullptr; }
    return rc;
}

#ifdef DPG_PLAN_TIMING
double dpg_plan_t_export[8];
#endif
// host half of a build alone (no device calls), for CPU timing of the incremental rebuild
int dpg_chol_plan_host(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                       const dpg_chol_sym* S, double* ms) {
    thread_local CholHost H;
    thread_local CholDev c;
    c.sym = *S;
    const double t0 = wall_ms();
    const int rc = chol_plan(&c, n, pair_lo, pair_hi, n_pairs, H);
    if (ms) *ms = wall_ms() - t0;
#ifdef DPG_PLAN_TIMING
    for (int k = 0; k < 8; ++k) dpg_plan_t_export[k] = g_plan_t[k];
#endif
    return rc;
}

int dpg_chol_fused(void* h) { return h && reinterpret_cast<const CholDev*>(h)->fused ? 1 : 0; }

void dpg_chol_build_times(void* h, double out[2]) {
    const CholDev* c = reinterpret_cast<const CholDev*>(h);
    out[0] = c ? c->t_build[0] : 0.0;
    out[1] = c ? c->t_build[1] : 0.0;
}

// L11^-1 of the large fronts from the fronts just factored (gate: the pipelined loop's, refactoring
// iterations only)
static void launch_inv(CholDev* c, hipStream_t st, const int32_t* gate) {
    if (c->n_inv_tasks > 0)
        hipLaunchKernelGGL(chol_inv_l11, dim3((unsigned)c->n_inv_tasks), dim3(kInvThreads), c->lds_inv, st, c->inv_tasks, c->sns,
                           c->fronts, c->linv, gate);
}

// the values in fronts now belong to the current analysis
static void note_factored(CholDev* c, int64_t refactored, int64_t kept, int64_t moved, int64_t pick_ns = 0) {
    c->pstats[0] = refactored;
    c->pstats[1] = kept;
    c->pstats[2] = moved;
    c->pstats[3] = pick_ns;
    if (!c->track) return;
    c->fac_valid = true;
    c->fac_ptr = c->fronts;
    c->fac_ysol = c->ysol;
    c->fac_acc = c->acc;
    c->sym_is_fac = true;
    c->fac_db = c->fused_db;
}

extern "C" int dpg_chol_solve(void* h, const double* hb, void* stream) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    note_factored(c, c->sym.ns, 0, 0);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dpg_chol_sym& S = c->sym;
    const double* g = hb + 9 * c->nnzb_upper;
    if (hipMemsetAsync(c->status, 0, sizeof(int32_t), st) != hipSuccess) return DPG_ERR_HIP;
    if (c->fused) {
        if (hipMemsetAsync(c->sync, 0, c->sync_bytes, st) != hipSuccess) return DPG_ERR_HIP;
        hipLaunchKernelGGL(chol_factor_dag, dim3((unsigned)c->n_tickets), dim3(kFT), c->lds_fused, st, c->order_fac,
                           c->sync, c->status, c->sns, c->omap, c->relmap, c->child_list, c->ftasks, c->fchild, hb, g,
                           c->perm, c->fronts,
                           c->ysol, c->acc, S.ns, c->fused_db ? 1 : 0, nullptr, nullptr);
        if (c->use_dinv && c->n_dblocks > 0)
            hipLaunchKernelGGL(chol_inv_diag, dim3((unsigned)c->n_dblocks), dim3(64), 0, st, c->dblocks, c->sns, c->fronts, c->dinv);
        hipLaunchKernelGGL(chol_backward_dag, dim3(S.ns), dim3(kT), c->lds_solve_max, st, c->order_bwd,
                           c->sync + 1 + 2 * S.ns, c->status, c->sns, c->rows, c->segs, c->fronts, c->ysol, c->xsol, c->solve_stage, c->solve_maxseg,
                           c->use_dinv ? c->dinv : nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
        // the inverse after the backward (which, as a refactoring iteration of the gated loop, chains):
        // the chord steps of dpg_chol_resolve then do the same arithmetic as the gated loop's
        c->inv_valid = c->keep_inv && c->n_inv_tasks > 0;
        if (c->inv_valid) launch_inv(c, st, nullptr);
        return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
    }
    int pid = 0;
    for (int32_t l = 0; l < S.n_levels; ++l) {
        const CholDev::Level& L = c->plan[(size_t)l];
        hipLaunchKernelGGL(chol_assemble, dim3(L.asm_cnt), dim3(kT), L.lds_asm, st, c->asm_tasks + L.asm_off,
                           c->asm_child, c->sns, c->omap, hb, c->relmap, c->fronts, pid++);
        for (const CholDev::Step& p : L.steps) {
            const int2* pt = c->panel_tasks + p.panel_off;
            if (p.rpt == 1) hipLaunchKernelGGL(chol_panel<kT>, dim3(p.panel_cnt), dim3(kT), 0, st, pt, c->sns, c->fronts, c->status, pid++);
            else if (p.rpt == 2) hipLaunchKernelGGL(chol_panel<2 * kT>, dim3(p.panel_cnt), dim3(2 * kT), 0, st, pt, c->sns, c->fronts, c->status, pid++);
            else hipLaunchKernelGGL(chol_panel<4 * kT>, dim3(p.panel_cnt), dim3(4 * kT), 0, st, pt, c->sns, c->fronts, c->status, pid++);
            if (p.upd_cnt > 0)
                hipLaunchKernelGGL(chol_update, dim3(p.upd_cnt), dim3(kT), 0, st, c->upd_tasks + p.upd_off, c->sns, c->fronts, pid++);
        }
    }
    if (hipMemsetAsync(c->sync, 0, c->sync_bytes, st) != hipSuccess) return DPG_ERR_HIP;
    int32_t* sync_f = c->sync;
    int32_t* sync_b = c->sync + 1 + S.ns;
    if (c->use_dinv && c->n_dblocks > 0)
        hipLaunchKernelGGL(chol_inv_diag, dim3((unsigned)c->n_dblocks), dim3(64), 0, st, c->dblocks, c->sns, c->fronts, c->dinv);
    const double* di = c->use_dinv ? c->dinv : nullptr;
    hipLaunchKernelGGL(chol_forward_dag, dim3(S.ns), dim3(kT), c->lds_solve_max, st, c->order_fwd, sync_f, c->status,
                       c->sns, c->child_list, c->relmap, c->fronts, g, c->perm, c->ysol, c->acc, c->solve_stage, di, nullptr,
                       nullptr);
    hipLaunchKernelGGL(chol_backward_dag, dim3(S.ns), dim3(kT), c->lds_solve_max, st, c->order_bwd, sync_b, c->status,
                       c->sns, c->rows, c->segs, c->fronts, c->ysol, c->xsol, c->solve_stage, c->solve_maxseg, di, nullptr, nullptr,
                       nullptr, nullptr, nullptr);
    c->inv_valid = c->keep_inv && c->n_inv_tasks > 0;
    if (c->inv_valid) launch_inv(c, st, nullptr);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" void dpg_chol_track_factor(void* h, int on) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    if (!c || c->track == (on != 0)) return;
    c->track = on != 0;
    c->fac_valid = false;
    c->sym_is_fac = false;
    c->cur_G.clear();   // the current analysis was planned untracked: its team sizes are unknown
}
extern "C" void dpg_chol_forget_factor(void* h) {
    if (h) reinterpret_cast<CholDev*>(h)->fac_valid = false;
}
extern "C" void dpg_chol_partial_stats(void* h, int64_t out[4]) {
    const CholDev* c = reinterpret_cast<const CholDev*>(h);
    for (int k = 0; k < 4; ++k) out[k] = c ? c->pstats[k] : 0;
}

// ISAM2's partial re-elimination (isam_->update, dpg_slam.cc:320, re-eliminates only the cliques
// the new factors touch and their ancestors), as a multifrontal refactorization that keeps every
// front whose values cannot have changed since the tracked factorization:
//   * the same columns (same first column, same count: positions are stable between reorders, the
//     caller checks the order is unchanged -- here: the old order is a prefix of the new), the same
//     rows, the same children (by first column, in order: the extend-add order), the same team
//     size and panel buffering (the arithmetic order of the factorization kernel);
//   * no dirty node's column in it (its H blocks are then the same sums of the same factors at the
//     same linearization point: the caller's contract);
//   * no dirty front below it (its children's update matrices are unchanged).
// The forward solve folded into the factorization keeps its values too: a kept front's nodes have
// the same gradient (no new factor on them, same theta) and its children are kept, so its part of y
// (at its column positions: unchanged between reorders) and its pending row updates for the parent
// are what a full refactorization would compute again.  A kept front the new layout moved -- its
// values and its pending updates -- goes through the scratch buffer (gather, scatter), then the
// factorization runs with the kept fronts only signalling their parents, then the backward solve
// over every front.  The result is bit-identical to dpg_chol_solve's.
extern "C" int dpg_chol_solve_partial(void* h, const double* hb, const int32_t* dirty_nodes, int64_t n_dirty,
                                      void* stream) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    const dpg_chol_sym& S = c->sym;
    const dpg_chol_sym& O = c->fac_sym;
    const bool usable = c->track && c->fac_valid && !c->sym_is_fac && c->fac_ptr == c->fronts &&
                        c->fac_ysol == c->ysol && c->fac_acc == c->acc && c->fused &&
                        !(c->use_dinv && c->n_dblocks > 0) && c->fac_db == c->fused_db && O.ns > 0 && O.n <= S.n &&
                        (int64_t)c->fac_G.size() == (int64_t)O.ns && (int64_t)c->cur_G.size() == (int64_t)S.ns &&
                        std::equal(O.perm.begin(), O.perm.end(), S.perm.begin());
    if (!usable) return dpg_chol_solve(h, hb, stream);
    const double t_pick = wall_ms();
    const int32_t ns = S.ns;
    std::vector<uint8_t>& keep = c->h_keep;
    std::vector<int32_t>& old = c->h_old;
    keep.assign((size_t)ns, 1);
    old.assign((size_t)ns, -1);
    for (int64_t q = 0; q < n_dirty; ++q) {
        const int32_t v = dirty_nodes[q];
        if (v < 0 || v >= S.n) return dpg_chol_solve(h, hb, stream);
        keep[(size_t)S.sn_of[(size_t)S.pos[(size_t)v]]] = 0;
    }
    int64_t kept = 0;
    for (int32_t sn = 0; sn < ns; ++sn) {   // children before parents (a parent's first column is later)
        if (keep[(size_t)sn]) {
            const int32_t c0 = S.sn_c0[(size_t)sn], c1 = S.sn_c0[(size_t)sn + 1];
            bool same = c1 <= O.n;
            int32_t os = -1;
            if (same) {
                os = O.sn_of[(size_t)c0];
                same = O.sn_c0[(size_t)os] == c0 && O.sn_c0[(size_t)os + 1] == c1 && c->fac_G[(size_t)os] == c->cur_G[(size_t)sn];
            }
            if (same) {
                const int64_t r0 = S.sn_rows_ptr[(size_t)sn], r1 = S.sn_rows_ptr[(size_t)sn + 1];
                const int64_t q0 = O.sn_rows_ptr[(size_t)os], q1 = O.sn_rows_ptr[(size_t)os + 1];
                same = r1 - r0 == q1 - q0 && std::equal(S.sn_rows.begin() + r0, S.sn_rows.begin() + r1, O.sn_rows.begin() + q0);
            }
            if (same) {
                const int64_t a0 = S.child_ptr[(size_t)sn], a1 = S.child_ptr[(size_t)sn + 1];
                const int64_t b0 = O.child_ptr[(size_t)os], b1 = O.child_ptr[(size_t)os + 1];
                same = a1 - a0 == b1 - b0;
                for (int64_t t = 0; same && t < a1 - a0; ++t)
                    same = S.sn_c0[(size_t)S.child_list[(size_t)(a0 + t)]] == O.sn_c0[(size_t)O.child_list[(size_t)(b0 + t)]];
            }
            if (same) {
                old[(size_t)sn] = os;
                ++kept;
            } else {
                keep[(size_t)sn] = 0;
            }
        }
        if (!keep[(size_t)sn] && S.sn_parent[(size_t)sn] >= 0) keep[(size_t)S.sn_parent[(size_t)sn]] = 0;
    }
    if (kept == 0) return dpg_chol_solve(h, hb, stream);
    // runs of kept fronts the layout moved: gather {old, scratch}, scatter {scratch, new}; the
    // pending updates of front s sit at 3 sn_rows_ptr[s] (chol_plan's acc_off)
    std::vector<int64_t>& runs = c->h_runs;
    runs.clear();
    int64_t moved = 0, max_run = 0;
    auto add_run = [&](int64_t src, int64_t dst, int64_t len, int64_t buf) {
        if (src == dst || len == 0) return;
        const size_t nr = runs.size();
        if (nr >= 4 && runs[nr - 1] == buf && runs[nr - 4] + runs[nr - 2] == src && runs[nr - 3] + runs[nr - 2] == dst) {
            runs[nr - 2] += len;
        } else {
            runs.push_back(src);
            runs.push_back(dst);
            runs.push_back(len);
            runs.push_back(buf);
        }
        max_run = std::max(max_run, runs[runs.size() - 2]);
        moved += len;
    };
    for (int32_t sn = 0; sn < ns; ++sn)
        if (keep[(size_t)sn])
            add_run(O.front_off[(size_t)old[(size_t)sn]], S.front_off[(size_t)sn],
                    S.front_off[(size_t)sn + 1] - S.front_off[(size_t)sn], 0);
    for (int32_t sn = 0; sn < ns; ++sn)
        if (keep[(size_t)sn])
            add_run(3 * O.sn_rows_ptr[(size_t)old[(size_t)sn]], 3 * S.sn_rows_ptr[(size_t)sn],
                    3 * (S.sn_rows_ptr[(size_t)sn + 1] - S.sn_rows_ptr[(size_t)sn]), 1);
    const int64_t nruns = (int64_t)runs.size() / 4;
    if (nruns > 65535) return dpg_chol_solve(h, hb, stream);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // keep flags + gather runs + scatter runs: one pinned buffer, one copy up
    const size_t keep_bytes = ((size_t)ns + 15) & ~size_t(15);
    const size_t run_bytes = sizeof(int64_t) * 4 * (size_t)nruns;
    const size_t bytes = keep_bytes + 2 * run_bytes;
    if (c->pev_set && hipEventSynchronize(c->pev) != hipSuccess) return DPG_ERR_HIP;
    if (bytes > c->c_pstage) {
        if (c->pstage) (void)hipHostFree(c->pstage);
        c->pstage = nullptr;
        const size_t want = std::max(bytes, c->c_pstage + c->c_pstage / 2);
        c->c_pstage = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&c->pstage), want) != hipSuccess) return DPG_ERR_HIP;
        c->c_pstage = want;
    }
    if (dreserve(&c->dpart, &c->c_dpart, bytes) || (moved > 0 && dreserve(&c->scratch, &c->c_scratch, (size_t)moved)))
        return DPG_ERR_HIP;
    memcpy(c->pstage, keep.data(), (size_t)ns);
    int64_t* gat = reinterpret_cast<int64_t*>(c->pstage + keep_bytes);
    int64_t* sca = gat + 4 * nruns;
    for (int64_t r = 0, off = 0; r < nruns; ++r) {
        const int64_t* q = runs.data() + 4 * r;
        const int64_t g4[4] = {q[0], off, q[2], q[3]}, s4[4] = {off, q[1], q[2], q[3]};
        std::copy(g4, g4 + 4, gat + 4 * r);
        std::copy(s4, s4 + 4, sca + 4 * r);
        off += q[2];
    }
    if (!c->pev && hipEventCreateWithFlags(&c->pev, hipEventDisableTiming) != hipSuccess) return DPG_ERR_HIP;
    if (hipMemcpyAsync(c->dpart, c->pstage, bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(c->pev, st) != hipSuccess)
        return DPG_ERR_HIP;
    c->pev_set = true;
    const uint8_t* keep_dev = reinterpret_cast<const uint8_t*>(c->dpart);
    const int64_t* gat_dev = reinterpret_cast<const int64_t*>(c->dpart + keep_bytes);
    const int64_t* sca_dev = gat_dev + 4 * nruns;
    if (nruns > 0) {
        const unsigned gx = (unsigned)std::min<int64_t>(64, std::max<int64_t>(1, (max_run + 2047) / 2048));
        hipLaunchKernelGGL(chol_copy_runs, dim3(gx, (unsigned)nruns), dim3(256), 0, st, c->fronts, c->acc, c->scratch,
                           c->scratch, gat_dev);
        hipLaunchKernelGGL(chol_copy_runs, dim3(gx, (unsigned)nruns), dim3(256), 0, st, c->scratch, c->scratch, c->fronts,
                           c->acc, sca_dev);
    }
    const double* g = hb + 9 * c->nnzb_upper;
    if (hipMemsetAsync(c->status, 0, sizeof(int32_t), st) != hipSuccess ||
        hipMemsetAsync(c->sync, 0, c->sync_bytes, st) != hipSuccess)
        return DPG_ERR_HIP;
    hipLaunchKernelGGL(chol_factor_dag, dim3((unsigned)c->n_tickets), dim3(kFT), c->lds_fused, st, c->order_fac,
                       c->sync, c->status, c->sns, c->omap, c->relmap, c->child_list, c->ftasks, c->fchild, hb, g,
                       c->perm, c->fronts, c->ysol, c->acc, ns, c->fused_db ? 1 : 0, nullptr, keep_dev);
    hipLaunchKernelGGL(chol_backward_dag, dim3(ns), dim3(kT), c->lds_solve_max, st, c->order_bwd,
                       c->sync + 1 + 2 * ns, c->status, c->sns, c->rows, c->segs, c->fronts, c->ysol, c->xsol,
                       c->solve_stage, c->solve_maxseg, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
    note_factored(c, ns - kept, kept, moved, (int64_t)((wall_ms() - t_pick) * 1e6));
    c->inv_valid = false;
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

// forward + backward solves with the fronts of the last factorization (the right-hand side from hb)
extern "C" int dpg_chol_resolve(void* h, const double* hb, void* stream) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dpg_chol_sym& S = c->sym;
    const double* g = hb + 9 * c->nnzb_upper;
    if (hipMemsetAsync(c->sync, 0, c->sync_bytes, st) != hipSuccess) return DPG_ERR_HIP;
    const double* di = c->use_dinv ? c->dinv : nullptr;   // inverted by the factorization's dpg_chol_solve
    const double* li = c->inv_valid ? c->linv : nullptr;
    hipLaunchKernelGGL(chol_forward_dag, dim3(S.ns), dim3(kT), c->lds_solve_max, st, c->order_fwd, c->sync, c->status,
                       c->sns, c->child_list, c->relmap, c->fronts, g, c->perm, c->ysol, c->acc, c->solve_stage, di, nullptr,
                       li);
    hipLaunchKernelGGL(chol_backward_dag, dim3(S.ns), dim3(kT), c->lds_solve_max, st, c->order_bwd,
                       c->sync + 1 + 2 * S.ns, c->status, c->sns, c->rows, c->segs, c->fronts, c->ysol, c->xsol, c->solve_stage,
                       c->solve_maxseg, di, nullptr, nullptr, nullptr, nullptr, li);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

// one Gauss-Newton iteration's solve with the path chosen on the device (gate, see gate_off):
// the fused factorization + forward solve, or the forward solve with the last factor, then the
// backward solve.  Only the fused plan without inverted diagonal blocks (dpg_chol_gated_ok).
extern "C" int dpg_chol_gated_ok(void* h) {
    const CholDev* c = reinterpret_cast<const CholDev*>(h);
    return c && c->fused && !(c->use_dinv && c->n_dblocks > 0) ? 1 : 0;
}

extern "C" void dpg_chol_sync_dev(void* h, int32_t** sync, int64_t* n_words) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    *sync = c->sync;
    *n_words = (int64_t)(c->sync_bytes / sizeof(int32_t));
}

// prezeroed: the caller's previous launch cleared the status word and the sync counters
extern "C" int dpg_chol_solve_gated(void* h, const double* hb, const int32_t* gate, int prezeroed, double* X,
                                    double* max_out, void* stream) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    if (!dpg_chol_gated_ok(h)) return DPG_ERR_STATE;
    c->fac_valid = false;   // (a Gauss-Newton loop's refactorizations are not tracked)
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dpg_chol_sym& S = c->sym;
    const double* g = hb + 9 * c->nnzb_upper;
    if (!prezeroed && (hipMemsetAsync(c->status, 0, sizeof(int32_t), st) != hipSuccess ||
                       hipMemsetAsync(c->sync, 0, c->sync_bytes, st) != hipSuccess))
        return DPG_ERR_HIP;
    const bool inv = c->n_inv_tasks > 0;
    if (inv) {   // this iteration's solves come after the previous iteration's inverse
        if (!c->aux) {
            if (hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&c->ev_fac, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&c->ev_inv[0], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&c->ev_inv[1], hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(c->ev_inv[0], c->aux) != hipSuccess || hipEventRecord(c->ev_inv[1], c->aux) != hipSuccess)
                return DPG_ERR_HIP;
        }
        if (hipStreamWaitEvent(st, c->ev_inv[c->inv_par ^ 1], 0) != hipSuccess) return DPG_ERR_HIP;
    }
    hipLaunchKernelGGL(chol_factor_dag, dim3((unsigned)c->n_tickets), dim3(kFT), c->lds_fused, st, c->order_fac,
                       c->sync, c->status, c->sns, c->omap, c->relmap, c->child_list, c->ftasks, c->fchild, hb, g,
                       c->perm, c->fronts, c->ysol, c->acc, S.ns, c->fused_db ? 1 : 0, gate, nullptr);
    if (inv) {   // L11^-1 of a refactoring iteration beside its backward solve (which does not use it)
        if (hipEventRecord(c->ev_fac, st) != hipSuccess || hipStreamWaitEvent(c->aux, c->ev_fac, 0) != hipSuccess)
            return DPG_ERR_HIP;
        launch_inv(c, c->aux, gate);
        if (hipEventRecord(c->ev_inv[c->inv_par], c->aux) != hipSuccess) return DPG_ERR_HIP;
        c->inv_par ^= 1;
    }
    hipLaunchKernelGGL(chol_forward_dag, dim3(S.ns), dim3(kT), c->lds_solve_max, st, c->order_fwd, c->sync, c->status,
                       c->sns, c->child_list, c->relmap, c->fronts, g, c->perm, c->ysol, c->acc, c->solve_stage,
                       nullptr, gate, c->linv);
    hipLaunchKernelGGL(chol_backward_dag, dim3(S.ns), dim3(kT), c->lds_solve_max, st, c->order_bwd,
                       c->sync + 1 + 2 * S.ns, c->status, c->sns, c->rows, c->segs, c->fronts, c->ysol, c->xsol,
                       c->solve_stage, c->solve_maxseg, nullptr, gate, c->perm, X, max_out, c->linv);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

// a Gauss-Newton graph's solver keeps L11^-1 for its chord steps (the incremental graph refactors
// every update and does not)
extern "C" void dpg_chol_keep_inverse(void* h, int on) {
    if (h) reinterpret_cast<CholDev*>(h)->keep_inv = on != 0;
}

// the gated loop's control kernel rewrites the gate the inverse kernel reads: it must come after
// this iteration's inverse (normally long finished: it ran beside the backward solve and assembly)
extern "C" int dpg_chol_join_aux(void* h, void* stream) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    if (!c || !c->aux) return DPG_OK;
    return hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), c->ev_inv[c->inv_par ^ 1], 0) == hipSuccess ? DPG_OK
                                                                                                       : DPG_ERR_HIP;
}

extern "C" const int32_t* dpg_chol_pos_dev(void* h) { return reinterpret_cast<CholDev*>(h)->pos; }
extern "C" const double* dpg_chol_x_dev(void* h) { return reinterpret_cast<CholDev*>(h)->xsol; }
extern "C" const int32_t* dpg_chol_status_dev(void* h) { return reinterpret_cast<CholDev*>(h)->status; }
extern "C" void dpg_chol_stats(void* h, double out[6]) {
    const dpg_chol_sym& S = reinterpret_cast<CholDev*>(h)->sym;
    out[0] = S.ns;
    out[1] = S.n_levels;
    out[2] = S.max_front;
    out[3] = S.flops;
    out[4] = (double)S.front_off[(size_t)S.ns] * 8.0;
    out[5] = (double)S.n;
}

#ifdef DPG_CHOL_TIMING
extern "C" int dpg_chol_prof_dump(unsigned long long* out, int n, unsigned long long* span) {
    if (hipMemcpyFromSymbol(span, HIP_SYMBOL(g_span), sizeof(unsigned long long) * kProfL * kProfW * 2) != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * (size_t)n) == hipSuccess ? 0 : -1;
}
extern "C" int dpg_chol_steps_dump(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_steps), sizeof(unsigned long long) * 16 * 8 * (size_t)n) == hipSuccess ? 0 : -1;
}
extern "C" int dpg_chol_panel_dump(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_panel), sizeof(unsigned long long) * 16 * 8 * (size_t)n) == hipSuccess ? 0 : -1;
}
extern "C" int dpg_chol_bwd_dump(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd), sizeof(unsigned long long) * 8 * (size_t)n) == hipSuccess ? 0 : -1;
}
extern "C" int dpg_chol_front_dump(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_front), sizeof(unsigned long long) * 8 * (size_t)n) == hipSuccess ? 0 : -1;
}
extern "C" void dpg_chol_tree(void* h, int32_t* parent, int32_t* m3, int32_t* k3) {
    const dpg_chol_sym& S = reinterpret_cast<CholDev*>(h)->sym;
    for (int32_t s = 0; s < S.ns; ++s) {
        parent[s] = S.sn_parent[(size_t)s];
        k3[s] = 3 * (S.sn_c0[(size_t)s + 1] - S.sn_c0[(size_t)s]);
        m3[s] = k3[s] + 3 * (int32_t)(S.sn_rows_ptr[(size_t)s + 1] - S.sn_rows_ptr[(size_t)s]);
    }
}
extern "C" int dpg_chol_prof_reset(void) {
    std::vector<unsigned long long> sp((size_t)kProfL * kProfW * 2, 0ull);
    std::vector<unsigned long long> z((size_t)4096 * kProfSlots, 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z.data(), z.size() * 8) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_span), sp.data(), sp.size() * 8) == hipSuccess ? 0 : -1;
}
#endif
