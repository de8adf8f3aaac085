// dpg_gn.hip -- pose-graph Gauss-Newton on gfx950: per-factor linearization + block-sparse
// (H, b) assembly, block-Jacobi PCG in fp64, Pose2 retraction.
//
// Replaces DpgSLAM::optimizeGraph (src/dpg_slam/dpg_slam.cc:316-329) -> GTSAM
// ISAM2/GaussNewtonOptimizer over PriorFactor<Pose2> / BetweenFactor<Pose2> (dpg_slam.cc:44-75,
// 178-183,227-238,331-338), restated with GTSAM 4.x default semantics:
//   Between: h = Xi^-1 Xj, e = Local(z, h) = z^-1 h as (x, y, theta); Jacobians of
//            Pose2::between (H1 = -AdjointMap(h^-1) inlined, H2 = I) -- BetweenFactor without
//            SLOW_BUT_CORRECT_BETWEENFACTOR applies no Local() Jacobian;
//   Prior:   e = -Local(x, prior), H = I;
//   whitened normal equations  H = sum A^T W A,  g = sum A^T W e,  solve H d = -g,
//   retract X <- X * Pose2(d) (ChartAtOrigin, no Expmap).
//
// Assembly is a deterministic GATHER (no float atomics): one lane per upper 3x3 block walks the
// factors that touch it in factor order.  The packed buffer [H upper | g | chi2] is exactly what
// the multi-GPU path all-reduces (one RCCL call per GN iteration).
// The solve: block-Jacobi preconditioned CG over the full BSR (two kernels per CG iteration,
// deterministic fixed-order partial sums), then one retraction kernel.

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <future>
#include <vector>

#include "dpg_chol.h"
#include "dpg_internal.h"
#include "dpg_gn_pipe.h"

namespace {

constexpr int kRowThreads = 256;

__device__ __forceinline__ void between_lin(const double* a, const double* b, double h[4], double H1[9]) {
    const double c1 = cos(a[2]), s1 = sin(a[2]), c2 = cos(b[2]), s2 = sin(b[2]);
    const double c = c1 * c2 + s1 * s2, s = -s1 * c2 + c1 * s2;
    const double dx = b[0] - a[0], dy = b[1] - a[1];
    h[0] = c1 * dx + s1 * dy;
    h[1] = -s1 * dx + c1 * dy;
    h[2] = c;
    h[3] = s;
    if (H1) {
        const double dt1 = -s2 * dx + c2 * dy, dt2 = -c2 * dx - s2 * dy;
        H1[0] = -c; H1[1] = -s; H1[2] = dt1;
        H1[3] = s;  H1[4] = -c; H1[5] = dt2;
        H1[6] = 0;  H1[7] = 0;  H1[8] = -1;
    }
}

// error e and Jacobian A_i (A_j = I for Between, prior has only A_i = I)
__device__ void linearize(const dpg_factor& f, const double* X, double e[3], double Ai[9]) {
    double h[4];
    if (f.kind == DPG_FACTOR_PRIOR) {
        between_lin(X + 3 * f.i, f.z, h, nullptr);
        e[0] = -h[0];
        e[1] = -h[1];
        e[2] = -atan2(h[3], h[2]);
#pragma unroll
        for (int q = 0; q < 9; ++q) Ai[q] = (q % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    between_lin(X + 3 * f.i, X + 3 * f.j, h, Ai);
    const double cz = cos(f.z[2]), sz = sin(f.z[2]);
    double ch = h[2], sh = h[3];
    const double n = ch * ch + sh * sh;
    if (fabs(n - 1.0) > 1e-10) { const double sc = 1.0 / sqrt(n); ch *= sc; sh *= sc; }
    const double c = cz * ch + sz * sh, s = -sz * ch + cz * sh;
    const double dx = h[0] - f.z[0], dy = h[1] - f.z[1];
    e[0] = cz * dx + sz * dy;
    e[1] = -sz * dx + cz * dy;
    e[2] = atan2(s, c);
}

// C += A^T diag(w) B
__device__ __forceinline__ void atwb_acc(const double* A, const double* w, const double* B, double* C) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) acc += A[3 * k + r] * w[k] * B[3 * k + c];
            C[3 * r + c] += acc;
        }
}

// linearization by contribution-list entry: entry q of the upper blocks' lists (factor fi, role)
// contributes 13 doubles to its block -- role 0 (diag i): A_i^T W A_i, the g_i term, the chi2 term;
// role 1 (diag j, A_j = I): the diagonal of W, the g_j term; role 2 / 3 (the (i, j) / (j, i) block):
// A_i^T W.  A factor is linearized once per entry (at most three times).
constexpr int kRec = 13;
__device__ __forceinline__ void lin_record(const dpg_factor& f, const double* X, int role, double (&C)[kRec]) {
    double e[3], Ai[9];
    linearize(f, X, e, Ai);
    const double* w = f.info;
#pragma unroll
    for (int k = 0; k < kRec; ++k) C[k] = 0.0;
    if (role == 0) {
        atwb_acc(Ai, w, Ai, C);
#pragma unroll
        for (int r = 0; r < 3; ++r) C[9 + r] = Ai[r] * w[0] * e[0] + Ai[3 + r] * w[1] * e[1] + Ai[6 + r] * w[2] * e[2];
        C[12] = 0.5 * (w[0] * e[0] * e[0] + w[1] * e[1] * e[1] + w[2] * e[2] * e[2]);
    } else if (role == 1) {
#pragma unroll
        for (int r = 0; r < 3; ++r) { C[r] = w[r]; C[9 + r] = w[r] * e[r]; }
    } else {
        const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        atwb_acc(Ai, w, I3, C);
    }
}

// Linearization + assembly, ONE launch.  A 64-lane workgroup owns a run of upper blocks -- 4
// diagonal ones (~8.5 entries each at config 4's degree) or 32 off-diagonal ones (~1 each), so
// either way at most one list entry per lane (8 diagonal blocks per workgroup: two rounds of
// linearization on most lanes, 25 -> 14.5 us per launch at 4): the lanes linearize the run's entries into LDS (a
// record per entry, kLgChunk at a time), then lane b adds block b's records in list (= factor)
// order -- no float atomics, deterministic.  Round 4 ran this as two launches (a linearization
// kernel writing the records to HBM, a gather kernel reading them back); same records, same order.
constexpr int kLgLanes = 64, kLgDiag = 4, kLgOff = 32, kLgChunk = 128;
__host__ __device__ inline int64_t lg_groups(int64_t n_nodes, int64_t nnzb_upper) {
    return (n_nodes + kLgDiag - 1) / kLgDiag + (nnzb_upper - n_nodes + kLgOff - 1) / kLgOff;
}
__global__ __launch_bounds__(kLgLanes) void lin_gather_kernel(const dpg_factor* __restrict__ F, const double* __restrict__ X,
                                                              const int32_t* __restrict__ cptr, const int32_t* __restrict__ clist,
                                                              int64_t n_nodes, int64_t nnzb_upper, int64_t shard_begin,
                                                              int64_t shard_end, const uint8_t* __restrict__ mine,
                                                              double* __restrict__ hb, double* __restrict__ chi2_node,
                                                              const int32_t* gate) {
    __shared__ double rec[kLgChunk * kRec];
    __shared__ int32_t code_s[kLgChunk];
    if (gate && !gate[0]) return;
    const int64_t nd = (n_nodes + kLgDiag - 1) / kLgDiag, wg = blockIdx.x;
    const int64_t u0 = wg < nd ? wg * kLgDiag : n_nodes + (wg - nd) * kLgOff;
    const int64_t u1 = wg < nd ? min(u0 + kLgDiag, n_nodes) : min(u0 + kLgOff, nnzb_upper);
    const int lane = threadIdx.x;
    const int64_t u = u0 + lane;
    const bool own = u < u1;
    const int32_t q0 = cptr[u0], q1 = cptr[u1];
    const int32_t qa = own ? cptr[u] : 0, qb = own ? cptr[u + 1] : 0;
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    double g[3] = {0, 0, 0};
    double chi2 = 0.0;
    for (int32_t c0 = q0; c0 < q1; c0 += kLgChunk) {
        const int32_t c1 = min(c0 + kLgChunk, q1);
        for (int32_t q = c0 + lane; q < c1; q += kLgLanes) {
            const int32_t code = clist[q], fi = code >> 2;
            const bool skip = mine ? !mine[fi] : (fi < shard_begin || fi >= shard_end);   // another rank's factor
            code_s[q - c0] = skip ? -1 : code;
            if (skip) continue;
            double C[kRec];
            lin_record(F[fi], X, code & 3, C);
            double* o = rec + kRec * (q - c0);
#pragma unroll
            for (int k = 0; k < kRec; ++k) o[k] = C[k];
        }
        __syncthreads();
        if (own) {
            for (int32_t q = max(qa, c0); q < min(qb, c1); ++q) {
                const int32_t code = code_s[q - c0];
                if (code < 0) continue;
                const double* v = rec + kRec * (q - c0);
                const int role = code & 3;
                if (role == 0) {          // diag i
#pragma unroll
                    for (int k = 0; k < 9; ++k) H[k] += v[k];
#pragma unroll
                    for (int r = 0; r < 3; ++r) g[r] += v[9 + r];
                    chi2 += v[12];
                } else if (role == 1) {   // diag j (A_j = I): W
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int k = 0; k < 3; ++k) H[3 * r + k] += r == k ? v[r] : 0.0;
#pragma unroll
                    for (int r = 0; r < 3; ++r) g[r] += v[9 + r];
                } else if (role == 2) {   // H(i, j) = A_i^T W, i < j
#pragma unroll
                    for (int k = 0; k < 9; ++k) H[k] += v[k];
                } else {                  // H(j, i) = W A_i, j < i
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int k = 0; k < 3; ++k) H[3 * r + k] += v[3 * k + r];
                }
            }
        }
        __syncthreads();
    }
    if (!own) return;
    double* o = hb + 9 * u;
#pragma unroll
    for (int q = 0; q < 9; ++q) o[q] = H[q];
    if (u < n_nodes) {
        double* gb = hb + 9 * nnzb_upper + 3 * u;
        gb[0] = g[0]; gb[1] = g[1]; gb[2] = g[2];
        chi2_node[u] = chi2;
    }
}

__device__ double block_sum(double v, double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    __syncthreads();
    return s;
}

// this thread's terms k = t, t + stride, ... in ascending k, eight loads in flight (the adds in the
// order of the plain strided loop: the terms are >= 0, so the padding zeros change nothing)
__device__ __forceinline__ double strided_sum(const double* __restrict__ v, int64_t n, int64_t t, int64_t stride) {
    double s = 0.0;
    for (int64_t k0 = t; k0 < n; k0 += 8 * stride) {
        double x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = k0 + j * stride < n ? v[k0 + j * stride] : 0.0;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += x[j];
    }
    return s;
}

// vote != NULL (multi-device forms, world > 1): this device's max |delta| and solver status into
// its own vote words (dpg_gn_dev.n_vote), summed by the all-reduce with the other devices' zeros
__global__ void chi2_kernel(const double* __restrict__ chi2_node, int64_t n, double* __restrict__ out,
                            const int32_t* gate, double* __restrict__ vote, const double* __restrict__ dinf,
                            const int32_t* __restrict__ status, int32_t world, int32_t rank) {
    __shared__ double red[16];
    if (gate && !gate[0]) return;
    double s = strided_sum(chi2_node, n, threadIdx.x, blockDim.x);
    s = block_sum(s, red);
    if (threadIdx.x == 0) {
        *out = s;
        if (vote) {
            vote[rank] = *dinf;
            vote[world + rank] = status ? (double)*status : 0.0;   // the PCG solver has no status word
        }
    }
}

// inverse of an SPD 3x3 block (adjugate / determinant)
__device__ void inv3(const double* A, double* B) {
    const double a = A[0], b = A[1], c = A[2], d = A[3], e = A[4], f = A[5], g = A[6], h = A[7], i = A[8];
    const double C00 = e * i - f * h, C01 = -(d * i - f * g), C02 = d * h - e * g;
    const double det = a * C00 + b * C01 + c * C02;
    if (!(fabs(det) > 0.0)) {
        for (int q = 0; q < 9; ++q) B[q] = (q % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    const double id = 1.0 / det;
    B[0] = C00 * id; B[1] = -(b * i - c * h) * id; B[2] = (b * f - c * e) * id;
    B[3] = C01 * id; B[4] = (a * i - c * g) * id;  B[5] = -(a * f - c * d) * id;
    B[6] = C02 * id; B[7] = -(a * h - b * g) * id; B[8] = (a * e - b * d) * id;
}

__device__ __forceinline__ void mv3(const double* M, const double* x, double* y) {
    y[0] = M[0] * x[0] + M[1] * x[1] + M[2] * x[2];
    y[1] = M[3] * x[0] + M[4] * x[1] + M[5] * x[2];
    y[2] = M[6] * x[0] + M[7] * x[1] + M[8] * x[2];
}

// expand the upper blocks into the full BSR, invert the diagonal, start PCG from x = 0
__global__ void pcg_init_kernel(const double* __restrict__ hb, const int32_t* __restrict__ rowptr,
                                const int32_t* __restrict__ src_up, int64_t n, int64_t nnzb_upper,
                                double* __restrict__ bsr, double* __restrict__ minv, double* __restrict__ x,
                                double* __restrict__ r, double* __restrict__ z, double* __restrict__ p0,
                                double* __restrict__ part_rz, double* __restrict__ part_rr) {
    __shared__ double red[16];
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double rz = 0.0, rr = 0.0;
    if (v < n) {
        for (int32_t s = rowptr[v]; s < rowptr[v + 1]; ++s) {
            const int32_t su = src_up[s];
            const double* U = hb + 9 * (int64_t)(su >= 0 ? su : -1 - su);
            double* D = bsr + 9 * (int64_t)s;
            if (su >= 0) {
#pragma unroll
                for (int q = 0; q < 9; ++q) D[q] = U[q];
            } else {
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int b = 0; b < 3; ++b) D[3 * a + b] = U[3 * b + a];
            }
        }
        double Mi[9];
        inv3(hb + 9 * v, Mi);
#pragma unroll
        for (int q = 0; q < 9; ++q) minv[9 * v + q] = Mi[q];
        const double* g = hb + 9 * nnzb_upper + 3 * v;
        double rv[3] = {-g[0], -g[1], -g[2]}, zv[3];
        mv3(Mi, rv, zv);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            x[3 * v + c] = 0.0;
            r[3 * v + c] = rv[c];
            z[3 * v + c] = zv[c];
            p0[3 * v + c] = zv[c];
            rz += rv[c] * zv[c];
            rr += rv[c] * rv[c];
        }
    }
    rz = block_sum(rz, red);
    rr = block_sum(rr, red);
    if (threadIdx.x == 0) { part_rz[blockIdx.x] = rz; part_rr[blockIdx.x] = rr; }
}

__device__ __forceinline__ double sum_partials(const double* __restrict__ p, int nb) {
    double s = 0.0;
    for (int k = 0; k < nb; ++k) s += p[k];
    return s;
}

// K_A(it): rz_it = sum(part_rz); beta = rz_it / rz_{it-1} (it > 0); p_new = z + beta p_old
// (redundantly for neighbour rows); q = H p_new; partial p_new . q
__global__ void pcg_spmv_kernel(int it, const double* __restrict__ bsr, const int32_t* __restrict__ rowptr,
                                const int32_t* __restrict__ colidx, int64_t n, const double* __restrict__ z,
                                const double* __restrict__ p_old, double* __restrict__ p_new,
                                double* __restrict__ q, const double* __restrict__ part_rz,
                                const double* __restrict__ part_rr, double* __restrict__ part_pq,
                                double* __restrict__ scal, int nb) {
    __shared__ double red[16];
    const double rz = sum_partials(part_rz, nb);
    const double beta = it > 0 ? (scal[2 * (it - 1)] != 0.0 ? rz / scal[2 * (it - 1)] : 0.0) : 0.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        scal[2 * it] = rz;
        scal[2 * it + 1] = sum_partials(part_rr, nb);
    }
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double pq = 0.0;
    if (v < n) {
        double acc[3] = {0, 0, 0};
        for (int32_t s = rowptr[v]; s < rowptr[v + 1]; ++s) {
            const int64_t c = colidx[s];
            double pc[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) pc[k] = it > 0 ? z[3 * c + k] + beta * p_old[3 * c + k] : p_old[3 * c + k];
            const double* B = bsr + 9 * (int64_t)s;
            acc[0] += B[0] * pc[0] + B[1] * pc[1] + B[2] * pc[2];
            acc[1] += B[3] * pc[0] + B[4] * pc[1] + B[5] * pc[2];
            acc[2] += B[6] * pc[0] + B[7] * pc[1] + B[8] * pc[2];
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double pv = it > 0 ? z[3 * v + k] + beta * p_old[3 * v + k] : p_old[3 * v + k];
            p_new[3 * v + k] = pv;
            q[3 * v + k] = acc[k];
            pq += pv * acc[k];
        }
    }
    pq = block_sum(pq, red);
    if (threadIdx.x == 0) part_pq[blockIdx.x] = pq;
}

// K_B(it): alpha = rz_it / (p.q); x += alpha p; r -= alpha q; z = M^-1 r; partial rz, rr
__global__ void pcg_update_kernel(int it, int64_t n, const double* __restrict__ minv,
                                  const double* __restrict__ p, const double* __restrict__ q,
                                  double* __restrict__ x, double* __restrict__ r, double* __restrict__ z,
                                  const double* __restrict__ part_rz_in, const double* __restrict__ part_pq,
                                  double* __restrict__ part_rz_out, double* __restrict__ part_rr, int nb) {
    __shared__ double red[16];
    const double rz = sum_partials(part_rz_in, nb);
    const double pq = sum_partials(part_pq, nb);
    const double alpha = pq != 0.0 ? rz / pq : 0.0;
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double rz_n = 0.0, rr = 0.0;
    if (v < n) {
        double rv[3], zv[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            x[3 * v + k] += alpha * p[3 * v + k];
            rv[k] = r[3 * v + k] - alpha * q[3 * v + k];
            r[3 * v + k] = rv[k];
        }
        mv3(minv + 9 * v, rv, zv);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            z[3 * v + k] = zv[k];
            rz_n += rv[k] * zv[k];
            rr += rv[k] * rv[k];
        }
    }
    rz_n = block_sum(rz_n, red);
    rr = block_sum(rr, red);
    if (threadIdx.x == 0) { part_rz_out[blockIdx.x] = rz_n; part_rr[blockIdx.x] = rr; }
}

// X <- X * Pose2(d); partial max |d|.  d is indexed by node, or by elimination position when
// pos != NULL (the Cholesky's solution vector).
__global__ void retract_kernel(double* __restrict__ X, const double* __restrict__ d, int64_t n,
                               const int32_t* __restrict__ pos, double* __restrict__ max_out, const int32_t* gate) {
    if (gate && !gate[0]) return;
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double m = 0.0;
    if (v < n) {
        const int64_t di = 3 * (int64_t)(pos ? pos[v] : v);
        m = pose_retract(X + 3 * v, d[di], d[di + 1], d[di + 2]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
    if ((threadIdx.x & 63) == 0)
        atomicMax(reinterpret_cast<unsigned long long*>(max_out), (unsigned long long)__double_as_longlong(m));
}

// scal3[1] = chi2 of hb, scal3[2] = solver status (the Cholesky's, or 0)
__global__ void scalars_kernel(const double* __restrict__ chi2, const int32_t* __restrict__ status,
                               double* __restrict__ scal3) {
    scal3[1] = *chi2;
    scal3[2] = status ? (double)*status : 0.0;
}

// ICP results -> BetweenFactor measurement + diagonal information (dpg_slam.cc:331-338)
__global__ void icp_to_factor_kernel(const dpg_icp_result* __restrict__ res, dpg_factor* __restrict__ F,
                                     int64_t first, int64_t count, int64_t n_always, double ix, double iy,
                                     double ith) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= count) return;
    dpg_factor& f = F[first + e];
    const dpg_icp_result r = res[e];
    const bool keep = e < n_always || (r.converged && r.status == DPG_ICP_OK);
    f.z[0] = r.z[0];
    f.z[1] = r.z[1];
    f.z[2] = r.z[2];
    f.info[0] = keep ? ix : 0.0;
    f.info[1] = keep ? iy : 0.0;
    f.info[2] = keep ? ith : 0.0;
}

template <typename T>
int dev_alloc(T** p, size_t n) {
    if (n == 0) n = 1;
    return hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)) == hipSuccess ? 0 : DPG_ERR_HIP;
}

template <typename T>
int up(T* dst, const std::vector<T>& src) {
    if (src.empty()) return 0;
    return hipMemcpy(dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice) == hipSuccess ? 0 : DPG_ERR_HIP;
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + kRowThreads - 1) / kRowThreads); }

}  // namespace

// [H upper 9 nnzb | g 3n | chi2 | pad | votes n_vote]
extern "C" int64_t dpg_gn_dev_vote_offset(const dpg_gn_dev* g) { return 9 * g->nnzb_upper + 3 * g->n_nodes + 2; }
extern "C" int64_t dpg_gn_dev_hb_size(const dpg_gn_dev* g) { return dpg_gn_dev_vote_offset(g) + g->n_vote; }

extern "C" void dpg_gn_dev_free(dpg_gn_dev* g) {
    void* ptrs[] = {g->factors, g->up_row, g->up_col, g->up_cptr, g->up_clist, g->node_fptr, g->node_flist,
                    g->rowptr, g->colidx, g->src_up, g->bsr, g->minv, g->poses, g->x, g->r, g->z,
                    g->p0, g->p1, g->q, g->partials, g->scal, g->hb_own, g->scal3, g->mine, g->hb_part};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (g->scal3_host) (void)hipHostFree(g->scal3_host);
    if (g->chol) dpg_chol_destroy(g->chol);
    memset(g, 0, sizeof(*g));
}

static double gn_wall_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

extern "C" int dpg_gn_dev_alloc(dpg_gn_dev* g, int64_t n, const dpg_factor* F, int64_t nf,
                                int64_t shard_begin, int64_t shard_end, const dpg_chol_opts* opts, void* sync_stream) {
    memset(g, 0, sizeof(*g));
    if (n <= 0 || nf < 0 || n > (int64_t)1 << 28) return DPG_ERR_ARG;
    const double t0 = gn_wall_ms();
    // unique pairs (lo, hi) of Between factors, as sorted 64-bit keys lo << 32 | hi; every
    // factor's pair index found once
    std::vector<uint64_t> fkey((size_t)nf, ~0ull);
    std::vector<uint64_t> pk;
    pk.reserve((size_t)nf);
    for (int64_t k = 0; k < nf; ++k) {
        const dpg_factor& f = F[k];
        if (f.kind == DPG_FACTOR_PRIOR) {
            if (f.i < 0 || f.i >= n) return DPG_ERR_ARG;
            continue;
        }
        if (f.kind != DPG_FACTOR_BETWEEN || f.i < 0 || f.j < 0 || f.i >= n || f.j >= n || f.i == f.j)
            return DPG_ERR_ARG;
        fkey[(size_t)k] = (uint64_t)std::min(f.i, f.j) << 32 | (uint64_t)std::max(f.i, f.j);
        pk.push_back(fkey[(size_t)k]);
    }
    std::sort(pk.begin(), pk.end());
    pk.erase(std::unique(pk.begin(), pk.end()), pk.end());
    const int64_t P = (int64_t)pk.size();
    const int64_t nu = n + P;
    // the Cholesky's symbolic analysis and host plan (no device call) need only the pairs: on a
    // thread of their own while this one builds the contribution lists and the BSR rows; all of
    // the setup's host work runs before the wait below, so a caller's kernels still running on
    // sync_stream (the batch's ICP) overlap it
    std::vector<int32_t> plo((size_t)P), phi((size_t)P);
    for (int64_t p = 0; p < P; ++p) { plo[(size_t)p] = (int32_t)(pk[(size_t)p] >> 32); phi[(size_t)p] = (int32_t)(pk[(size_t)p] & 0xffffffffu); }
    const dpg_chol_opts copt = opts ? *opts : dpg_chol_opts{};
    double sym_ms = 0.0;
    std::future<void*> sym_job = std::async(std::launch::async, [&]() -> void* {
        const double ts = gn_wall_ms();
        void* ch = nullptr;
        dpg_chol_opts o = copt;
        dpg_chol_sym S;
        if (dpg_chol_symbolic(n, plo.data(), phi.data(), P, &o, &S) ||
            dpg_chol_create_sym_plan(&ch, n, plo.data(), phi.data(), P, &S, &o))
            ch = nullptr;   // the PCG solver still works; dpg_gn_dev_solve reports which ran
        sym_ms = gn_wall_ms() - ts;
        return ch;
    });
    std::vector<int32_t> fpair((size_t)nf, -1);
    for (int64_t k = 0; k < nf; ++k)
        if (fkey[(size_t)k] != ~0ull)
            fpair[(size_t)k] = (int32_t)(std::lower_bound(pk.begin(), pk.end(), fkey[(size_t)k]) - pk.begin());
    // contribution lists per upper block (factor order)
    std::vector<int32_t> cnt((size_t)nu + 1, 0);
    for (int64_t k = 0; k < nf; ++k) {
        const dpg_factor& f = F[k];
        cnt[(size_t)f.i + 1]++;
        if (f.kind == DPG_FACTOR_BETWEEN) {
            cnt[(size_t)f.j + 1]++;
            cnt[(size_t)(n + fpair[(size_t)k]) + 1]++;
        }
    }
    for (int64_t u = 0; u < nu; ++u) cnt[(size_t)u + 1] += cnt[(size_t)u];
    std::vector<int32_t> cptr = cnt, clist((size_t)cnt[(size_t)nu]);
    std::vector<int32_t> cur(cnt.begin(), cnt.end() - 1);
    for (int64_t k = 0; k < nf; ++k) {
        const dpg_factor& f = F[k];
        clist[(size_t)cur[(size_t)f.i]++] = (int32_t)(k << 2 | 0);
        if (f.kind == DPG_FACTOR_BETWEEN) {
            clist[(size_t)cur[(size_t)f.j]++] = (int32_t)(k << 2 | 1);
            clist[(size_t)cur[(size_t)(n + fpair[(size_t)k])]++] = (int32_t)(k << 2 | (f.i < f.j ? 2 : 3));
        }
    }
    // full BSR rows, by column: row v is the pairs (u, v) with u < v in ascending u (the key order
    // deals them so, bucketed by v), the diagonal block, then the pairs (v, w) in ascending w
    std::vector<int32_t> rowptr((size_t)n + 1, 0);
    for (int64_t v = 0; v < n; ++v) rowptr[(size_t)v + 1] = 1;
    for (uint64_t key : pk) { rowptr[(size_t)(key >> 32) + 1]++; rowptr[(size_t)(key & 0xffffffffu) + 1]++; }
    for (int64_t v = 0; v < n; ++v) rowptr[(size_t)v + 1] += rowptr[(size_t)v];
    std::vector<int32_t> colidx((size_t)rowptr[(size_t)n]), srcup((size_t)rowptr[(size_t)n]);
    {
        std::vector<int32_t> at(rowptr.begin(), rowptr.end() - 1);
        for (int64_t p = 0; p < P; ++p) {   // row hi: (lo, pair), ascending lo
            const int32_t lo = (int32_t)(pk[(size_t)p] >> 32), hi = (int32_t)(pk[(size_t)p] & 0xffffffffu);
            colidx[(size_t)at[(size_t)hi]] = lo;
            srcup[(size_t)at[(size_t)hi]++] = (int32_t)(-1 - (n + p));
        }
        for (int64_t v = 0; v < n; ++v) {   // the diagonal block after them
            colidx[(size_t)at[(size_t)v]] = (int32_t)v;
            srcup[(size_t)at[(size_t)v]++] = (int32_t)v;
        }
        for (int64_t p = 0; p < P; ++p) {   // row lo: (hi, pair), ascending hi
            const int32_t lo = (int32_t)(pk[(size_t)p] >> 32), hi = (int32_t)(pk[(size_t)p] & 0xffffffffu);
            colidx[(size_t)at[(size_t)lo]] = hi;
            srcup[(size_t)at[(size_t)lo]++] = (int32_t)(n + p);
        }
    }
    const double t1 = gn_wall_ms();
    void* chol = sym_job.get();
    const double t2 = gn_wall_ms();
    if (sync_stream && hipStreamSynchronize(reinterpret_cast<hipStream_t>(sync_stream)) != hipSuccess) {
        if (chol) dpg_chol_destroy(chol);
        return DPG_ERR_HIP;
    }
    g->n_nodes = n;
    g->n_factors = nf;
    g->nnzb_upper = nu;
    g->nnzb_full = (int64_t)colidx.size();
    g->shard_begin = shard_begin < 0 ? 0 : shard_begin;
    g->shard_end = shard_end > nf ? nf : shard_end;
    g->n_blocks_rows = (int32_t)nblk(n);
    int rc = 0;
    rc |= dev_alloc(&g->factors, (size_t)nf);
    rc |= dev_alloc(&g->up_cptr, cptr.size());
    rc |= dev_alloc(&g->up_clist, clist.size());
    rc |= dev_alloc(&g->rowptr, rowptr.size());
    rc |= dev_alloc(&g->colidx, colidx.size());
    rc |= dev_alloc(&g->src_up, srcup.size());
    rc |= dev_alloc(&g->bsr, 9 * colidx.size());
    rc |= dev_alloc(&g->minv, 9 * (size_t)n);
    rc |= dev_alloc(&g->poses, 3 * (size_t)n);
    rc |= dev_alloc(&g->x, 3 * (size_t)n);
    rc |= dev_alloc(&g->r, 3 * (size_t)n);
    rc |= dev_alloc(&g->z, 3 * (size_t)n);
    rc |= dev_alloc(&g->p0, 3 * (size_t)n);
    rc |= dev_alloc(&g->p1, 3 * (size_t)n);
    rc |= dev_alloc(&g->q, 3 * (size_t)n);
    rc |= dev_alloc(&g->partials, 6 * (size_t)g->n_blocks_rows + (size_t)n);
    rc |= dev_alloc(&g->scal, 2 * (size_t)65536);
    rc |= dev_alloc(&g->hb_own, (size_t)dpg_gn_dev_hb_size(g));
    rc |= dev_alloc(&g->scal3, 4);
    if (!rc && hipHostMalloc(reinterpret_cast<void**>(&g->scal3_host), 4 * sizeof(double)) != hipSuccess) rc = DPG_ERR_HIP;
    if (rc) { if (chol) dpg_chol_destroy(chol); dpg_gn_dev_free(g); return DPG_ERR_HIP; }
    if (nf && hipMemcpy(g->factors, F, (size_t)nf * sizeof(dpg_factor), hipMemcpyHostToDevice) != hipSuccess) rc = DPG_ERR_HIP;
    rc |= up(g->up_cptr, cptr);
    rc |= up(g->up_clist, clist);
    rc |= up(g->rowptr, rowptr);
    rc |= up(g->colidx, colidx);
    rc |= up(g->src_up, srcup);
    if (rc) { if (chol) dpg_chol_destroy(chol); dpg_gn_dev_free(g); return DPG_ERR_HIP; }
    // the supernodal Cholesky's device structures (once per pattern)
    g->chol = chol;
    if (g->chol && dpg_chol_create_sym_upload(&g->chol)) g->chol = nullptr;   // (destroyed on error)
    if (g->chol) dpg_chol_keep_inverse(g->chol, 1);   // chord steps reuse the factor: L11^-1 for their solves
    const double t3 = gn_wall_ms();
    double bt[2] = {0.0, 0.0};
    if (g->chol) dpg_chol_build_times(g->chol, bt);
    g->setup_ms[0] = t1 - t0;                             // (beside the next two from the pairs on)
    g->setup_ms[1] = std::max(0.0, sym_ms - bt[0]);       // the symbolic analysis (ordering, supernodes)
    g->setup_ms[2] = bt[0];                               // its host plan
    g->setup_ms[3] = std::max(0.0, (t3 - t2) - bt[1]);   // waiting for the stream, allocations, uploads
    g->setup_ms[4] = bt[1];                               // the Cholesky's upload
    return DPG_OK;
}

extern "C" int dpg_gn_dev_icp_to_factors(dpg_gn_dev* g, const dpg_icp_result* res, int64_t first, int64_t count,
                                         int64_t n_always, double ix, double iy, double ith, void* stream) {
    if (count <= 0) return DPG_OK;
    if (first < 0 || first + count > g->n_factors) return DPG_ERR_ARG;
    hipLaunchKernelGGL(icp_to_factor_kernel, dim3(nblk(count)), dim3(kRowThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), res, g->factors, first, count, n_always, ix, iy, ith);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

static int assemble_gated(dpg_gn_dev* g, double* hb, hipStream_t s, const int32_t* gate, bool chi2 = true) {
    double* chi2_node = g->partials + 6 * (size_t)g->n_blocks_rows;
    const int64_t ng = lg_groups(g->n_nodes, g->nnzb_upper);
    if (ng > 0)
        hipLaunchKernelGGL(lin_gather_kernel, dim3((unsigned)ng), dim3(kLgLanes), 0, s, g->factors, g->poses, g->up_cptr,
                           g->up_clist, g->n_nodes, g->nnzb_upper, g->shard_begin, g->shard_end, g->mine, hb, chi2_node, gate);
    if (chi2) {
        // the vote words go with the partial buffer only (the sum gives every device all of them)
        const bool vote = hb == g->hb_part && g->n_vote > 0;
        hipLaunchKernelGGL(chi2_kernel, dim3(1), dim3(1024), 0, s, chi2_node, g->n_nodes,
                           hb + 9 * g->nnzb_upper + 3 * g->n_nodes, gate, vote ? hb + dpg_gn_dev_vote_offset(g) : nullptr,
                           g->scal3, vote && g->chol ? dpg_chol_status_dev(g->chol) : nullptr, g->world, g->rank);
    }
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_gn_dev_assemble(dpg_gn_dev* g, double* hb, void* stream) {
    return assemble_gated(g, hb, reinterpret_cast<hipStream_t>(stream), nullptr);
}

// ---- multi-device forms ----
__global__ void own_kernel(uint8_t* __restrict__ mine, int64_t nf, int32_t world, int32_t rank) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f < nf) mine[f] = (f % world) == rank ? 1 : 0;
}

// icp_to_factor_kernel's expressions for this device's results, written to the caller's slots
__global__ void icp_to_factor_scatter_kernel(const dpg_icp_result* __restrict__ res, const int32_t* __restrict__ idx,
                                             dpg_factor* __restrict__ F, uint8_t* __restrict__ mine, int64_t first,
                                             int64_t n_local, int64_t n_always, double ix, double iy, double ith) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_local) return;
    const int64_t e = idx[j];
    dpg_factor& f = F[first + e];
    const dpg_icp_result r = res[j];
    const bool keep = e < n_always || (r.converged && r.status == DPG_ICP_OK);
    f.z[0] = r.z[0];
    f.z[1] = r.z[1];
    f.z[2] = r.z[2];
    f.info[0] = keep ? ix : 0.0;
    f.info[1] = keep ? iy : 0.0;
    f.info[2] = keep ? ith : 0.0;
    mine[first + e] = 1;
}

struct VsumArgs {
    const double* parts[16];
    double* outs[16];
};
// virtual devices' all-reduce: every output the same rank-order sum
__global__ void vsum_kernel(VsumArgs a, int32_t k, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double s = a.parts[0][i];
        for (int32_t q = 1; q < k; ++q) s += a.parts[q][i];
        for (int32_t q = 0; q < k; ++q) a.outs[q][i] = s;
    }
}

extern "C" int dpg_gn_dev_set_ownership(dpg_gn_dev* g, int32_t world, int32_t rank, void* stream) {
    if (world < 1 || rank < 0 || rank >= world) return DPG_ERR_ARG;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int32_t nv = world > 1 ? 2 * world : 0;
    if (nv != g->n_vote) {   // the packed buffers grow by the vote words
        if (hipStreamSynchronize(s) != hipSuccess) return DPG_ERR_HIP;
        if (g->hb_own) (void)hipFree(g->hb_own);
        if (g->hb_part) (void)hipFree(g->hb_part);
        g->hb_own = g->hb_part = nullptr;
        g->n_vote = nv;
        if (dev_alloc(&g->hb_own, (size_t)dpg_gn_dev_hb_size(g))) return DPG_ERR_HIP;
    }
    if (!g->mine && dev_alloc(&g->mine, (size_t)g->n_factors)) return DPG_ERR_HIP;
    if (!g->hb_part && dev_alloc(&g->hb_part, (size_t)dpg_gn_dev_hb_size(g))) return DPG_ERR_HIP;
    // the other devices' vote words stay zero in this device's partial buffer
    if (hipMemsetAsync(g->hb_part, 0, sizeof(double) * (size_t)dpg_gn_dev_hb_size(g), s) != hipSuccess) return DPG_ERR_HIP;
    g->world = world;
    g->rank = rank;
    if (g->n_factors > 0)
        hipLaunchKernelGGL(own_kernel, dim3(nblk(g->n_factors)), dim3(kRowThreads), 0, reinterpret_cast<hipStream_t>(stream),
                           g->mine, g->n_factors, world, rank);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_gn_dev_icp_to_factors_scatter(dpg_gn_dev* g, const dpg_icp_result* res, const int32_t* idx,
                                                 int64_t n_local, int64_t first, int64_t count, int64_t n_always,
                                                 double ix, double iy, double ith, void* stream) {
    if (!g->mine || first < 0 || count < n_local || first + count > g->n_factors) return DPG_ERR_ARG;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (count > 0 && hipMemsetAsync(g->mine + first, 0, (size_t)count, s) != hipSuccess) return DPG_ERR_HIP;
    if (n_local > 0)
        hipLaunchKernelGGL(icp_to_factor_scatter_kernel, dim3(nblk(n_local)), dim3(kRowThreads), 0, s, res, idx, g->factors,
                           g->mine, first, n_local, n_always, ix, iy, ith);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_gn_dev_assemble_part(dpg_gn_dev* g, const int32_t* gate, void* stream) {
    if (!g->hb_part) return DPG_ERR_STATE;
    return assemble_gated(g, g->hb_part, reinterpret_cast<hipStream_t>(stream), gate, true);
}

extern "C" int dpg_launch_vsum(const double* const* parts, double* const* outs, int32_t k, int64_t n, void* stream) {
    if (k < 1 || k > 16 || n <= 0) return k >= 1 && k <= 16 ? DPG_OK : DPG_ERR_ARG;
    VsumArgs a;
    for (int q = 0; q < 16; ++q) {
        a.parts[q] = q < k ? parts[q] : nullptr;
        a.outs[q] = q < k ? outs[q] : nullptr;
    }
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 1023) / 1024, 2048);
    hipLaunchKernelGGL(vsum_kernel, dim3(blocks), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream), a, k, n);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

static int pcg_solve(dpg_gn_dev* g, const double* hb, const dpg_gn_params* gp, hipStream_t s);

extern "C" int dpg_gn_dev_solve_async(dpg_gn_dev* g, const double* hb, const dpg_gn_params* gp, void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const double* xout = g->x;
    const int32_t* xpos = nullptr;
    g->last_pcg_iters = 0;
    g->last_used_chol = gp->linear_solver == DPG_SOLVER_CHOLESKY && g->chol;
    if (g->last_used_chol) {
        // chord steps once the step is small -- while they keep contracting: a chord step that
        // shrank the step by less than 10x (linear convergence gone slow, e.g. a sweep far from the
        // optimum) hands back to a fresh factorization
        const bool slow = g->last_was_chord && g->last_delta_inf > 0.1 * g->prev_delta_inf;
        const bool reuse = gp->reuse_factorization && g->have_factor && g->last_delta_inf < gp->refactor_delta && !slow;
        g->last_was_chord = reuse ? 1 : 0;
        const int rc = reuse ? dpg_chol_resolve(g->chol, hb, stream) : dpg_chol_solve(g->chol, hb, stream);
        if (rc) return rc;
        if (!reuse) {
            g->have_factor = 1;
            ++g->n_factorizations;
        }
        xout = dpg_chol_x_dev(g->chol);
        xpos = dpg_chol_pos_dev(g->chol);
    } else {
        const int it = pcg_solve(g, hb, gp, s);
        if (it < 0) return DPG_ERR_HIP;
        g->last_pcg_iters = it;
    }
    if (hipMemsetAsync(g->scal3, 0, sizeof(double), s) != hipSuccess) return DPG_ERR_HIP;
    hipLaunchKernelGGL(retract_kernel, dim3(g->n_blocks_rows), dim3(kRowThreads), 0, s, g->poses, xout, g->n_nodes,
                       xpos, g->scal3, nullptr);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

// ---- the pipelined loop (dpg_gn_pipe.h) ----
// clear what the next fused solve counts on (as dpg_chol_solve's memsets)
__device__ __forceinline__ void clear_sync(int32_t* sync, int64_t n_words, int32_t* status) {
    int4* s4 = reinterpret_cast<int4*>(sync);   // 16-B aligned, n_words a multiple of 4
    for (int64_t k = threadIdx.x; k < n_words / 4; k += blockDim.x) s4[k] = make_int4(0, 0, 0, 0);
    if (threadIdx.x == 0) *status = 0;
}

// a report into host memory: the fields, then the tag the host polls.  The slot is fine-grained
// (coherent, uncached) host memory (dpg_api.hip ensure_pipe): the fields go out as system-scope
// stores, and the tag only after all of them have been acknowledged (s_waitcnt vmcnt(0)), so the
// host never sees the tag before the fields -- without __threadfence_system's write-back of the
// whole L2, which holds nothing of the slot's
__device__ __forceinline__ void sys_st64(void* p, uint64_t v) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
static_assert(offsetof(dpg_gn_slot, reuse) == 24 && offsetof(dpg_gn_slot, active) == 28 &&
              offsetof(dpg_gn_slot, final_) == 32 && offsetof(dpg_gn_slot, it) == 36 && offsetof(dpg_gn_slot, tag) == 40,
              "post_slot stores the int pairs as 8-byte words");
__device__ __forceinline__ void post_slot(dpg_gn_slot* slot, const dpg_gn_slot& o, uint64_t tag) {
    sys_st64(&slot->dinf, (uint64_t)__double_as_longlong(o.dinf));
    sys_st64(&slot->error, (uint64_t)__double_as_longlong(o.error));
    sys_st64(&slot->status, (uint64_t)__double_as_longlong(o.status));
    sys_st64(&slot->reuse, (uint64_t)(uint32_t)o.reuse | (uint64_t)(uint32_t)o.active << 32);
    sys_st64(&slot->final_, (uint64_t)(uint32_t)o.final_ | (uint64_t)(uint32_t)o.it << 32);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sys_st64(&slot->tag, tag);
}

__global__ void pipe_init_kernel(dpg_gn_ctl* ctl, int32_t reuse, int32_t last_was_chord, int32_t have_factor,
                                 double last_dinf, double prev_dinf, const double* cur_dev, dpg_gn_slot* init,
                                 double* max_out, int32_t* sync, int64_t n_words, int32_t* status, uint32_t loop) {
    clear_sync(sync, n_words, status);
    if (threadIdx.x != 0) return;
    const double cur = *cur_dev;   // the assembled initial error (the host loop reads it back first)
    {
        dpg_gn_slot o{};
        o.error = cur;
        post_slot(init, o, (uint64_t)loop << 32);
    }
    ctl->loop = loop;
    ctl->active = !(cur <= 0.0) ? 1 : 0;   // the host loop's entry test
    ctl->reuse = reuse;
    ctl->last_was_chord = last_was_chord;
    ctl->have_factor = have_factor;
    ctl->it = 0;
    ctl->last_dinf = last_dinf;
    ctl->prev_dinf = prev_dinf;
    ctl->cur_error = cur;
    *max_out = 0.0;
}

// the end of one iteration: the error (chi2_kernel's sum, same order), its report, then the next
// iteration decided exactly as the host loop does (dpg_api.hip gn_loop: the stop rule;
// dpg_gn_dev_solve_async: the chord rule), and the solver's counters cleared for it
// chi2_sum != NULL (multi-device forms): the error is the all-reduced sum already in hb, not this
// device's per-node terms.  vote != NULL (world > 1): max |delta| and the status are taken from the
// all-reduced vote words -- the largest |delta| and the largest status over the devices -- so every
// device decides from the same numbers; devices whose |delta| differ (they solved different systems)
// end the loop together with status DPG_GN_STATUS_DIVERGED
__global__ __launch_bounds__(1024) void pipe_ctl_kernel(dpg_gn_ctl* ctl, const double* __restrict__ chi2_node, int64_t n,
                                                        double* chi2, const double* chi2_sum, int32_t* status,
                                                        double* max_out, dpg_gn_params P, dpg_gn_slot* slot,
                                                        int32_t* sync, int64_t n_words, const double* __restrict__ vote,
                                                        int32_t world) {
    __shared__ double red[16];
    if (!ctl->active) return;   // uniform: nothing ran this iteration, nothing to report
    double sum = 0.0;
    if (chi2_sum) {
        sum = *chi2_sum;
    } else {
        sum = block_sum(strided_sum(chi2_node, n, threadIdx.x, blockDim.x), red);
    }
    const double st_word = (double)*status;
    __syncthreads();   // every lane has read the status word before it is cleared
    clear_sync(sync, n_words, status);
    if (threadIdx.x != 0) return;
    *chi2 = sum;
    dpg_gn_slot o;
    o.reuse = ctl->reuse;
    o.active = ctl->active;
    o.it = ctl->it;
    o.final_ = 1;
    o.dinf = 0.0;
    o.error = 0.0;
    o.status = 0.0;
    if (ctl->active) {
        double dinf = *max_out, st = st_word;
        if (vote) {
            const unsigned long long d0 = (unsigned long long)__double_as_longlong(vote[0]);
            bool diverged = false;
            dinf = vote[0];
            st = vote[world];
            for (int32_t r = 1; r < world; ++r) {
                diverged |= (unsigned long long)__double_as_longlong(vote[r]) != d0;
                dinf = fmax(dinf, vote[r]);
                st = fmax(st, vote[world + r]);
            }
            if (diverged) st = (double)DPG_GN_STATUS_DIVERGED;
        }
        const double nw = sum;
        const int it = ctl->it + 1;
        o.dinf = dinf;
        o.error = nw;
        o.status = st;
        o.it = it;
        bool fin = st != 0.0 || it >= P.max_iterations;
        if (!fin) {
            const double cur = ctl->cur_error;
            if (P.use_error_criteria) {
                bool conv = nw <= 0.0;
                if (!conv) {
                    const double abs_dec = cur - nw, rel_dec = abs_dec / cur;
                    conv = (P.relative_error_tol != 0.0 && rel_dec <= P.relative_error_tol) ||
                           abs_dec <= P.absolute_error_tol;
                }
                fin = conv || !isfinite(cur);
            } else {
                fin = dinf < P.delta_tol;
            }
        }
        o.final_ = fin ? 1 : 0;
        // chord bookkeeping after the fetch: prev <- last, last <- dinf; the step just taken
        ctl->prev_dinf = ctl->last_dinf;
        ctl->last_dinf = dinf;
        ctl->last_was_chord = ctl->reuse;
        ctl->have_factor = 1;
        ctl->cur_error = nw;
        ctl->it = it;
        const bool slow = ctl->last_was_chord && ctl->last_dinf > 0.1 * ctl->prev_dinf;
        ctl->reuse = (P.reuse_factorization && ctl->have_factor && ctl->last_dinf < P.refactor_delta && !slow) ? 1 : 0;
        ctl->active = fin ? 0 : 1;
        *max_out = 0.0;
    }
    post_slot(slot, o, ((uint64_t)ctl->loop << 32) | (uint32_t)o.it);
}

extern "C" int dpg_gn_pipe_init(dpg_gn_dev* g, const dpg_gn_params* gp, dpg_gn_ctl* ctl, const double* cur_dev,
                                dpg_gn_slot* init, uint32_t loop, void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // iteration 1's chord decision from the host bookkeeping (as dpg_gn_dev_solve_async takes it)
    const bool slow = g->last_was_chord && g->last_delta_inf > 0.1 * g->prev_delta_inf;
    const bool reuse = gp->reuse_factorization && g->have_factor && g->last_delta_inf < gp->refactor_delta && !slow;
    int32_t* sync;
    int64_t n_words;
    dpg_chol_sync_dev(g->chol, &sync, &n_words);
    hipLaunchKernelGGL(pipe_init_kernel, dim3(1), dim3(1024), 0, s, ctl, reuse ? 1 : 0, g->last_was_chord, g->have_factor,
                       g->last_delta_inf, g->prev_delta_inf, cur_dev, init, g->scal3, sync, n_words,
                       const_cast<int32_t*>(dpg_chol_status_dev(g->chol)), loop);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_gn_pipe_issue_solve(dpg_gn_dev* g, dpg_gn_ctl* ctl, int part, void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int32_t* gate = &ctl->active;
    if (!g->chol || !dpg_chol_gated_ok(g->chol) || (part && !g->hb_part)) return DPG_ERR_STATE;
    int rc = dpg_chol_solve_gated(g->chol, g->hb_own, gate, 1, g->poses, g->scal3, stream);
    if (rc) return rc;
    return part ? assemble_gated(g, g->hb_part, s, gate, true) : assemble_gated(g, g->hb_own, s, gate, false);
}

extern "C" int dpg_gn_pipe_issue_ctl(dpg_gn_dev* g, const dpg_gn_params* gp, dpg_gn_ctl* ctl, dpg_gn_slot* slot,
                                     int part, void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int32_t* sync;
    int64_t n_words;
    if (dpg_chol_join_aux(g->chol, stream)) return DPG_ERR_HIP;
    dpg_chol_sync_dev(g->chol, &sync, &n_words);
    double* chi2 = g->hb_own + 9 * g->nnzb_upper + 3 * g->n_nodes;
    hipLaunchKernelGGL(pipe_ctl_kernel, dim3(1), dim3(1024), 0, s, ctl, g->partials + 6 * (size_t)g->n_blocks_rows,
                       g->n_nodes, chi2, part ? chi2 : nullptr, const_cast<int32_t*>(dpg_chol_status_dev(g->chol)),
                       g->scal3, *gp, slot, sync, n_words,
                       part && g->n_vote > 0 ? g->hb_own + dpg_gn_dev_vote_offset(g) : nullptr, g->world);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_gn_pipe_issue(dpg_gn_dev* g, const dpg_gn_params* gp, dpg_gn_ctl* ctl, dpg_gn_slot* slot,
                                 void* stream) {
    const int rc = dpg_gn_pipe_issue_solve(g, ctl, 0, stream);
    return rc ? rc : dpg_gn_pipe_issue_ctl(g, gp, ctl, slot, 0, stream);
}

extern "C" int dpg_gn_dev_fetch(dpg_gn_dev* g, const double* hb, void* stream, double out[3]) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool chol = g->chol != nullptr && g->last_used_chol;
    hipLaunchKernelGGL(scalars_kernel, dim3(1), dim3(1), 0, s, hb + 9 * g->nnzb_upper + 3 * g->n_nodes,
                       chol ? dpg_chol_status_dev(g->chol) : nullptr, g->scal3);
    if (hipMemcpyAsync(g->scal3_host, g->scal3, 3 * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return DPG_ERR_HIP;
    out[0] = g->scal3_host[0];
    out[1] = g->scal3_host[1];
    out[2] = g->scal3_host[2];
    g->prev_delta_inf = g->last_delta_inf;
    g->last_delta_inf = out[0];
    return DPG_OK;
}

extern "C" int dpg_gn_dev_solve(dpg_gn_dev* g, const double* hb, const dpg_gn_params* gp, void* stream,
                                double* delta_inf, double* error, int32_t* pcg_iters) {
    int rc = dpg_gn_dev_solve_async(g, hb, gp, stream);
    if (rc) return rc;
    double sc[3];
    if ((rc = dpg_gn_dev_fetch(g, hb, stream, sc))) return rc;
    if (gp->linear_solver == DPG_SOLVER_CHOLESKY && g->chol && sc[2] != 0.0) return DPG_ERR_NUMERIC;
    if (delta_inf) *delta_inf = sc[0];
    if (error) *error = sc[1];
    if (pcg_iters) *pcg_iters = g->last_pcg_iters;
    return DPG_OK;
}

// block-Jacobi PCG on the full BSR; returns the iteration count (< 0 on a HIP error)
static int pcg_solve(dpg_gn_dev* g, const double* hb, const dpg_gn_params* gp, hipStream_t s) {
    const int nb = g->n_blocks_rows;
    const int64_t n = g->n_nodes;
    double* part_rz_a = g->partials;
    double* part_rz_b = g->partials + nb;
    double* part_rr = g->partials + 2 * (size_t)nb;
    double* part_pq = g->partials + 3 * (size_t)nb;
    hipLaunchKernelGGL(pcg_init_kernel, dim3(nb), dim3(kRowThreads), 0, s, hb, g->rowptr, g->src_up, n, g->nnzb_upper,
                       g->bsr, g->minv, g->x, g->r, g->z, g->p0, part_rz_a, part_rr);
    double host_scal[2] = {0, 0};
    double rr0 = -1.0;
    const int check = gp->pcg_check_every > 0 ? gp->pcg_check_every : 16;
    const int max_it = std::min(gp->pcg_max_iterations > 0 ? gp->pcg_max_iterations : 20000, 65535);
    const double tol2 = gp->pcg_rel_tol * gp->pcg_rel_tol;
    int it = 0;
    double* pbuf[2] = {g->p0, g->p1};
    double* rzbuf[2] = {part_rz_a, part_rz_b};
    for (; it < max_it; ++it) {
        double* p_old = pbuf[it & 1];
        double* p_new = pbuf[(it + 1) & 1];
        hipLaunchKernelGGL(pcg_spmv_kernel, dim3(nb), dim3(kRowThreads), 0, s, it, g->bsr, g->rowptr, g->colidx, n,
                           g->z, p_old, p_new, g->q, rzbuf[it & 1], part_rr, part_pq, g->scal, nb);
        if (it % check == 0) {
            if (hipMemcpyAsync(host_scal, g->scal + 2 * it, 2 * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return -1;
            if (rr0 < 0) rr0 = host_scal[1];
            if (!(host_scal[1] > tol2 * rr0) || !(rr0 > 0)) break;   // converged (or zero rhs)
        }
        hipLaunchKernelGGL(pcg_update_kernel, dim3(nb), dim3(kRowThreads), 0, s, it, n, g->minv, p_new, g->q, g->x,
                           g->r, g->z, rzbuf[it & 1], part_pq, rzbuf[(it + 1) & 1], part_rr, nb);
    }
    return it;
}

// the rank form's host collective (dpg_api.hip, dpg_ctx::HostColl): the stream waits here until the
// collective thread has stored this iteration's tag.  One lane; vector loads at system scope (the
// word is host memory), s_sleep between polls, a 120 s bound on the 100 MHz clock.
__global__ void host_wait_kernel(const uint32_t* flag, uint32_t tag, uint32_t* timed_out) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    for (;;) {
        const uint32_t v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((int32_t)(v - tag) >= 0) return;
        if (wall_clock64() - t0 > 12000000000ull) {   // 120 s
            __hip_atomic_store(timed_out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

extern "C" int dpg_launch_host_wait(const uint32_t* flag, uint32_t tag, uint32_t* timed_out, void* stream) {
    hipLaunchKernelGGL(host_wait_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), flag, tag, timed_out);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}
