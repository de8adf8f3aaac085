// dpg_chol.hip -- supernodal multifrontal Cholesky of the pose-graph normal equations on gfx950.
//
// The CHOLESKY solve that GTSAM runs inside GaussNewtonOptimizer / ISAM2 as a
// level-scheduled GPU factorization: the symbolic analysis (dpg_chol_sym.cpp) runs once per
// sparsity pattern; each GN iteration then runs, per elimination-tree level, ONE kernel launch
// for all fronts of that level (one 256-thread workgroup per front):
//   factor: zero the dense front, scatter the original 3x3 blocks of H, extend-add the
//           children's update matrices (in child order: deterministic, no atomics), partial
//           Cholesky of the pivot columns in LDS panels, Schur complement left in place;
//   forward:  L y = -g  (children's pending row updates gathered, diagonal blocks solved by one
//             wave from LDS, L21 y passed up);
//   backward: L^T x = y (ancestors' x gathered by row position).
// fp64 throughout; the fronts of one factorization stay resident in HBM (tens of MB).

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "dpg_chol.h"
#include "dpg_internal.h"

namespace {

constexpr int kT = 256;     // threads per front workgroup
constexpr int kNB = 32;     // factorization panel width (scalar columns)
constexpr int kSB = 64;     // triangular-solve diagonal block

struct SnDev {
    int32_t c0, k, r, nchild;   // k, r in 3x3 blocks
    int64_t front_off;          // doubles
    int64_t rows_off;           // into rows / relmap
    int64_t child_off;          // into child_list
    int64_t omap_off;
    int64_t acc_off;            // doubles (3r pending row updates of the forward solve)
    int32_t omap_n, pad;
};

struct OEnt {                   // one upper 3x3 block of H -> its front position
    int32_t u;                  // block index in the packed hb buffer
    int16_t a, b;               // local block row / column in the front
    int32_t tr, pad;            // 1: the front wants H(lo,hi)^T
};

__global__ __launch_bounds__(kT) void chol_factor_level(const int32_t* __restrict__ level_sn,
                                                        const SnDev* __restrict__ sns,
                                                        const OEnt* __restrict__ omap,
                                                        const double* __restrict__ hb,
                                                        const int32_t* __restrict__ child_list,
                                                        const int32_t* __restrict__ relmap,
                                                        double* __restrict__ fronts, int32_t* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) double P[];
    const int tid = threadIdx.x;
    const int s = level_sn[blockIdx.x];
    const SnDev S = sns[s];
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k;
    double* F = fronts + S.front_off;
    for (int e = tid; e < m3 * m3; e += kT) F[e] = 0.0;
    __syncthreads();
    for (int q = tid; q < S.omap_n * 9; q += kT) {
        const OEnt o = omap[S.omap_off + q / 9];
        const int ii = (q % 9) / 3, jj = q % 3;
        const double* B = hb + 9 * (int64_t)o.u;
        F[(3 * o.b + jj) * m3 + 3 * o.a + ii] = o.tr ? B[3 * jj + ii] : B[3 * ii + jj];
    }
    __syncthreads();
    for (int ci = 0; ci < S.nchild; ++ci) {   // extend-add, one child at a time
        const int c = child_list[S.child_off + ci];
        const SnDev C = sns[c];
        const int r3c = 3 * C.r, k3c = 3 * C.k, m3c = 3 * (C.k + C.r);
        const double* Fc = fronts + C.front_off;
        const int32_t* rm = relmap + C.rows_off;
        for (int e = tid; e < r3c * r3c; e += kT) {
            const int i = e % r3c, j = e / r3c;
            if (i < j) continue;
            const int pi = 3 * rm[i / 3] + i % 3, pj = 3 * rm[j / 3] + j % 3;
            F[pj * m3 + pi] += Fc[(k3c + j) * m3c + k3c + i];
        }
        __syncthreads();
    }
    // blocked right-looking partial Cholesky of the first k3 columns:
    //   panel (R x w, R = rows from j0 down) in LDS, factored Crout-style (2 barriers / column),
    //   then the trailing lower triangle updated by 4x4 register tiles (lower-triangle tiles only).
    for (int j0 = 0; j0 < k3; j0 += kNB) {
        const int w = min(kNB, k3 - j0), R = m3 - j0;
        for (int e = tid; e < w * R; e += kT) {
            const int t = e / R, i = e - t * R;
            P[e] = F[(j0 + t) * m3 + j0 + i];
        }
        __syncthreads();
        for (int t = 0; t < w; ++t) {
            // column t: subtract the contributions of the panel's earlier columns (rows i >= t)
            if (t > 0) {
                for (int i = t + tid; i < R; i += kT) {
                    double acc = 0.0;
                    for (int s2 = 0; s2 < t; ++s2) acc += P[s2 * R + i] * P[s2 * R + t];
                    P[t * R + i] -= acc;
                }
                __syncthreads();
            }
            double piv = P[t * R + t];
            if (!(piv > 0.0)) {
                if (tid == 0) atomicExch(status, 1);
                piv = 1.0;
            }
            piv = sqrt(piv);
            const double inv = 1.0 / piv;
            __syncthreads();   // everyone has read the pivot before row t is overwritten
            for (int i = t + tid; i < R; i += kT) P[t * R + i] = (i == t) ? piv : P[t * R + i] * inv;
            __syncthreads();
        }
        for (int e = tid; e < w * R; e += kT) {
            const int t = e / R, i = e - t * R;
            if (i >= t) F[(j0 + t) * m3 + j0 + i] = P[e];
        }
        // trailing update: F(i, l) -= sum_t P(i, t) P(l, t) for w <= l <= i < R (panel-local)
        const int T = R - w;
        const int nt = (T + 3) >> 2;
        const int ntiles = nt * (nt + 1) / 2;
        for (int q = tid; q < ntiles; q += kT) {
            int ti = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
            while (ti * (ti + 1) / 2 > q) --ti;
            while ((ti + 1) * (ti + 2) / 2 <= q) ++ti;
            const int tl = q - ti * (ti + 1) / 2;
            const int i0 = w + 4 * ti, l0 = w + 4 * tl;
            double acc[4][4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = 0.0;
            for (int t = 0; t < w; ++t) {
                const double* Pt = P + t * R;
                double a[4], b[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) a[r] = (i0 + r < R) ? Pt[i0 + r] : 0.0;
#pragma unroll
                for (int c = 0; c < 4; ++c) b[c] = (l0 + c < R) ? Pt[l0 + c] : 0.0;
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[r][c] += a[r] * b[c];
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int l = l0 + c;
                if (l >= R) continue;
                double* col = F + (int64_t)(j0 + l) * m3 + j0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = i0 + r;
                    if (i < R && i >= l) col[i] -= acc[r][c];
                }
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kT) void chol_forward_level(const int32_t* __restrict__ level_sn,
                                                         const SnDev* __restrict__ sns,
                                                         const int32_t* __restrict__ child_list,
                                                         const int32_t* __restrict__ relmap,
                                                         const double* __restrict__ fronts,
                                                         const double* __restrict__ g,
                                                         const int32_t* __restrict__ perm,
                                                         double* __restrict__ ysol, double* __restrict__ acc) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int s = level_sn[blockIdx.x];
    const SnDev S = sns[s];
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k, r3 = 3 * S.r;
    const double* F = fronts + S.front_off;
    double* D = sm;                  // kSB x kSB diagonal block
    double* y = sm + kSB * kSB;      // k3
    double* aR = y + k3;             // r3
    for (int t = tid; t < k3; t += kT) {
        const int node = perm[S.c0 + t / 3];
        y[t] = -g[3 * node + t % 3];
    }
    for (int t = tid; t < r3; t += kT) aR[t] = 0.0;
    __syncthreads();
    for (int ci = 0; ci < S.nchild; ++ci) {
        const int c = child_list[S.child_off + ci];
        const SnDev C = sns[c];
        const int32_t* rm = relmap + C.rows_off;
        for (int t = tid; t < 3 * C.r; t += kT) {
            const int li = 3 * rm[t / 3] + t % 3;
            const double v = acc[C.acc_off + t];
            if (li < k3) y[li] -= v;
            else aR[li - k3] += v;
        }
        __syncthreads();
    }
    for (int jb = 0; jb < k3; jb += kSB) {
        const int bw = min(kSB, k3 - jb);
        for (int e = tid; e < bw * bw; e += kT) {
            const int i = e % bw, j = e / bw;
            D[j * kSB + i] = F[(jb + j) * m3 + jb + i];
        }
        __syncthreads();
        if (wave == 0) {
            double yl = lane < bw ? y[jb + lane] : 0.0;
            for (int j = 0; j < bw; ++j) {
                const double yj = __shfl(yl, j, 64) / D[j * kSB + j];
                if (lane == j) yl = yj;
                else if (lane > j && lane < bw) yl -= D[j * kSB + lane] * yj;
            }
            if (lane < bw) y[jb + lane] = yl;
        }
        __syncthreads();
        for (int i = jb + bw + tid; i < k3; i += kT) {
            double sacc = 0.0;
            for (int j = 0; j < bw; ++j) sacc += F[(jb + j) * m3 + i] * y[jb + j];
            y[i] -= sacc;
        }
        __syncthreads();
    }
    for (int t = tid; t < r3; t += kT) {
        double sacc = 0.0;
        for (int j = 0; j < k3; ++j) sacc += F[j * m3 + k3 + t] * y[j];
        acc[S.acc_off + t] = aR[t] + sacc;
    }
    for (int t = tid; t < k3; t += kT) ysol[3 * (int64_t)S.c0 + t] = y[t];
}

__global__ __launch_bounds__(kT) void chol_backward_level(const int32_t* __restrict__ level_sn,
                                                          const SnDev* __restrict__ sns,
                                                          const int32_t* __restrict__ rows,
                                                          const double* __restrict__ fronts,
                                                          const double* __restrict__ ysol,
                                                          double* __restrict__ xsol) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int s = level_sn[blockIdx.x];
    const SnDev S = sns[s];
    const int m3 = 3 * (S.k + S.r), k3 = 3 * S.k, r3 = 3 * S.r;
    const double* F = fronts + S.front_off;
    double* D = sm;
    double* z = sm + kSB * kSB;      // k3
    double* xr = z + k3;             // r3
    for (int t = tid; t < r3; t += kT) xr[t] = xsol[3 * (int64_t)rows[S.rows_off + t / 3] + t % 3];
    __syncthreads();
    for (int j = tid; j < k3; j += kT) {
        double sacc = 0.0;
        for (int t = 0; t < r3; ++t) sacc += F[j * m3 + k3 + t] * xr[t];
        z[j] = ysol[3 * (int64_t)S.c0 + j] - sacc;
    }
    __syncthreads();
    const int nblk = (k3 + kSB - 1) / kSB;
    for (int b = nblk - 1; b >= 0; --b) {
        const int jb = b * kSB, bw = min(kSB, k3 - jb);
        for (int e = tid; e < bw * bw; e += kT) {
            const int i = e % bw, j = e / bw;
            D[j * kSB + i] = F[(jb + j) * m3 + jb + i];
        }
        __syncthreads();
        if (wave == 0) {
            double zl = lane < bw ? z[jb + lane] : 0.0;
            for (int j = bw - 1; j >= 0; --j) {
                const double xj = __shfl(zl, j, 64) / D[j * kSB + j];
                if (lane == j) zl = xj;
                else if (lane < j) zl -= D[lane * kSB + j] * xj;   // L(jb+j, jb+lane)
            }
            if (lane < bw) z[jb + lane] = zl;
        }
        __syncthreads();
        for (int j = tid; j < jb; j += kT) {
            double sacc = 0.0;
            for (int i = 0; i < bw; ++i) sacc += F[j * m3 + jb + i] * z[jb + i];
            z[j] -= sacc;
        }
        __syncthreads();
    }
    for (int j = tid; j < k3; j += kT) xsol[3 * (int64_t)S.c0 + j] = z[j];
}

template <typename T>
int dalloc_copy(T** d, const std::vector<T>& h) {
    const size_t n = std::max<size_t>(h.size(), 1);
    if (hipMalloc(reinterpret_cast<void**>(d), n * sizeof(T)) != hipSuccess) return DPG_ERR_HIP;
    if (!h.empty() && hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
        return DPG_ERR_HIP;
    return DPG_OK;
}

struct CholDev {
    dpg_chol_sym sym;
    int64_t n = 0;
    SnDev* sns = nullptr;
    OEnt* omap = nullptr;
    int32_t* child_list = nullptr;
    int32_t* relmap = nullptr;
    int32_t* rows = nullptr;
    int32_t* level_list = nullptr;
    int32_t* perm = nullptr;
    int32_t* pos = nullptr;
    double* fronts = nullptr;
    double* acc = nullptr;
    double* ysol = nullptr;
    double* xsol = nullptr;
    int32_t* status = nullptr;
    std::vector<int32_t> level_ptr;
    std::vector<size_t> lds_factor, lds_solve;   // per level
    int64_t nnzb_upper = 0;
};

}  // namespace

extern "C" void dpg_chol_destroy(void* h) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    if (!c) return;
    void* ptrs[] = {c->sns, c->omap, c->child_list, c->relmap, c->rows, c->level_list, c->perm, c->pos,
                    c->fronts, c->acc, c->ysol, c->xsol, c->status};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete c;
}

extern "C" int dpg_chol_create(void** out, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi,
                               int64_t n_pairs) {
    *out = nullptr;
    CholDev* c = new CholDev();
    dpg_chol_opts o{64, 0.3};
    if (dpg_chol_symbolic(n, pair_lo, pair_hi, n_pairs, &o, &c->sym)) {
        delete c;
        return DPG_ERR_NUMERIC;
    }
    const dpg_chol_sym& S = c->sym;
    c->n = n;
    c->nnzb_upper = n + n_pairs;
    // omap: every upper block of H -> (front, local block row, local block col, transpose)
    std::vector<std::vector<OEnt>> per((size_t)S.ns);
    auto local_index = [&](int32_t s, int32_t p) -> int32_t {
        const int32_t c0 = S.sn_c0[(size_t)s], k = S.sn_c0[(size_t)s + 1] - c0;
        if (p >= c0 && p < c0 + k) return p - c0;
        const int32_t* b = S.sn_rows.data() + S.sn_rows_ptr[(size_t)s];
        const int32_t* e = S.sn_rows.data() + S.sn_rows_ptr[(size_t)s + 1];
        const int32_t* it = std::lower_bound(b, e, p);
        if (it == e || *it != p) return -1;
        return k + (int32_t)(it - b);
    };
    for (int64_t v = 0; v < n; ++v) {
        const int32_t p = S.pos[(size_t)v], s = S.sn_of[(size_t)p];
        const int32_t l = local_index(s, p);
        per[(size_t)s].push_back(OEnt{(int32_t)v, (int16_t)l, (int16_t)l, 0, 0});
    }
    for (int64_t q = 0; q < n_pairs; ++q) {
        const int32_t lo = pair_lo[q], hi = pair_hi[q];
        const int32_t plo = S.pos[(size_t)lo], phi = S.pos[(size_t)hi];
        const int32_t later = plo > phi ? plo : phi, earlier = plo > phi ? phi : plo;
        const int32_t s = S.sn_of[(size_t)earlier];
        const int32_t a = local_index(s, later), b = local_index(s, earlier);
        if (a < 0 || b < 0) { delete c; return DPG_ERR_NUMERIC; }
        // front wants A(later, earlier) = H(later_node, earlier_node); hb holds H(lo, hi)
        per[(size_t)s].push_back(OEnt{(int32_t)(n + q), (int16_t)a, (int16_t)b, plo > phi ? 0 : 1, 0});
    }
    std::vector<OEnt> omap;
    std::vector<SnDev> sns((size_t)S.ns);
    int64_t acc_total = 0;
    for (int32_t s = 0; s < S.ns; ++s) {
        SnDev& d = sns[(size_t)s];
        d.c0 = S.sn_c0[(size_t)s];
        d.k = S.sn_c0[(size_t)s + 1] - d.c0;
        d.r = (int32_t)(S.sn_rows_ptr[(size_t)s + 1] - S.sn_rows_ptr[(size_t)s]);
        d.nchild = (int32_t)(S.child_ptr[(size_t)s + 1] - S.child_ptr[(size_t)s]);
        d.front_off = S.front_off[(size_t)s];
        d.rows_off = S.sn_rows_ptr[(size_t)s];
        d.child_off = S.child_ptr[(size_t)s];
        d.omap_off = (int64_t)omap.size();
        d.omap_n = (int32_t)per[(size_t)s].size();
        d.acc_off = acc_total;
        d.pad = 0;
        acc_total += 3 * d.r;
        omap.insert(omap.end(), per[(size_t)s].begin(), per[(size_t)s].end());
    }
    c->level_ptr = S.level_ptr;
    c->lds_factor.assign((size_t)S.n_levels, 0);
    c->lds_solve.assign((size_t)S.n_levels, 0);
    for (int32_t l = 0; l < S.n_levels; ++l) {
        size_t mf = 0, ms = 0;
        for (int32_t q = S.level_ptr[(size_t)l]; q < S.level_ptr[(size_t)l + 1]; ++q) {
            const SnDev& d = sns[(size_t)S.level_list[(size_t)q]];
            mf = std::max(mf, (size_t)(3 * (d.k + d.r)) * kNB * sizeof(double));
            ms = std::max(ms, (size_t)(kSB * kSB + 3 * (d.k + d.r)) * sizeof(double));
        }
        c->lds_factor[(size_t)l] = mf;
        c->lds_solve[(size_t)l] = ms;
        if (mf > 160 * 1024 || ms > 160 * 1024) { dpg_chol_destroy(c); return DPG_ERR_SIZE; }
    }
    int rc = 0;
    rc |= dalloc_copy(&c->sns, sns);
    rc |= dalloc_copy(&c->omap, omap);
    rc |= dalloc_copy(&c->child_list, S.child_list);
    rc |= dalloc_copy(&c->relmap, S.relmap);
    rc |= dalloc_copy(&c->rows, S.sn_rows);
    rc |= dalloc_copy(&c->level_list, S.level_list);
    rc |= dalloc_copy(&c->perm, S.perm);
    rc |= dalloc_copy(&c->pos, S.pos);
    rc |= hipMalloc(reinterpret_cast<void**>(&c->fronts), std::max<size_t>((size_t)S.front_off[(size_t)S.ns], 1) * 8) != hipSuccess;
    rc |= hipMalloc(reinterpret_cast<void**>(&c->acc), std::max<size_t>((size_t)acc_total, 1) * 8) != hipSuccess;
    rc |= hipMalloc(reinterpret_cast<void**>(&c->ysol), (size_t)(3 * n) * 8) != hipSuccess;
    rc |= hipMalloc(reinterpret_cast<void**>(&c->xsol), (size_t)(3 * n) * 8) != hipSuccess;
    rc |= hipMalloc(reinterpret_cast<void**>(&c->status), sizeof(int32_t)) != hipSuccess;
    if (rc) { dpg_chol_destroy(c); return DPG_ERR_HIP; }
    *out = c;
    return DPG_OK;
}

extern "C" int dpg_chol_solve(void* h, const double* hb, void* stream) {
    CholDev* c = reinterpret_cast<CholDev*>(h);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dpg_chol_sym& S = c->sym;
    const double* g = hb + 9 * c->nnzb_upper;
    if (hipMemsetAsync(c->status, 0, sizeof(int32_t), st) != hipSuccess) return DPG_ERR_HIP;
    for (int32_t l = 0; l < S.n_levels; ++l) {
        const int32_t b = c->level_ptr[(size_t)l], cnt = c->level_ptr[(size_t)l + 1] - b;
        hipLaunchKernelGGL(chol_factor_level, dim3(cnt), dim3(kT), c->lds_factor[(size_t)l], st, c->level_list + b,
                           c->sns, c->omap, hb, c->child_list, c->relmap, c->fronts, c->status);
    }
    for (int32_t l = 0; l < S.n_levels; ++l) {
        const int32_t b = c->level_ptr[(size_t)l], cnt = c->level_ptr[(size_t)l + 1] - b;
        hipLaunchKernelGGL(chol_forward_level, dim3(cnt), dim3(kT), c->lds_solve[(size_t)l], st, c->level_list + b,
                           c->sns, c->child_list, c->relmap, c->fronts, g, c->perm, c->ysol, c->acc);
    }
    for (int32_t l = S.n_levels - 1; l >= 0; --l) {
        const int32_t b = c->level_ptr[(size_t)l], cnt = c->level_ptr[(size_t)l + 1] - b;
        hipLaunchKernelGGL(chol_backward_level, dim3(cnt), dim3(kT), c->lds_solve[(size_t)l], st, c->level_list + b,
                           c->sns, c->rows, c->fronts, c->ysol, c->xsol);
    }
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
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
