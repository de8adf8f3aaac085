// chol_bench.cpp -- standalone timing + residual check of the GPU supernodal Cholesky
// (dpg_chol_create / dpg_chol_solve in libdpg.so) on a pose-graph sparsity pattern.
// The system is a random SPD matrix with that pattern (diagonally dominant), not a GN system.
// usage: chol_bench PAIRS.bin [iters]   (PAIRS.bin: int64 n, int64 P, int32 lo[P], int32 hi[P])
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "../dpg-slam_amd/csrc/dpg_chol.h"

extern "C" {
int dpg_chol_create(void** chol, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                    const dpg_chol_opts* opts);
void dpg_chol_destroy(void* chol);
int dpg_chol_solve(void* chol, const double* hb, void* stream);
int dpg_chol_resolve(void* chol, const double* hb, void* stream);
const int32_t* dpg_chol_pos_dev(void* chol);
const double* dpg_chol_x_dev(void* chol);
const int32_t* dpg_chol_status_dev(void* chol);
void dpg_chol_stats(void* chol, double out[6]);
#ifdef DPG_CHOL_TIMING
int dpg_chol_prof_dump(unsigned long long* out, int n, unsigned long long* span);
int dpg_chol_prof_reset(void);
int dpg_chol_front_dump(unsigned long long* out, int n);
int dpg_chol_bwd_dump(unsigned long long* out, int n);
int dpg_chol_panel_dump(unsigned long long* out, int n);
int dpg_chol_steps_dump(unsigned long long* out, int n);
void dpg_chol_tree(void* h, int32_t* parent, int32_t* m3, int32_t* k3);
#endif
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s PAIRS.bin [iters] [solve_inv_cols]\n", argv[0]);
        return 2;
    }
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int64_t n = 0, P = 0;
    if (fread(&n, 8, 1, f) != 1 || fread(&P, 8, 1, f) != 1) return 2;
    std::vector<int32_t> lo((size_t)P), hi((size_t)P);
    if (fread(lo.data(), 4, (size_t)P, f) != (size_t)P || fread(hi.data(), 4, (size_t)P, f) != (size_t)P) return 2;
    fclose(f);
    // hb: [9 (n + P) upper blocks | 3n g | chi2 | pad]
    const int64_t nb = n + P;
    std::vector<double> hb((size_t)(9 * nb + 3 * n + 2), 0.0);
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::vector<double> rowsum((size_t)(3 * n), 0.0);
    for (int64_t q = 0; q < P; ++q) {
        double* B = hb.data() + 9 * (n + q);
        for (int e = 0; e < 9; ++e) {
            B[e] = U(rng);
            rowsum[(size_t)(3 * lo[(size_t)q] + e / 3)] += fabs(B[e]);
            rowsum[(size_t)(3 * hi[(size_t)q] + e % 3)] += fabs(B[e]);
        }
    }
    for (int64_t v = 0; v < n; ++v) {
        double* D = hb.data() + 9 * v;
        for (int a = 0; a < 3; ++a)
            for (int b = a; b < 3; ++b) {
                const double x = 0.1 * U(rng);
                D[3 * a + b] = x;
                D[3 * b + a] = x;
            }
        for (int a = 0; a < 3; ++a) D[4 * a] = rowsum[(size_t)(3 * v + a)] + 1.0;
    }
    double* g = hb.data() + 9 * nb;
    for (int64_t t = 0; t < 3 * n; ++t) g[t] = U(rng);

    void* ch = nullptr;
    dpg_chol_opts co;
    if (argc > 3) co.solve_inv_cols = atoi(argv[3]);
    int rc = dpg_chol_create(&ch, n, lo.data(), hi.data(), P, &co);
    if (rc) {
        fprintf(stderr, "dpg_chol_create failed %d\n", rc);
        return 1;
    }
    double st[6];
    dpg_chol_stats(ch, st);
    double* d_hb = nullptr;
    CK(hipMalloc(&d_hb, hb.size() * 8));
    CK(hipMemcpy(d_hb, hb.data(), hb.size() * 8, hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w)
        if (dpg_chol_solve(ch, d_hb, s)) return 1;
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int it = 0; it < iters; ++it)
        if (dpg_chol_solve(ch, d_hb, s)) return 1;
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // forward + backward solves alone with the factor of the last solve (the chord steps of GN)
    float ms_re = 0.f;
    CK(hipEventRecord(e0, s));
    for (int it = 0; it < iters; ++it)
        if (dpg_chol_resolve(ch, d_hb, s)) return 1;
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms_re, e0, e1));
    std::vector<double> x((size_t)(3 * n));
    std::vector<int32_t> pos((size_t)n);
    int32_t status = 0;
    CK(hipMemcpy(x.data(), dpg_chol_x_dev(ch), x.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(pos.data(), dpg_chol_pos_dev(ch), pos.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&status, dpg_chol_status_dev(ch), 4, hipMemcpyDeviceToHost));
    // residual of H x = -g, x in node order
    std::vector<double> xn((size_t)(3 * n)), r((size_t)(3 * n));
    for (int64_t v = 0; v < n; ++v)
        for (int a = 0; a < 3; ++a) xn[(size_t)(3 * v + a)] = x[(size_t)(3 * pos[(size_t)v] + a)];
    for (int64_t t = 0; t < 3 * n; ++t) r[(size_t)t] = g[t];
    for (int64_t v = 0; v < n; ++v) {
        const double* D = hb.data() + 9 * v;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) r[(size_t)(3 * v + a)] += D[3 * a + b] * xn[(size_t)(3 * v + b)];
    }
    for (int64_t q = 0; q < P; ++q) {
        const double* B = hb.data() + 9 * (n + q);
        const int64_t i = lo[(size_t)q], j = hi[(size_t)q];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                r[(size_t)(3 * i + a)] += B[3 * a + b] * xn[(size_t)(3 * j + b)];
                r[(size_t)(3 * j + b)] += B[3 * a + b] * xn[(size_t)(3 * i + a)];
            }
    }
    double rmax = 0.0, gmax = 0.0;
    for (int64_t t = 0; t < 3 * n; ++t) {
        rmax = fmax(rmax, fabs(r[(size_t)t]));
        gmax = fmax(gmax, fabs(g[t]));
    }
    printf("{\"n\": %lld, \"pairs\": %lld, \"supernodes\": %.0f, \"levels\": %.0f, \"max_front\": %.0f, "
           "\"mflop\": %.1f, \"ms_per_solve\": %.4f, \"ms_per_resolve\": %.4f, \"residual_rel\": %.3e, \"status\": %d}\n",
           (long long)n, (long long)P, st[0], st[1], st[2], st[3] / 1e6, ms / iters, ms_re / iters, rmax / gmax, status);
#ifdef DPG_CHOL_TIMING
    {
        // fused path: per-front stamps of the last solve -> the critical path through the tree
        const int ns = (int)st[0];
        std::vector<unsigned long long> fm((size_t)ns * 8, 0ull);
        if (dpg_chol_prof_reset()) return 1;
        if (dpg_chol_solve(ch, d_hb, s)) return 1;
        CK(hipStreamSynchronize(s));
        std::vector<int32_t> par((size_t)ns), m3v((size_t)ns), k3v((size_t)ns);
        dpg_chol_tree(ch, par.data(), m3v.data(), k3v.data());
        if (dpg_chol_front_dump(fm.data(), ns) == 0 && fm[4] != 0) {
            unsigned long long t0 = ~0ull, t1 = 0;
            int root = -1;
            for (int q = 0; q < ns; ++q) {
                t0 = std::min(t0, fm[(size_t)q * 8]);
                if (fm[(size_t)q * 8 + 4] > t1) { t1 = fm[(size_t)q * 8 + 4]; root = q; }
            }
            printf("fused factor span %.1f us (last front %d)\n", (t1 - t0) / 100.0, root);
            double sw = 0, sa = 0, sf = 0, so = 0, sl = 0;
            int depth = 0;
            std::vector<int> crit;
            for (int q = root; q >= 0;) {
                crit.push_back(q);
                const unsigned long long* m = fm.data() + (size_t)q * 8;
                int last = -1;
                for (int c = 0; c < ns; ++c)
                    if (par[(size_t)c] == q && (last < 0 || fm[(size_t)c * 8 + 4] > fm[(size_t)last * 8 + 4])) last = c;
                const double lat = last >= 0 ? ((double)m[1] - (double)fm[(size_t)last * 8 + 4]) / 100.0 : 0.0;
                // large fronts: stamp 3 is the right-hand side owner's (a helper), stamp 4 the chain's
                const double out = m[4] >= m[3] ? (m[4] - m[3]) / 100.0 : 0.0;
                const double fac = ((double)(m[4] >= m[3] ? m[3] : m[4]) - (double)m[2]) / 100.0;
                printf("  front %5d m3 %3d k3 %3d | claim %8.2f wait %7.2f (signal->ready %5.2f) asm %6.2f factor %7.2f out %6.2f\n", q,
                       m3v[(size_t)q], k3v[(size_t)q], (m[0] - t0) / 100.0, ((double)m[1] - (double)m[0]) / 100.0, lat,
                       (m[2] - m[1]) / 100.0, fac, out);
                sw += lat; sa += (m[2] - m[1]) / 100.0; sf += fac; so += out;
                sl += 0; ++depth;
                q = last;
            }
            std::vector<unsigned long long> pm((size_t)ns * 16 * 8, 0ull);
            if (dpg_chol_panel_dump(pm.data(), ns) == 0) {
                for (int q : crit) {
                    if (k3v[(size_t)q] <= 24) continue;
                    printf("  panels of front %d (k3 %d):", q, k3v[(size_t)q]);
                    for (int pp = 0; pp < 16; ++pp) {
                        const unsigned long long* m = pm.data() + ((size_t)q * 16 + pp) * 8;
                        if (!m[4]) continue;
                        printf(" [p%d pub %.1f", pp, ((double)m[4] - (double)t0) / 100.0);
                        if (m[0]) printf(" wake->ld %.1f upd %.1f fac %.1f (ld %.1f potrf %.1f trsm %.1f) pub %.1f", ((double)m[1] - (double)m[0]) / 100.0,
                                         ((double)m[2] - (double)m[1]) / 100.0, ((double)m[3] - (double)m[2]) / 100.0,
                                         ((double)m[5] - (double)m[2]) / 100.0, ((double)m[6] - (double)m[5]) / 100.0,
                                         ((double)m[7] - (double)m[6]) / 100.0, ((double)m[4] - (double)m[3]) / 100.0);
                        printf("]");
                    }
                    printf("\n");
                }
            }
            printf("critical path: %d fronts, hand-off %.1f + assembly %.1f + factor %.1f + out %.1f us\n", depth, sw, sa, sf, so);
        }
        std::vector<unsigned long long> bm((size_t)ns * 8, 0ull), sm2((size_t)ns * 16 * 8, 0ull);
        if (dpg_chol_bwd_dump(bm.data(), ns) == 0 && bm[4] != 0) {
            // backward: the last front to finish, then its parents up to the root
            unsigned long long t0 = ~0ull, t1 = 0;
            int last = -1;
            for (int q = 0; q < ns; ++q) {
                t0 = std::min(t0, bm[(size_t)q * 8]);
                if (bm[(size_t)q * 8 + 4] > t1) { t1 = bm[(size_t)q * 8 + 4]; last = q; }
            }
            printf("backward span %.1f us (last front %d)\n", (t1 - t0) / 100.0, last);
            double sw = 0, sz = 0, sd = 0, so = 0;
            int depth = 0;
            for (int q = last; q >= 0; q = par[(size_t)q]) {
                const unsigned long long* m = bm.data() + (size_t)q * 8;
                const int pq = par[(size_t)q];
                const double lat = pq >= 0 ? ((double)m[1] - (double)bm[(size_t)pq * 8 + 4]) / 100.0 : 0.0;
                printf("  bwd front %5d m3 %3d k3 %3d | claim %8.2f wait %7.2f (parent->ready %5.2f) z %6.2f diag %6.2f out %6.2f\n", q,
                       m3v[(size_t)q], k3v[(size_t)q], (m[0] - t0) / 100.0, ((double)m[1] - (double)m[0]) / 100.0, lat,
                       (m[2] - m[1]) / 100.0, (m[3] - m[2]) / 100.0, (m[4] - m[3]) / 100.0);
                sw += lat; sz += (m[2] - m[1]) / 100.0; sd += (m[3] - m[2]) / 100.0; so += (m[4] - m[3]) / 100.0;
                if (k3v[(size_t)q] > 24 && dpg_chol_steps_dump(sm2.data(), ns) == 0) {   // per diagonal block: load, chain, column dots
                    printf("      diag blocks:");
                    for (int b = 3; b >= 0; --b) {
                        const unsigned long long* d = sm2.data() + ((size_t)q * 16 + 8 + b) * 8;
                        if (b * 64 >= k3v[(size_t)q] || !d[3]) continue;
                        printf(" [b%d load %.2f chain %.2f dots %.2f]", b, ((double)d[1] - (double)d[0]) / 100.0,
                               ((double)d[2] - (double)d[1]) / 100.0, ((double)d[3] - (double)d[2]) / 100.0);
                    }
                    printf("\n");
                }
                ++depth;
            }
            printf("backward critical path: %d fronts, hand-off %.1f + z %.1f + diag %.1f + out %.1f us\n", depth, sw, sz, sd, so);
        }
    }
    {
        // phase marks of workgroup 0 of every factor launch of the last solve (10 ns ticks)
        const int slots = 40, nl = 512, nw = 2048;
        std::vector<unsigned long long> pr((size_t)slots * 4096, 0ull), span((size_t)nl * nw * 2);
        if (dpg_chol_prof_reset()) return 1;
        if (dpg_chol_solve(ch, d_hb, s)) return 1;
        CK(hipStreamSynchronize(s));
        if (dpg_chol_prof_dump(pr.data(), slots * 4096, span.data()) == 0) {
            unsigned long long prev_end = 0;
            double tot = 0.0;
            for (int l = 0; l < nl; ++l) {
                const unsigned long long* m = pr.data() + (size_t)l * slots;
                if (!m[0]) break;
                unsigned long long smin = ~0ull, smax = 0, emax = 0;
                int nwg = 0, slow = 0;
                double dmax = 0.0;
                for (int b = 0; b < nw; ++b) {
                    const unsigned long long s0 = span[((size_t)l * nw + b) * 2], e0 = span[((size_t)l * nw + b) * 2 + 1];
                    if (!s0) break;
                    ++nwg;
                    smin = s0 < smin ? s0 : smin;
                    smax = s0 > smax ? s0 : smax;
                    emax = e0 > emax ? e0 : emax;
                    if ((double)(e0 - s0) > dmax) { dmax = (double)(e0 - s0); slow = b; }
                }
                unsigned long long last = m[0];
                printf("L%03d gap %5.2f span %6.2f wgs %4d last-start %6.2f slowest wg %4d %6.2f | wg0:", l,
                       prev_end ? ((double)smin - (double)prev_end) / 100.0 : 0.0, (double)(emax - smin) / 100.0, nwg,
                       (double)(smax - smin) / 100.0, slow, dmax / 100.0);
                tot += (double)(emax - smin) / 100.0;
                for (int k = 1; k < slots; ++k)
                    if (m[k]) {
                        printf(" %d:%.2f", k, (double)(m[k] - last) / 100.0);
                        last = m[k];
                    }
                printf("\n");
                prev_end = emax;
            }
            printf("sum of spans %.1f us\n", tot);
        }
    }
#endif
    dpg_chol_destroy(ch);
    return (rmax / gmax < 1e-9 && status == 0) ? 0 : 3;
}
