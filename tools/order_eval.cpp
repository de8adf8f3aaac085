// order_eval.cpp -- compare fill-reducing orders for the GPU Cholesky on a pose graph (host only):
// minimum degree vs nested dissection (several leaf sizes).  For each: fill (blocks), factor Mflop,
// supernodes, elimination-tree levels, largest front and the critical-path estimate the fused DAG
// factorization schedules by (dpg_chol.hip chol_plan: 4 + 0.06 m3 + 0.9 k3 us for a small front, 10 + 20 us
// per 24-column panel for a large one, summed along the longest leaf-to-root path), plus the
// ordering time.
// usage: order_eval PAIRS.bin        (int32 n, int32 P, then P x (lo, hi))
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <algorithm>
#include <vector>

#include "../dpg-slam_amd/csrc/dpg_chol.h"

static double now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

static void report(const char* name, double ms, const dpg_chol_sym& S) {
    int64_t nnz = 0;
    for (int32_t s = 0; s < S.ns; ++s) {
        const int64_t k = S.sn_c0[(size_t)s + 1] - S.sn_c0[(size_t)s], r = S.sn_rows_ptr[(size_t)s + 1] - S.sn_rows_ptr[(size_t)s];
        nnz += k * (k - 1) / 2 + k * r;
    }
    std::vector<double> cp((size_t)S.ns, 0.0);
    double crit = 0.0, work = 0.0;
    for (int32_t s = S.ns - 1; s >= 0; --s) {   // parents after children: walk down from the roots
        const int32_t k = S.sn_c0[(size_t)s + 1] - S.sn_c0[(size_t)s];
        const int32_t r = (int32_t)(S.sn_rows_ptr[(size_t)s + 1] - S.sn_rows_ptr[(size_t)s]);
        const int32_t nch = (int32_t)(S.child_ptr[(size_t)s + 1] - S.child_ptr[(size_t)s]);
        const int32_t m3 = 3 * (k + r);
        const double est = (m3 <= 96 && nch <= 8) ? 4.0 + 0.06 * m3 + 0.9 * (3 * k) : 10.0 + 20.0 * ((3 * k + 23) / 24);
        const int32_t p = S.sn_parent[(size_t)s];
        cp[(size_t)s] = est + (p >= 0 ? cp[(size_t)p] : 0.0);
        crit = std::max(crit, cp[(size_t)s]);
        work += est;
    }
    printf("%-10s order %8.2f ms | fill %8lld blocks, %8.1f Mflop, %5d supernodes, %4d levels, max front %4d | "
           "critical path ~%7.0f us, work ~%8.0f us\n",
           name, ms, (long long)nnz, S.flops * 1e-6, S.ns, S.n_levels, S.max_front, crit, work);
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t n, P;
    if (fread(&n, 4, 1, f) != 1 || fread(&P, 4, 1, f) != 1) return 2;
    std::vector<int32_t> lo((size_t)P), hi((size_t)P);
    for (int32_t q = 0; q < P; ++q)
        if (fread(&lo[(size_t)q], 4, 1, f) != 1 || fread(&hi[(size_t)q], 4, 1, f) != 1) return 2;
    fclose(f);
    printf("graph: %d nodes, %d pairs\n", n, P);
    dpg_chol_opts o{64, 0.3};
    {
        std::vector<int32_t> perm;
        std::vector<std::vector<int32_t>> pat;
        const double t = now_ms();
        dpg_chol_order(n, lo.data(), hi.data(), P, perm, pat);
        const double ms = now_ms() - t;
        dpg_chol_sym S;
        dpg_chol_sym_from_patterns(n, perm, pat, &o, &S);
        report("min-degree", ms, S);
    }
    for (int k = 0; k < 4; ++k) {   // the batch analysis' candidates (dpg_chol_symbolic picks the shortest path)
        static const int prm[4][3] = {{0, 5, 0}, {2, 4, 2}, {8, 4, 2}, {4, 5, 1}};
        std::vector<int32_t> perm;
        std::vector<std::vector<int32_t>> pat;
        const double t = now_ms();
        if (dpg_chol_order_nd_sep(n, lo.data(), hi.data(), P, 16, prm[k][0], prm[k][1], prm[k][2], k > 0, perm, pat)) return 3;
        const double ms = now_ms() - t;
        dpg_chol_sym S;
        if (dpg_chol_sym_from_patterns(n, perm, pat, &o, &S)) return 4;
        char name[32];
        snprintf(name, sizeof(name), "sep/%d", k);
        report(name, ms, S);
    }
    {
        const double t = now_ms();
        dpg_chol_sym S;
        if (dpg_chol_symbolic(n, lo.data(), hi.data(), P, &o, &S)) return 5;
        report("batch-pick", now_ms() - t, S);
    }
    for (int leaf : {32, 64, 128, 256, 512}) {
        std::vector<int32_t> perm;
        std::vector<std::vector<int32_t>> pat;
        const double t = now_ms();
        if (dpg_chol_order_nd(n, lo.data(), hi.data(), P, leaf, perm, pat)) return 3;
        const double ms = now_ms() - t;
        dpg_chol_sym S;
        if (dpg_chol_sym_from_patterns(n, perm, pat, &o, &S)) return 4;
        char name[32];
        snprintf(name, sizeof(name), "nd/%d", leaf);
        report(name, ms, S);
    }
    return 0;
}
