// chol_analyze.cpp -- host-only: symbolic analysis statistics of a pose-graph pattern (per level:
// fronts, largest front, flops; the elimination tree's critical path in flops).
// usage: chol_analyze PAIRS.bin [max_cols relax]
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include "../dpg-slam_amd/csrc/dpg_chol.h"

int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    int64_t n = 0, P = 0;
    if (!f || fread(&n, 8, 1, f) != 1 || fread(&P, 8, 1, f) != 1) return 2;
    std::vector<int32_t> lo((size_t)P), hi((size_t)P);
    if (fread(lo.data(), 4, (size_t)P, f) != (size_t)P || fread(hi.data(), 4, (size_t)P, f) != (size_t)P) return 2;
    dpg_chol_opts o{argc > 2 ? atoi(argv[2]) : 64, argc > 3 ? atof(argv[3]) : 0.3};
    dpg_chol_sym S;
    if (dpg_chol_symbolic(n, lo.data(), hi.data(), P, &o, &S)) return 3;
    std::vector<double> fl((size_t)S.ns), cp((size_t)S.ns, 0.0);
    int64_t nnzL = 0;
    for (int s = 0; s < S.ns; ++s) {
        const double k = 3.0 * (S.sn_c0[s + 1] - S.sn_c0[s]), r = 3.0 * (S.sn_rows_ptr[s + 1] - S.sn_rows_ptr[s]);
        fl[s] = k * k * k / 3 + k * k * r + k * r * r;
        nnzL += (int64_t)(k * (k + 1) / 2 + k * r);
    }
    double crit = 0, crit_us = 0;
    std::vector<double> cl((size_t)S.ns, 0.0);
    for (int s = 0; s < S.ns; ++s) {   // children precede parents
        cp[s] += fl[s];
        if (S.sn_parent[s] >= 0) cp[S.sn_parent[s]] = std::max(cp[S.sn_parent[s]], cp[s]);
        else crit = std::max(crit, cp[s]);
        // latency model of the DAG kernel: LDS small front ~3 us, team front ~8 us + 25 us per 24-col panel
        const int k3 = 3 * (S.sn_c0[s + 1] - S.sn_c0[s]), m3 = k3 + 3 * (int)(S.sn_rows_ptr[s + 1] - S.sn_rows_ptr[s]);
        cl[s] += m3 <= 96 ? 3.0 : 8.0 + 25.0 * ((k3 + 23) / 24);
        if (S.sn_parent[s] >= 0) cl[S.sn_parent[s]] = std::max(cl[S.sn_parent[s]], cl[s]);
        else crit_us = std::max(crit_us, cl[s]);
    }
    printf("latency-model critical path %.0f us\n", crit_us);
    printf("n=%lld ns=%d levels=%d max_front=%d flops=%.3g nnzL=%lld fronts=%.1f MB crit_path_flops=%.3g\n",
           (long long)n, S.ns, S.n_levels, S.max_front, S.flops, (long long)nnzL, S.front_off[S.ns] * 8e-6, crit);
    {
        const int edges[] = {24, 48, 64, 96, 128, 160, 192, 256, 320, 100000};
        int cnt[10] = {0};
        double fl_b[10] = {0};
        for (int s = 0; s < S.ns; ++s) {
            const int m3 = 3 * (S.sn_c0[s + 1] - S.sn_c0[s] + (int)(S.sn_rows_ptr[s + 1] - S.sn_rows_ptr[s]));
            int b = 0;
            while (m3 > edges[b]) ++b;
            ++cnt[b]; fl_b[b] += fl[s];
        }
        int nch_hist[6] = {0};
        for (int s = 0; s < S.ns; ++s) {
            const int m3 = 3 * (S.sn_c0[s + 1] - S.sn_c0[s] + (int)(S.sn_rows_ptr[s + 1] - S.sn_rows_ptr[s]));
            if (m3 > 96) continue;
            const int64_t nc = S.child_ptr[s + 1] - S.child_ptr[s];
            nch_hist[nc == 0 ? 0 : nc <= 2 ? 1 : nc <= 4 ? 2 : nc <= 8 ? 3 : nc <= 16 ? 4 : 5]++;
        }
        printf("small-front children: 0:%d <=2:%d <=4:%d <=8:%d <=16:%d >16:%d\n", nch_hist[0], nch_hist[1], nch_hist[2], nch_hist[3], nch_hist[4], nch_hist[5]);
        printf("m3 histogram:");
        for (int b = 0; b < 10; ++b) printf(" <=%d:%d(%.2g)", edges[b], cnt[b], fl_b[b]);
        printf("\n");
    }
    for (int l = 0; l < S.n_levels; ++l) {
        int cnt = 0, mk = 0, mm = 0; double lf = 0, mf = 0;
        for (int q = S.level_ptr[l]; q < S.level_ptr[l + 1]; ++q) {
            int s = S.level_list[q]; ++cnt;
            int k = S.sn_c0[s + 1] - S.sn_c0[s], r = (int)(S.sn_rows_ptr[s + 1] - S.sn_rows_ptr[s]);
            mk = std::max(mk, 3 * k); mm = std::max(mm, 3 * (k + r)); lf += fl[s]; mf = std::max(mf, fl[s]);
        }
        printf("L%2d fronts=%5d max_k3=%4d max_m3=%4d flops=%.3g max_front_flops=%.3g\n", l, cnt, mk, mm, lf, mf);
    }
    return 0;
}
