// incsym_bench.cpp -- CPU timing of the incremental path's host symbolic work per update
// (dpg_inc_update, dpg-slam_amd/csrc/dpg_inc.hip: ordering kept/extended or refreshed every 64
// nodes, the derived structures, the GPU solver's host plan) on a recorded arrival sequence
// (tools/dump_inc_edges.py).  No device calls.
// usage: incsym_bench EDGES.bin [TAIL]   prints mean ms per part over the last TAIL updates
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <algorithm>
#include <vector>

#include "../dpg-slam_amd/csrc/dpg_chol.h"

#ifdef DPG_PLAN_TIMING
extern double dpg_plan_t_export[8];
extern double dpg_csr_t[8];
#endif
static double now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: incsym_bench EDGES.bin [TAIL]\n"); return 2; }
    const int tail = argc > 2 ? atoi(argv[2]) : 500;
    const int every = argc > 3 ? atoi(argv[3]) : 64;
    const double grow = argc > 4 ? atof(argv[4]) : 1.5;
    double flops = 0, maxf = 0, levels = 0, crit_sum = 0;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<int32_t> buf;
    int32_t x;
    while (fread(&x, 4, 1, f) == 1) buf.push_back(x);
    fclose(f);
    size_t at = 0;
    const int V = buf[at++];
    std::vector<std::vector<std::pair<int32_t, int32_t>>> by((size_t)V);
    for (int v = 0; v < V; ++v) {
        const int c = buf[at++];
        for (int k = 0; k < c; ++k, at += 2) by[(size_t)v].emplace_back(buf[at], buf[at + 1]);
    }
    dpg_chol_incsym I;
    dpg_chol_sym S;
    dpg_chol_opts o{64, 0.3};
    std::vector<int32_t> plo, phi;
    int64_t V_at = 0, nnz_at = 0;
    double acc[4] = {0, 0, 0, 0};
    int cnt = 0, reorders = 0;
    double t_reset = 0, t_order = 0, pt0[8] = {0}, ct0[8] = {0};
    for (int v = 0; v < V; ++v) {
        const int64_t V1 = v + 1;
#ifdef DPG_PLAN_TIMING
        if (v == V - tail) for (int k = 0; k < 8; ++k) { pt0[k] = dpg_plan_t_export[k]; ct0[k] = dpg_csr_t[k]; }
#endif
        if (I.n > 0) dpg_incsym_append(&I, 1);
        for (auto& e : by[(size_t)v]) { plo.push_back(e.first); phi.push_back(e.second); }
        const double t0 = now_ms();
        bool re = false;
        const double expect = V_at > 0 ? (double)nnz_at * (double)V1 / (double)V_at : 0.0;
        if (I.n == 0 || V1 - V_at >= every) re = true;
        else {
            for (auto& e : by[(size_t)v]) dpg_incsym_add_edge(&I, e.first, e.second);
            if ((double)I.nnz > grow * expect + 64.0) re = true;
        }
        if (re) {
            const double tr = now_ms();
            if (dpg_incsym_reset(&I, V1, plo.data(), phi.data(), (int64_t)plo.size())) return 3;
            V_at = V1;
            nnz_at = I.nnz;
            ++reorders;
            if (v >= V - tail) {
                t_reset += now_ms() - tr;
                std::vector<int32_t> pm;
                std::vector<std::vector<int32_t>> pt;
                const double to = now_ms();
                dpg_chol_order(V1, plo.data(), phi.data(), (int64_t)plo.size(), pm, pt);
                t_order += now_ms() - to;
            }
        }
        const double t1 = now_ms();
        if (dpg_incsym_derive(&I, &o, &S)) return 4;
        const double t2 = now_ms();
        if (v >= V - tail) {   // the derive split: pattern extraction alone
            const double te = now_ms();
            static std::vector<int64_t> cp;
            static std::vector<int32_t> rows;
            const int64_t n = I.n, nw = (n + 63) / 64;
            cp.resize((size_t)n + 1);
            rows.clear();
            cp[0] = 0;
            for (int64_t p = 0; p < n; ++p) {
                const uint64_t* row = &I.bits[(size_t)(p * I.words)];
                for (int64_t w = (p + 1) / 64; w < nw; ++w) {
                    uint64_t m = row[w];
                    while (m) { rows.push_back((int32_t)(w * 64 + __builtin_ctzll(m))); m &= m - 1; }
                }
                cp[(size_t)p + 1] = (int64_t)rows.size();
            }
            (void)te;
            static dpg_chol_sym S2;
            const double tf = now_ms();
            dpg_chol_sym_from_csr(n, I.perm.data(), cp.data(), rows.data(), &o, &S2);
            acc[3] += now_ms() - tf;
        }
#ifdef DPG_PLAN_VERIFY
        // the incremental prepare builds the plan's H-block buckets from I's order beside the
        // derivation (dpg_chol_plan_blocks): that order must be the one the analysis carries, and
        // the plan checks the prebuilt buckets against its own (every 50th update: host only)
        if (I.perm != S.perm || I.pos != S.pos) { fprintf(stderr, "update %d: I and S orders differ\n", v); abort(); }
        if (v % 50 == 49) {
            static void* hv = nullptr;
            dpg_chol_sym S3 = S;
            if (dpg_chol_plan_blocks(&hv, V1, I.pos.data(), I.perm.data(), plo.data(), phi.data(), (int64_t)plo.size()) ||
                dpg_chol_create_sym_plan(&hv, V1, plo.data(), phi.data(), (int64_t)plo.size(), &S3, &o))
                return 6;
        }
#endif
        double plan = 0;
        if (dpg_chol_plan_host(V1, plo.data(), phi.data(), (int64_t)plo.size(), &S, &plan)) return 5;
        if (v >= V - tail) {
            acc[0] += t1 - t0;
            acc[1] += t2 - t1;
            acc[2] += plan;
            flops += S.flops;
            maxf = std::max<double>(maxf, S.max_front);
            levels += S.n_levels;
            // the critical-path estimate the fused factorization schedules by (dpg_chol.hip chol_plan)
            std::vector<double> cpe((size_t)S.ns, 0.0);
            double crit = 0.0;
            for (int32_t s = S.ns - 1; s >= 0; --s) {
                const int32_t k = S.sn_c0[(size_t)s + 1] - S.sn_c0[(size_t)s];
                const int32_t r = (int32_t)(S.sn_rows_ptr[(size_t)s + 1] - S.sn_rows_ptr[(size_t)s]);
                const int32_t nch = (int32_t)(S.child_ptr[(size_t)s + 1] - S.child_ptr[(size_t)s]);
                const int32_t m3 = 3 * (k + r);
                const double est = (m3 <= 96 && nch <= 8) ? 4.0 + 0.05 * m3 : 10.0 + 20.0 * ((3 * k + 23) / 24);
                const int32_t pa = S.sn_parent[(size_t)s];
                cpe[(size_t)s] = est + (pa >= 0 ? cpe[(size_t)pa] : 0.0);
                crit = std::max(crit, cpe[(size_t)s]);
            }
            crit_sum += crit;
            ++cnt;
        }
    }
    printf("V=%d pairs=%zu nnz=%lld supernodes=%d reorders=%d | last %d updates, mean ms: incsym %.3f derive %.3f "
           "plan %.3f total %.3f (derive's from_csr alone %.3f, reorder %.3f, of which the ordering %.3f)\n",
           V, plo.size(), (long long)I.nnz, S.ns, reorders, cnt, acc[0] / cnt, acc[1] / cnt, acc[2] / cnt,
           (acc[0] + acc[1] + acc[2]) / cnt, acc[3] / cnt, t_reset / cnt, t_order / cnt);
    printf("mean factor Mflop %.1f, max front %.0f blocks, mean levels %.1f, mean critical-path estimate %.0f us\n",
           flops / cnt * 1e-6, maxf, levels / cnt, crit_sum / cnt);
#ifdef DPG_PLAN_TIMING
    printf("plan parts, mean ms over the tail:");
    for (int k = 1; k < 8; ++k)
        printf(" %d:%.3f", k, (dpg_plan_t_export[k] - pt0[k] - dpg_plan_t_export[k - 1] + pt0[k - 1]) / cnt);
    printf("\nfrom_csr parts, mean ms over the tail (derive + the bench's own call):");
    for (int k = 1; k < 6; ++k) printf(" %d:%.3f", k, (dpg_csr_t[k] - ct0[k] - dpg_csr_t[k - 1] + ct0[k - 1]) / cnt);
    printf("\n");
#endif
    return 0;
}
