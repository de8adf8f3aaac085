#include "dpg_chol.h"
#include <cstdio>
#include <chrono>
#include <vector>
#include <cstdlib>
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "r"); long n; fscanf(f, "%ld", &n);
    std::vector<int32_t> lo, hi; int a, b;
    while (fscanf(f, "%d %d", &a, &b) == 2) { lo.push_back(a); hi.push_back(b); }
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    for (int rep = 0; rep < 5; ++rep) {
        double t0 = now();
        std::vector<int32_t> pm; std::vector<std::vector<int32_t>> pt;
        dpg_chol_order_nd_sep(n, lo.data(), hi.data(), lo.size(), 16, 8, 4, 2, true, pm, pt, argc > 2 ? atoi(argv[2]) : true);
        double t1 = now();
        dpg_chol_sym T; dpg_chol_sym_from_patterns(n, pm, pt, nullptr, &T);
        double t2 = now();
        double cp = dpg_chol_critical_path_us(T);
        double t3 = now();
        std::vector<int32_t> pm0; std::vector<std::vector<int32_t>> pt0;
        dpg_chol_order_nd_sep(n, lo.data(), hi.data(), lo.size(), 16, 0, 5, 0, true, pm0, pt0, true);
        double t4 = now();
        dpg_chol_sym S; dpg_chol_symbolic(n, lo.data(), hi.data(), lo.size(), nullptr, &S);
        double t5 = now();
        unsigned long h = 1469598103934665603ul; for (int32_t v : pm) h = (h ^ (unsigned)v) * 1099511628211ul;
        printf("cand1 order %.2f sym %.2f cp %.2f | cand0 order %.2f | symbolic %.2f  hash %lx cp %.1f\n", t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, h, cp);
    }
}
