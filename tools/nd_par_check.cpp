// nd_par_check.cpp -- the nested dissection's threaded forms give the serial form's orders
// (dpg_chol_sym.cpp: the halves of a large part on two threads, a large part's starts on up to
// four, the level structures reused): the same permutation and column patterns, for both
// candidate rules, on generated pose-graph-like graphs (a route with local and long loop
// closures, several components).  usage: nd_par_check N SEED  -> prints "ok" or the mismatch
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <set>
#include <utility>
#include <vector>

#include "../dpg-slam_amd/csrc/dpg_chol.h"

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 6000;
    const unsigned seed = argc > 2 ? (unsigned)atoi(argv[2]) : 1;
    std::mt19937 rng(seed);
    std::set<std::pair<int32_t, int32_t>> pairs;
    const int comps = 1 + (int)(seed % 3);   // 1-3 components
    const int per = n / comps;
    for (int c = 0; c < comps; ++c) {
        const int b = c * per, e = c == comps - 1 ? n : b + per;
        for (int v = b; v + 1 < e; ++v) pairs.insert({v, v + 1});
        std::uniform_int_distribution<int> any(b, e - 1), near(-60, 60);
        for (int k = 0; k < 3 * (e - b); ++k) {
            const int i = any(rng);
            const int j = k % 4 == 0 ? any(rng) : std::min(e - 1, std::max(b, i + near(rng)));
            if (i != j) pairs.insert({std::min(i, j), std::max(i, j)});
        }
    }
    std::vector<int32_t> lo, hi;
    for (auto& p : pairs) { lo.push_back(p.first); hi.push_back(p.second); }
    const struct { int32_t starts, bal, score; bool cover; } rules[] = {{0, 5, 0, false}, {8, 4, 2, true}};
    for (auto& r : rules) {
        std::vector<int32_t> p0, p1;
        std::vector<std::vector<int32_t>> t0, t1;
        if (dpg_chol_order_nd_sep(n, lo.data(), hi.data(), (int64_t)lo.size(), 16, r.starts, r.bal, r.score, r.cover, p0, t0, false) ||
            dpg_chol_order_nd_sep(n, lo.data(), hi.data(), (int64_t)lo.size(), 16, r.starts, r.bal, r.score, r.cover, p1, t1, true)) {
            printf("order failed\n");
            return 1;
        }
        if (p0 != p1 || t0 != t1) {
            printf("mismatch: starts %d\n", r.starts);
            return 1;
        }
    }
    std::vector<int32_t> q0, q1;
    std::vector<std::vector<int32_t>> u0, u1;
    if (dpg_incsym_order(n, lo.data(), hi.data(), (int64_t)lo.size(), q0, u0, nullptr, false) ||
        dpg_incsym_order(n, lo.data(), hi.data(), (int64_t)lo.size(), q1, u1, nullptr, true) || q0 != q1 || u0 != u1) {
        printf("incsym order mismatch\n");
        return 1;
    }
    printf("ok %zu pairs\n", lo.size());
    return 0;
}
