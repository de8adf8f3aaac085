// incsym_check.cpp -- CPU check of the incremental symbolic analysis (dpg_chol_incsym): a random
// pose graph grown node by node (chain + loop closures to older nodes, some between two older
// nodes), starting from a minimum-degree order of its first part; after every step the maintained
// column patterns must equal a from-scratch symbolic elimination of the current graph in the
// maintained order.  usage: incsym_check N0 STEPS SEED [split|-] [LEAD]   (exit 0 = all equal)
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <set>
#include <vector>

#include "../dpg-slam_amd/csrc/dpg_chol.h"

static std::vector<std::set<int>> eliminate(int64_t n, const std::vector<int32_t>& pos,
                                            const std::vector<std::pair<int, int>>& edges) {
    std::vector<std::set<int>> col((size_t)n);
    for (auto& e : edges) {
        int a = pos[(size_t)e.first], b = pos[(size_t)e.second];
        if (a > b) std::swap(a, b);
        col[(size_t)a].insert(b);
    }
    for (int64_t j = 0; j < n; ++j) {
        if (col[(size_t)j].empty()) continue;
        const int p = *col[(size_t)j].begin();
        for (int r : col[(size_t)j])
            if (r != p) col[(size_t)p].insert(r);
    }
    return col;
}

int main(int argc, char** argv) {
    const int n0 = argc > 1 ? atoi(argv[1]) : 200, steps = argc > 2 ? atoi(argv[2]) : 100;
    std::mt19937 rng(argc > 3 ? atoi(argv[3]) : 1);
    // "split": the initial graph is several components (chain breaks every 40 nodes, no closures
    // across them) and some nodes are isolated -- the nested dissection's component handling
    const bool split = argc > 4 && argv[4][0] == 's';
    std::vector<std::pair<int, int>> edges;
    for (int v = 1; v < n0; ++v) {
        if (split && (v % 40 == 0 || v % 97 == 5)) continue;
        edges.emplace_back(v - 1, v);
        if (v > 10 && rng() % 3 == 0) {
            const int j = (int)(rng() % (v - 5));
            if (!split || j / 40 == v / 40) edges.emplace_back(j, v);
        }
    }
    std::vector<int32_t> lo, hi;
    for (auto& e : edges) { lo.push_back(e.first); hi.push_back(e.second); }
    dpg_chol_incsym I;
    // lead > 0: the background reorder's path (dpg_inc.hip) -- the order of a snapshot of the graph
    // `lead` nodes earlier (dpg_incsym_order + dpg_incsym_init), the nodes since appended at its
    // end and their edges added, instead of a fresh order of the whole initial graph
    const int lead = argc > 5 ? atoi(argv[5]) : 0;
    if (lead > 0 && lead < n0) {
        const int ns = n0 - lead;
        int64_t k = 0;
        while (k < (int64_t)edges.size() && edges[(size_t)k].second < ns) ++k;   // edges arrive by their later node
        std::vector<int32_t> perm;
        std::vector<std::vector<int32_t>> pat;
        if (dpg_incsym_order(ns, lo.data(), hi.data(), k, perm, pat)) return 3;
        dpg_incsym_init(&I, ns, perm, pat);
        dpg_incsym_append(&I, lead);
        for (int64_t q = k; q < (int64_t)edges.size(); ++q) dpg_incsym_add_edge(&I, edges[(size_t)q].first, edges[(size_t)q].second);
    } else if (dpg_incsym_reset(&I, n0, lo.data(), hi.data(), (int64_t)lo.size())) {
        return 3;
    }
    int64_t n = n0;
    for (int s = 0; s < steps; ++s) {
        dpg_incsym_append(&I, 1);
        const int v = (int)n++;
        std::vector<std::pair<int, int>> add{{v - 1, v}};
        for (int q = 0; q < 3; ++q)
            if (rng() % 2) add.emplace_back((int)(rng() % (v - 2)), v - 1);   // loop closure to the previous node
        if (rng() % 5 == 0) add.emplace_back((int)(rng() % (v / 2)), (int)(v / 2 + rng() % (v / 2 - 1)));
        for (auto& e : add) {
            edges.push_back(e);
            dpg_incsym_add_edge(&I, e.first, e.second);
        }
        const auto ref = eliminate(n, I.pos, edges);
        int64_t nnz = 0;
        for (int64_t j = 0; j < n; ++j) {
            for (int64_t r = j + 1; r < n; ++r) {
                const bool a = (I.bits[(size_t)(j * I.words + r / 64)] >> (r % 64)) & 1ull;
                const bool b = ref[(size_t)j].count((int)r) != 0;
                if (a != b) { printf("step %d: column %lld row %lld: inc %d ref %d\n", s, (long long)j, (long long)r, a, b); return 1; }
            }
            nnz += (int64_t)ref[(size_t)j].size();
            const int pref = ref[(size_t)j].empty() ? -1 : *ref[(size_t)j].begin();
            if (pref != I.parent[(size_t)j]) { printf("step %d: parent of %lld: %d vs %d\n", s, (long long)j, I.parent[(size_t)j], pref); return 1; }
        }
        if (nnz != I.nnz) { printf("step %d: nnz %lld vs %lld\n", s, (long long)I.nnz, (long long)nnz); return 1; }
        if (s % 3 == 0) {   // the CSR patterns derive keeps up to date (merged every few steps)
            dpg_chol_sym S;
            dpg_chol_opts o{64, 0.3};
            if (dpg_incsym_derive(&I, &o, &S)) { printf("step %d: derive failed\n", s); return 1; }
            for (int64_t j = 0; j < n; ++j) {
                const std::vector<int> csr(I.rows.begin() + I.cp[(size_t)j], I.rows.begin() + I.cp[(size_t)j + 1]);
                const std::vector<int> want(ref[(size_t)j].begin(), ref[(size_t)j].end());
                if (csr != want) { printf("step %d: CSR column %lld differs\n", s, (long long)j); return 1; }
            }
        }
    }
    dpg_chol_sym S;
    dpg_chol_opts o{64, 0.3};
    if (dpg_incsym_derive(&I, &o, &S)) return 4;
    printf("ok: n=%lld nnz=%lld supernodes=%d\n", (long long)n, (long long)I.nnz, S.ns);
    return 0;
}
