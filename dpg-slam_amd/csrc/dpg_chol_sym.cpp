// dpg_chol_sym.cpp -- symbolic analysis of the block-sparse pose-graph system for the GPU
// supernodal multifrontal Cholesky (the CHOLESKY linear solver GTSAM runs inside
// ISAM2 / GaussNewtonOptimizer).  Host code, run once per sparsity pattern
// (dpg_gn_setup); the numeric factorization and solves are in dpg_chol.hip.
//
//   1. fill-reducing order on the 3x3-block graph: nested dissection (BFS level separators) down
//      to parts of <= 16 nodes, ordered by minimum degree (bitset elimination graphs, ties ->
//      lowest node index) -- shallow elimination trees for the GPU's critical path
//   2. column structure of L and the elimination tree
//   3. fundamental supernodes, merged further while the added explicit zeros stay small
//      (relaxed amalgamation), and the supernodal elimination tree
//   4. level schedule (leaves = level 0) and the maps the GPU kernels need: original H blocks
//      -> front positions, child update matrix rows -> parent front rows
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <future>
#include <memory>
#include <queue>
#include <vector>

#include "dpg_chol.h"

namespace {

// Minimum-degree ordering over the block graph.  adjacency: CSR of the symmetric graph without
// self loops.  Returns perm (elimination order) and the L column patterns (later nodes, by pos).
void min_degree(int64_t n, const std::vector<int64_t>& aptr, const std::vector<int32_t>& adj,
                std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pattern) {
    const int64_t W = (n + 63) / 64;
    std::vector<uint64_t> bits((size_t)(n * W), 0ull);
    // [wlo, whi): a word range of each row holding all its set bits (pose-graph neighbourhoods are
    // mostly local in node id, so the row operations below touch few words)
    std::vector<int32_t> wlo((size_t)n, (int32_t)W), whi((size_t)n, 0);
    for (int64_t v = 0; v < n; ++v)
        for (int64_t q = aptr[v]; q < aptr[v + 1]; ++q) {
            const int32_t u = adj[(size_t)q];
            bits[(size_t)(v * W + u / 64)] |= 1ull << (u % 64);
            wlo[(size_t)v] = std::min(wlo[(size_t)v], u / 64);
            whi[(size_t)v] = std::max(whi[(size_t)v], u / 64 + 1);
        }
    std::vector<int32_t> deg((size_t)n);
    for (int64_t v = 0; v < n; ++v) deg[(size_t)v] = (int32_t)(aptr[v + 1] - aptr[v]);
    std::vector<char> done((size_t)n, 0);
    perm.assign((size_t)n, -1);
    pattern.assign((size_t)n, {});
    std::vector<int32_t> nb;
    nb.reserve(1024);
    // the uneliminated node of least degree, ties -> lowest index: a min-heap of (degree, node) with
    // lazy deletion (an entry is current iff its degree is the node's degree now)
    std::priority_queue<std::pair<int32_t, int32_t>, std::vector<std::pair<int32_t, int32_t>>,
                        std::greater<std::pair<int32_t, int32_t>>> heap;
    for (int64_t v = 0; v < n; ++v) heap.emplace(deg[(size_t)v], (int32_t)v);
    for (int64_t p = 0; p < n; ++p) {
        int32_t v = -1;
        while (!heap.empty()) {
            const auto top = heap.top();
            heap.pop();
            if (!done[(size_t)top.second] && top.first == deg[(size_t)top.second]) { v = top.second; break; }
        }
        done[(size_t)v] = 1;
        perm[(size_t)p] = v;
        nb.clear();
        uint64_t* bv = &bits[(size_t)(v * W)];
        const int32_t vlo = wlo[(size_t)v], vhi = whi[(size_t)v];
        for (int64_t w = vlo; w < vhi; ++w) {
            uint64_t b = bv[w];
            while (b) {
                const int t = __builtin_ctzll(b);
                b &= b - 1;
                nb.push_back((int32_t)(w * 64 + t));
            }
        }
        pattern[(size_t)p] = nb;   // node ids; converted to positions after the ordering is known
        for (int32_t u : nb) {
            uint64_t* bu = &bits[(size_t)(u * W)];
            for (int64_t w = vlo; w < vhi; ++w) bu[w] |= bv[w];
            bu[u / 64] &= ~(1ull << (u % 64));
            bu[v / 64] &= ~(1ull << (v % 64));
            int32_t lo = std::min(wlo[(size_t)u], vlo), hi = std::max(whi[(size_t)u], vhi);
            while (lo < hi && bu[lo] == 0) ++lo;
            while (hi > lo && bu[hi - 1] == 0) --hi;
            wlo[(size_t)u] = lo;
            whi[(size_t)u] = hi;
            int32_t d = 0;
            for (int64_t w = lo; w < hi; ++w) d += __builtin_popcountll(bu[w]);
            if (d != deg[(size_t)u]) heap.emplace(d, u);
            deg[(size_t)u] = d;
        }
        for (int64_t w = vlo; w < vhi; ++w) bv[w] = 0;
    }
}

// ---- nested dissection (shallow elimination trees)
// Minimum degree minimises fill but on a long, thin pose graph (a route driven several times: a
// ladder a few nodes wide and thousands long) it eliminates from the ends inwards and the
// elimination tree becomes a path hundreds of supernodes deep -- and the GPU factorization's
// critical path is the tree's height.  Nested dissection splits such a graph at its middle by a
// separator a few nodes wide (a BFS level structure from a pseudo-peripheral node: the smallest
// level in the middle half), orders both halves recursively and the separator last: height
// O(log n) separators.  Parts of at most `leaf` nodes are ordered by minimum degree.
//
// Separator choice (round 3): `starts` = 0 is round 2's rule (one level structure from the
// pseudo-peripheral node, the smallest level with a fifth of the part on either side).  With
// starts > 0 the search covers the cuts between consecutive levels of several level structures
// (the pseudo-peripheral start, the far end of its BFS, and starts - 1 more spread over its BFS
// order, for parts of at least 256 nodes), each cut's trimmed separator counted in one pass over
// the edges, and keeps the cut with both sides >= 1 / bal of the part that minimises
// |S| sqrt(N / min(|A|, |B|)) (score 2; score 1: |S| N / min, score 0: |S|) -- small separators
// high in the tree are what the GPU factorization's critical path pays for (dpg_chol_symbolic
// picks among such orders by that path's estimate).
struct NdParams {
    int32_t starts = 0, bal = 5, score = 0;
    bool cover = false;   // the chosen cut's separator as a minimum vertex cover of its crossing edges
    bool par = false;     // the two halves of a large part ordered on two threads (same order)
};
// Per-vertex scratch shared by the parallel halves of a split (the parts are disjoint: a part only
// writes its own vertices; it reads a neighbour's stamp, which another part may be writing, only
// to compare it with its own id -- relaxed atomic accesses for the stamps, the levels and the
// cover marks are only touched for the part's own vertices)
// fptr / fcnt: each vertex's neighbours inside its current part, a range of that part's filtered
// adjacency (NdState.fadj; built once per part, in the graph's adjacency order, so every traversal
// visits what the unfiltered one with the stamp test would, in the same order)
struct NdShared {
    std::vector<int32_t> stamp, lvl, aux;
    std::vector<int64_t> fptr;
    std::vector<int32_t> fcnt;
    std::atomic<int32_t> next_id{0};
};
struct NdState {
    int64_t n;
    const int64_t* aptr;
    const int32_t* adj;
    const int32_t* fadj = nullptr;   // the current part's filtered adjacency
    int32_t leaf;
    NdParams prm;
    NdShared* sh;
    std::vector<int32_t> queue;
    std::vector<int32_t>* out;
};
inline int32_t stamp_of(const NdState& st, int32_t v) { return __atomic_load_n(&st.sh->stamp[(size_t)v], __ATOMIC_RELAXED); }
inline void stamp_set(NdState& st, int32_t v, int32_t id) { __atomic_store_n(&st.sh->stamp[(size_t)v], id, __ATOMIC_RELAXED); }
inline int32_t nd_new_id(NdState& st) { return st.sh->next_id.fetch_add(1, std::memory_order_relaxed) + 1; }

inline const int32_t* nbr_begin(const NdState& st, int32_t v) { return st.fadj + st.sh->fptr[(size_t)v]; }
inline const int32_t* nbr_end(const NdState& st, int32_t v) { return st.fadj + st.sh->fptr[(size_t)v] + st.sh->fcnt[(size_t)v]; }

// the part's filtered adjacency (its vertices are stamped `id`): into `fadj`, which must outlive
// the part's own traversals (its sub-parts build their own)
void nd_filter(NdState& st, const std::vector<int32_t>& sub, int32_t id, std::vector<int32_t>& fadj) {
    size_t tot = 0;
    for (int32_t v : sub) tot += (size_t)(st.aptr[v + 1] - st.aptr[v]);
    fadj.clear();
    fadj.reserve(tot);
    for (int32_t v : sub) {
        st.sh->fptr[(size_t)v] = (int64_t)fadj.size();
        for (int64_t t = st.aptr[v]; t < st.aptr[v + 1]; ++t) {
            const int32_t u = st.adj[(size_t)t];
            if (stamp_of(st, u) == id) fadj.push_back(u);
        }
        st.sh->fcnt[(size_t)v] = (int32_t)((int64_t)fadj.size() - st.sh->fptr[(size_t)v]);
    }
    st.fadj = fadj.data();
}

// BFS over the current part from `src` into the level array `lvl` (-1 = not reached) and `queue`
// (visit order); returns the height
int32_t nd_bfs_into(const NdState& st, int32_t id, int32_t src, int32_t* lvl, std::vector<int32_t>& queue) {
    (void)id;
    // branch-free visit (the new-or-not test of a neighbour is data-dependent, mispredicted about
    // half the time): every neighbour is written at the queue's tail, which advances only when it
    // is new -- the same visit order as a test-and-push
    if (queue.size() < (size_t)st.n + 1) queue.resize((size_t)st.n + 1);
    int32_t* q = queue.data();
    size_t qh = 0, qt = 1;
    q[0] = src;
    lvl[src] = 0;
    int32_t h = 0;
    while (qh < qt) {
        const int32_t v = q[qh++];
        const int32_t lv = lvl[v];
        h = std::max(h, lv);
        for (const int32_t *p = nbr_begin(st, v), *e = nbr_end(st, v); p != e; ++p) {
            const int32_t u = *p;
            const int32_t lu = lvl[u];
            const bool fresh = lu < 0;
            lvl[u] = fresh ? lv + 1 : lu;
            q[qt] = u;
            qt += fresh;
        }
    }
    queue.resize(qt);
    return h + 1;
}
int32_t nd_bfs(NdState& st, int32_t id, int32_t src) { return nd_bfs_into(st, id, src, st.sh->lvl.data(), st.queue); }

int32_t nd_degree(const NdState& st, int32_t id, int32_t v) {
    (void)id;
    return st.sh->fcnt[(size_t)v];
}

// min_degree's order (no patterns) of a part of at most 64 nodes: one bitmask row per node, the
// same choices -- the uneliminated node of least (degree, index), its neighbourhood made a clique
// in ascending index order -- without min_degree's allocations (the nested dissection orders a
// thousand such parts per order)
void min_degree_small(int32_t n, uint64_t* row, int32_t* perm) {
    int32_t deg[64];
    uint64_t left = n == 64 ? ~0ull : ((1ull << n) - 1);
    for (int32_t v = 0; v < n; ++v) deg[v] = __builtin_popcountll(row[v]);
    for (int32_t p = 0; p < n; ++p) {
        int32_t v = -1;
        for (uint64_t m = left; m; m &= m - 1) {
            const int32_t u = __builtin_ctzll(m);
            if (v < 0 || deg[u] < deg[v]) v = u;
        }
        left &= ~(1ull << v);
        perm[p] = v;
        const uint64_t bv = row[v];
        for (uint64_t m = bv; m; m &= m - 1) {
            const int32_t u = __builtin_ctzll(m);
            row[u] = (row[u] | bv) & ~(1ull << u) & ~(1ull << v);
            deg[u] = __builtin_popcountll(row[u]);
        }
        row[v] = 0;
    }
}

void nd_min_degree(NdState& st, const std::vector<int32_t>& sub) {
    const int32_t id = nd_new_id(st);
    for (size_t i = 0; i < sub.size(); ++i) { stamp_set(st, sub[i], id); st.sh->lvl[(size_t)sub[i]] = (int32_t)i; }
    if (sub.size() <= 64) {
        uint64_t row[64];
        int32_t lp[64];
        const int32_t n = (int32_t)sub.size();
        for (int32_t i = 0; i < n; ++i) {
            const int32_t v = sub[(size_t)i];
            row[i] = 0;
            for (int64_t t = st.aptr[v]; t < st.aptr[v + 1]; ++t)
                if (stamp_of(st, st.adj[(size_t)t]) == id) row[i] |= 1ull << st.sh->lvl[(size_t)st.adj[(size_t)t]];
        }
        min_degree_small(n, row, lp);
        for (int32_t k = 0; k < n; ++k) st.out->push_back(sub[(size_t)lp[k]]);
        return;
    }
    std::vector<int64_t> ap(sub.size() + 1, 0);
    std::vector<int32_t> aj;
    for (size_t i = 0; i < sub.size(); ++i) {
        const int32_t v = sub[i];
        for (int64_t t = st.aptr[v]; t < st.aptr[v + 1]; ++t)
            if (stamp_of(st, st.adj[(size_t)t]) == id) aj.push_back(st.sh->lvl[(size_t)st.adj[(size_t)t]]);
        ap[i + 1] = (int64_t)aj.size();
    }
    std::vector<int32_t> lp;
    std::vector<std::vector<int32_t>> lpat;
    min_degree((int64_t)sub.size(), ap, aj, lp, lpat);
    for (int32_t l : lp) st.out->push_back(sub[(size_t)l]);
}

void nd_rec(NdState& st, std::vector<int32_t>& sub);

// after a split: A's order, B's order, then the separator.  With prm.par a large part's two halves
// are ordered at once, B into its own list on a second thread -- the same order as one thread
// (each half's recursion sees only its own vertices; the ids only need to be distinct)
constexpr size_t kNdParMin = 1024;
void nd_halves(NdState& st, std::vector<int32_t>& A, std::vector<int32_t>& B, const std::vector<int32_t>& S) {
    if (st.prm.par && A.size() + B.size() >= kNdParMin) {
        std::vector<int32_t> outB;
        NdState sb;
        sb.n = st.n;
        sb.aptr = st.aptr;
        sb.adj = st.adj;
        sb.leaf = st.leaf;
        sb.prm = st.prm;
        sb.sh = st.sh;
        sb.out = &outB;
        std::future<void> fb = std::async(std::launch::async, [&sb, &B] { nd_rec(sb, B); });
        nd_rec(st, A);
        fb.get();
        st.out->insert(st.out->end(), outB.begin(), outB.end());
    } else {
        nd_rec(st, A);
        nd_rec(st, B);
    }
    for (int32_t v : S) st.out->push_back(v);
}

// the best cut between consecutive levels of the level structure from s0 (bm < 0: none admissible)
struct NdCut {
    int32_t bm = -1;
    bool up = false;
    double sc = 0.0;
    int64_t imb = 0;
};
constexpr size_t kNdStartsParMin = 2048;
constexpr size_t kNdStartsThreads = 4;
// (have_h > 0: lvl already holds the level structure from s0, of height have_h)
NdCut nd_best_cut(const NdState& st, const std::vector<int32_t>& sub, int32_t id, int32_t s0, int32_t* lvl,
                  std::vector<int32_t>& queue, int32_t have_h = 0) {
    NdCut best;
    const int64_t N = (int64_t)sub.size();
    int32_t hh = have_h;
    if (hh <= 0) {
        for (int32_t v : sub) lvl[v] = -1;
        hh = nd_bfs_into(st, id, s0, lvl, queue);
    }
    if (hh < 3) return best;
    std::vector<int64_t> cnt((size_t)hh, 0), slo((size_t)hh, 0), shi((size_t)hh, 0);
    for (int32_t v : sub) {
        const int32_t l = lvl[v];
        cnt[(size_t)l]++;
        bool up = false, dn = false;
        for (const int32_t *p = nbr_begin(st, v), *e = nbr_end(st, v); p != e; ++p) {
            const int32_t lu = lvl[*p];
            up |= lu == l + 1;
            dn |= lu == l - 1;
        }
        slo[(size_t)l] += up;                    // on level l, touching l + 1
        if (l > 0) shi[(size_t)l - 1] += dn;     // on level l, touching l - 1
    }
    int64_t below = 0;
    for (int32_t l = 0; l + 1 < hh; ++l) {   // the cut between levels l and l + 1
        const bool up = shi[(size_t)l] < slo[(size_t)l];
        const int64_t sz = up ? shi[(size_t)l] : slo[(size_t)l];
        const int64_t a_sz = below + cnt[(size_t)l] - (up ? 0 : sz), b_sz = N - a_sz - sz;
        below += cnt[(size_t)l];
        if (l == 0 || (int64_t)st.prm.bal * a_sz < N || (int64_t)st.prm.bal * b_sz < N) continue;
        const double mn = (double)std::min(a_sz, b_sz);
        const double sc = st.prm.score == 2 ? (double)sz * sqrt((double)N / mn)
                          : st.prm.score == 1 ? (double)sz * (double)N / mn : (double)sz;
        const int64_t imb = a_sz > b_sz ? a_sz - b_sz : b_sz - a_sz;
        if (best.bm < 0 || sc < best.sc || (sc == best.sc && imb < best.imb)) {
            best.bm = l; best.up = up; best.sc = sc; best.imb = imb;
        }
    }
    return best;
}

// the separator search with several level structures (NdParams, starts > 0); src is the part's
// pseudo-peripheral node, `id` its stamp; have_h > 0: the shared level array and queue hold the
// level structure from src already (of height have_h: the pseudo-peripheral search's last BFS).
// A level structure already in the shared array is not recomputed -- src's for the first start,
// the last start's for the chosen cut -- with the same result.
void nd_split_multi(NdState& st, std::vector<int32_t>& sub, int32_t id, int32_t src, int32_t have_h) {
    const int64_t N = (int64_t)sub.size();
    const int T = N >= 256 ? st.prm.starts : 1;
    std::vector<int32_t> starts{src};
    int32_t h_src = have_h;
    {
        if (h_src <= 0) {
            for (int32_t v : sub) st.sh->lvl[(size_t)v] = -1;
            h_src = nd_bfs(st, id, src);
        }
        const std::vector<int32_t> order(st.queue.begin(), st.queue.end());
        for (int t = 1; t < T; ++t) starts.push_back(order[(size_t)((int64_t)t * (N - 1) / T)]);
        starts.push_back(order.back());
    }
    // every start's best cut (the first of the smallest (score, imbalance) along its levels), then
    // the first best over the starts in order -- the same pick as one scan over all (start, cut);
    // a large part's starts are searched on several threads, each with its own level array
    std::vector<NdCut> cuts(starts.size());
    const int W = st.prm.par && (size_t)N >= kNdStartsParMin ? (int)std::min<size_t>(kNdStartsThreads, starts.size()) : 1;
    // worker 0 (this thread) works in the shared array: its first start is src (already there)
    size_t k_shared = 0;   // the start whose level structure the shared array holds at the end
    for (size_t k = 0; k < starts.size(); k += (size_t)W) {
        cuts[k] = nd_best_cut(st, sub, id, starts[k], st.sh->lvl.data(), st.queue, k == 0 ? h_src : 0);
        k_shared = k;
        if (k == 0 && W > 1) {   // the other workers start once src's cut is taken
            break;
        }
    }
    if (W > 1) {
        auto work = [&](int w) {
            std::unique_ptr<int32_t[]> lv(new int32_t[(size_t)st.n]);
            std::vector<int32_t> q;
            for (size_t k = (size_t)w; k < starts.size(); k += (size_t)W) cuts[k] = nd_best_cut(st, sub, id, starts[k], lv.get(), q);
        };
        std::vector<std::future<void>> fs;
        for (int w = 1; w < W; ++w) fs.push_back(std::async(std::launch::async, work, w));
        for (size_t k = (size_t)W; k < starts.size(); k += (size_t)W) {
            cuts[k] = nd_best_cut(st, sub, id, starts[k], st.sh->lvl.data(), st.queue);
            k_shared = k;
        }
        for (auto& f : fs) f.get();
    }
    int32_t bsrc = -1, bm = -1;
    bool bupper = false;
    double bsc = 0.0;
    int64_t bimb = 0;
    for (size_t k = 0; k < starts.size(); ++k) {
        const NdCut& c = cuts[k];
        if (c.bm >= 0 && (bm < 0 || c.sc < bsc || (c.sc == bsc && c.imb < bimb))) {
            bsrc = starts[k]; bm = c.bm; bupper = c.up; bsc = c.sc; bimb = c.imb;
        }
    }
    if (bm < 0) { nd_min_degree(st, sub); return; }
    if (bsrc != starts[k_shared]) {
        for (int32_t v : sub) st.sh->lvl[(size_t)v] = -1;
        nd_bfs(st, id, bsrc);
    }
    auto touches = [&](int32_t v, int32_t l) {
        for (const int32_t *p = nbr_begin(st, v), *e = nbr_end(st, v); p != e; ++p)
            if (st.sh->lvl[(size_t)*p] == l) return true;
        return false;
    };
    std::vector<int32_t> A, B, S;
    if (st.prm.cover) {
        // the cut's crossing edges join X (level bm, touching bm + 1) and Y (level bm + 1, touching
        // bm); a minimum vertex cover of that bipartite graph (maximum matching, Konig) is the
        // smallest separator this cut admits -- never larger than either side's boundary
        std::vector<int32_t> X, Y;
        for (int32_t v : sub) {
            const int32_t l = st.sh->lvl[(size_t)v];
            if (l == bm && touches(v, bm + 1)) { st.sh->aux[(size_t)v] = (int32_t)X.size(); X.push_back(v); }
            else if (l == bm + 1 && touches(v, bm)) { st.sh->aux[(size_t)v] = (int32_t)Y.size(); Y.push_back(v); }
        }
        std::vector<int64_t> xp(X.size() + 1, 0);
        std::vector<int32_t> xa;
        for (size_t i = 0; i < X.size(); ++i) {
            const int32_t v = X[i];
            for (const int32_t *p = nbr_begin(st, v), *e = nbr_end(st, v); p != e; ++p)
                if (st.sh->lvl[(size_t)*p] == bm + 1) xa.push_back(st.sh->aux[(size_t)*p]);
            xp[i + 1] = (int64_t)xa.size();
        }
        std::vector<int32_t> mx(X.size(), -1), my(Y.size(), -1), seen(Y.size(), -1);
        // Kuhn's augmenting paths, iterative (the path stack holds (x, next edge))
        std::vector<std::pair<int32_t, int64_t>> stk;
        for (int32_t x0 = 0; x0 < (int32_t)X.size(); ++x0) {
            stk.assign(1, {x0, xp[(size_t)x0]});
            bool found = false;
            while (!stk.empty() && !found) {
                auto& top = stk.back();
                const int32_t x = top.first;
                if (top.second == xp[(size_t)x + 1]) { stk.pop_back(); continue; }
                const int32_t y = xa[(size_t)top.second++];
                if (seen[(size_t)y] == x0) continue;
                seen[(size_t)y] = x0;
                if (my[(size_t)y] < 0) {   // augment along the stack
                    int32_t yy = y;
                    for (size_t k = stk.size(); k-- > 0;) {
                        const int32_t xx = stk[k].first, prev = mx[(size_t)xx];
                        mx[(size_t)xx] = yy;
                        my[(size_t)yy] = xx;
                        yy = prev;
                    }
                    found = true;
                } else {
                    stk.push_back({my[(size_t)y], xp[(size_t)my[(size_t)y]]});
                }
            }
        }
        // Konig: Z = reachable from the unmatched X by alternating paths; cover = (X \ Z) + (Y in Z)
        std::vector<char> zx(X.size(), 0), zy(Y.size(), 0);
        std::vector<int32_t> q;
        for (int32_t x = 0; x < (int32_t)X.size(); ++x)
            if (mx[(size_t)x] < 0) { zx[(size_t)x] = 1; q.push_back(x); }
        for (size_t qi = 0; qi < q.size(); ++qi) {
            const int32_t x = q[qi];
            for (int64_t t = xp[(size_t)x]; t < xp[(size_t)x + 1]; ++t) {
                const int32_t y = xa[(size_t)t];
                if (zy[(size_t)y] || mx[(size_t)x] == y) continue;
                zy[(size_t)y] = 1;
                const int32_t x2 = my[(size_t)y];
                if (x2 >= 0 && !zx[(size_t)x2]) { zx[(size_t)x2] = 1; q.push_back(x2); }
            }
        }
        for (size_t i = 0; i < X.size(); ++i) st.sh->aux[(size_t)X[i]] = zx[i] ? -1 : -2;   // -2: in the cover
        for (size_t j = 0; j < Y.size(); ++j) st.sh->aux[(size_t)Y[j]] = zy[j] ? -2 : -1;
        for (int32_t v : sub) {
            const int32_t l = st.sh->lvl[(size_t)v];
            const bool in_cover = (l == bm || l == bm + 1) && st.sh->aux[(size_t)v] == -2;
            (in_cover ? S : l <= bm ? A : B).push_back(v);
        }
        for (int32_t v : X) st.sh->aux[(size_t)v] = -1;
        for (int32_t v : Y) st.sh->aux[(size_t)v] = -1;
    } else {
        for (int32_t v : sub) {
            const int32_t l = st.sh->lvl[(size_t)v];
            if (!bupper) {
                if (l < bm) A.push_back(v);
                else if (l > bm) B.push_back(v);
                else (touches(v, bm + 1) ? S : A).push_back(v);
            } else {
                if (l <= bm) A.push_back(v);
                else if (l > bm + 1) B.push_back(v);
                else (touches(v, bm) ? S : B).push_back(v);
            }
        }
    }
    nd_halves(st, A, B, S);
}

void nd_rec(NdState& st, std::vector<int32_t>& sub) {
    if ((int32_t)sub.size() <= st.leaf) { nd_min_degree(st, sub); return; }
    const int32_t id = nd_new_id(st);
    for (int32_t v : sub) { stamp_set(st, v, id); st.sh->lvl[(size_t)v] = -1; }
    std::vector<int32_t> fadj;   // this part's filtered adjacency (st.fadj while the part splits)
    nd_filter(st, sub, id, fadj);
    // connected components, each ordered on its own
    std::vector<std::vector<int32_t>> comps;
    int32_t comp_h = 0;   // one component: the level structure from sub[0] is in the shared array
    for (int32_t v : sub)
        if (st.sh->lvl[(size_t)v] < 0) {
            comp_h = nd_bfs(st, id, v);
            comps.emplace_back(st.queue.begin(), st.queue.end());
        }
    if (comps.size() > 1) {
        for (auto& c : comps) {
            std::sort(c.begin(), c.end());
            nd_rec(st, c);
        }
        return;
    }
    // pseudo-peripheral start: repeat BFS from a least-degree node of the last level while the
    // height grows
    int32_t src = sub[0], h = 0;
    int32_t bfs_src = -1, bfs_h = 0;   // the level structure the shared array holds
    for (int it = 0; it < 4; ++it) {
        int32_t hh = it == 0 ? comp_h : 0;   // the components' BFS was from sub[0] = src
        if (hh <= 0) {
            for (int32_t v : sub) st.sh->lvl[(size_t)v] = -1;
            hh = nd_bfs(st, id, src);
        }
        bfs_src = src;
        bfs_h = hh;
        if (hh <= h) break;
        h = hh;
        int32_t best = -1, bd = 1 << 30;
        for (int32_t v : st.queue)
            if (st.sh->lvl[(size_t)v] == h - 1) {
                const int32_t d = nd_degree(st, id, v);
                if (d < bd || (d == bd && v < best)) { bd = d; best = v; }
            }
        if (best == src) break;
        src = best;
    }
    if (st.prm.starts > 0) { nd_split_multi(st, sub, id, src, bfs_src == src ? bfs_h : 0); return; }
    for (int32_t v : sub) st.sh->lvl[(size_t)v] = -1;
    h = nd_bfs(st, id, src);
    const int64_t N = (int64_t)sub.size();
    if (h < 3) { nd_min_degree(st, sub); return; }
    std::vector<int64_t> cnt((size_t)h, 0);
    for (int32_t v : sub) cnt[(size_t)st.sh->lvl[(size_t)v]]++;
    // separator level: the smallest in the middle (both sides >= N/5), ties -> the most balanced
    int32_t m = -1;
    int64_t below = 0, best_sz = 0, best_imb = 0;
    for (int32_t l = 0; l < h; ++l) {
        const int64_t above = N - below - cnt[(size_t)l];
        if (l > 0 && l < h - 1 && 5 * below >= N && 5 * above >= N) {
            const int64_t imb = below > above ? below - above : above - below;
            if (m < 0 || cnt[(size_t)l] < best_sz || (cnt[(size_t)l] == best_sz && imb < best_imb)) {
                m = l;
                best_sz = cnt[(size_t)l];
                best_imb = imb;
            }
        }
        below += cnt[(size_t)l];
    }
    if (m < 0) {   // no level leaves both sides a fifth: the level that halves the count
        below = 0;
        for (m = 0; m < h - 1 && 2 * (below + cnt[(size_t)m]) < N; ++m) below += cnt[(size_t)m];
        m = std::min(std::max(m, 1), h - 2);
    }
    // the separator: the level-m nodes with a neighbour on level m + 1 (the others join the lower
    // side), or the level-(m + 1) nodes with a neighbour on level m (the others join the upper
    // side), whichever is smaller
    auto touches = [&](int32_t v, int32_t l) {
        for (const int32_t *p = nbr_begin(st, v), *e = nbr_end(st, v); p != e; ++p)
            if (st.sh->lvl[(size_t)*p] == l) return true;
        return false;
    };
    int64_t s_lo = 0, s_hi = 0;
    for (int32_t v : sub) {
        const int32_t l = st.sh->lvl[(size_t)v];
        if (l == m) s_lo += touches(v, m + 1);
        else if (l == m + 1) s_hi += touches(v, m);
    }
    const bool upper = s_hi < s_lo;
    std::vector<int32_t> A, B, S;
    for (int32_t v : sub) {
        const int32_t l = st.sh->lvl[(size_t)v];
        if (!upper) {
            if (l < m) A.push_back(v);
            else if (l > m) B.push_back(v);
            else (touches(v, m + 1) ? S : A).push_back(v);
        } else {
            if (l <= m) A.push_back(v);
            else if (l > m + 1) B.push_back(v);
            else (touches(v, m) ? S : B).push_back(v);
        }
    }
    nd_halves(st, A, B, S);
}

// column patterns of L (positions, sorted) for a given order: each column's later neighbours and
// its elimination-tree children's patterns
void patterns_of_order(int64_t n, const std::vector<int64_t>& aptr, const std::vector<int32_t>& adj,
                       const std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat) {
    std::vector<int32_t> pos((size_t)n);
    for (int64_t p = 0; p < n; ++p) pos[(size_t)perm[(size_t)p]] = (int32_t)p;
    pat.assign((size_t)n, {});
    std::vector<std::vector<int32_t>> kids((size_t)n);
    std::vector<int32_t> rows, tmp;
    for (int64_t p = 0; p < n; ++p) {
        const int32_t v = perm[(size_t)p];
        rows.clear();
        for (int64_t t = aptr[v]; t < aptr[v + 1]; ++t)
            if (pos[(size_t)adj[(size_t)t]] > p) rows.push_back(pos[(size_t)adj[(size_t)t]]);
        std::sort(rows.begin(), rows.end());
        rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
        for (int32_t c : kids[(size_t)p]) {
            const std::vector<int32_t>& pc = pat[(size_t)c];   // pc[0] == p
            tmp.resize(rows.size() + pc.size());
            tmp.resize((size_t)(std::set_union(rows.begin(), rows.end(), pc.begin() + 1, pc.end(), tmp.begin()) - tmp.begin()));
            rows.swap(tmp);
        }
        std::vector<int32_t>().swap(kids[(size_t)p]);
        pat[(size_t)p] = rows;
        if (!rows.empty()) kids[(size_t)rows[0]].push_back((int32_t)p);
    }
}

}  // namespace

int dpg_chol_order_nd(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs, int32_t leaf,
                      std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat) {
    return dpg_chol_order_nd_sep(n, pair_lo, pair_hi, n_pairs, leaf, 0, 5, 0, false, perm, pat);
}

int dpg_chol_order_nd_sep(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs, int32_t leaf,
                          int32_t starts, int32_t bal, int32_t score, bool cover, std::vector<int32_t>& perm,
                          std::vector<std::vector<int32_t>>& pat, bool par) {
    if (n <= 0) return -1;
    std::vector<int64_t> aptr((size_t)n + 1, 0);
    for (int64_t p = 0; p < n_pairs; ++p) { aptr[(size_t)pair_lo[p] + 1]++; aptr[(size_t)pair_hi[p] + 1]++; }
    for (int64_t v = 0; v < n; ++v) aptr[(size_t)v + 1] += aptr[(size_t)v];
    std::vector<int32_t> adj((size_t)aptr[(size_t)n]);
    {
        std::vector<int64_t> cur(aptr.begin(), aptr.end() - 1);
        for (int64_t p = 0; p < n_pairs; ++p) {
            adj[(size_t)cur[(size_t)pair_lo[p]]++] = pair_hi[p];
            adj[(size_t)cur[(size_t)pair_hi[p]]++] = pair_lo[p];
        }
    }
    NdState st;
    st.n = n;
    st.aptr = aptr.data();
    st.adj = adj.data();
    st.leaf = std::max<int32_t>(leaf, 4);
    st.prm.starts = starts;
    st.prm.bal = std::max<int32_t>(bal, 2);
    st.prm.score = score;
    st.prm.cover = cover && starts > 0;
    st.prm.par = par;
    NdShared sh;
    sh.aux.assign((size_t)n, -1);
    sh.stamp.assign((size_t)n, 0);
    sh.lvl.assign((size_t)n, -1);
    sh.fptr.assign((size_t)n, 0);
    sh.fcnt.assign((size_t)n, 0);
    st.sh = &sh;
    perm.clear();
    perm.reserve((size_t)n);
    st.out = &perm;
    std::vector<int32_t> all((size_t)n);
    for (int64_t v = 0; v < n; ++v) all[(size_t)v] = (int32_t)v;
    nd_rec(st, all);
    if ((int64_t)perm.size() != n) return -1;
    patterns_of_order(n, aptr, adj, perm, pat);
    return 0;
}

int dpg_chol_order(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                   std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat, bool md) {
    if (n <= 0) return -1;
    // nested dissection with minimum-degree parts of <= 16 nodes (tools/order_job.sh: the GPU
    // factorization 1.1x faster than under plain minimum degree on config 4's graph, 1.5x on config
    // 3's, 16x on config 5's four-pass route); md: plain minimum degree (DPG_ORDER_MD)
    if (!md) return dpg_chol_order_nd(n, pair_lo, pair_hi, n_pairs, 16, perm, pat);
    // ---- graph
    std::vector<int64_t> aptr((size_t)n + 1, 0);
    for (int64_t p = 0; p < n_pairs; ++p) { aptr[(size_t)pair_lo[p] + 1]++; aptr[(size_t)pair_hi[p] + 1]++; }
    for (int64_t v = 0; v < n; ++v) aptr[(size_t)v + 1] += aptr[(size_t)v];
    std::vector<int32_t> adj((size_t)aptr[(size_t)n]);
    {
        std::vector<int64_t> cur(aptr.begin(), aptr.end() - 1);
        for (int64_t p = 0; p < n_pairs; ++p) {
            adj[(size_t)cur[(size_t)pair_lo[p]]++] = pair_hi[p];
            adj[(size_t)cur[(size_t)pair_hi[p]]++] = pair_lo[p];
        }
    }
    // ---- ordering + column patterns (in positions)
    min_degree(n, aptr, adj, perm, pat);
    std::vector<int32_t> pos((size_t)n);
    for (int64_t p = 0; p < n; ++p) pos[(size_t)perm[(size_t)p]] = (int32_t)p;
    for (int64_t p = 0; p < n; ++p) {
        for (int32_t& u : pat[(size_t)p]) u = pos[(size_t)u];
        std::sort(pat[(size_t)p].begin(), pat[(size_t)p].end());
    }
    return 0;
}

// The fused factorization's critical path estimate (us) of a symbolic analysis: the same per-front
// model chol_plan orders its tickets by (dpg_chol.hip: a front of <= 96 rows and <= 8 children is
// factored in LDS, 4 + 0.06 m3 + 0.9 k3; a larger one by a team, 10 + 20 per 24-column panel),
// summed along the longest leaf-to-root path
double dpg_chol_critical_path_us(const dpg_chol_sym& S) {
    std::vector<double> cp((size_t)S.ns, 0.0);
    double crit = 0.0;
    for (int32_t s = S.ns - 1; s >= 0; --s) {   // parents after their children: walk down from the roots
        const int32_t k = S.sn_c0[(size_t)s + 1] - S.sn_c0[(size_t)s];
        const int32_t r = (int32_t)(S.sn_rows_ptr[(size_t)s + 1] - S.sn_rows_ptr[(size_t)s]);
        const int32_t nch = (int32_t)(S.child_ptr[(size_t)s + 1] - S.child_ptr[(size_t)s]);
        const int32_t m3 = 3 * (k + r);
        const double est = (m3 <= 96 && nch <= 8) ? 4.0 + 0.06 * m3 + 0.9 * (3 * k) : 10.0 + 20.0 * ((3 * k + 23) / 24);
        const int32_t p = S.sn_parent[(size_t)s];
        cp[(size_t)s] = est + (p >= 0 ? cp[(size_t)p] : 0.0);
        crit = std::max(crit, cp[(size_t)s]);
    }
    return crit;
}

// The batch symbolic analysis (once per pattern): nested-dissection orders under two separator
// rules (round 2's, and the 8-start search with the sqrt-ratio score and minimum-vertex-cover
// separators), each carried through the supernodal analysis, and the one whose critical-path
// estimate is shortest is kept.  Config 4 (tools/nd_ab2_job.sh, profiles/r03/v15_nd_cover_ab.txt):
// factor + solve 0.860 -> 0.716 ms, chord-step solves 0.251 -> 0.230 ms; config 3 keeps round 2's
// order (0.282 ms; the others 0.29-0.34).
// The incremental graph (dpg_incsym_order) reorders every 64 nodes with the same pick, on a worker
// thread (dpg_inc.hip).
// opts->order DPG_ORDER_ND (2) keeps round 2's single order, DPG_ORDER_MD (1) plain minimum degree.
int dpg_chol_symbolic(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                      const dpg_chol_opts* opts, dpg_chol_sym* S) {
    std::vector<int32_t> perm;
    std::vector<std::vector<int32_t>> pat;
    const int32_t order = opts ? opts->order : 0;
    if (order != 0 || n < 256) {
        if (dpg_chol_order(n, pair_lo, pair_hi, n_pairs, perm, pat, order == 1)) return -1;
        return dpg_chol_sym_from_patterns(n, perm, pat, opts, S);
    }
    struct Cand { int32_t starts, bal, score; };
    static const Cand cands[] = {{0, 5, 0}, {8, 4, 2}};
    struct Res {
        int rc = 0;
        double cp = 0.0;
        dpg_chol_sym T;
    };
    // both candidates at once (thread-local scratch); the first kept unless the second is shorter
    auto run = [&](int k) {
        Res r;
        std::vector<int32_t> pm;
        std::vector<std::vector<int32_t>> pt;
        if (dpg_chol_order_nd_sep(n, pair_lo, pair_hi, n_pairs, 16, cands[k].starts, cands[k].bal, cands[k].score, true,
                                  pm, pt, true) ||
            dpg_chol_sym_from_patterns(n, pm, pt, opts, &r.T))
            r.rc = -1;
        else
            r.cp = dpg_chol_critical_path_us(r.T);
        return r;
    };
    std::future<Res> second = std::async(std::launch::async, run, 1);
    Res r0 = run(0);
    Res r1 = second.get();
    if (r0.rc || r1.rc) return -1;
    *S = std::move(r1.cp < r0.cp ? r1.T : r0.T);
    return 0;
}

int dpg_chol_sym_from_patterns(int64_t n, const std::vector<int32_t>& perm, const std::vector<std::vector<int32_t>>& pat,
                               const dpg_chol_opts* opts, dpg_chol_sym* S) {
    if (n <= 0 || (int64_t)perm.size() != n || (int64_t)pat.size() != n) return -1;
    std::vector<int64_t> cp((size_t)n + 1, 0);
    for (int64_t p = 0; p < n; ++p) cp[(size_t)p + 1] = cp[(size_t)p] + (int64_t)pat[(size_t)p].size();
    std::vector<int32_t> rows((size_t)cp[(size_t)n]);
    for (int64_t p = 0; p < n; ++p) std::copy(pat[(size_t)p].begin(), pat[(size_t)p].end(), rows.begin() + cp[(size_t)p]);
    return dpg_chol_sym_from_csr(n, perm.data(), cp.data(), rows.data(), opts, S);
}

#ifdef DPG_PLAN_TIMING
double dpg_csr_t[8];
static double csr_now() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}
#define CSR_T(k) dpg_csr_t[k] += csr_now()
#else
#define CSR_T(k) do { } while (0)
#endif

static int sym_from_csr(int64_t n, const int32_t* perm, const int64_t* cp, const int32_t* prow, const dpg_chol_opts* opts,
                        dpg_chol_sym* S, bool exact);

int dpg_chol_sym_from_csr(int64_t n, const int32_t* perm, const int64_t* cp, const int32_t* prow,
                          const dpg_chol_opts* opts, dpg_chol_sym* S) {
    return sym_from_csr(n, perm, cp, prow, opts, S, false);
}

// exact = the patterns are the exact structure of L (the incremental state: a fresh elimination
// extended by exact fill updates).  Then every column's pattern minus its parent lies in the
// parent's pattern (the elimination-tree property), and a supernode is a parent chain, so the row
// set of a supernode -- the union of its columns' rows past its last column -- is the last column's
// pattern: no merge, no inclusion test.  Built with DPG_PLAN_VERIFY the union is checked anyway.
static int sym_from_csr(int64_t n, const int32_t* perm, const int64_t* cp, const int32_t* prow, const dpg_chol_opts* opts,
                        dpg_chol_sym* S, bool exact) {
    if (n <= 0) return -1;
    CSR_T(0);
    auto psize = [&](int64_t p) { return cp[p + 1] - cp[p]; };
    // scratch reused across calls (the incremental solver derives every update)
    thread_local std::vector<int32_t> parent, nchild, sn_first, mark, rowbuf, stamp, mergebuf;
    parent.assign((size_t)n, -1);
    nchild.assign((size_t)n, 0);
    for (int64_t p = 0; p < n; ++p)
        if (psize(p) > 0) { parent[(size_t)p] = prow[cp[p]]; nchild[(size_t)parent[(size_t)p]]++; }
    // ---- fundamental supernodes, then relaxed merging of chains
    // column p+1 joins p's supernode when p's parent is p+1 and the patterns nest (fundamental),
    // or when the explicit zeros added stay within the budget.
    S->sn_of.resize((size_t)n);
    sn_first.clear();
    const int32_t max_cols = opts && opts->max_supernode_cols > 0 ? opts->max_supernode_cols : 64;
    const double relax = opts ? opts->relax_fraction : 0.0;
    // a column joins its child's supernode whatever its other children (they hang off the merged
    // front, whose index set holds their rows): nested dissection's separators become one front
    // each instead of a chain of fronts split at every subtree root attached to them.
    // opts->merge_single restores the single-child rule.
    const bool any_child = !(opts && opts->merge_single);
    {
        int32_t s = -1;
        int64_t zeros = 0, cols = 0;
        for (int64_t p = 0; p < n; ++p) {
            bool join = false;
            if (p > 0 && s >= 0) {
                const int64_t q = p - 1;
                const int64_t cq = psize(q), cpp = psize(p);
                const int64_t ncols = p - sn_first[(size_t)s] + 1;
                // (a merge past another child keeps the front within 127 blocks: the fused
                // factorization's two LDS panel buffers still fit)
                const bool chain = parent[(size_t)q] == (int32_t)p &&
                                   (nchild[(size_t)p] == 1 || (any_child && ncols + cpp <= 127));
                if (chain && ncols <= max_cols) {
                    if (cq == cpp + 1) join = true;   // fundamental
                    else if (relax > 0.0) {
                        // every earlier column of the supernode would carry p's pattern: the rows
                        // of pat[p] missing from pat[q] \ {p} become explicit zeros in them
                        const int64_t add = std::max<int64_t>(0, cpp - (cq - 1)) * cols;
                        if ((double)(zeros + add) <= relax * (double)((cols + 1) * (cpp + 1))) { join = true; zeros += add; }
                    }
                }
            }
            if (!join) { sn_first.push_back((int32_t)p); ++s; zeros = 0; cols = 0; }
            S->sn_of[(size_t)p] = s;
            ++cols;
        }
    }
    const int32_t ns = (int32_t)sn_first.size();
    sn_first.push_back((int32_t)n);
    CSR_T(1);
    // ---- supernode row sets: union of its columns' patterns beyond its last column
    S->n = n;
    S->ns = ns;
    S->perm.assign(perm, perm + n);
    S->pos.resize((size_t)n);
    for (int64_t p = 0; p < n; ++p) S->pos[(size_t)perm[p]] = (int32_t)p;
    S->sn_c0.assign(sn_first.begin(), sn_first.end());
    S->sn_rows_ptr.assign((size_t)ns + 1, 0);
    S->sn_rows.clear();
    S->sn_parent.assign((size_t)ns, -1);
    mark.assign((size_t)n, -1);
    for (int32_t s = 0; s < ns; ++s) {
        const int32_t c0 = sn_first[(size_t)s], c1 = sn_first[(size_t)s + 1];
        // sorted union of the columns' rows >= c1, merged from the last column down (the last
        // column's rows all qualify; in a fundamental supernode every merge adds nothing)
#ifndef DPG_PLAN_VERIFY
        if (exact) {   // straight from the last column's pattern
            const int32_t *b = prow + cp[c1 - 1], *e = prow + cp[c1];
            S->sn_rows.insert(S->sn_rows.end(), b, e);
            S->sn_rows_ptr[(size_t)s + 1] = (int64_t)S->sn_rows.size();
            if (e > b) S->sn_parent[(size_t)s] = S->sn_of[(size_t)*b];
            continue;
        }
#endif
        rowbuf.assign(prow + cp[c1 - 1], prow + cp[c1]);
        for (int32_t c = c1 - 2; c >= c0; --c) {
            const int32_t* b = std::lower_bound(prow + cp[c], prow + cp[c + 1], c1);
            const int32_t* e = prow + cp[c + 1];
            if (std::includes(rowbuf.begin(), rowbuf.end(), b, e)) continue;
#ifdef DPG_PLAN_VERIFY
            if (exact) {
                fprintf(stderr, "exact patterns: column %d's rows past its supernode are not in the last column's\n", c);
                abort();
            }
#endif
            mergebuf.resize(rowbuf.size() + (size_t)(e - b));
            mergebuf.resize((size_t)(std::set_union(rowbuf.begin(), rowbuf.end(), b, e, mergebuf.begin()) - mergebuf.begin()));
            rowbuf.swap(mergebuf);
        }
        S->sn_rows.insert(S->sn_rows.end(), rowbuf.begin(), rowbuf.end());
        S->sn_rows_ptr[(size_t)s + 1] = (int64_t)S->sn_rows.size();
        if (!rowbuf.empty()) S->sn_parent[(size_t)s] = S->sn_of[(size_t)rowbuf[0]];
    }
    CSR_T(2);
    // ---- levels
    S->sn_level.assign((size_t)ns, 0);
    for (int32_t s = 0; s < ns; ++s) {   // children precede parents in elimination order
        const int32_t p = S->sn_parent[(size_t)s];
        if (p >= 0) S->sn_level[(size_t)p] = std::max(S->sn_level[(size_t)p], S->sn_level[(size_t)s] + 1);
    }
    int32_t nl = 0;
    for (int32_t s = 0; s < ns; ++s) nl = std::max(nl, S->sn_level[(size_t)s] + 1);
    S->n_levels = nl;
    S->level_ptr.assign((size_t)nl + 1, 0);
    for (int32_t s = 0; s < ns; ++s) S->level_ptr[(size_t)S->sn_level[(size_t)s] + 1]++;
    for (int32_t l = 0; l < nl; ++l) S->level_ptr[(size_t)l + 1] += S->level_ptr[(size_t)l];
    S->level_list.resize((size_t)ns);
    {
        rowbuf.assign(S->level_ptr.begin(), S->level_ptr.end() - 1);
        for (int32_t s = 0; s < ns; ++s) S->level_list[(size_t)rowbuf[(size_t)S->sn_level[(size_t)s]]++] = s;
    }
    CSR_T(3);
    // ---- children lists and relative maps (child update rows -> parent front index)
    S->child_ptr.assign((size_t)ns + 1, 0);
    for (int32_t s = 0; s < ns; ++s)
        if (S->sn_parent[(size_t)s] >= 0) S->child_ptr[(size_t)S->sn_parent[(size_t)s] + 1]++;
    for (int32_t s = 0; s < ns; ++s) S->child_ptr[(size_t)s + 1] += S->child_ptr[(size_t)s];
    S->child_list.resize((size_t)S->child_ptr[(size_t)ns]);
    {
        rowbuf.resize((size_t)ns);
        for (int32_t s = 0; s < ns; ++s) rowbuf[(size_t)s] = (int32_t)S->child_ptr[(size_t)s];
        for (int32_t s = 0; s < ns; ++s)
            if (S->sn_parent[(size_t)s] >= 0) S->child_list[(size_t)rowbuf[(size_t)S->sn_parent[(size_t)s]]++] = s;
    }
    // relmap: a parent's front row index by position (mark holds it while its children are mapped,
    // stamp says which parent's front the position is in)
    S->relmap.resize(S->sn_rows.size());
    stamp.assign((size_t)n, -1);
    for (int32_t p = 0; p < ns; ++p) {
        if (S->child_ptr[(size_t)p + 1] == S->child_ptr[(size_t)p]) continue;
        const int32_t pc0 = sn_first[(size_t)p], pk = sn_first[(size_t)p + 1] - pc0;
        for (int32_t c = 0; c < pk; ++c) { mark[(size_t)(pc0 + c)] = c; stamp[(size_t)(pc0 + c)] = p; }
        for (int64_t t = S->sn_rows_ptr[(size_t)p]; t < S->sn_rows_ptr[(size_t)p + 1]; ++t) {
            mark[(size_t)S->sn_rows[(size_t)t]] = pk + (int32_t)(t - S->sn_rows_ptr[(size_t)p]);
            stamp[(size_t)S->sn_rows[(size_t)t]] = p;
        }
        for (int64_t ci = S->child_ptr[(size_t)p]; ci < S->child_ptr[(size_t)p + 1]; ++ci) {
            const int32_t s = S->child_list[(size_t)ci];
            for (int64_t t = S->sn_rows_ptr[(size_t)s]; t < S->sn_rows_ptr[(size_t)s + 1]; ++t) {
                const int32_t row = S->sn_rows[(size_t)t];
                // child rows must lie in the parent's front (its columns or its rows)
                if (stamp[(size_t)row] != p) return -2;
                S->relmap[(size_t)t] = mark[(size_t)row];
            }
        }
    }
    CSR_T(4);
    // ---- front offsets (doubles), stats
    S->front_off.assign((size_t)ns + 1, 0);
    double flops = 0.0;
    int32_t maxm = 0;
    for (int32_t s = 0; s < ns; ++s) {
        const int64_t k = sn_first[(size_t)s + 1] - sn_first[(size_t)s];
        const int64_t r = S->sn_rows_ptr[(size_t)s + 1] - S->sn_rows_ptr[(size_t)s];
        const int64_t m3 = 3 * (k + r);
        // rounded up to an even count: every front starts 16-B aligned (the fused factorization's
        // 16-B sc1 hand-offs, dpg_chol.hip front_rsrc)
        S->front_off[(size_t)s + 1] = S->front_off[(size_t)s] + ((m3 * m3 + 1) & ~(int64_t)1);
        maxm = std::max<int32_t>(maxm, (int32_t)(k + r));
        const double k3 = 3.0 * (double)k, r3 = 3.0 * (double)r;
        flops += k3 * k3 * k3 / 3.0 + k3 * k3 * r3 + k3 * r3 * r3;
    }
    S->max_front = maxm;
    S->flops = flops;
    CSR_T(5);
    return 0;
}

// ---------------------------------------------------------------- incremental symbolic state
namespace {

void incsym_grow_words(dpg_chol_incsym* I, int64_t need_bits) {
    if (need_bits <= I->words * 64) return;
    int64_t w = std::max<int64_t>(64, I->words * 2);
    while (w * 64 < need_bits) w *= 2;
    const int64_t sw = (w + 63) / 64;
    std::vector<uint64_t> nb((size_t)(I->n * w), 0ull), ns((size_t)(I->n * sw), 0ull);
    for (int64_t p = 0; p < I->n; ++p) {
        memcpy(&nb[(size_t)(p * w)], &I->bits[(size_t)(p * I->words)], sizeof(uint64_t) * (size_t)I->words);
        memcpy(&ns[(size_t)(p * sw)], &I->summ[(size_t)(p * I->swords)], sizeof(uint64_t) * (size_t)I->swords);
    }
    I->bits.swap(nb);
    I->summ.swap(ns);
    I->words = w;
    I->swords = sw;
}

inline bool has(const dpg_chol_incsym* I, int64_t j, int64_t r) {
    return (I->bits[(size_t)(j * I->words + r / 64)] >> (r % 64)) & 1ull;
}

inline void set_bit(dpg_chol_incsym* I, int64_t j, int64_t r) {
    const int64_t w = r / 64;
    I->bits[(size_t)(j * I->words + w)] |= 1ull << (r % 64);
    I->summ[(size_t)(j * I->swords + w / 64)] |= 1ull << (w % 64);
}

// the set positions > `after` of column j, in increasing order, through the summary words
template <typename F>
inline void for_rows_after(const dpg_chol_incsym* I, int64_t j, int64_t after, F&& f) {
    const uint64_t* row = &I->bits[(size_t)(j * I->words)];
    const uint64_t* sm = &I->summ[(size_t)(j * I->swords)];
    const int64_t w0 = (after + 1) / 64;
    for (int64_t sw = w0 / 64; sw < I->swords; ++sw) {
        uint64_t s = sm[sw];
        if (sw == w0 / 64) s &= ~0ull << (w0 % 64);
        while (s) {
            const int64_t w = sw * 64 + __builtin_ctzll(s);
            s &= s - 1;
            uint64_t m = row[w];
            if (w == w0) m &= ~0ull << ((after + 1) % 64);
            while (m) {
                f(w * 64 + __builtin_ctzll(m));
                m &= m - 1;
            }
        }
    }
}

}  // namespace

int dpg_incsym_order(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                     std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat,
                     const dpg_chol_opts* opts, bool concurrent) {
    // The batch analysis's pick (opts->order DPG_ORDER_AUTO) -- round 2's separator rule or the
    // 8-start search with cover separators, each carried through the supernodal analysis under the
    // incremental solver's options, the shorter critical-path estimate kept.  It costs two orders
    // and two analyses per reorder, which dpg_inc computes on a worker thread ahead of time
    // (dpg_inc.hip, DPG_INC_BG_LEAD), so the per-node latency does not pay for it: config 4 at V = 5000
    // p50 2.14 -> 1.96 ms, 456 -> 487 nodes/s; config 5 413 vs 411 nodes/s
    // (profiles/r03/v24_incbg_ab.txt).  DPG_ORDER_ND: round 2's rule alone; DPG_ORDER_MD: minimum
    // degree.
    // The two candidates are independent (their scratch is thread-local): with `concurrent` the
    // second is computed on a thread of its own beside the first (a sweep's fresh order at 10 k
    // nodes is on its caller's path); the first is kept unless the second's estimate is strictly
    // shorter.
    const int32_t order = opts ? opts->order : 0;
    int rc = 0;
    if (order == 0 && n >= 256) {
        const dpg_chol_opts o = opts ? *opts : dpg_chol_opts{};
        struct Cand {
            int rc = 0;
            double cp = 0.0;
            std::vector<int32_t> pm;
            std::vector<std::vector<int32_t>> pt;
        };
        auto run = [&](int k) {
            Cand c;
            // (dpg_chol_order's nested dissection; a waiting caller's orders also split their
            // large parts over threads -- the same orders)
            c.rc = k == 0 ? dpg_chol_order_nd_sep(n, pair_lo, pair_hi, n_pairs, 16, 0, 5, 0, false, c.pm, c.pt, concurrent)
                          : dpg_chol_order_nd_sep(n, pair_lo, pair_hi, n_pairs, 16, 8, 4, 2, true, c.pm, c.pt, concurrent);
            if (c.rc == 0) {
                dpg_chol_sym T;
                if (dpg_chol_sym_from_patterns(n, c.pm, c.pt, &o, &T)) c.rc = -1;
                else c.cp = dpg_chol_critical_path_us(T);
            }
            return c;
        };
        std::future<Cand> second = std::async(concurrent ? std::launch::async : std::launch::deferred, run, 1);
        Cand c0 = run(0);
        Cand c1 = second.get();
        if (c0.rc || c1.rc) return -1;
        Cand& b = c1.cp < c0.cp ? c1 : c0;
        perm.swap(b.pm);
        pat.swap(b.pt);
    } else {
        rc = dpg_chol_order(n, pair_lo, pair_hi, n_pairs, perm, pat, order == 1);
    }
    return rc ? -1 : 0;
}

int dpg_incsym_reset(dpg_chol_incsym* I, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                     const dpg_chol_opts* opts) {
    std::vector<int32_t> perm;
    std::vector<std::vector<int32_t>> pat;
    if (dpg_incsym_order(n, pair_lo, pair_hi, n_pairs, perm, pat, opts, true)) return -1;
    dpg_incsym_init(I, n, perm, pat);
    return 0;
}

void dpg_incsym_init(dpg_chol_incsym* I, int64_t n, std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat) {
    I->n = n;
    I->words = std::max<int64_t>(64, (n + 63) / 64 * 2);
    I->swords = (I->words + 63) / 64;
    I->perm.swap(perm);
    I->pos.assign((size_t)n, 0);
    const std::vector<int32_t>& pm = I->perm;
    for (int64_t p = 0; p < n; ++p) I->pos[(size_t)pm[(size_t)p]] = (int32_t)p;
    I->bits.assign((size_t)(n * I->words), 0ull);
    I->summ.assign((size_t)(n * I->swords), 0ull);
    I->parent.assign((size_t)n, -1);
    I->nnz = 0;
    I->cp.assign((size_t)n + 1, 0);
    I->rows.clear();
    I->added.clear();
    for (int64_t p = 0; p < n; ++p) {
        for (int32_t r : pat[(size_t)p]) set_bit(I, p, r);
        I->rows.insert(I->rows.end(), pat[(size_t)p].begin(), pat[(size_t)p].end());
        I->cp[(size_t)p + 1] = (int64_t)I->rows.size();
        if (!pat[(size_t)p].empty()) I->parent[(size_t)p] = pat[(size_t)p][0];
        I->nnz += (int64_t)pat[(size_t)p].size();
    }
}

void dpg_incsym_append(dpg_chol_incsym* I, int64_t k) {
    if (k <= 0) return;
    incsym_grow_words(I, I->n + k);
    for (int64_t q = 0; q < k; ++q) {
        I->perm.push_back((int32_t)(I->n + q));   // new node n + q (ids are dense) -> the next position
        I->pos.push_back((int32_t)(I->n + q));
        I->parent.push_back(-1);
    }
    I->n += k;
    I->bits.resize((size_t)(I->n * I->words), 0ull);
    I->summ.resize((size_t)(I->n * I->swords), 0ull);
    I->cp.resize((size_t)I->n + 1, I->cp.empty() ? 0 : I->cp.back());   // the new columns: empty
}

// Row r enters column j's pattern (j < r, positions) and everything the elimination implies: it
// propagates up the elimination tree, and when r becomes a column's new parent, that column's
// other rows above r enter column r as well.
int64_t dpg_incsym_add_edge(dpg_chol_incsym* I, int32_t a, int32_t b) {
    int64_t pa = I->pos[(size_t)a], pb = I->pos[(size_t)b];
    if (pa == pb) return 0;
    if (pa > pb) std::swap(pa, pb);
    int64_t added = 0;
    std::vector<std::pair<int64_t, int64_t>> work{{pa, pb}};
    while (!work.empty()) {
        int64_t j = work.back().first;
        const int64_t r = work.back().second;
        work.pop_back();
        while (j >= 0 && j < r) {
            if (has(I, j, r)) break;
            set_bit(I, j, r);
            I->added.emplace_back((int32_t)j, (int32_t)r);
            ++added;
            const int64_t p_old = I->parent[(size_t)j];
            if (p_old < 0 || r < p_old) {
                I->parent[(size_t)j] = (int32_t)r;
                // column r inherits column j's rows above r
                for_rows_after(I, j, r, [&](int64_t t) { work.emplace_back(r, t); });
                break;
            }
            j = p_old;
        }
    }
    I->nnz += added;
    return added;
}

int dpg_incsym_derive(dpg_chol_incsym* I, const dpg_chol_opts* opts, dpg_chol_sym* S) {
    const int64_t n = I->n;
    if ((int64_t)I->cp.size() != n + 1) return -3;
    if (!I->added.empty()) {
        // merge the entries added since the last derive into the CSR patterns, in one pass
        std::sort(I->added.begin(), I->added.end());
        std::vector<int32_t>& out = I->rows_tmp;
        out.resize(I->rows.size() + I->added.size());
        size_t a = 0, o = 0;
        int64_t prev = 0;
        for (int64_t p = 0; p < n; ++p) {
            const int64_t b = prev, e = I->cp[(size_t)p + 1];
            prev = e;
            I->cp[(size_t)p] = (int64_t)o;
            if (a == I->added.size() || I->added[a].first != p) {
                if (e > b) memcpy(out.data() + o, I->rows.data() + b, sizeof(int32_t) * (size_t)(e - b));
                o += (size_t)(e - b);
                continue;
            }
            int64_t t = b;
            while (a < I->added.size() && I->added[a].first == p) {
                const int32_t r = I->added[a++].second;
                while (t < e && I->rows[(size_t)t] < r) out[o++] = I->rows[(size_t)t++];
                out[o++] = r;
            }
            while (t < e) out[o++] = I->rows[(size_t)t++];
        }
        I->cp[(size_t)n] = (int64_t)o;
        out.resize(o);
        I->rows.swap(out);
        I->added.clear();
    }
    if (I->cp[(size_t)n] != I->nnz) return -3;
    return sym_from_csr(n, I->perm.data(), I->cp.data(), I->rows.data(), opts, S, true);
}
