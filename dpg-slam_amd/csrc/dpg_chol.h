// dpg_chol.h -- GPU supernodal multifrontal Cholesky for the 3x3-block pose-graph system
// (private, C++).  Symbolic analysis in dpg_chol_sym.cpp, numeric factorization + solves in
// dpg_chol.hip.
#ifndef DPG_CHOL_H
#define DPG_CHOL_H

#include <stdint.h>

#include <vector>

// The solver's options (the public dpg_solver_options, dpg_slam_c.h, set per context)
struct dpg_chol_opts {
    int32_t max_supernode_cols = 64;   // cap on columns (3x3 blocks) per supernode
    double relax_fraction = 0.3;       // explicit-zero budget of relaxed amalgamation (0 = fundamental)
    int32_t order = 0;                 // DPG_ORDER_AUTO | DPG_ORDER_MD | DPG_ORDER_ND
    int32_t merge_single = 0;          // supernodes merge only along single-child chains (round 1's rule)
    int32_t fused = 1;                 // one-launch DAG factorization when the fronts fit LDS
    int32_t solve_stage = -1;          // doubles of L staged in LDS by the solves (-1: what fills 80 KB)
    int32_t solve_maxseg = -1;         // ancestor row segments in the backward solve (-1: all)
    int32_t solve_dinv = 0;            // solves with inverted diagonal blocks
    int32_t solve_inv_cols = 0;        // fronts of at least this many pivot columns get L11^-1 after the
                                       // factorization: the solves' diagonal part is then one product
                                       // instead of a substitution chain (0: never; measured slower,
                                       // DESIGN.md K4 round 5)
};

// Everything is indexed by block positions p = pos[node] in the elimination order.
struct dpg_chol_sym {
    int64_t n = 0;                    // block columns (nodes)
    int32_t ns = 0;                   // supernodes
    int32_t n_levels = 0;
    int32_t max_front = 0;            // largest front, in blocks
    double flops = 0.0;               // factorization flop estimate
    std::vector<int32_t> perm, pos;   // perm[p] = node, pos[node] = p
    std::vector<int32_t> sn_c0;       // [ns+1] first column position of each supernode
    std::vector<int32_t> sn_of;       // [n] supernode of each column position
    std::vector<int64_t> sn_rows_ptr; // [ns+1]
    std::vector<int32_t> sn_rows;     // row positions below each supernode (sorted)
    std::vector<int32_t> sn_parent;   // [ns]
    std::vector<int32_t> sn_level;    // [ns]
    std::vector<int32_t> level_ptr;   // [n_levels+1] into level_list
    std::vector<int32_t> level_list;  // supernodes grouped by level
    std::vector<int64_t> child_ptr;   // [ns+1]
    std::vector<int32_t> child_list;
    std::vector<int32_t> relmap;      // parallel to sn_rows: index of that row in the parent front
    std::vector<int64_t> front_off;   // [ns+1] doubles: front s is a (3m x 3m) column-major matrix
};

int dpg_chol_symbolic(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                      const dpg_chol_opts* opts, dpg_chol_sym* S);
// the two halves of dpg_chol_symbolic: the minimum-degree order with the column patterns of L
// (in elimination positions, sorted), and everything derived from an order + patterns
// (md: minimum degree alone; otherwise nested dissection with minimum-degree parts of <= 16 nodes)
int dpg_chol_order(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                   std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat, bool md = false);
// nested dissection (BFS level separators; parts of <= leaf nodes by minimum degree): shallow trees
int dpg_chol_order_nd(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs, int32_t leaf,
                      std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat);
// the same with the separator rule of the multi-start search (starts = 0: round 2's rule; bal:
// both sides >= 1 / bal of the part; score 0 |S|, 1 |S| N / min side, 2 |S| sqrt(N / min side);
// cover: the chosen cut's separator as a minimum vertex cover of its crossing edges)
int dpg_chol_order_nd_sep(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs, int32_t leaf,
                          int32_t starts, int32_t bal, int32_t score, bool cover, std::vector<int32_t>& perm,
                          std::vector<std::vector<int32_t>>& pat, bool par = false);
int dpg_chol_sym_from_patterns(int64_t n, const std::vector<int32_t>& perm, const std::vector<std::vector<int32_t>>& pat,
                               const dpg_chol_opts* opts, dpg_chol_sym* S);
// the fused factorization's critical-path estimate (us) of an analysis (the chol_plan ticket model)
double dpg_chol_critical_path_us(const dpg_chol_sym& S);
// the same from patterns in CSR form: column p's rows are prow[cp[p] .. cp[p + 1]) (sorted)
int dpg_chol_sym_from_csr(int64_t n, const int32_t* perm, const int64_t* cp, const int32_t* prow,
                          const dpg_chol_opts* opts, dpg_chol_sym* S);

// Incremental symbolic state of a growing pose graph (dpg_inc.hip): the elimination order is kept
// and new nodes are appended at its end; the column patterns of L are bitsets over positions,
// updated along the elimination-tree paths a new edge touches (no re-ordering).
struct dpg_chol_incsym {
    int64_t n = 0, words = 0;               // nodes, 64-bit words per pattern row (capacity)
    std::vector<int32_t> perm, pos;         // elimination order
    std::vector<uint64_t> bits;             // [n][words]: later positions in column p's pattern
    int64_t swords = 0;                     // summary words per row: (words + 63) / 64
    std::vector<uint64_t> summ;             // [n][swords]: bit w set when bits word w may be nonzero
    std::vector<int32_t> parent;            // elimination-tree parent position (-1: root)
    int64_t nnz = 0;                        // pattern entries (blocks below the diagonal)
    // the same patterns in CSR form (column p: rows[cp[p] .. cp[p + 1]), sorted), as of the last
    // derive, and the entries added since (merged in by the next derive)
    std::vector<int64_t> cp;
    std::vector<int32_t> rows, rows_tmp;
    std::vector<std::pair<int32_t, int32_t>> added;
};
// a fresh minimum-degree order of the graph (pairs) -> state
int dpg_incsym_reset(dpg_chol_incsym* I, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                     const dpg_chol_opts* opts = nullptr);
// the two halves of dpg_incsym_reset: the order and column patterns of the graph (a pure function
// of its arguments, safe on a worker thread), and the state built from them (perm, pat consumed)
// (concurrent: the two candidates of the automatic rule on two threads -- for callers waiting on
// the order; the incremental graph's ahead-of-time order on its worker thread runs them in turn)
int dpg_incsym_order(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                     std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat,
                     const dpg_chol_opts* opts = nullptr, bool concurrent = false);
void dpg_incsym_init(dpg_chol_incsym* I, int64_t n, std::vector<int32_t>& perm, std::vector<std::vector<int32_t>>& pat);
// nodes n .. n + k - 1 appended at the end of the order
void dpg_incsym_append(dpg_chol_incsym* I, int64_t k);
// edge (a, b) of the graph (nodes); returns the number of pattern entries it added (fill)
int64_t dpg_incsym_add_edge(dpg_chol_incsym* I, int32_t a, int32_t b);
// the derived structures of the current state
int dpg_incsym_derive(dpg_chol_incsym* I, const dpg_chol_opts* opts, dpg_chol_sym* S);


// GPU solver structures (dpg_chol.hip) for a given symbolic analysis; *h is reused -- its device
// buffers grow only when needed -- or created when NULL.  On error *h is destroyed and NULL.  The
// analysis is moved into *h: *S is left holding *h's previous one (or nothing).
int dpg_chol_create_sym(void** h, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                        dpg_chol_sym* S, const dpg_chol_opts* opts = nullptr);
// the same in two halves: the plan (host only, no device call) and its upload (the same thread,
// no other build in between); on error *h is destroyed and NULL
int dpg_chol_create_sym_plan(void** h, int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                             dpg_chol_sym* S, const dpg_chol_opts* opts = nullptr);
int dpg_chol_create_sym_upload(void** h);
// the plan's first part (H's blocks bucketed by column position) ahead of the next
// dpg_chol_create_sym_plan of a graph with n nodes and these n_pairs pairs, whose analysis carries
// the ordering pos / perm; creates *h when NULL.  Host only, not concurrently with a plan or an
// upload of the same object (the incremental prepare runs it beside dpg_incsym_derive)
int dpg_chol_plan_blocks(void** h, int64_t n, const int32_t* pos, const int32_t* perm, const int32_t* pair_lo,
                         const int32_t* pair_hi, int64_t n_pairs);
/* drops buckets prebuilt by dpg_chol_plan_blocks (the next plan builds its own) */
void dpg_chol_blocks_invalidate(void* h);
// host time (ms) of the last build of h: structures, uploads
void dpg_chol_build_times(void* h, double out[2]);
// 1 when h factors with the fused DAG kernel (every front fits its LDS budget), 0 on the level path
int dpg_chol_fused(void* h);
// the host half of a build alone (no device calls; tools/incsym_bench.cpp times it on the CPU)
int dpg_chol_plan_host(int64_t n, const int32_t* pair_lo, const int32_t* pair_hi, int64_t n_pairs,
                       const dpg_chol_sym* S, double* ms);

#endif
