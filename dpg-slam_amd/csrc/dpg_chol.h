// dpg_chol.h -- GPU supernodal multifrontal Cholesky for the 3x3-block pose-graph system
// (private, C++).  Symbolic analysis in dpg_chol_sym.cpp, numeric factorization + solves in
// dpg_chol.hip.
#ifndef DPG_CHOL_H
#define DPG_CHOL_H

#include <stdint.h>

#include <vector>

struct dpg_chol_opts {
    int32_t max_supernode_cols;   // cap on columns (3x3 blocks) per supernode
    double relax_fraction;        // explicit-zero budget of relaxed amalgamation (0 = fundamental)
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

#endif
