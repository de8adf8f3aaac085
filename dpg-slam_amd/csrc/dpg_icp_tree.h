// dpg_icp_tree.h -- the fixed fp64 reduction tree of the ICP rigid-fit sums (R5), shared by the
// three ICP kernels and restated by the CPU oracle (oracle/dpg_oracle.c lane_tree).
//
// The sums: [0] count, [1] sum d, [2..3] sum p, [4..5] sum q, [6] sum (px qx + py qy), [7] sum
// (px qy - py qx) -- p the moved source point, q its target, d the fp32 squared distance; each
// pair's terms are exact fp64 products with one rounded add/subtract.  The count is an integer,
// exact in any order.  The tree for sums [1..7] (DPG_ICP_LANES = 512 lanes = 8 waves of 64):
//   * lane l accumulates the accepted pairs of the source points i with i mod 512 == l, in
//     ascending i, starting from 0.0;
//   * inside each wave, for off = 32, 16, 8, 4, 2, 1: acc[k] = acc[k] + acc[k + off] (k < off);
//     lane 0 then holds the wave partial W_w;
//   * S = ((W0 + W1) + (W2 + W3)) + ((W4 + W5) + (W6 + W7)).
// Any fixed tree gives the same result on every run; this one costs the GPU one DPP/swizzle/
// bpermute step per level and nothing in LDS.  (PCL's Umeyama sums in float in its own order,
// which is unpinned -- SURVEY §8a R5.)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpg_tree {

constexpr int kSums = 8;        // cnt, d, px, py, qx, qy, dot, cross
constexpr int kLanes = 512;     // == DPG_ICP_LANES
constexpr int kWaves = kLanes / 64;

// lane k (< off) receives lane k + off's value; other lanes' results are never used
template <int OFF>
__device__ __forceinline__ double down(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    int lo = (int)(uint32_t)b, hi = (int)(uint32_t)(b >> 32);
    if constexpr (OFF == 32) {
        lo = __shfl_down(lo, 32, 64);
        hi = __shfl_down(hi, 32, 64);
    } else if constexpr (OFF == 16) {   // ds_swizzle, bit mode: lane ^ 16 inside each 32-lane half
        lo = __builtin_amdgcn_ds_swizzle(lo, 0x401F);
        hi = __builtin_amdgcn_ds_swizzle(hi, 0x401F);
    } else {                            // DPP row_shl:OFF (lane k reads lane k + OFF of its row)
        lo = __builtin_amdgcn_update_dpp(0, lo, 0x100 + OFF, 0xF, 0xF, false);
        hi = __builtin_amdgcn_update_dpp(0, hi, 0x100 + OFF, 0xF, 0xF, false);
    }
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

// the in-wave part of the tree for sums [FIRST, kSums): lane 0 ends with W_w
template <int FIRST = 0>
__device__ __forceinline__ void wave_fold(double (&acc)[kSums]) {
#pragma unroll
    for (int q = FIRST; q < kSums; ++q) acc[q] = acc[q] + down<32>(acc[q]);
#pragma unroll
    for (int q = FIRST; q < kSums; ++q) acc[q] = acc[q] + down<16>(acc[q]);
#pragma unroll
    for (int q = FIRST; q < kSums; ++q) acc[q] = acc[q] + down<8>(acc[q]);
#pragma unroll
    for (int q = FIRST; q < kSums; ++q) acc[q] = acc[q] + down<4>(acc[q]);
#pragma unroll
    for (int q = FIRST; q < kSums; ++q) acc[q] = acc[q] + down<2>(acc[q]);
#pragma unroll
    for (int q = FIRST; q < kSums; ++q) acc[q] = acc[q] + down<1>(acc[q]);
}

namespace detail {
__device__ __forceinline__ uint32_t lo32(double v) { return (uint32_t)(uint64_t)__double_as_longlong(v); }
__device__ __forceinline__ uint32_t hi32(double v) { return (uint32_t)((uint64_t)__double_as_longlong(v) >> 32); }
__device__ __forceinline__ double mk(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// v_permlane32_swap / v_permlane16_swap on a pair of doubles: a keeps its own lower part (lanes
// 0-31, resp. rows 0 and 2) and receives b's, b the mirror -- then a + b is the tree's sum
// "lower lane + upper lane" of a in the lower part and of b in the upper part
template <int W>
__device__ __forceinline__ double swap_add(double a, double b) {
    uint32_t al = lo32(a), ah = hi32(a), bl = lo32(b), bh = hi32(b);
    if constexpr (W == 32) {
        const auto l = __builtin_amdgcn_permlane32_swap(al, bl, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(ah, bh, false, false);
        al = l[0]; bl = l[1]; ah = h[0]; bh = h[1];
    } else {
        const auto l = __builtin_amdgcn_permlane16_swap(al, bl, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
        al = l[0]; bl = l[1]; ah = h[0]; bh = h[1];
    }
    return mk(al, ah) + mk(bl, bh);
}
}  // namespace detail

// The same in-wave tree as wave_fold for all eight sums, with the work of each level spread
// over the lanes: at off = 32 the lower half adds sums 0-3 and the upper half sums 4-7 (one
// permlane32 swap per pair instead of a shuffle per sum), at off = 16 the rows split them again,
// at off = 8 the half-rows, and the last three levels fold one sum per 8-lane group.  Every
// partial is the same two operands added in the same order as in wave_fold, so the results are
// bit-identical.  Lane 8 g ends with W_w[fold_sum(g)]; the other lanes' values are not used.
__device__ __forceinline__ int fold_sum(int g) { return 4 * (g >> 2) + 2 * (g & 1) + ((g >> 1) & 1); }
__device__ __forceinline__ double wave_fold_t(const double (&acc)[kSums]) {
    static_assert(kSums == 8, "the transposed fold is written for eight sums");
    const int lane = threadIdx.x & 63;
    double u0 = detail::swap_add<32>(acc[0], acc[4]);
    double u1 = detail::swap_add<32>(acc[1], acc[5]);
    double u2 = detail::swap_add<32>(acc[2], acc[6]);
    double u3 = detail::swap_add<32>(acc[3], acc[7]);
    const double s0 = detail::swap_add<16>(u0, u1);
    const double s1 = detail::swap_add<16>(u2, u3);
    // off = 8 inside each 16-lane row: lanes 0-7 add s0, lanes 8-15 add s1
    const bool lo8 = (lane & 15) < 8;
    const double t = lo8 ? s1 : s0;
    const double r = detail::mk((uint32_t)__builtin_amdgcn_update_dpp(0, (int)detail::lo32(t), 0x128, 0xF, 0xF, false),
                                (uint32_t)__builtin_amdgcn_update_dpp(0, (int)detail::hi32(t), 0x128, 0xF, 0xF, false));
    double z = lo8 ? s0 + r : r + s1;
    z = z + down<4>(z);
    z = z + down<2>(z);
    z = z + down<1>(z);
    return z;
}

// the cross-wave part: W[w * stride + q] -> S[q]
__device__ __forceinline__ double combine(const double* W, int stride, int q) {
    return ((W[0 * stride + q] + W[1 * stride + q]) + (W[2 * stride + q] + W[3 * stride + q])) +
           ((W[4 * stride + q] + W[5 * stride + q]) + (W[6 * stride + q] + W[7 * stride + q]));
}

// one accepted pair (source p moved, target q, fp32 squared distance d) into a lane's sums
__device__ __forceinline__ void add_pair(double (&acc)[kSums], float sx, float sy, float tx, float ty, float d) {
    const double px = sx, py = sy, qx = tx, qy = ty;
    acc[0] = acc[0] + 1.0;
    acc[1] = acc[1] + (double)d;
    acc[2] = acc[2] + px;
    acc[3] = acc[3] + py;
    acc[4] = acc[4] + qx;
    acc[5] = acc[5] + qy;
    acc[6] = acc[6] + (px * qx + py * qy);
    acc[7] = acc[7] + (px * qy - py * qx);
}

// R5 closed form from the reduced sums: a = S_dot - (Sp . Sq) / n, b = S_cross - (Sp x Sq) / n
__device__ __forceinline__ void fit_ab(const double* S, double& a, double& b) {
    const double n = S[0];
    a = S[6] - (S[2] * S[4] + S[3] * S[5]) / n;
    b = S[7] - (S[2] * S[5] - S[3] * S[4]) / n;
}

}  // namespace dpg_tree
