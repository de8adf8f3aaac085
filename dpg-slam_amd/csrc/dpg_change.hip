// dpg_change.hip -- DPG change detection on the GPU: DpgSLAM::executeDPG (dpg_slam.cc:865-886) and
// getActiveAndDynamicMapPoints (:832-863) over a device-resident node store (dpg_dpg).
//
// The reference keeps one hash-map occupancy grid per node (dpg_slam.h:45-260), merges them into a
// greedy submap one candidate at a time and compares cell by cell.  Here every grid that matters is
// one bit-plane of a single dense window of cells around the current pose chain (only cells of the
// chain's own grids are ever queried or counted: detection looks up the submap at chain cells, the
// coverage counts chain cells, removed points lie in chain cells):
//   word[cell] bit 2k / 2k+1 : chain node k's grid has the cell FREE-marked / OCCUPIED-marked
//   word[cell] bit 30 / 31   : the submap has it FREE-marked / OCCUPIED-marked
// A grid's status is OCCUPIED if any occupied point fell in the cell, else FREE if a ray crossed it
// (setFreeCells never overwrites OCCUPIED, setOccupiedCells always wins, combineOccupancyGrids
// prefers OCCUPIED -- :931-956,1015-1029), so all marking is order-free atomicOr.
// The sequential greedy submap (:646-695) reduces to "candidate c joins iff it is the FIRST
// candidate (in node order) to cover some chain cell": a cell's first coverer always finds it
// uncovered, and a later candidate only finds cells uncovered that no earlier one covers.  So one
// atomicMin pass gives first[cell], a histogram per candidate gives the coverage curve, and the
// threshold stop is a prefix walk over the (few) candidates.
//
// Kernels (all one thread per beam, 256-thread blocks, blockIdx.y = node of a short list):
//   raster_kernel<MODE>   ray-march a node's included beams (getIntermediateFreeCellsInFOV,
//                         :1059-1082) into the window: MODE 0 chain bits, 1 first coverer, 2 submap bits
//   hist_kernel           chain cells per first coverer; accept_kernel the greedy prefix walk
//   added_kernel / removed_kernel   per-point detection (:745-766) + bins of the score (:782-830)
//   commit_kernel, apply_added_kernel, apply_removed_kernel   labels + sector of REMOVED (:714-743)
//   deactivate_kernel     updateNodesAndSectorStatus (:888-911, dpg_node.cc:28-96): one block per
//                         past node over the removed points
// Every fp32 expression is evaluated as the reference writes it (-ffp-contract=off); the trig of
// node frames is taken on the host with the same libm calls the oracle uses.  Q8 fixes: see
// include/dpg_slam_c.h and DESIGN.md §3.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <vector>

#include "dpg_atan2f.h"
#include "dpg_internal.h"

namespace {

constexpr int kT = 256;
constexpr int32_t kInf = 0x7f7f7f7f;
constexpr uint32_t kSubFree = 1u << 30, kSubOcc = 1u << 31;

struct Ctl {                     // device counters, fetched once at the end of a call
    unsigned long long chain_cells, samples, oob, n_added, n_removed, sect_off, nodes_off, pad;
    int32_t n_acc, uncovered_lo, uncovered_hi, pad2;
};

struct Box { int32_t x0, y0, w, h; };

struct DS {                      // device view of the node store + per-call scratch
    const int64_t* off;
    const float2* plaser;
    const float* range;
    uint8_t* label;
    const uint8_t* sector;
    const float4* geom;          // amin, amax, rmax, angle_inc
    uint32_t* sect;              // per node: bit s = sector s active
    uint32_t* active;
    const float4* frame;         // [2V]: (lmx, lmy, cos a, sin a), (cos -a, sin -a, 0, 0)
    uint32_t* grid;
    int32_t* first;
    const int32_t* chain;        // chain node ids
    const int32_t* slot;         // [chain]: bit-plane slot of chain node k (bits 2 slot, 2 slot + 1)
    const int32_t* rast;         // chain indices whose grid is (re)rasterised this call
    const float4* cframe;        // [2 chain]: frames of the chain nodes at their CHAIN poses (grids)
    int32_t chain_sep;           // 1: some chain pose differs from that node's estimate
    uint32_t chain_bits;         // planes of the current chain nodes
    uint32_t keep_mask;          // planes kept from the previous call (window reused)
    int32_t rebuild;             // 1: window (re)built, every plane starts empty
    const int32_t* cand;         // candidate node ids, node order
    int32_t* cand_cnt;
    int32_t* acc;
    uint32_t* bins;              // [chain][bin_words]
    int32_t* inrange;            // [chain]
    int32_t* commit;             // [chain + 1]: flags, [chain] = mask
    uint8_t* added;              // [chain][max_beams]
    uint16_t* rmask;             // [n_cand][max_beams]
    float2* removed_xy;
    Ctl* ctl;
    double res, inv_res;
    int32_t max_beams, n_chain, n_cand, bin_words, total_bins, num_sectors;
    float min_pct;
    double change_thr, cover_thr;
    Box box;
};

// round((double)v / res) exactly (convertToKeyForm, :923-929): v * (1/res) is within ~2 ulp of the
// quotient, so unless its fraction lies within 1e-6 of one half it rounds to the same integer as
// the correctly rounded division; only those rare near-ties pay for the fp64 division
__device__ __forceinline__ int key_of(const DS& d, float v) {
    const double q = (double)v * d.inv_res;
    const double fl = floor(q), fr = q - fl;
    if (fabs(fr - 0.5) > 1e-6) return (int)(fr < 0.5 ? fl : fl + 1.0);
    return (int)round((double)v / d.res);
}

__device__ __forceinline__ bool cell_of(const DS& d, float x, float y, int64_t* idx) {
    const int kx = key_of(d, x);
    const int ky = key_of(d, y);
    const int ix = kx - d.box.x0, iy = ky - d.box.y0;
    if (ix < 0 || iy < 0 || ix >= d.box.w || iy >= d.box.h) return false;
    *idx = (int64_t)iy * d.box.w + ix;
    return true;
}

// map-frame point of beam b of node v: transformPoint(getPointInLaserFrame, 0, lidar pose) (:844)
__device__ __forceinline__ float2 map_point(const DS& d, int64_t v, int64_t b) {
    const float4 f = d.frame[2 * v];
    const float2 p = d.plaser[b];
    const float ns = -f.w;
    const float rx = f.z * p.x + ns * p.y;
    const float ry = f.w * p.x + f.z * p.y;
    return make_float2(f.x + rx, f.y + ry);
}

// the same with the frame given (a chain node's grid pose)
__device__ __forceinline__ float2 map_point_at(const float4 f, float2 p) {
    const float ns = -f.w;
    const float rx = f.z * p.x + ns * p.y;
    const float ry = f.w * p.x + f.z * p.y;
    return make_float2(f.x + rx, f.y + ry);
}

// inverseTransformPoint(q, 0, lidar pose of v) (math_utils.cc:21-35)
__device__ __forceinline__ float2 rel_lidar(const DS& d, int64_t v, float2 q) {
    const float4 f = d.frame[2 * v];
    const float4 g = d.frame[2 * v + 1];
    const float tx = q.x - f.x, ty = q.y - f.y;
    const float ns = -g.y;
    return make_float2(g.x * tx + ns * ty, g.y * tx + g.x * ty);
}

// beam of an included point: node active, sector active (:917,982; every label is included,
// NOT_YET_LABELED as STATIC -- Q8 fix)
__device__ __forceinline__ bool included(const DS& d, int64_t v, int64_t b) {
    return d.active[v] && ((d.sect[v] >> d.sector[b]) & 1u);
}

// bin of the change score relative to chain node k (:815-821); -1 outside the scan's range
__device__ __forceinline__ void score_bin(const DS& d, int k, float2 q) {
    const int64_t c = d.chain[k];
    const float4 gm = d.geom[c];
    const float2 r = rel_lidar(d, c, q);
    const float a = dpg_atan2f(r.y, r.x);   // the host libm's atan2f, bit for bit
    if (a > gm.y || a < gm.x) return;
    const float inc = (gm.y - gm.x) / (float)d.total_bins;
    const uint32_t bin = (uint16_t)((a - gm.x) / inc);
    atomicOr(&d.bins[(int64_t)k * d.bin_words + (bin >> 5)], 1u << (bin & 31));
    d.inrange[k] = 1;
}

// kG lanes share a beam: every lane steps the float t chain (one add per sample, the reference's
// exact sequence) and marks one contiguous kG-th of the samples; a block covers kT / kG adjacent beams of one
// scan.  Near the lidar those rays cross the same cells over and over (hundreds of rays per cell
// within a metre), so each block first inserts a cell into an LDS hash set and only the first
// insertion issues the global atomic; the marking is a set union, so dropping repeats is exact.
#ifndef DPG_RASTER_G
#define DPG_RASTER_G 32
#endif
#ifndef DPG_RASTER_BLOCK
#define DPG_RASTER_BLOCK 1024
#endif
constexpr int kG = DPG_RASTER_G;
constexpr int kRB = DPG_RASTER_BLOCK;   // raster workgroup: kRB / kG beams
#ifndef DPG_RASTER_HASH
#define DPG_RASTER_HASH 16384
#endif
constexpr int kH = DPG_RASTER_HASH > 0 ? DPG_RASTER_HASH : 1;   // LDS hash slots (4 B each)
constexpr uint32_t kEmpty = 0xffffffffu;

template <int MODE>
__device__ __forceinline__ void mark_cell(const DS& d, uint32_t* hset, int64_t c, bool occ, int k,
                                          uint32_t chain_mask, uint32_t fbit, uint32_t obit) {
    const uint32_t key = ((uint32_t)c << 1) | (occ ? 1u : 0u);      // c < 2^28
    uint32_t h = (key * 2654435761u) >> (32 - (kH > 1 ? __builtin_ctz(kH) : 1));   // multiplicative hash
    bool fresh = true;
    for (int probe = 0; DPG_RASTER_HASH > 0 && probe < 8; ++probe, h = (h + 1) & (kH - 1)) {
        const uint32_t old = atomicCAS(&hset[h], kEmpty, key);
        if (old == kEmpty) break;
        if (old == key) { fresh = false; break; }
    }
    if (!fresh) return;
    // fire-and-forget atomics (no return value, so the wave does not wait on them); first[] of a
    // cell outside the chain grids is never read
    if (MODE == 1) atomicMin(&d.first[c], k);
    else atomicOr(&d.grid[c], occ ? obit : fbit);
}

template <int MODE>
__global__ __launch_bounds__(kRB) void raster_kernel(DS d) {
    __shared__ uint32_t hset[kH];
    __shared__ unsigned long long red[2];
    const int k = blockIdx.y;
    const int lane = threadIdx.x % kG;
    for (int q = threadIdx.x; q < kH; q += kRB) hset[q] = kEmpty;
    if (threadIdx.x == 0) { red[0] = 0; red[1] = 0; }
    __syncthreads();
    bool live = !(MODE == 2 && !d.acc[k]);
    const int kc = MODE == 0 ? d.rast[k] : k;                 // chain index (MODE 0)
    const int64_t v = MODE == 0 ? d.chain[kc] : d.cand[k];
    const int64_t i = (int64_t)blockIdx.x * (kRB / kG) + threadIdx.x / kG;
    const int64_t b0 = d.off[v], nb = d.off[v + 1] - b0;
    const int64_t b = b0 + i;
    live = live && i < nb && included(d, v, b);
    const uint32_t chain_mask = d.chain_bits;
    const int sl = MODE == 0 ? d.slot[kc] : 0;
    const uint32_t fbit = MODE == 0 ? 1u << (2 * sl) : kSubFree;
    const uint32_t obit = MODE == 0 ? 1u << (2 * sl + 1) : kSubOcc;
    unsigned long long oob = 0, ns = 0;
    if (live) {
        // a chain node's grid sits at its chain pose (current_pass_nodes_, dpg_slam.cc:591-620)
        const float4 f = MODE == 0 ? d.cframe[2 * kc] : d.frame[2 * v];
        const float2 m = MODE == 0 ? map_point_at(f, d.plaser[b]) : map_point(d, v, b);
        int64_t c;
        if (lane == 0 && d.label[b] != DPG_LABEL_MAX_RANGE) {      // occupied end point (:993-997)
            if (cell_of(d, m.x, m.y, &c)) mark_cell<MODE>(d, hset, c, true, k, chain_mask, fbit, obit);
            else ++oob;
        }
        // getIntermediateFreeCellsInFOV: num_bins = round(range / res), t += 1.0 / num_bins in float
        const uint32_t nbins = (uint32_t)round((double)d.range[b] / d.res);
        const float inc = (float)(1.0 / (double)nbins);
        // lane l takes the l-th contiguous chunk of the ~nbins + 1 steps (the last lane runs on to
        // the chain's true end): it first replays the float t chain up to its chunk, then marks
        const uint32_t chunk = (nbins + kG) / kG;
        const uint32_t s0 = (uint32_t)lane * chunk, s1 = lane == kG - 1 ? 0xffffffffu : s0 + chunk;
        uint32_t step = 0;
        float t = 0.0f;
        for (; step < s0 && (double)t < 1.0; ++step) t = t + inc;
        for (; step < s1 && (double)t < 1.0; t = t + inc, ++step) {
            const float ix = (1 - t) * f.x + t * m.x;
            const float iy = (1 - t) * f.y + t * m.y;
            ++ns;
            if (!cell_of(d, ix, iy, &c)) { ++oob; continue; }
            mark_cell<MODE>(d, hset, c, false, k, chain_mask, fbit, obit);
        }
    }
    if (ns) atomicAdd(&red[0], ns);
    if (oob) atomicAdd(&red[1], oob);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (red[0]) atomicAdd(&d.ctl->samples, red[0]);
        if (MODE == 0 && red[1]) atomicAdd(&d.ctl->oob, red[1]);   // chain grids must fit the window
    }
}

// per-call reset of the window and the small scratch (one launch instead of seven memsets)
__global__ __launch_bounds__(kT) void init_kernel(DS d, int64_t n_cells) {
    const int64_t stride = (int64_t)gridDim.x * kT;
    const int64_t n4 = n_cells >> 2;   // 16-byte accesses (hipMalloc buffers are 256-B aligned)
    uint4* g4 = reinterpret_cast<uint4*>(d.grid);
    int4* f4 = reinterpret_cast<int4*>(d.first);
    for (int64_t c = (int64_t)blockIdx.x * kT + threadIdx.x; c < n4; c += stride) {
        uint4 w = make_uint4(0u, 0u, 0u, 0u);
        if (!d.rebuild) {
            w = g4[c];
            w.x &= d.keep_mask; w.y &= d.keep_mask; w.z &= d.keep_mask; w.w &= d.keep_mask;
        }
        g4[c] = w;
        f4[c] = make_int4(kInf, kInf, kInf, kInf);
    }
    for (int64_t c = 4 * n4 + (int64_t)blockIdx.x * kT + threadIdx.x; c < n_cells; c += stride) {
        d.grid[c] = d.rebuild ? 0u : (d.grid[c] & d.keep_mask);
        d.first[c] = kInf;
    }
    if (blockIdx.x == 0) {
        for (int k = threadIdx.x; k < d.n_cand; k += kT) { d.cand_cnt[k] = 0; d.acc[k] = 0; }
        for (int k = threadIdx.x; k < d.n_chain * d.bin_words; k += kT) d.bins[k] = 0u;
        for (int k = threadIdx.x; k < d.n_chain; k += kT) d.inrange[k] = 0;
        if (threadIdx.x == 0) memset(d.ctl, 0, sizeof(Ctl));
    }
}

// chain cells (the uncovered set at the start) and cells per first coverer: grid-stride blocks
// with an LDS histogram (up to kHist candidates), flushed once per block
constexpr int kHist = 1024;
__global__ __launch_bounds__(kT) void hist_kernel(DS d, int64_t n_cells) {
    __shared__ int32_t h[kHist];
    __shared__ unsigned long long tot;
    const bool lds = d.n_cand <= kHist;
    for (int q = threadIdx.x; q < kHist; q += kT) h[q] = 0;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    const uint32_t chain_mask = d.chain_bits;
    int in = 0;
    const int64_t stride = (int64_t)gridDim.x * kT;
    auto count = [&](uint32_t w, int32_t f) {
        if (!(w & chain_mask)) return;
        ++in;
        if (f != kInf) {
            if (lds) atomicAdd(&h[f], 1);
            else atomicAdd(&d.cand_cnt[f], 1);
        }
    };
    const int64_t n4 = n_cells >> 2;   // 16-byte loads; first[] only where a chain cell is
    const uint4* g4 = reinterpret_cast<const uint4*>(d.grid);
    const int4* f4 = reinterpret_cast<const int4*>(d.first);
    for (int64_t c = (int64_t)blockIdx.x * kT + threadIdx.x; c < n4; c += stride) {
        const uint4 w = g4[c];
        if (!((w.x | w.y | w.z | w.w) & chain_mask)) continue;
        const int4 f = f4[c];
        count(w.x, f.x); count(w.y, f.y); count(w.z, f.z); count(w.w, f.w);
    }
    for (int64_t c = 4 * n4 + (int64_t)blockIdx.x * kT + threadIdx.x; c < n_cells; c += stride)
        count(d.grid[c], d.first[c]);
    if (in) atomicAdd(&tot, (unsigned long long)in);
    __syncthreads();
    if (threadIdx.x == 0 && tot) atomicAdd(&d.ctl->chain_cells, tot);
    if (lds)
        for (int q = threadIdx.x; q < d.n_cand; q += kT)
            if (h[q]) atomicAdd(&d.cand_cnt[q], h[q]);
}

// the greedy walk of getSubMapCoveringCurrPoseChain (:646-695) over the candidates in node order
__global__ void accept_kernel(DS d) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const unsigned long long total = d.ctl->chain_cells;
    unsigned long long cur = total;
    bool stop = false;
    int32_t n = 0;
    for (int k = 0; k < d.n_cand; ++k) {
        d.acc[k] = 0;
        if (stop) continue;
        if (d.cand_cnt[k] > 0) {
            d.acc[k] = 1;
            cur -= (unsigned long long)d.cand_cnt[k];
            ++n;
        }
        const double coverage = 1 - ((double)cur) / (double)total;
        if (coverage >= d.cover_thr) stop = true;
    }
    d.ctl->n_acc = n;
    d.ctl->uncovered_lo = (int32_t)(cur & 0xffffffffull);
    d.ctl->uncovered_hi = (int32_t)(cur >> 32);
}

// added points of chain node k: its occupied points whose cell the submap has FREE (:757-759)
__global__ __launch_bounds__(kT) void added_kernel(DS d) {
    const int k = blockIdx.y;
    const int64_t v = d.chain[k];
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    const int64_t b0 = d.off[v], nb = d.off[v + 1] - b0;
    if (i >= nb) return;
    const int64_t b = b0 + i;
    uint8_t is_added = 0;
    if (included(d, v, b) && d.label[b] != DPG_LABEL_MAX_RANGE) {
        // the cell from the chain grid's pose; the bin score from the node's estimate (:786-800)
        const float2 m = map_point_at(d.cframe[2 * k], d.plaser[b]);
        int64_t c;
        if (cell_of(d, m.x, m.y, &c)) {
            const uint32_t w = d.grid[c];
            if ((w & kSubFree) && !(w & kSubOcc)) {
                is_added = 1;
                score_bin(d, k, d.chain_sep ? map_point(d, v, b) : m);
            }
        }
    }
    d.added[(int64_t)k * d.max_beams + i] = is_added;
}

// removed points: occupied points of submap nodes in cells chain node k has FREE (:761-763)
__global__ __launch_bounds__(kT) void removed_kernel(DS d) {
    const int j = blockIdx.y;
    if (!d.acc[j]) return;
    const int64_t v = d.cand[j];
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    const int64_t b0 = d.off[v], nb = d.off[v + 1] - b0;
    if (i >= nb) return;
    const int64_t b = b0 + i;
    uint32_t mask = 0;
    if (included(d, v, b) && d.label[b] != DPG_LABEL_MAX_RANGE) {
        const float2 m = map_point(d, v, b);
        int64_t c;
        if (cell_of(d, m.x, m.y, &c)) {
            const uint32_t w = d.grid[c];
            for (int k = 0; k < d.n_chain; ++k) {
                if (((w >> (2 * d.slot[k])) & 3u) == 1u) {     // FREE in chain node k's grid
                    mask |= 1u << k;
                    score_bin(d, k, m);
                }
            }
        }
    }
    d.rmask[(int64_t)j * d.max_beams + i] = (uint16_t)mask;
}

// computeBinScoreAndCommitLabelsForNode's verdict (:802-829): |bins| / totalBins >= threshold,
// evaluated only if some changed point fell inside the scan's angle range
__global__ void commit_kernel(DS d) {
    __shared__ int32_t mask;
    if (threadIdx.x == 0) mask = 0;
    __syncthreads();
    for (int k = threadIdx.x; k < d.n_chain; k += blockDim.x) {
        int pop = 0;
        for (int w = 0; w < d.bin_words; ++w) pop += __popc(d.bins[(int64_t)k * d.bin_words + w]);
        const int ok = d.inrange[k] && ((double)pop / (double)d.total_bins >= d.change_thr);
        d.commit[k] = ok;
        if (ok) atomicOr(&mask, 1 << k);
    }
    __syncthreads();
    if (threadIdx.x == 0) d.commit[d.n_chain] = mask;
}

__global__ __launch_bounds__(kT) void apply_added_kernel(DS d) {
    const int k = blockIdx.y;
    if (!d.commit[k]) return;
    const int64_t v = d.chain[k];
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    const int64_t b0 = d.off[v], nb = d.off[v + 1] - b0;
    const bool a = i < nb && d.added[(int64_t)k * d.max_beams + i];
    if (a) d.label[b0 + i] = DPG_LABEL_ADDED;
    const int cnt = __syncthreads_count(a);
    if (threadIdx.x == 0 && cnt) atomicAdd(&d.ctl->n_added, (unsigned long long)cnt);
}

// setPointLabel(REMOVED) on the point's own node (Q8 fix of :739): label + sector off
__global__ __launch_bounds__(kT) void apply_removed_kernel(DS d) {
    const int j = blockIdx.y;
    if (!d.acc[j]) return;
    const int64_t v = d.cand[j];
    const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
    const int64_t b0 = d.off[v], nb = d.off[v + 1] - b0;
    if (i >= nb) return;
    if (!(d.rmask[(int64_t)j * d.max_beams + i] & (uint32_t)d.commit[d.n_chain])) return;
    const int64_t b = b0 + i;
    d.label[b] = DPG_LABEL_REMOVED;
    const uint32_t bit = 1u << d.sector[b];
    const uint32_t old = atomicAnd(&d.sect[v], ~bit);
    if (old & bit) atomicAdd(&d.ctl->sect_off, 1ull);
    const unsigned long long slot = atomicAdd(&d.ctl->n_removed, 1ull);
    d.removed_xy[slot] = map_point(d, v, b);
}

// DpgNode::deactivateIntersectingSectors for every past node (dpg_node.cc:28-96), Q8 fix: a point
// in an already inactive sector is skipped (continue) instead of ending the loop (break)
__global__ __launch_bounds__(kT) void deactivate_kernel(DS d) {
    const int64_t v = blockIdx.x;
    if (!d.active[v]) return;
    const int64_t n_removed = (int64_t)d.ctl->n_removed;   // written by apply_removed_kernel
    __shared__ uint32_t mask;
    const uint32_t m0 = d.sect[v];
    if (threadIdx.x == 0) mask = m0;
    __syncthreads();
    const float4 gm = d.geom[v];                 // amin, amax, rmax, angle_inc
    const float sector_size = (gm.y - gm.x) / (float)d.num_sectors;
    const int64_t b0 = d.off[v], nb = d.off[v + 1] - b0;
    for (int64_t q = threadIdx.x; q < n_removed; q += kT) {
        const float2 r = rel_lidar(d, v, d.removed_xy[q]);
        const float norm = __fsqrt_rn(r.x * r.x + r.y * r.y);
        if (norm > gm.z) continue;
        const float a = dpg_atan2f(r.y, r.x);   // the host libm's atan2f, bit for bit
        if (a > gm.y || a < gm.x) continue;
        const uint32_t s = (uint8_t)((a - gm.x) / sector_size);
        if ((int)s >= d.num_sectors || !((mask >> s) & 1u)) continue;
        const float approx = (a - gm.x) / gm.w;
        int64_t fl = (int64_t)floorf(approx);
        fl = fl < 0 ? 0 : (fl > nb - 1 ? nb - 1 : fl);   // bounds guard (the reference indexes unchecked)
        float fov = d.range[b0 + fl];
        if (fl < nb - 1) fov = fminf(fov, d.range[b0 + fl + 1]);
        if (fov > norm) atomicAnd(&mask, ~(1u << s));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t m = mask;
        d.sect[v] = m;
        const int off = __popc(m0 & ~m);
        if (off) atomicAdd(&d.ctl->sect_off, (unsigned long long)off);
        const uint32_t full = (1u << d.num_sectors) - 1u;
        if (d.min_pct > ((float)__popc(m & full)) / (float)d.num_sectors) {
            d.active[v] = 0;
            atomicAdd(&d.ctl->nodes_off, 1ull);
        }
    }
}

// getActiveAndDynamicMapPoints: per node, the four category flags of each beam packed as 16-bit
// lanes of a u64, scanned over the block so each list keeps node/beam order
__device__ __forceinline__ uint64_t categories(const DS& d, int64_t v, int64_t b) {
    const uint8_t l = d.label[b];
    if (l == DPG_LABEL_NOT_YET_LABELED || l == DPG_LABEL_MAX_RANGE) return 0;
    uint64_t f = 0;
    if (d.active[v] && ((d.sect[v] >> d.sector[b]) & 1u)) {
        if (l == DPG_LABEL_STATIC) f |= 1ull;
        else if (l == DPG_LABEL_ADDED) f |= 1ull << 16;
    }
    if (l == DPG_LABEL_ADDED) f |= 1ull << 48;
    else if (l == DPG_LABEL_REMOVED) f |= 1ull << 32;
    return f;
}

template <bool WRITE>
__global__ __launch_bounds__(kT) void map_lists_kernel(DS d, int64_t* counts /*[V][4]*/, const int64_t* base /*[4]*/,
                                                       float2* out, int64_t cap) {
    const int64_t v = blockIdx.x;
    const int64_t b0 = d.off[v], nb = d.off[v + 1] - b0;
    __shared__ uint64_t scan[kT];
    int64_t run[4] = {0, 0, 0, 0};
    if (WRITE)
        for (int l = 0; l < 4; ++l) run[l] = base[l] + counts[4 * v + l];
    for (int64_t i0 = 0; i0 < nb; i0 += kT) {
        const int64_t i = i0 + threadIdx.x;
        const uint64_t f = i < nb ? categories(d, v, b0 + i) : 0;
        scan[threadIdx.x] = f;
        __syncthreads();
        for (int s = 1; s < kT; s <<= 1) {     // inclusive Hillis-Steele over the packed lanes
            const uint64_t add = threadIdx.x >= s ? scan[threadIdx.x - s] : 0;
            __syncthreads();
            scan[threadIdx.x] += add;
            __syncthreads();
        }
        const uint64_t incl = scan[threadIdx.x], tot = scan[kT - 1];
        if (WRITE && f) {
            const float2 m = map_point(d, v, b0 + i);
            const uint64_t excl = incl - f;
            for (int l = 0; l < 4; ++l) {
                if ((f >> (16 * l)) & 0xffff) {
                    const int64_t pos = run[l] + (int64_t)((excl >> (16 * l)) & 0xffff);
                    if (pos < cap) out[pos] = m;
                }
            }
        }
        for (int l = 0; l < 4; ++l) run[l] += (int64_t)((tot >> (16 * l)) & 0xffff);
        __syncthreads();
    }
    if (!WRITE && threadIdx.x == 0)
        for (int l = 0; l < 4; ++l) counts[4 * v + l] = run[l];
}

template <typename T>
struct Buf {
    T* p = nullptr;
    size_t cap = 0;
    int reserve(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return -1;
        cap = n;
        return 0;
    }
    ~Buf() { if (p) (void)hipFree(p); }
};

double now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

// math_utils::AngleMod<float> (math_utils.h:13-16)
float angle_mod_f(float a) {
    double ad = (double)a;
    ad -= (M_PI * 2.0) * rint(ad / (M_PI * 2.0));
    return (float)ad;
}

}  // namespace

struct dpg_dpg {
    dpg_ctx* ctx = nullptr;
    hipStream_t s = nullptr;
    int device = 0;
    dpg_change_params p{};
    int64_t V = 0, B = 0;
    int32_t max_beams = 0;
    std::vector<int64_t> off;
    std::vector<float> geom;          // [V][4]
    std::vector<float> rmax_beam;     // largest range of each node's beams (window size)
    std::vector<uint8_t> active_h;    // host mirror of the node activity
    std::vector<float> h_pose;        // [V][3] pose bits the cached frames were computed from (NaN: none)
    float* h_frames = nullptr;        // [V][8] cached node frames, pinned (see upload_frames)
    int64_t h_cap = 0;                // nodes the pinned mirrors (h_frames, h_act) hold
    unsigned char* h_app = nullptr;   // pinned staging of dpg_dpg_append's uploads
    size_t app_cap = 0;
    // pinned staging of the per-call inputs/outputs: one H2D copy of [chain 16 | slot 16 | rast 16 |
    // chain frames 128 | candidates], one D2H of the node activity and the commit flags
    int32_t* h_stage = nullptr;
    int64_t stage_cap = 0;
    uint32_t* h_act = nullptr;
    int32_t* h_commit = nullptr;
    // the window kept across calls: chain grids of nodes still in the chain (same pose) stay as
    // planes; only the new chain node is rasterised (see dpg_execute_dpg)
    Box win{};
    bool win_valid = false;
    int32_t slot_node[15];
    float slot_pose[15][3];
    Buf<int64_t> d_off;
    Buf<float2> d_plaser;
    Buf<float> d_range;
    Buf<uint8_t> d_label, d_sector;
    Buf<float4> d_geom, d_frame;
    Buf<uint32_t> d_sect, d_active, d_grid, d_bins;
    Buf<int32_t> d_first, d_stage, d_cand_cnt, d_acc, d_inrange, d_commit;
    Buf<uint8_t> d_added;
    Buf<uint16_t> d_rmask;
    Buf<float2> d_removed, d_map_out;
    Buf<Ctl> d_ctl;
    Buf<int64_t> d_counts, d_base;
    Ctl* h_ctl = nullptr;             // pinned
    hipEvent_t ev[2] = {};
};

#define DTRY(expr)                                                                     \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) return dpg_set_error(DPG_ERR_HIP, hipGetErrorString(_e)); \
    } while (0)

namespace {

constexpr int64_t kStageCand = 48 + 128;   // int32 offset of the candidates in the staging block

DS make_ds(dpg_dpg* d) {
    DS s;
    memset(&s, 0, sizeof(s));
    s.off = d->d_off.p; s.plaser = d->d_plaser.p; s.range = d->d_range.p; s.label = d->d_label.p;
    s.sector = d->d_sector.p; s.geom = d->d_geom.p; s.sect = d->d_sect.p; s.active = d->d_active.p;
    s.frame = d->d_frame.p; s.grid = d->d_grid.p; s.first = d->d_first.p; s.chain = d->d_stage.p;
    s.slot = d->d_stage.p ? d->d_stage.p + 16 : nullptr; s.rast = d->d_stage.p ? d->d_stage.p + 32 : nullptr;
    s.cframe = d->d_stage.p ? reinterpret_cast<const float4*>(d->d_stage.p + 48) : nullptr;
    s.cand = d->d_stage.p ? d->d_stage.p + kStageCand : nullptr; s.cand_cnt = d->d_cand_cnt.p; s.acc = d->d_acc.p; s.bins = d->d_bins.p;
    s.inrange = d->d_inrange.p; s.commit = d->d_commit.p; s.added = d->d_added.p; s.rmask = d->d_rmask.p;
    s.removed_xy = d->d_removed.p; s.ctl = d->d_ctl.p;
    s.res = d->p.occ_grid_resolution; s.inv_res = 1.0 / d->p.occ_grid_resolution; s.max_beams = d->max_beams; s.num_sectors = d->p.num_sectors;
    s.total_bins = d->p.num_bins_for_change_detection;
    s.bin_words = (d->p.num_bins_for_change_detection + 2 + 31) / 32;
    s.min_pct = d->p.minimum_percent_active_sectors;
    s.change_thr = d->p.delta_change_threshold;
    s.cover_thr = d->p.current_pose_graph_coverage_threshold;
    return s;
}

// node frames: lidar pose in the map (transformPoint(laser, node pose), dpg_node.cc:34-36) with
// Rotation2Df(a) and Rotation2Df(-a) coefficients from the host libm.  Cached per node and keyed
// by the pose bits: only nodes whose estimate changed since the last call are recomputed and
// uploaded (a call after a re-optimisation refreshes them all).
void node_frame(const dpg_dpg* d, const float* e, float* f) {
    const float th = e[2];
    const float c0 = cosf(th), s0 = sinf(th), ns0 = -s0;
    const float lx = e[0] + (c0 * d->p.laser[0] + ns0 * d->p.laser[1]);
    const float ly = e[1] + (s0 * d->p.laser[0] + c0 * d->p.laser[1]);
    const float a = angle_mod_f(th + d->p.laser[2]);
    f[0] = lx; f[1] = ly; f[2] = cosf(a); f[3] = sinf(a); f[4] = cosf(-a); f[5] = sinf(-a); f[6] = 0.f; f[7] = 0.f;
}

// active_only: executeDPG reads the frames of active nodes only (inactive nodes have no grid and
// skip the sector update), so after a re-optimisation only those are recomputed; a stale frame of
// an inactive node keeps its old pose bits in h_pose and is refreshed when the map lists need it
int upload_frames(dpg_dpg* d, int64_t V, const float* est, bool active_only = false) {
    int64_t lo = V, hi = -1;
    for (int64_t v = 0; v < V; ++v) {
        if (active_only && !d->active_h[(size_t)v]) continue;
        float* c = &d->h_pose[(size_t)(3 * v)];
        if (memcmp(c, est + 3 * v, 3 * sizeof(float)) == 0) continue;
        memcpy(c, est + 3 * v, 3 * sizeof(float));
        node_frame(d, est + 3 * v, &d->h_frames[(size_t)(8 * v)]);
        lo = std::min(lo, v);
        hi = v;
    }
    if (hi >= lo)
        DTRY(hipMemcpyAsync(d->d_frame.p + 2 * lo, &d->h_frames[(size_t)(8 * lo)], sizeof(float) * 8 * (hi - lo + 1),
                            hipMemcpyHostToDevice, d->s));
    return DPG_OK;
}

}  // namespace

namespace {
int finish_call(dpg_dpg* d, int64_t V, int64_t chain_n, double t0, dpg_change_stats* st);
}  // namespace

extern "C" {

void dpg_change_params_default(dpg_change_params* p) {
    memset(p, 0, sizeof(*p));
    p->num_sectors = 5;
    p->current_pose_chain_len = 5;
    p->num_bins_for_change_detection = 36;
    p->delta_change_threshold = 0.20;
    p->current_pose_graph_coverage_threshold = 1.0;
    p->occ_grid_resolution = 0.05;
    p->minimum_percent_active_sectors = 0.5f;
    p->distance_threshold_for_local_submap_nodes = 5.0f;
    p->laser[0] = 0.2f; p->laser[1] = 0.f; p->laser[2] = 0.f;
}

dpg_dpg* dpg_dpg_create(dpg_ctx* ctx, int64_t V, const int64_t* off, const float* ranges, const float* geom,
                        const dpg_change_params* p) {
    if (!ctx || V <= 0 || !off || !ranges || !geom || !p) { dpg_set_error(DPG_ERR_ARG, "bad arguments"); return nullptr; }
    if (p->num_sectors < 1 || p->num_sectors > 8 || p->current_pose_chain_len < 0 || p->current_pose_chain_len > 15 ||
        p->num_bins_for_change_detection < 1 || p->num_bins_for_change_detection > 65534 || !(p->occ_grid_resolution > 0)) {
        dpg_set_error(DPG_ERR_ARG, "change params out of range (sectors 1..8, chain 0..15, bins 1..65534, resolution > 0)");
        return nullptr;
    }
    dpg_dpg* d = new dpg_dpg();
    d->ctx = ctx;
    d->s = reinterpret_cast<hipStream_t>(dpg_ctx_stream_of(ctx));
    d->device = dpg_ctx_device_of(ctx);
    d->p = *p;
    d->V = V;
    d->B = off[V];
    d->off.assign(off, off + V + 1);
    d->geom.resize((size_t)(4 * V));
    d->rmax_beam.assign((size_t)V, 0.f);
    d->active_h.assign((size_t)V, 1);
    d->h_pose.assign((size_t)(3 * V), NAN);
    for (int q = 0; q < 15; ++q) d->slot_node[q] = -1;
    std::vector<float2> pl((size_t)d->B);
    std::vector<uint8_t> lab((size_t)d->B), sec((size_t)d->B);
    for (int64_t v = 0; v < V; ++v) {
        const int64_t nb = off[v + 1] - off[v];
        if (nb < 2 || nb > 65535) { delete d; dpg_set_error(DPG_ERR_SIZE, "beams per scan must be in [2, 65535]"); return nullptr; }
        d->max_beams = std::max<int32_t>(d->max_beams, (int32_t)nb);
        const float amin = geom[3 * v], amax = geom[3 * v + 1], rmax = geom[3 * v + 2];
        // createNode (dpg_slam.cc:497-507) and MeasurementPoint (dpg_measurement.h:41-46,102-104)
        const float ainc = (float)((double)(amax - amin) / ((double)nb - 1.0));
        const float per_sector = ((float)nb) / (float)p->num_sectors;
        d->geom[(size_t)(4 * v)] = amin; d->geom[(size_t)(4 * v + 1)] = amax;
        d->geom[(size_t)(4 * v + 2)] = rmax; d->geom[(size_t)(4 * v + 3)] = ainc;
        for (int64_t i = 0; i < nb; ++i) {
            const int64_t b = off[v] + i;
            const float angle = ainc * (float)i + amin;
            const float r = ranges[b];
            pl[(size_t)b] = make_float2(r * cosf(angle), r * sinf(angle));
            lab[(size_t)b] = r >= rmax ? DPG_LABEL_MAX_RANGE : DPG_LABEL_NOT_YET_LABELED;
            sec[(size_t)b] = (uint8_t)((float)i / per_sector);
            d->rmax_beam[(size_t)v] = std::max(d->rmax_beam[(size_t)v], r);
        }
    }
    std::vector<uint32_t> sect((size_t)V, (1u << p->num_sectors) - 1u), act((size_t)V, 1u);
    // error paths free what was allocated so far (pinned mirrors, events, device buffers)
    auto bad = [&](const char* m) { dpg_dpg_destroy(d); dpg_set_error(DPG_ERR_HIP, m); return (dpg_dpg*)nullptr; };
    if (hipSetDevice(d->device) != hipSuccess) return bad("hipSetDevice failed");
    if (d->d_off.reserve((size_t)(V + 1)) || d->d_plaser.reserve((size_t)d->B) || d->d_range.reserve((size_t)d->B) ||
        d->d_label.reserve((size_t)d->B) || d->d_sector.reserve((size_t)d->B) || d->d_geom.reserve((size_t)V) ||
        d->d_sect.reserve((size_t)V) || d->d_active.reserve((size_t)V) || d->d_ctl.reserve(1) ||
        d->d_frame.reserve((size_t)(2 * V)))
        return bad("hipMalloc failed");
    if (hipHostMalloc(reinterpret_cast<void**>(&d->h_ctl), sizeof(Ctl), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&d->h_frames), sizeof(float) * 8 * V, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&d->h_act), sizeof(uint32_t) * V, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&d->h_commit), sizeof(int32_t) * 16, hipHostMallocDefault) != hipSuccess)
        return bad("hipHostMalloc failed");
    memset(d->h_frames, 0, sizeof(float) * 8 * V);
    d->h_cap = V;
    hipStream_t s = d->s;
    if (hipMemcpyAsync(d->d_off.p, off, sizeof(int64_t) * (V + 1), hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d->d_plaser.p, pl.data(), sizeof(float2) * d->B, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d->d_range.p, ranges, sizeof(float) * d->B, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d->d_label.p, lab.data(), d->B, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d->d_sector.p, sec.data(), d->B, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d->d_geom.p, d->geom.data(), sizeof(float) * 4 * V, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d->d_sect.p, sect.data(), sizeof(uint32_t) * V, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d->d_active.p, act.data(), sizeof(uint32_t) * V, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return bad("upload of the node store failed");
    for (auto& e : d->ev) (void)hipEventCreate(&e);
    dpg_ctx_adopt(ctx, d, [](void* x) { dpg_dpg_destroy(static_cast<dpg_dpg*>(x)); });
    return d;
}

// One node per call on the DpgSLAM path: the cost is per call, so nothing here is O(V) -- the
// device arrays and the pinned mirrors grow by 1.5x with their contents kept, the new nodes' data
// are built straight into one pinned staging block and go up from it (only the new offsets, not
// the whole offset array), and the stream is not waited on at the end (the next call, or any
// executeDPG, is queued behind these copies; the staging block is reused only after the stream
// synchronisation that opens the next call).
int dpg_dpg_append(dpg_dpg* d, int64_t n_new, const int64_t* off_rel, const float* ranges, const float* geom) {
    if (!d || n_new < 0 || (n_new > 0 && (!off_rel || !ranges || !geom))) return dpg_set_error(DPG_ERR_ARG, "bad arguments");
    if (n_new == 0) return DPG_OK;
    DTRY(hipSetDevice(d->device));
    hipStream_t s = d->s;
    DTRY(hipStreamSynchronize(s));
    const int64_t V0 = d->V, B0 = d->B, V1 = V0 + n_new, nb_new = off_rel[n_new] - off_rel[0];
    int32_t max_beams = d->max_beams;
    for (int64_t k = 0; k < n_new; ++k) {
        const int64_t nb = off_rel[k + 1] - off_rel[k];
        if (nb < 2 || nb > 65535) return dpg_set_error(DPG_ERR_SIZE, "beams per scan must be in [2, 65535]");
        max_beams = std::max<int32_t>(max_beams, (int32_t)nb);
    }
    // staging layout (16-B aligned parts): offsets [n_new] i64 | plaser [nb] float2 | range [nb] f32 |
    // geom [n_new] float4 | sect [n_new] u32 | active [n_new] u32 | label [nb] u8 | sector [nb] u8
    auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
    const size_t o_off = 0, o_pl = al(o_off + 8 * (size_t)n_new), o_rg = al(o_pl + 8 * (size_t)nb_new),
                 o_gm = al(o_rg + 4 * (size_t)nb_new), o_sc = al(o_gm + 16 * (size_t)n_new),
                 o_ac = al(o_sc + 4 * (size_t)n_new), o_lb = al(o_ac + 4 * (size_t)n_new), o_sr = al(o_lb + (size_t)nb_new),
                 need = al(o_sr + (size_t)nb_new);
    if (need > d->app_cap) {
        unsigned char* nb = nullptr;
        const size_t cap = std::max(need, d->app_cap + d->app_cap / 2);
        if (hipHostMalloc(reinterpret_cast<void**>(&nb), cap, hipHostMallocDefault) != hipSuccess)
            return dpg_set_error(DPG_ERR_HIP, "hipHostMalloc(append staging) failed");
        if (d->h_app) (void)hipHostFree(d->h_app);
        d->h_app = nb;
        d->app_cap = cap;
    }
    unsigned char* st = d->h_app;
    int64_t* off_new = reinterpret_cast<int64_t*>(st + o_off);
    float2* pl = reinterpret_cast<float2*>(st + o_pl);
    float* rg = reinterpret_cast<float*>(st + o_rg);
    float* gm = reinterpret_cast<float*>(st + o_gm);
    uint32_t* sect = reinterpret_cast<uint32_t*>(st + o_sc);
    uint32_t* act = reinterpret_cast<uint32_t*>(st + o_ac);
    uint8_t* lab = st + o_lb;
    uint8_t* sec = st + o_sr;
    // the new nodes' largest ranges and the beam maximum are committed to d only after every
    // allocation and copy below succeeded (as off and V)
    std::vector<float> rmax_new((size_t)n_new);
    int64_t last = d->off.back();
    for (int64_t k = 0; k < n_new; ++k) {
        const int64_t nb = off_rel[k + 1] - off_rel[k];
        const float amin = geom[3 * k], amax = geom[3 * k + 1], rmax = geom[3 * k + 2];
        const float ainc = (float)((double)(amax - amin) / ((double)nb - 1.0));   // createNode (dpg_slam.cc:497)
        const float per_sector = ((float)nb) / (float)d->p.num_sectors;
        gm[4 * k] = amin; gm[4 * k + 1] = amax; gm[4 * k + 2] = rmax; gm[4 * k + 3] = ainc;
        float rm = 0.f;
        for (int64_t i = 0; i < nb; ++i) {
            const int64_t b = off_rel[k] - off_rel[0] + i;
            const float angle = ainc * (float)i + amin;
            const float r = ranges[b];
            pl[b] = make_float2(r * cosf(angle), r * sinf(angle));
            rg[b] = r;
            lab[b] = r >= rmax ? DPG_LABEL_MAX_RANGE : DPG_LABEL_NOT_YET_LABELED;
            sec[b] = (uint8_t)((float)i / per_sector);
            rm = std::max(rm, r);
        }
        last += nb;
        off_new[k] = last;
        rmax_new[(size_t)k] = rm;
        sect[k] = (1u << d->p.num_sectors) - 1u;
        act[k] = 1u;
    }
    // device arrays grow with their contents kept (amortised x1.5)
    auto grow = [&](auto& b, size_t used, size_t need_n) -> int {
        using T = std::remove_pointer_t<decltype(b.p)>;
        if (need_n <= b.cap) return 0;
        const size_t cap = std::max(need_n, b.cap + b.cap / 2);
        T* np = nullptr;
        if (hipMalloc(reinterpret_cast<void**>(&np), cap * sizeof(T)) != hipSuccess) return -1;
        if (used && hipMemcpyAsync(np, b.p, used * sizeof(T), hipMemcpyDeviceToDevice, s) != hipSuccess) { (void)hipFree(np); return -1; }
        if (hipStreamSynchronize(s) != hipSuccess) { (void)hipFree(np); return -1; }
        if (b.p) (void)hipFree(b.p);
        b.p = np;
        b.cap = cap;
        return 0;
    };
    const size_t B1 = (size_t)(B0 + nb_new);
    if (grow(d->d_off, (size_t)(V0 + 1), (size_t)(V1 + 1)) || grow(d->d_plaser, (size_t)B0, B1) || grow(d->d_range, (size_t)B0, B1) ||
        grow(d->d_label, (size_t)B0, B1) || grow(d->d_sector, (size_t)B0, B1) || grow(d->d_geom, (size_t)V0, (size_t)V1) ||
        grow(d->d_sect, (size_t)V0, (size_t)V1) || grow(d->d_active, (size_t)V0, (size_t)V1) ||
        grow(d->d_frame, (size_t)(2 * V0), (size_t)(2 * V1)))
        return dpg_set_error(DPG_ERR_HIP, "hipMalloc(node store growth) failed");
    // pinned host mirrors, amortised x1.5
    if (V1 > d->h_cap) {
        const int64_t cap = std::max<int64_t>(V1, d->h_cap + d->h_cap / 2);
        float* nf = nullptr;
        uint32_t* na = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&nf), sizeof(float) * 8 * cap, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&na), sizeof(uint32_t) * cap, hipHostMallocDefault) != hipSuccess) {
            if (nf) (void)hipHostFree(nf);
            return dpg_set_error(DPG_ERR_HIP, "hipHostMalloc(node store growth) failed");
        }
        memcpy(nf, d->h_frames, sizeof(float) * 8 * V0);
        (void)hipHostFree(d->h_frames);
        (void)hipHostFree(d->h_act);
        d->h_frames = nf;
        d->h_act = na;
        d->h_cap = cap;
    }
    memset(d->h_frames + 8 * V0, 0, sizeof(float) * 8 * n_new);
    DTRY(hipMemcpyAsync(d->d_off.p + V0 + 1, off_new, sizeof(int64_t) * n_new, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(d->d_plaser.p + B0, pl, sizeof(float2) * nb_new, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(d->d_range.p + B0, rg, sizeof(float) * nb_new, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(d->d_label.p + B0, lab, nb_new, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(d->d_sector.p + B0, sec, nb_new, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(d->d_geom.p + V0, gm, sizeof(float) * 4 * n_new, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(d->d_sect.p + V0, sect, sizeof(uint32_t) * n_new, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(d->d_active.p + V0, act, sizeof(uint32_t) * n_new, hipMemcpyHostToDevice, s));
    d->h_pose.resize((size_t)(3 * V1), NAN);
    d->active_h.resize((size_t)V1, 1);
    d->geom.insert(d->geom.end(), gm, gm + 4 * n_new);
    d->off.insert(d->off.end(), off_new, off_new + n_new);
    d->V = V1;
    d->B = (int64_t)B1;
    d->rmax_beam.insert(d->rmax_beam.end(), rmax_new.begin(), rmax_new.end());
    d->max_beams = max_beams;
    return DPG_OK;
}

void dpg_dpg_destroy(dpg_dpg* d) {
    if (!d) return;
    dpg_ctx_release_child(d->ctx, d);
    (void)hipSetDevice(d->device);
    (void)hipStreamSynchronize(d->s);
    if (d->h_ctl) (void)hipHostFree(d->h_ctl);
    if (d->h_frames) (void)hipHostFree(d->h_frames);
    if (d->h_act) (void)hipHostFree(d->h_act);
    if (d->h_commit) (void)hipHostFree(d->h_commit);
    if (d->h_stage) (void)hipHostFree(d->h_stage);
    if (d->h_app) (void)hipHostFree(d->h_app);
    for (auto& e : d->ev) if (e) (void)hipEventDestroy(e);
    delete d;
}

int dpg_execute_dpg(dpg_dpg* d, int64_t V, int64_t cur_len, const float* est, dpg_change_stats* st) {
    return dpg_execute_dpg_chain(d, V, cur_len, est, nullptr, st);
}

int dpg_execute_dpg_chain(dpg_dpg* d, int64_t V, int64_t cur_len, const float* est, const float* chain_poses,
                          dpg_change_stats* st) {
    if (!d || !est || V <= 0 || V > d->V || cur_len < 0 || cur_len > V) return dpg_set_error(DPG_ERR_ARG, "bad arguments");
    const double t0 = now_ms();
    dpg_change_stats local;
    if (!st) st = &local;
    memset(st, 0, sizeof(*st));
    DTRY(hipSetDevice(d->device));
    hipStream_t s = d->s;
    const dpg_change_params& p = d->p;
    const int64_t n_past = V - cur_len;
    const int64_t chain_n = std::min<int64_t>(cur_len, p.current_pose_chain_len);
    st->n_chain = chain_n;
    std::vector<int32_t> chain;
    for (int64_t k = 0; k < chain_n; ++k) chain.push_back((int32_t)(V - chain_n + k));
    // the pose of chain node k for its grid and the proximity search: the caller's chain pose
    // (current_pass_nodes_, dpg_slam.cc:591-620,646-668) or the node's estimate
    auto cpose = [&](int64_t k) { return chain_poses ? chain_poses + 3 * k : est + 3 * (int64_t)chain[(size_t)k]; };
    // candidates: active past nodes within the proximity threshold of a chain node (:646-668)
    std::vector<int32_t> cand;
    for (int64_t j = 0; j < n_past && chain_n > 0; ++j) {
        if (!d->active_h[(size_t)j]) continue;
        for (int64_t k = 0; k < chain_n; ++k) {
            const float* c = cpose(k);
            const float dx = c[0] - est[3 * j], dy = c[1] - est[3 * j + 1];
            if (sqrtf(dx * dx + dy * dy) <= p.distance_threshold_for_local_submap_nodes) { cand.push_back((int32_t)j); break; }
        }
    }
    st->n_candidates = (int64_t)cand.size();
    int rc = upload_frames(d, V, est, true);
    if (rc) return rc;
    if (d->d_ctl.reserve(1)) return dpg_set_error(DPG_ERR_HIP, "hipMalloc(ctl) failed");
    if (chain_n == 0) {   // no pose chain: only the sector/node update of the (empty) removed set runs
        DS ds = make_ds(d);
        DTRY(hipEventRecord(d->ev[0], s));
        DTRY(hipMemsetAsync(d->d_ctl.p, 0, sizeof(Ctl), s));
        if (n_past > 0) deactivate_kernel<<<(unsigned)n_past, kT, 0, s>>>(ds);
        DTRY(hipGetLastError());
        DTRY(hipEventRecord(d->ev[1], s));
        return finish_call(d, V, 0, t0, st);
    }
    // window: every chain ray stays within its longest range of the lidar
    float cfr[15][8];   // chain frames at the chain poses
    int32_t chain_sep = 0;
    for (int64_t k = 0; k < chain_n; ++k) {
        const float* c = cpose(k);
        const int32_t v = chain[(size_t)k];
        if (!std::isfinite(c[0]) || !std::isfinite(c[1]) || !std::isfinite(c[2]) ||
            !std::isfinite(est[3 * v]) || !std::isfinite(est[3 * v + 1]) || !std::isfinite(est[3 * v + 2]))
            return dpg_set_error(DPG_ERR_ARG, "non-finite pose in the pose chain");
        node_frame(d, c, cfr[k]);
        if (memcmp(c, est + 3 * v, 3 * sizeof(float)) != 0) chain_sep = 1;
    }
    double xlo = 1e300, xhi = -1e300, ylo = 1e300, yhi = -1e300;
    for (int64_t k = 0; k < chain_n; ++k) {
        const double r = d->rmax_beam[(size_t)chain[(size_t)k]];
        xlo = std::min(xlo, cfr[k][0] - r); xhi = std::max(xhi, cfr[k][0] + r);
        ylo = std::min(ylo, cfr[k][1] - r); yhi = std::max(yhi, cfr[k][1] + r);
    }
    Box need;
    need.x0 = (int32_t)floor(xlo / p.occ_grid_resolution) - 4;
    need.y0 = (int32_t)floor(ylo / p.occ_grid_resolution) - 4;
    need.w = (int32_t)ceil(xhi / p.occ_grid_resolution) + 4 - need.x0 + 1;
    need.h = (int32_t)ceil(yhi / p.occ_grid_resolution) + 4 - need.y0 + 1;
    const Box& w0 = d->win;
    const bool reuse = d->win_valid && need.x0 >= w0.x0 && need.y0 >= w0.y0 && need.x0 + need.w <= w0.x0 + w0.w &&
                       need.y0 + need.h <= w0.y0 + w0.h;
    if (!reuse) {   // new window with a margin, so the next chain nodes usually still fit
        const int32_t m = (int32_t)ceil(4.0 / p.occ_grid_resolution);
        Box nw{need.x0 - m, need.y0 - m, need.w + 2 * m, need.h + 2 * m};
        if ((int64_t)nw.w * nw.h > (int64_t)1 << 28) nw = need;
        if ((int64_t)nw.w * nw.h > (int64_t)1 << 28)
            return dpg_set_error(DPG_ERR_SIZE, "change-detection window exceeds 2^28 cells");
        if (d->d_grid.reserve((size_t)nw.w * nw.h) || d->d_first.reserve((size_t)nw.w * nw.h))
            return dpg_set_error(DPG_ERR_HIP, "hipMalloc(window) failed");
        d->win = nw;
        d->win_valid = true;
        for (int q = 0; q < 15; ++q) d->slot_node[q] = -1;
    }
    const Box box = d->win;
    const int64_t cells = (int64_t)box.w * box.h;
    st->grid_cells = cells;
    // bit-plane slots: a chain node keeps its plane while it stays in the chain with the same pose
    std::vector<int32_t> slot((size_t)chain_n, -1), rast;
    uint32_t keep = 0, chain_bits = 0;
    for (int q = 0; q < 15; ++q) {
        const int32_t v = d->slot_node[q];
        if (v < 0) continue;
        int64_t k = v - (V - chain_n);
        if (k >= 0 && k < chain_n && memcmp(d->slot_pose[q], cpose(k), 3 * sizeof(float)) == 0) {
            slot[(size_t)k] = q;
            keep |= 3u << (2 * q);
        } else {
            d->slot_node[q] = -1;
        }
    }
    for (int64_t k = 0; k < chain_n; ++k) {
        if (slot[(size_t)k] < 0) {
            int q = 0;
            while (d->slot_node[q] >= 0) ++q;   // chain_n <= 15 planes: always one free
            d->slot_node[q] = chain[(size_t)k];
            memcpy(d->slot_pose[q], cpose(k), 3 * sizeof(float));
            slot[(size_t)k] = q;
            rast.push_back((int32_t)k);
        }
        chain_bits |= 3u << (2 * slot[(size_t)k]);
    }
    const int64_t nc = (int64_t)cand.size();
    const int32_t bin_words = (p.num_bins_for_change_detection + 2 + 31) / 32;
    if (d->stage_cap < kStageCand + nc) {
        if (d->h_stage) (void)hipHostFree(d->h_stage);
        d->h_stage = nullptr;
        d->stage_cap = 0;
        const int64_t cap = kStageCand + std::max<int64_t>(2 * nc, 256);
        if (hipHostMalloc(reinterpret_cast<void**>(&d->h_stage), sizeof(int32_t) * cap, hipHostMallocDefault) != hipSuccess)
            return dpg_set_error(DPG_ERR_HIP, "hipHostMalloc(stage) failed");
        d->stage_cap = cap;
    }
    if (d->d_stage.reserve((size_t)d->stage_cap) || d->d_cand_cnt.reserve((size_t)std::max<int64_t>(nc, 1)) ||
        d->d_acc.reserve((size_t)std::max<int64_t>(nc, 1)) || d->d_bins.reserve((size_t)(chain_n * bin_words)) ||
        d->d_inrange.reserve((size_t)chain_n) || d->d_commit.reserve((size_t)chain_n + 1) ||
        d->d_added.reserve((size_t)(chain_n * d->max_beams)) ||
        d->d_rmask.reserve((size_t)(std::max<int64_t>(nc, 1) * d->max_beams)) ||
        d->d_removed.reserve((size_t)(std::max<int64_t>(nc, 1) * d->max_beams)))
        return dpg_set_error(DPG_ERR_HIP, "hipMalloc(change scratch) failed");
    DTRY(hipEventRecord(d->ev[0], s));
    int32_t* hs = d->h_stage;   // the previous call ended with a stream synchronisation
    memcpy(hs, chain.data(), sizeof(int32_t) * chain_n);
    memcpy(hs + 16, slot.data(), sizeof(int32_t) * chain_n);
    if (!rast.empty()) memcpy(hs + 32, rast.data(), sizeof(int32_t) * rast.size());
    memcpy(hs + 48, cfr, sizeof(float) * 8 * chain_n);
    if (nc) memcpy(hs + kStageCand, cand.data(), sizeof(int32_t) * nc);
    DTRY(hipMemcpyAsync(d->d_stage.p, hs, sizeof(int32_t) * (kStageCand + nc), hipMemcpyHostToDevice, s));
    DS ds = make_ds(d);
    ds.n_chain = (int32_t)chain_n;
    ds.n_cand = (int32_t)nc;
    ds.box = box;
    ds.chain_bits = chain_bits;
    ds.chain_sep = chain_sep;
    ds.keep_mask = keep;
    ds.rebuild = reuse ? 0 : 1;
    const unsigned gx = (unsigned)((d->max_beams + kT - 1) / kT);
    const unsigned gr = (unsigned)((d->max_beams + kRB / kG - 1) / (kRB / kG));
    init_kernel<<<(unsigned)std::min<int64_t>((cells + kT - 1) / kT, 2048), kT, 0, s>>>(ds, cells);
    if (!rast.empty()) raster_kernel<0><<<dim3(gr, (unsigned)rast.size()), kRB, 0, s>>>(ds);
    if (nc) raster_kernel<1><<<dim3(gr, (unsigned)nc), kRB, 0, s>>>(ds);
    hist_kernel<<<(unsigned)std::min<int64_t>((cells + kT - 1) / kT, 1024), kT, 0, s>>>(ds, cells);
    accept_kernel<<<1, 64, 0, s>>>(ds);
    if (nc) raster_kernel<2><<<dim3(gr, (unsigned)nc), kRB, 0, s>>>(ds);
    added_kernel<<<dim3(gx, (unsigned)chain_n), kT, 0, s>>>(ds);
    if (nc) removed_kernel<<<dim3(gx, (unsigned)nc), kT, 0, s>>>(ds);
    commit_kernel<<<1, 64, 0, s>>>(ds);
    apply_added_kernel<<<dim3(gx, (unsigned)chain_n), kT, 0, s>>>(ds);
    if (nc) apply_removed_kernel<<<dim3(gx, (unsigned)nc), kT, 0, s>>>(ds);
    // every active past node re-checks its active-sector fraction, removed points or not (dpg_node.cc:93-95)
    if (n_past > 0) deactivate_kernel<<<(unsigned)n_past, kT, 0, s>>>(ds);
    DTRY(hipGetLastError());
    DTRY(hipEventRecord(d->ev[1], s));
    return finish_call(d, V, chain_n, t0, st);
}

}  // extern "C"

namespace {

// read back the counters and the node activity of one dpg_execute_dpg (one synchronisation)
int finish_call(dpg_dpg* d, int64_t V, int64_t chain_n, double t0, dpg_change_stats* st) {
    hipStream_t s = d->s;
    DTRY(hipMemcpyAsync(d->h_ctl, d->d_ctl.p, sizeof(Ctl), hipMemcpyDeviceToHost, s));
    uint32_t* act = d->h_act;
    DTRY(hipMemcpyAsync(act, d->d_active.p, sizeof(uint32_t) * V, hipMemcpyDeviceToHost, s));
    int32_t* cm = d->h_commit;
    if (chain_n) DTRY(hipMemcpyAsync(cm, d->d_commit.p, sizeof(int32_t) * (chain_n + 1), hipMemcpyDeviceToHost, s));
    DTRY(hipStreamSynchronize(s));
    for (int64_t v = 0; v < V; ++v) d->active_h[(size_t)v] = act[(size_t)v] ? 1 : 0;
    const Ctl& c = *d->h_ctl;
    if (c.oob) return dpg_set_error(DPG_ERR_STATE, "a pose-chain ray left the change-detection window");
    st->n_submap_nodes = c.n_acc;
    st->n_chain_cells = (int64_t)c.chain_cells;
    st->n_uncovered = (int64_t)(((uint64_t)(uint32_t)c.uncovered_hi << 32) | (uint32_t)c.uncovered_lo);
    st->n_added = (int64_t)c.n_added;
    st->n_removed = (int64_t)c.n_removed;
    st->n_sectors_deactivated = (int64_t)c.sect_off;
    st->n_nodes_deactivated = (int64_t)c.nodes_off;
    st->n_samples = (int64_t)c.samples;
    for (int64_t k = 0; k < chain_n; ++k) st->n_committed += cm[(size_t)k] != 0;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, d->ev[0], d->ev[1]);
    st->ms_kernels = ms;
    st->ms_total = now_ms() - t0;
    return DPG_OK;
}

}  // namespace

extern "C" {

int dpg_dpg_fetch(dpg_dpg* d, uint8_t* labels, uint8_t* sector_active, uint8_t* node_active) {
    if (!d) return dpg_set_error(DPG_ERR_ARG, "bad arguments");
    DTRY(hipSetDevice(d->device));
    DTRY(hipStreamSynchronize(d->s));
    if (labels) DTRY(hipMemcpy(labels, d->d_label.p, d->B, hipMemcpyDeviceToHost));
    std::vector<uint32_t> t((size_t)d->V);
    if (sector_active) {
        DTRY(hipMemcpy(t.data(), d->d_sect.p, sizeof(uint32_t) * d->V, hipMemcpyDeviceToHost));
        for (int64_t v = 0; v < d->V; ++v) sector_active[v] = (uint8_t)t[(size_t)v];
    }
    if (node_active) {
        DTRY(hipMemcpy(t.data(), d->d_active.p, sizeof(uint32_t) * d->V, hipMemcpyDeviceToHost));
        for (int64_t v = 0; v < d->V; ++v) node_active[v] = t[(size_t)v] ? 1 : 0;
    }
    return DPG_OK;
}

int dpg_dpg_load(dpg_dpg* d, const uint8_t* labels, const uint8_t* sector_active, const uint8_t* node_active) {
    if (!d) return dpg_set_error(DPG_ERR_ARG, "bad arguments");
    DTRY(hipSetDevice(d->device));
    DTRY(hipStreamSynchronize(d->s));
    d->win_valid = false;   // the kept chain planes may no longer match the node state
    if (labels) DTRY(hipMemcpy(d->d_label.p, labels, d->B, hipMemcpyHostToDevice));
    std::vector<uint32_t> t((size_t)d->V);
    if (sector_active) {
        const uint32_t full = (1u << d->p.num_sectors) - 1u;
        for (int64_t v = 0; v < d->V; ++v) t[(size_t)v] = sector_active[v] & full;
        DTRY(hipMemcpy(d->d_sect.p, t.data(), sizeof(uint32_t) * d->V, hipMemcpyHostToDevice));
    }
    if (node_active) {
        for (int64_t v = 0; v < d->V; ++v) { t[(size_t)v] = node_active[v] ? 1u : 0u; d->active_h[(size_t)v] = node_active[v] ? 1 : 0; }
        DTRY(hipMemcpy(d->d_active.p, t.data(), sizeof(uint32_t) * d->V, hipMemcpyHostToDevice));
    }
    return DPG_OK;
}

int64_t dpg_active_dynamic_points(dpg_dpg* d, int64_t V, const float* est, float* out, int64_t cap, int64_t counts[4]) {
    if (!d || !est || V <= 0 || V > d->V || !counts) return dpg_set_error(DPG_ERR_ARG, "bad arguments");
    DTRY(hipSetDevice(d->device));
    hipStream_t s = d->s;
    int rc = upload_frames(d, V, est);
    if (rc) return rc;
    if (d->d_counts.reserve((size_t)(4 * V)) || d->d_base.reserve(4))
        return dpg_set_error(DPG_ERR_HIP, "hipMalloc(map lists) failed");
    DS ds = make_ds(d);
    map_lists_kernel<false><<<(unsigned)V, kT, 0, s>>>(ds, d->d_counts.p, nullptr, nullptr, 0);
    DTRY(hipGetLastError());
    std::vector<int64_t> cnt((size_t)(4 * V));
    DTRY(hipMemcpyAsync(cnt.data(), d->d_counts.p, sizeof(int64_t) * 4 * V, hipMemcpyDeviceToHost, s));
    DTRY(hipStreamSynchronize(s));
    // per-node exclusive offsets inside each list, then list bases
    int64_t tot[4] = {0, 0, 0, 0};
    for (int64_t v = 0; v < V; ++v)
        for (int l = 0; l < 4; ++l) { const int64_t c = cnt[(size_t)(4 * v + l)]; cnt[(size_t)(4 * v + l)] = tot[l]; tot[l] += c; }
    int64_t base[4], total = 0;
    for (int l = 0; l < 4; ++l) { base[l] = total; total += tot[l]; counts[l] = tot[l]; }
    if (!out || cap <= 0 || total == 0) return total;
    if (d->d_map_out.reserve((size_t)std::min(cap, total))) return dpg_set_error(DPG_ERR_HIP, "hipMalloc(map out) failed");
    DTRY(hipMemcpyAsync(d->d_counts.p, cnt.data(), sizeof(int64_t) * 4 * V, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(d->d_base.p, base, sizeof(base), hipMemcpyHostToDevice, s));
    map_lists_kernel<true><<<(unsigned)V, kT, 0, s>>>(ds, d->d_counts.p, d->d_base.p, d->d_map_out.p, std::min(cap, total));
    DTRY(hipGetLastError());
    DTRY(hipMemcpyAsync(out, d->d_map_out.p, sizeof(float2) * std::min(cap, total), hipMemcpyDeviceToHost, s));
    DTRY(hipStreamSynchronize(s));
    return total;
}

}  // extern "C"
