// dpg_reopt.hip -- loop-closure candidate search of the re-linearisation sweep
// (DpgSLAM::reoptimize, dpg_slam.cc:91-98): for every node i and every j < i - 1, the pair (j, i)
// is a candidate when the float distance between the two ESTIMATED positions,
// (p_j - p_i).norm() = sqrt(dx*dx + dy*dy) (Eigen Vector2f, correctly rounded), is <= the
// threshold of the pair: maximum_node_dist_within_pass_scan_comparison_ (5.0) when both nodes are
// of the same pass, maximum_node_dist_across_passes_scan_comparison_ (2.0) otherwise
// (parameters.h:212,224).  The reference tests all O(V^2) pairs node by node; here one thread per
// node i scans j ascending twice -- count, then (after a host prefix sum) write -- so the output is
// the reference's own order: i ascending, j ascending.  Built with -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dpg_internal.h"

namespace {

constexpr int kRT = 256;
constexpr int kTile = 1024;   // nodes staged per LDS tile (float2 + pass)

__device__ __forceinline__ bool close_pair(float2 pj, int passj, float2 pi, int passi, float within, float across) {
    const float dx = pj.x - pi.x, dy = pj.y - pi.y;
    const float d = __fsqrt_rn(dx * dx + dy * dy);
    return d <= (passj == passi ? within : across);
}

// WRITE = false: count[i] = number of candidates of node i; true: write them at out + 2 * off[i]
template <bool WRITE>
__global__ __launch_bounds__(kRT) void lc_candidates_kernel(const float* __restrict__ poses /*[V][3]*/,
                                                            const int32_t* __restrict__ pass, int64_t V,
                                                            float within, float across, int32_t* __restrict__ count,
                                                            const int64_t* __restrict__ off, int32_t* __restrict__ out) {
    __shared__ float2 tp[kTile];
    __shared__ int32_t tpass[kTile];
    const int64_t i = (int64_t)blockIdx.x * kRT + threadIdx.x;
    const bool live = i < V;
    const float2 pi = live ? make_float2(poses[3 * i], poses[3 * i + 1]) : make_float2(0.f, 0.f);
    const int passi = live ? pass[i] : 0;
    // this block's nodes need j < i - 1 <= (last i of the block) - 1
    const int64_t jmax = min((int64_t)(blockIdx.x + 1) * kRT, V) - 1;
    int32_t n = 0;
    int64_t w = (WRITE && live) ? 2 * off[i] : 0;
    for (int64_t j0 = 0; j0 < jmax; j0 += kTile) {
        __syncthreads();
        for (int k = threadIdx.x; k < kTile && j0 + k < V; k += kRT) {
            const int64_t j = j0 + k;
            tp[k] = make_float2(poses[3 * j], poses[3 * j + 1]);
            tpass[k] = pass[j];
        }
        __syncthreads();
        const int64_t jend = live ? min(j0 + kTile, i - 1) : j0;   // j < i - 1
        for (int64_t j = j0; j < jend; ++j) {
            const int k = (int)(j - j0);
            if (close_pair(tp[k], tpass[k], pi, passi, within, across)) {
                if (WRITE) {
                    out[w] = (int32_t)j;
                    out[w + 1] = (int32_t)i;
                    w += 2;
                } else {
                    ++n;
                }
            }
        }
    }
    if (!WRITE && live) count[i] = n;
}

}  // namespace

extern "C" int dpg_launch_lc_count(const float* poses_dev, const int32_t* pass_dev, int64_t V, float within,
                                   float across, int32_t* count_dev, void* stream) {
    if (V <= 0) return DPG_OK;
    hipLaunchKernelGGL(lc_candidates_kernel<false>, dim3((unsigned)((V + kRT - 1) / kRT)), dim3(kRT), 0,
                       reinterpret_cast<hipStream_t>(stream), poses_dev, pass_dev, V, within, across, count_dev,
                       nullptr, nullptr);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

extern "C" int dpg_launch_lc_write(const float* poses_dev, const int32_t* pass_dev, int64_t V, float within,
                                   float across, const int64_t* off_dev, int32_t* pairs_dev, void* stream) {
    if (V <= 0) return DPG_OK;
    hipLaunchKernelGGL(lc_candidates_kernel<true>, dim3((unsigned)((V + kRT - 1) / kRT)), dim3(kRT), 0,
                       reinterpret_cast<hipStream_t>(stream), poses_dev, pass_dev, V, within, across, nullptr,
                       off_dev, pairs_dev);
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}

// ---- map assembly (DpgSLAM::GetMap, dpg_slam.cc:555-575) ----
// Every node's base_link cloud into the map frame with the node's estimated pose
// (math_utils::transformPoint(p, 0, pos, angle): Rotation2Df(angle) * p + pos), keeping the points
// whose running index over all nodes is a multiple of display_points_fraction_.  cos/sin of each
// node's angle come from the host (float cosf/sinf, what Eigen's Rotation2Df evaluates) so the
// device does only the multiply-adds -- bit-identical.  One workgroup per node; a streaming,
// HBM-bound kernel (8 B read per point, 8 B written per kept point).
namespace {
__global__ __launch_bounds__(kRT) void map_points_kernel(const float2* __restrict__ pts,
                                                         const int64_t* __restrict__ off,
                                                         const float4* __restrict__ frame /* x, y, c, s */,
                                                         int32_t fraction, float2* __restrict__ out) {
    const int v = blockIdx.x;
    const int64_t b = off[v], e = off[v + 1];
    const float4 f = frame[v];
    const float ns = -f.w;
    int64_t g = b + threadIdx.x;
    int64_t r = g % fraction;
    for (; g < e; g += kRT) {
        if (r == 0) {
            const float2 p = pts[g];
            out[g / fraction] = make_float2(f.x + (f.z * p.x + ns * p.y), f.y + (f.w * p.x + f.z * p.y));
        }
        r += kRT % fraction;
        if (r >= fraction) r -= fraction;
    }
}
}  // namespace

extern "C" int dpg_launch_map_points(const float* pts_dev, const int64_t* off_dev, const float* frames_dev, int64_t V,
                                     int32_t fraction, float* out_dev, void* stream) {
    if (V <= 0) return DPG_OK;
    if (fraction <= 0) return DPG_ERR_ARG;
    hipLaunchKernelGGL(map_points_kernel, dim3((unsigned)V), dim3(kRT), 0, reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const float2*>(pts_dev), off_dev, reinterpret_cast<const float4*>(frames_dev),
                       fraction, reinterpret_cast<float2*>(out_dev));
    return hipGetLastError() == hipSuccess ? DPG_OK : DPG_ERR_HIP;
}
