// clock_probe.hip -- diagnostics only (tools/clock_probe.py): the shader clock over time inside a
// kernel, from the ratio of s_memtime (shader clock) to s_memrealtime (100 MHz), per window of
// real time; and a bounded VALU load ("heater") for concurrency experiments.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void clk_trace(uint64_t* out, int n_win, int win_ticks) {
    float x = (float)threadIdx.x * 1e-3f;
    for (int w = 0; w < n_win; ++w) {
        const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
        uint64_t r1 = r0;
        while (r1 - r0 < (uint64_t)win_ticks) {
#pragma unroll
            for (int k = 0; k < 64; ++k) x = fmaf(x, 0.999f, 1e-4f);
            r1 = __builtin_amdgcn_s_memrealtime();
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            out[2 * w] = t1 - t0;
            out[2 * w + 1] = r1 - r0;
        }
    }
    if (x == 12345.0f) out[0] = 0;   // keeps the chain live
}

__global__ void heat(int iters, float* sink) {
    float x = (float)threadIdx.x * 1e-3f;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 64; ++k) x = fmaf(x, 0.999f, 1e-4f);
    }
    if (x == 12345.0f) sink[threadIdx.x] = x;
}

extern "C" int clk_trace_launch(void* out, int blocks, int threads, int n_win, int win_ticks, void* stream) {
    hipLaunchKernelGGL(clk_trace, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, (uint64_t*)out, n_win, win_ticks);
    return (int)hipGetLastError();
}

extern "C" int heat_launch(int blocks, int threads, int iters, void* sink, void* stream) {
    hipLaunchKernelGGL(heat, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, iters, (float*)sink);
    return (int)hipGetLastError();
}
