// ubench2.hip -- single-wave THROUGHPUT probes: independent fp64 fmas, independent readlanes,
// independent broadcast ds_read_b64, to price the Cholesky panel's per-step work.
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ double rdl(double v, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

__global__ void probe(double* out, unsigned long long* t, int n) {
    __shared__ double sh[256];
    sh[threadIdx.x] = threadIdx.x;
    __syncthreads();
    double a[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = threadIdx.x + k;
    const double y = 1.0000001;
    unsigned long long c0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = fma(a[k], y, 1e-9);   // 16 independent chains
    }
    unsigned long long c1 = clock64();
    double s = 0.0;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) s += rdl(a[k], (i + k) & 63) * 0.0 + 1.0;   // readlane pairs
    }
    unsigned long long c2 = clock64();
    double u = 0.0;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) u += sh[(i + k) & 255];   // broadcast ds_read_b64
    }
    unsigned long long c3 = clock64();
    double v = 0.0;
    for (int i = 0; i < n; ++i) {
        double p[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) p[k] = sh[(i * 16 + k) & 255];   // 16 loads then 16 fmas
#pragma unroll
        for (int k = 0; k < 16; ++k) v = fma(p[k], y, v);
    }
    unsigned long long c4 = clock64();
    double acc = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += a[k];
    out[threadIdx.x] = acc + s + u + v;
    if (threadIdx.x == 0) { t[0] = c1 - c0; t[1] = c2 - c1; t[2] = c3 - c2; t[3] = c4 - c3; }
}

int main() {
    double* d; unsigned long long* t;
    (void)hipMalloc(&d, 256 * 8); (void)hipMalloc(&t, 64);
    const int n = 1024;
    for (int rep = 0; rep < 2; ++rep) { hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, t, n); (void)hipDeviceSynchronize(); }
    unsigned long long h[4];
    (void)hipMemcpy(h, t, 32, hipMemcpyDeviceToHost);
    printf("independent fp64 fma        %.1f clk/op\n", (double)h[0] / (n * 16));
    printf("readlane pair (+add chain)  %.1f clk/op\n", (double)h[1] / (n * 16));
    printf("broadcast ds_read_b64 (+add chain) %.1f clk/op\n", (double)h[2] / (n * 16));
    printf("16 ds_read then 16 dep fma  %.1f clk/iter-element\n", (double)h[3] / (n * 16));
    return 0;
}
