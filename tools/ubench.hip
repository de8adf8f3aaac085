// ubench.hip -- latency microbenchmarks on one wave (clock rate, dependent fp64 fma, v_rsq_f64,
// v_readlane, ds_read_b64), to price the sequential chains of the Cholesky panel.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void probe(double* out, unsigned long long* t, int n, double a) {
    double x = a + threadIdx.x, y = 1.0 + 1e-9 * threadIdx.x;
    __shared__ double sh[256];
    sh[threadIdx.x] = x;
    __syncthreads();
    unsigned long long w0 = wall_clock64(), c0 = clock64();
    for (int i = 0; i < n; ++i) x = fma(x, y, 1e-7);              // dependent fp64 fma
    unsigned long long w1 = wall_clock64(), c1 = clock64();
    for (int i = 0; i < n; ++i) x = __builtin_amdgcn_rsq(x) + 1.0;   // dependent rsq + add
    unsigned long long w2 = wall_clock64(), c2 = clock64();
    for (int i = 0; i < n; ++i) {                                  // dependent readlane chain
        const int lo = __builtin_amdgcn_readlane(__double2loint(x), i & 31);
        const int hi = __builtin_amdgcn_readlane(__double2hiint(x), i & 31);
        x = __hiloint2double(hi, lo) * y;
    }
    unsigned long long w3 = wall_clock64(), c3 = clock64();
    int idx = threadIdx.x;
    for (int i = 0; i < n; ++i) {                                  // dependent LDS read chain
        x += sh[idx & 255];
        idx = (int)x & 7;
    }
    unsigned long long w4 = wall_clock64(), c4 = clock64();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) {
        t[0] = w1 - w0; t[1] = c1 - c0; t[2] = w2 - w1; t[3] = c2 - c1;
        t[4] = w3 - w2; t[5] = c3 - c2; t[6] = w4 - w3; t[7] = c4 - c3;
    }
}

int main() {
    double* d; unsigned long long* t;
    hipMalloc(&d, 256 * 8); hipMalloc(&t, 64);
    const int n = 4096;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, t, n, 1.0);
        hipDeviceSynchronize();
    }
    unsigned long long h[8];
    hipMemcpy(h, t, 64, hipMemcpyDeviceToHost);
    const char* nm[4] = {"fma_f64 dep", "rsq_f64+add dep", "readlane x2 + mul dep", "ds_read_b64 dep"};
    for (int k = 0; k < 4; ++k)
        printf("%-24s %.1f ns/iter  %.1f clk/iter  (clock %.2f GHz)\n", nm[k], h[2 * k] * 10.0 / n,
               (double)h[2 * k + 1] / n, (double)h[2 * k + 1] / (h[2 * k] * 10.0));
    return 0;
}
