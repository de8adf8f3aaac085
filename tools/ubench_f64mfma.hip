// ubench_f64mfma.hip -- fp64 throughput on gfx950: v_mfma_f64_16x16x4_f64 vs v_fma_f64, the
// two ways to run the Cholesky's tile updates (round-1 verdict: "use fp64 MFMA for the large-front
// tile updates and panel TRSM").  Every wave runs ITER steps of independent accumulator chains;
// the grid fills the chip (8 waves per SIMD).  Prints TFLOP/s of each and checks one MFMA tile
// against a scalar product (layout per cdna_hip_programming.md: A[l&15][k=l>>4], B[k=l>>4][l&15],
// D col = l&15, row = (l>>4) + 4 r).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 4096;

__global__ __launch_bounds__(256) void mfma_loop(double* out, double a0, double b0) {
    const int l = threadIdx.x & 63;
    double a = a0 + 1e-9 * l, b = b0 - 1e-9 * l;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int it = 0; it < ITER; ++it) {   // four independent chains hide the MFMA latency
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
    const d4 s = c0 + c1 + c2 + c3;
    out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(256) void fma_loop(double* out, double a0, double b0) {
    const int l = threadIdx.x;
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = a0 + 1e-9 * (l + q);
    const double m = b0;
    for (int it = 0; it < ITER; ++it)
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = fma(x[q], m, 1e-12);   // eight independent chains
    double s = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += x[q];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ void mfma_check(const double* A, const double* B, double* D) {   // A 16x4, B 4x16 row-major
    const int l = threadIdx.x;
    d4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = c[r];
}

int main() {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = cus * 8;   // 256-thread blocks: 4 waves each, 8 blocks = 8 waves per SIMD
    double* out;
    if (hipMalloc(&out, sizeof(double) * blocks * 256) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float ms;
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, 1.0, 1.0);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        // per wave per step: 4 MFMA x 16x16x4 x 2 flop
        const double fl_m = (double)blocks * 4 * ITER * 4 * 16 * 16 * 4 * 2;
        const double tf_m = fl_m / (ms * 1e-3) / 1e12;
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(256), 0, 0, out, 1.0, 1.0);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms2;
        (void)hipEventElapsedTime(&ms2, e0, e1);
        const double fl_v = (double)blocks * 256 * ITER * 8 * 2;
        const double tf_v = fl_v / (ms2 * 1e-3) / 1e12;
        if (rep) printf("CUs %d | v_mfma_f64_16x16x4: %.1f TFLOP/s (%.2f ms) | v_fma_f64: %.1f TFLOP/s (%.2f ms)\n", cus, tf_m, ms,
                        tf_v, ms2);
    }
    // layout check with exact small integers
    std::vector<double> A(64), B(64), D(256), ref(256, 0.0);
    for (int i = 0; i < 64; ++i) { A[i] = (i * 7) % 11 - 5; B[i] = (i * 5) % 13 - 6; }
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j)
            for (int k = 0; k < 4; ++k) ref[i * 16 + j] += A[i * 4 + k] * B[k * 16 + j];
    double *dA, *dB, *dD;
    if (hipMalloc(&dA, 512) || hipMalloc(&dB, 512) || hipMalloc(&dD, 2048)) return 1;
    (void)hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma_check, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    (void)hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += D[i] != ref[i];
    printf("layout check: %d of 256 wrong\n", bad);
    return bad ? 2 : 0;
}
