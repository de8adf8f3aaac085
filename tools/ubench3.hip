// ubench3.hip -- accuracy of v_rsq_f64 / v_rcp_f64 against correctly rounded 1/sqrt, 1/x
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
__global__ void k(const double* x, double* r0, double* r1, double* r2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double y = __builtin_amdgcn_rsq(x[i]);
    r0[i] = y;
    double h = 0.5 * x[i];
    double y1 = y * fma(-h * y, y, 1.5);
    r1[i] = y1;
    r2[i] = __builtin_amdgcn_rcp(x[i]);
}
int main() {
    const int n = 1 << 20;
    double *x, *a, *b, *c;
    (void)hipMallocManaged(&x, n * 8); (void)hipMallocManaged(&a, n * 8); (void)hipMallocManaged(&b, n * 8); (void)hipMallocManaged(&c, n * 8);
    unsigned long long s = 1;
    for (int i = 0; i < n; ++i) { s = s * 6364136223846793005ull + 1442695040888963407ull; x[i] = ldexp((double)(s >> 11) / 9007199254740992.0 + 0.5, (int)(s % 40) - 20); }
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, x, a, b, c, n);
    (void)hipDeviceSynchronize();
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; ++i) {
        long double t = 1.0L / sqrtl((long double)x[i]);
        e0 = fmax(e0, (double)fabsl((a[i] - t) / t));
        e1 = fmax(e1, (double)fabsl((b[i] - t) / t));
        long double u = 1.0L / (long double)x[i];
        e2 = fmax(e2, (double)fabsl((c[i] - u) / u));
    }
    printf("v_rsq_f64 max rel err %.3e; + 1 Newton %.3e; v_rcp_f64 %.3e (ulp %.3e)\n", e0, e1, e2, ldexp(1.0, -53));
    return 0;
}
