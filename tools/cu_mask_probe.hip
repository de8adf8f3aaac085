// Which physical compute unit (XCC, shader engine, CU) each bit of a HIP CU mask
// (hipExtStreamCreateWithCUMask) selects on this device: for a few single-bit masks, 64 one-wave
// workgroups record their hardware ids (vector stores), and the distinct ids are printed.
// build: hipcc --offload-arch=gfx950 -O2 -o cu_mask_probe tools/cu_mask_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <set>
#include <tuple>
#include <vector>

__global__ void hwid_kernel(unsigned* out) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", ncu);
    unsigned* d;
    hipMalloc(&d, 2 * 64 * sizeof(unsigned));
    const int bits[] = {0, 1, 2, 7, 8, 31, 32, 33, 64, 65, 255};
    for (int b : bits) {
        uint32_t mask[8] = {};
        mask[b >> 5] = 1u << (b & 31);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, 8, mask) != hipSuccess) { printf("bit %d: mask refused\n", b); continue; }
        hipLaunchKernelGGL(hwid_kernel, dim3(64), dim3(64), 0, s, d);
        std::vector<unsigned> h(128);
        hipMemcpyAsync(h.data(), d, 128 * sizeof(unsigned), hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> ids;   // xcc, se, sh, cu
        for (int k = 0; k < 64; ++k) {
            const unsigned hw = h[2 * k], xcc = h[2 * k + 1] & 0xf;
            ids.insert({xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xf});
        }
        printf("bit %3d ->", b);
        for (auto& t : ids) printf(" (xcc %u se %u sh %u cu %u)", std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t));
        printf("\n");
        hipStreamDestroy(s);
    }
    // the whole device, for reference: the distinct (xcc, se, cu) of 2048 workgroups
    return 0;
}
