// Host -> device copy of a pageable 200 MB buffer (the config-4 scan store's full clouds): plain
// hipMemcpy from pageable memory against hipHostRegister + copy + hipHostUnregister, and a pinned
// staging ring of 8 MB chunks (memcpy into pinned, async DMA, double-buffered).
// build: hipcc --offload-arch=gfx950 -O2 -o tools/build_h2d_probe tools/h2d_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <vector>
static double ms() { timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec * 1e3 + t.tv_nsec * 1e-6; }
int main() {
    const size_t B = (size_t)200 << 20;
    std::vector<char> h(B);
    for (size_t i = 0; i < B; i += 4096) h[i] = (char)i;
    void* d = nullptr;
    if (hipMalloc(&d, B) != hipSuccess) return 1;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    const size_t C = (size_t)8 << 20;
    char* pin[2];
    if (hipHostMalloc((void**)&pin[0], C, 0) != hipSuccess || hipHostMalloc((void**)&pin[1], C, 0) != hipSuccess) return 1;
    hipEvent_t ev[2];
    for (auto& e : ev) if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return 1;
    for (int r = 0; r < 4; ++r) {
        double t0 = ms();
        if (hipMemcpyAsync(d, h.data(), B, hipMemcpyHostToDevice, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) return 2;
        double t1 = ms();
        if (hipHostRegister(h.data(), B, hipHostRegisterDefault) != hipSuccess) return 3;
        double t2 = ms();
        if (hipMemcpyAsync(d, h.data(), B, hipMemcpyHostToDevice, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) return 4;
        double t3 = ms();
        if (hipHostUnregister(h.data()) != hipSuccess) return 5;
        double t4 = ms();
        // staging ring: memcpy chunk k into pin[k & 1] while chunk k - 1 is in flight
        for (size_t o = 0, k = 0; o < B; o += C, ++k) {
            const size_t n = o + C <= B ? C : B - o;
            if (k >= 2 && hipEventSynchronize(ev[k & 1]) != hipSuccess) return 6;
            memcpy(pin[k & 1], h.data() + o, n);
            if (hipMemcpyAsync((char*)d + o, pin[k & 1], n, hipMemcpyHostToDevice, s) != hipSuccess) return 7;
            if (hipEventRecord(ev[k & 1], s) != hipSuccess) return 8;
        }
        if (hipStreamSynchronize(s) != hipSuccess) return 9;
        double t5 = ms();
        printf("pageable %.1f ms | register %.1f + copy %.1f + unregister %.1f ms | pinned ring %.1f ms\n", t1 - t0, t2 - t1,
               t3 - t2, t4 - t3, t5 - t4);
    }
    return 0;
}
