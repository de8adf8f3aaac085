// Host-only check (no GPU needed): dpg_atan2f (dpg-slam_amd/csrc/dpg_atan2f.h) against the C
// library's atan2f on 40 M random arguments plus the special cases.  Build + run:
//   hipcc -O2 -ffp-contract=off -o /tmp/atan2f_check tools/atan2f_check.hip && /tmp/atan2f_check
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

#include "../dpg-slam_amd/csrc/dpg_atan2f.h"

static int same(float a, float b) { return memcmp(&a, &b, 4) == 0 || (a != a && b != b); }

int main() {
    uint64_t s = 88172645463325252ull;
    long bad = 0, n = 0;
    for (long i = 0; i < 40000000; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        float x = ((int32_t)(s & 0xffffffff)) / 2147483648.0f * 30.f;
        float y = ((int32_t)(s >> 32)) / 2147483648.0f * 30.f;
        switch (i % 6) {
            case 0: y *= 1e-6f; break;                   // near the +-pi seam and 0
            case 1: x = -fabsf(x); y *= 1e-4f; break;
            case 2: memcpy(&x, &s, 4); { uint32_t u = (uint32_t)(s >> 32); memcpy(&y, &u, 4); } break;  // any bits
            case 3: x = 1.0f; break;
            default: break;
        }
        float a = atan2f(y, x), b = dpg_atan2f(y, x);
        ++n;
        if (!same(a, b)) {
            if (bad < 5) printf("y=%a x=%a libm=%a dpg=%a\n", y, x, a, b);
            ++bad;
        }
    }
    const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-38f, -1e-38f, 3e38f, -3e38f};
    for (float y : sp)
        for (float x : sp) {
            ++n;
            if (!same(atan2f(y, x), dpg_atan2f(y, x))) { if (bad < 10) printf("special y=%a x=%a\n", y, x); ++bad; }
        }
    printf("atan2f mismatches: %ld of %ld\n", bad, n);
    return bad != 0;
}
