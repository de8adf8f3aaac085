// dpg_atan2f.h -- atan2f with the host libm's exact results, for the DPG angle tests.
//
// The reference takes the bearing of a point with atan2(float, float) (dpg_slam.cc:817,
// dpg_node.cc:51), i.e. the C library's atan2f.  The image's glibc (2.35) implements it with the
// float fdlibm algorithm (sysdeps/ieee754/flt-32/e_atan2f.c + s_atanf.c): argument reduction to
// one of four breakpoints and an 11-term odd polynomial in float arithmetic.  It is not correctly
// rounded (about 8 % of random arguments differ by one ulp from the rounded true value), so a
// different atan2f on the GPU would move points across bin and sector boundaries.  This is that
// algorithm restated (constants as bit patterns, as the library binary holds them: its atan
// polynomial's first coefficient is 0x3eaaaaab), evaluated with -ffp-contract=off; it is checked
// against the host atan2f on 40 M random arguments by tools/atan2f_check.hip and through the DPG
// parity tests.
//
// The algorithm restated here is fdlibm's (as carried by glibc's float port); its notice:
//   Conversion to float by Ian Lance Taylor, Cygnus Support, ian@cygnus.com.
//   ====================================================
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//
//   Developed at SunPro, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this
//   software is freely granted, provided that this notice
//   is preserved.
//   ====================================================
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__host__ __device__ inline float dpg_bits_f(uint32_t u) {
    union { uint32_t u; float f; } c;
    c.u = u;
    return c.f;
}
__host__ __device__ inline int32_t dpg_f_bits(float f) {
    union { float f; int32_t i; } c;
    c.f = f;
    return c.i;
}

// __atanf (s_atanf.c)
__host__ __device__ inline float dpg_atanf(float x) {
    const float atanhi[4] = {dpg_bits_f(0x3eed6338u), dpg_bits_f(0x3f490fdau), dpg_bits_f(0x3f7b985eu),
                             dpg_bits_f(0x3fc90fdau)};
    const float atanlo[4] = {dpg_bits_f(0x31ac3769u), dpg_bits_f(0x33222168u), dpg_bits_f(0x33140fb4u),
                             dpg_bits_f(0x33a22168u)};
    const float aT0 = dpg_bits_f(0x3eaaaaabu), aT1 = dpg_bits_f(0xbe4ccccdu), aT2 = dpg_bits_f(0x3e124925u),
                aT3 = dpg_bits_f(0xbde38e38u), aT4 = dpg_bits_f(0x3dba2e6eu), aT5 = dpg_bits_f(0xbd9d8795u),
                aT6 = dpg_bits_f(0x3d886b35u), aT7 = dpg_bits_f(0xbd6ef16bu), aT8 = dpg_bits_f(0x3d4bda59u),
                aT9 = dpg_bits_f(0xbd15a221u), aT10 = dpg_bits_f(0x3c8569d7u);
    const float one = 1.0f;
    const int32_t hx = dpg_f_bits(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {                 // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;  // NaN
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {                  // |x| < 0.4375
        if (ix < 0x31000000) return x;      // |x| < 2^-29
        id = -1;
    } else {
        x = x < 0 ? -x : x;
        if (ix < 0x3f980000) {              // |x| < 1.1875
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - one) / (2.0f + x); }
            else { id = 1; x = (x - one) / (x + one); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (one + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

// __ieee754_atan2f (e_atan2f.c)
__host__ __device__ inline float dpg_atan2f(float y, float x) {
    const float tiny = 1.0e-30f;
    const float pi_o_4 = dpg_bits_f(0x3f490fdbu), pi_o_2 = dpg_bits_f(0x3fc90fdbu), pi = dpg_bits_f(0x40490fdbu),
                pi_lo = dpg_bits_f(0xb3bbbd2eu);
    const int32_t hx = dpg_f_bits(x), ix = hx & 0x7fffffff;
    const int32_t hy = dpg_f_bits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;       // NaN
    if (hx == 0x3f800000) return dpg_atanf(y);                  // x = 1.0
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);          // 2 * sign(x) + sign(y)
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;                      // |y/x| > 2^60
    else if (hx < 0 && k < -60) z = 0.0f;                       // |y|/x < -2^60
    else z = dpg_atanf(dpg_bits_f((uint32_t)dpg_f_bits(y / x) & 0x7fffffffu));   // fabsf: sign bit cleared
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}
