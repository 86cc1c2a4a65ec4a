// Counter-based CEM proposal sampler (device side).
//
// Philox4x32-10 (Salmon et al., SC'11; Random123 constants) keyed by a 64-bit seed, counter
// (global candidate n, timestep t, CEM iteration, action group d>>2). Each call yields 4 words ->
// two Box-Muller pairs -> 4 standard normals for dims 4g..4g+3.
//
// The normal transform uses only correctly rounded float32 operations (__fadd_rn / __fmul_rn /
// __fdiv_rn / __fsqrt_rn, exact int->float) in a fixed order with contraction disabled, so it is
// bit-identical to the NumPy restatement in oracle/philox.py (the test checker).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mbrl {

struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ float f32_from_bits(uint32_t b) { return __uint_as_float(b); }

// Correctly rounded sqrt for finite x >= 0. gfx950's v_sqrt_f32 (what sqrtf / __fsqrt_rn lower to)
// is not correctly rounded; NumPy's is. Start from it and fix the last bit against the exact
// midpoints: squares of float32 values and of their midpoints are exact in fp64 (<= 50 bits).
__device__ __forceinline__ float exact_sqrt(float x) {
    if (!(x > 0.0f) || isinf(x)) return sqrtf(x);
    float y = sqrtf(x);
    const double xd = (double)x;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const float lo = __uint_as_float(__float_as_uint(y) - 1u);
        const float hi = __uint_as_float(__float_as_uint(y) + 1u);
        const double mlo = 0.5 * ((double)lo + (double)y);
        const double mhi = 0.5 * ((double)y + (double)hi);
        if (xd < mlo * mlo) y = lo;
        else if (xd > mhi * mhi) y = hi;
    }
    return y;
}

// ln(u), u in (0, 1]; mirrors oracle/philox.py:_log_f32 operation for operation.
__device__ __forceinline__ float exact_log(float u) {
#pragma clang fp contract(off)
    const uint32_t bits = __float_as_uint(u);
    int e = (int)(bits >> 23) - 127;
    float m = __uint_as_float((bits & 0x007FFFFFu) | 0x3F800000u);
    if (m > f32_from_bits(0x3FB504F3u)) { m = __fmul_rn(m, 0.5f); e += 1; }
    const float f = __fadd_rn(m, -1.0f);
    const float s = __fdiv_rn(f, __fadd_rn(2.0f, f));
    const float z = __fmul_rn(s, s);
    float p = __fadd_rn(f32_from_bits(0x3DE38E39u), __fmul_rn(z, f32_from_bits(0x3DBA2E8Cu)));
    p = __fadd_rn(f32_from_bits(0x3E124925u), __fmul_rn(z, p));
    p = __fadd_rn(f32_from_bits(0x3E4CCCCDu), __fmul_rn(z, p));
    p = __fadd_rn(f32_from_bits(0x3EAAAAABu), __fmul_rn(z, p));
    p = __fmul_rn(z, p);
    const float s2 = __fadd_rn(s, s);
    const float lnm = __fadd_rn(s2, __fmul_rn(s2, p));
    return __fadd_rn(__fmul_rn((float)e, f32_from_bits(0x3F317218u)), lnm);
}

// (sin, cos) of 2*pi*v, v in [0, 1); mirrors oracle/philox.py:_sincos_turn_f32.
__device__ __forceinline__ void exact_sincos_turn(float v, float& sn_out, float& cs_out) {
#pragma clang fp contract(off)
    const float v4 = __fmul_rn(v, 4.0f);
    int q = (int)floorf(v4);
    float f = __fadd_rn(v4, -(float)q);
    if (f >= 0.5f) { f = __fadd_rn(f, -1.0f); q += 1; }
    q &= 3;
    const float x = __fmul_rn(f, f32_from_bits(0x3FC90FDBu));
    const float x2 = __fmul_rn(x, x);
    float ps = __fadd_rn(f32_from_bits(0x39500D01u), -__fmul_rn(x2, f32_from_bits(0x3638EF1Du)));
    ps = __fadd_rn(f32_from_bits(0x3C088889u), -__fmul_rn(x2, ps));
    ps = __fadd_rn(f32_from_bits(0x3E2AAAABu), -__fmul_rn(x2, ps));
    const float sn = __fadd_rn(x, -__fmul_rn(__fmul_rn(x, x2), ps));
    float pc = __fadd_rn(f32_from_bits(0x37D00D01u), -__fmul_rn(x2, f32_from_bits(0x3493F27Eu)));
    pc = __fadd_rn(f32_from_bits(0x3AB60B61u), -__fmul_rn(x2, pc));
    pc = __fadd_rn(f32_from_bits(0x3D2AAAABu), -__fmul_rn(x2, pc));
    pc = __fadd_rn(0.5f, -__fmul_rn(x2, pc));
    const float cs = __fadd_rn(1.0f, -__fmul_rn(x2, pc));
    switch (q) {
        case 0: sn_out = sn; cs_out = cs; break;
        case 1: sn_out = cs; cs_out = -sn; break;
        case 2: sn_out = -sn; cs_out = -cs; break;
        default: sn_out = -cs; cs_out = sn; break;
    }
}

__device__ __forceinline__ void box_muller(uint32_t x0, uint32_t x1, float& z0, float& z1) {
#pragma clang fp contract(off)
    const float u1 = __fmul_rn((float)((x0 >> 8) + 1u), 5.9604644775390625e-8f);  // (0, 1]
    const float u2 = __fmul_rn((float)(x1 >> 8), 5.9604644775390625e-8f);         // [0, 1)
    const float r = exact_sqrt(__fmul_rn(-2.0f, exact_log(u1)));
    float sn, cs;
    exact_sincos_turn(u2, sn, cs);
    z0 = __fmul_rn(r, cs);
    z1 = __fmul_rn(r, sn);
}

// 4 standard normals for action dims 4g..4g+3 of (candidate n, step t, iteration it).
__device__ __forceinline__ void cem_normal4(uint64_t seed, uint32_t n, uint32_t t, uint32_t it,
                                            uint32_t g, float z[4]) {
    const u32x4 w = philox4x32_10(u32x4{n, t, it, g}, (uint32_t)seed, (uint32_t)(seed >> 32));
    box_muller(w.x, w.y, z[0], z[1]);
    box_muller(w.z, w.w, z[2], z[3]);
}

// clip(mu + sigma * eps, lo, hi) without contraction (oracle/philox.py:cem_actions).
__device__ __forceinline__ float cem_action(float mu, float sigma, float eps, float lo, float hi) {
#pragma clang fp contract(off)
    const float x = __fadd_rn(mu, __fmul_rn(sigma, eps));
    return fminf(fmaxf(x, lo), hi);
}

}  // namespace mbrl
