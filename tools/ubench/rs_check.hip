// The GD kernel's wave reduce-scatter (gd.hip wave_reduce_scatter32) against the ds_bpermute form it
// replaced, on random inputs: prints the number of lanes whose results differ (bitwise).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../mujoco-mbrl_amd/csrc/mbrl_internal.h"

namespace {
__device__ float rs_old(const float (&v)[32], int lane) {
    float a16[16], a8[8], a4[4], a2[2];
    for (int j = 0; j < 16; ++j) { const bool hi = lane & 32; const float keep = hi ? v[j + 16] : v[j], send = hi ? v[j] : v[j + 16]; a16[j] = keep + __shfl_xor(send, 32, 64); }
    for (int j = 0; j < 8; ++j) { const bool hi = lane & 16; const float keep = hi ? a16[j + 8] : a16[j], send = hi ? a16[j] : a16[j + 8]; a8[j] = keep + __shfl_xor(send, 16, 64); }
    for (int j = 0; j < 4; ++j) { const bool hi = lane & 8; const float keep = hi ? a8[j + 4] : a8[j], send = hi ? a8[j] : a8[j + 4]; a4[j] = keep + __shfl_xor(send, 8, 64); }
    for (int j = 0; j < 2; ++j) { const bool hi = lane & 4; const float keep = hi ? a4[j + 2] : a4[j], send = hi ? a4[j] : a4[j + 2]; a2[j] = keep + __shfl_xor(send, 4, 64); }
    const bool hi = lane & 2; const float keep = hi ? a2[1] : a2[0], send = hi ? a2[0] : a2[1];
    const float a1 = keep + __shfl_xor(send, 2, 64);
    return a1 + __shfl_xor(a1, 1, 64);
}
// v_permlane32_swap / v_permlane16_swap as inline asm: both registers are read and written. (The
// ROCm 7.2 clang builtins return the swapped pair wrongly here: __builtin_amdgcn_permlane32_swap's two
// results were read from ONE register, v_add_f32 vX, vY, vY after the swap -- tools/ubench/rs_check.hip.)
// The s_nops cover the VALU-write -> permlane-read and permlane-write -> VALU-read hazards, which the
// compiler's hazard recognizer does not see through inline asm.
__device__ __forceinline__ void permlane32_swap(float& x, float& y) {
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void permlane16_swap(float& x, float& y) {
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
}
#define GC_DPP(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, (v)), (ctrl), 0xF, 0xF, false))
__device__ float rs_new(const float (&v)[32], int lane) {
    float a16[16], a8[8], a4[4], a2[2];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        float x = v[j], y = v[j + 16];
        permlane32_swap(x, y);
        a16[j] = x + y;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float x = a16[j], y = a16[j + 8];
        permlane16_swap(x, y);
        a8[j] = x + y;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { const bool hi = lane & 8; const float keep = hi ? a8[j + 4] : a8[j], send = hi ? a8[j] : a8[j + 4]; a4[j] = keep + GC_DPP(send, 0x128); }
#pragma unroll
    for (int j = 0; j < 2; ++j) { const bool hi = lane & 4; const float keep = hi ? a4[j + 2] : a4[j], send = hi ? a4[j] : a4[j + 2]; a2[j] = keep + GC_DPP(GC_DPP(send, 0x141), 0x1B); }
    const bool hi = lane & 2; const float keep = hi ? a2[1] : a2[0], send = hi ? a2[0] : a2[1];
    const float a1 = keep + GC_DPP(send, 0x4E);
    return a1 + GC_DPP(a1, 0xB1);
}
}  // namespace

namespace {
__device__ float rs_A(const float (&v)[32], int lane) {   // permlane for ^32 / ^16, shfl for the rest
    float a16[16], a8[8], a4[4], a2[2];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v[j]), __builtin_bit_cast(unsigned, v[j + 16]), false, false);
        a16[j] = __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a16[j]), __builtin_bit_cast(unsigned, a16[j + 8]), false, false);
        a8[j] = __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
    }
    for (int j = 0; j < 4; ++j) { const bool hi = lane & 8; const float keep = hi ? a8[j + 4] : a8[j], send = hi ? a8[j] : a8[j + 4]; a4[j] = keep + __shfl_xor(send, 8, 64); }
    for (int j = 0; j < 2; ++j) { const bool hi = lane & 4; const float keep = hi ? a4[j + 2] : a4[j], send = hi ? a4[j] : a4[j + 2]; a2[j] = keep + __shfl_xor(send, 4, 64); }
    const bool hi = lane & 2; const float keep = hi ? a2[1] : a2[0], send = hi ? a2[0] : a2[1];
    const float a1 = keep + __shfl_xor(send, 2, 64);
    return a1 + __shfl_xor(a1, 1, 64);
}
__device__ float rs_B(const float (&v)[32], int lane) {   // shfl for ^32 / ^16, DPP for the rest
    float a16[16], a8[8], a4[4], a2[2];
    for (int j = 0; j < 16; ++j) { const bool hi = lane & 32; const float keep = hi ? v[j + 16] : v[j], send = hi ? v[j] : v[j + 16]; a16[j] = keep + __shfl_xor(send, 32, 64); }
    for (int j = 0; j < 8; ++j) { const bool hi = lane & 16; const float keep = hi ? a16[j + 8] : a16[j], send = hi ? a16[j] : a16[j + 8]; a8[j] = keep + __shfl_xor(send, 16, 64); }
#pragma unroll
    for (int j = 0; j < 4; ++j) { const bool hi = lane & 8; const float keep = hi ? a8[j + 4] : a8[j], send = hi ? a8[j] : a8[j + 4]; a4[j] = keep + GC_DPP(send, 0x128); }
#pragma unroll
    for (int j = 0; j < 2; ++j) { const bool hi = lane & 4; const float keep = hi ? a4[j + 2] : a4[j], send = hi ? a4[j] : a4[j + 2]; a2[j] = keep + GC_DPP(GC_DPP(send, 0x141), 0x1B); }
    const bool hi = lane & 2; const float keep = hi ? a2[1] : a2[0], send = hi ? a2[0] : a2[1];
    const float a1 = keep + GC_DPP(send, 0x4E);
    return a1 + GC_DPP(a1, 0xB1);
}
}  // namespace

__global__ void k(const float* in, float* o1, float* o2, int which) {
    const int l = threadIdx.x & 63;
    float v[32];
    for (int j = 0; j < 32; ++j) v[j] = in[threadIdx.x * 32 + j];
    o1[threadIdx.x] = rs_old(v, l);
    o2[threadIdx.x] = which == 0 ? rs_new(v, l) : which == 1 ? rs_A(v, l) : rs_B(v, l);
}

int main() {
    const int T = 512;
    float h[T * 32], r1[T], r2[T];
    srand(1);
    for (int i = 0; i < T * 32; ++i) h[i] = (float)rand() / RAND_MAX - 0.5f;
    float *d, *d1, *d2;
    if (hipMalloc(&d, sizeof(h)) || hipMalloc(&d1, sizeof(r1)) || hipMalloc(&d2, sizeof(r2))) return 1;
    if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice)) return 1;
    int bad = 0;
    for (int which = 0; which < 3; ++which) {
        hipLaunchKernelGGL(k, dim3(1), dim3(T), 0, 0, d, d1, d2, which);
        if (hipMemcpy(r1, d1, sizeof(r1), hipMemcpyDeviceToHost) || hipMemcpy(r2, d2, sizeof(r2), hipMemcpyDeviceToHost)) return 1;
        bad = 0;
        for (int i = 0; i < T; ++i) if (r1[i] != r2[i]) { if (bad < 4) printf("variant %d lane %d: old %.9g new %.9g\n", which, i, r1[i], r2[i]); ++bad; }
        printf("variant %d (0 asm permlane + dpp, 1 builtin permlane + shfl, 2 shfl + dpp): %d differing lanes\n", which, bad);
    }
    // the expected sum for lane 0 (k = 0 over wave 0's 64 lanes)
    double e = 0; for (int l = 0; l < 64; ++l) e += h[l * 32 + 0];
    printf("differing lanes: %d of %d; lane 0 old %.7g new %.7g exact %.7g\n", bad, T, r1[0], r2[0], e);
    return 0;
}
