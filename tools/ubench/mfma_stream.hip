// Microbenchmark: v_mfma_f32_16x16x4_f32 chunk loop (32 MFMAs, 8 accumulators per chunk, like the
// rollout kernel's hidden layers) with and without a concurrent L2-resident weight stream.
//   MODE 0: MFMA only (B operands fixed in registers)
//   MODE 1: MFMA + 8 x global_load_dwordx4 per chunk into a 4-deep ring, loaded data feeds the MFMAs
//   MODE 2: like 1, but the MFMAs read a fixed register set; the loads land in a sink (no dependency)
//   MODE 3: like 1 but loads via buffer_load with a descriptor (SGPR base, 32-bit voffset)
//   MODE 4: LDS-DMA (global_load_lds_dwordx4, inline asm, counted vmcnt) into a 2-chunk LDS ring per
//           wave, B fragments read back with ds_read_b128
//   MODE 5: ds_read_b128 of the B fragments from a fixed LDS region only (no global traffic)
//   MODE 6: like 1, but the loads write AGPRs (inline asm "=a") and the MFMAs read them from there
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define PIN() __builtin_amdgcn_sched_barrier(0)

template <int MODE, int NS = 2>
__global__ void __launch_bounds__(256) kern(const f32x4* __restrict__ w, int chunks, float* out,
                                            unsigned long long* cyc) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f32x4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0, 0, 0, 0};
    f32x4 ring[4][8];
    f32x4 fixed[8];
    for (int j = 0; j < 8; ++j) fixed[j] = f32x4{1.f * lane, 2.f, 3.f, 4.f};
    const f32x4* p = w + wave * 8 * 64 + lane;
    const int cs = 4 * 8 * 64;
    const int wrap = 68;
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, 68 * 32768, 0x00020000);
    auto ld = [&](f32x4 (&b)[8], int g) {
        g = g % wrap;
        if constexpr (MODE == 6) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                f32x4 v;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(v) : "v"(p + (size_t)g * cs + j * 64) : "memory");
                b[j] = v;
            }
        } else if constexpr (MODE == 3) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                b[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                           rsrc, (unsigned)(((g * cs) + wave * 8 * 64 + j * 64 + lane) * 16), 0, 0));
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j] = p[(size_t)g * cs + j * 64];
        }
    };
    f32x4 a = {0.5f, 0.25f, 0.125f, 1.f};
    // LDS ring for MODE 4/5: per wave 2 slots x 8 KiB
    float* wl = lds + wave * NS * 2048;
    const unsigned wl_addr = (unsigned)(size_t)wl;
    auto dma = [&](int slot, int g) {
        g = g % wrap;
        const f32x4* src = p + (size_t)g * cs;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            unsigned keep;
            const unsigned dst = __builtin_amdgcn_readfirstlane(wl_addr + slot * 8192 + j * 1024);
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(src + j * 64), "s"(dst) : "memory");
        }
    };
    if constexpr (MODE == 1 || MODE == 2 || MODE == 3 || MODE == 6)
        for (int q = 0; q < 3; ++q) ld(ring[q], q);
    if constexpr (MODE == 4)
        for (int q = 0; q < NS - 1; ++q) dma(q, q);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < chunks; c += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (MODE == 4 || MODE == 5) {
                if constexpr (MODE == 4) {
                    dma((c + u + NS - 1) % NS, c + u + NS - 1);
                    if constexpr (NS == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                    if constexpr (NS == 4) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
                }
                const float* rb = wl + (MODE == 4 ? ((c + u) % NS) * 2048 : 0);
#pragma unroll
                for (int j = 0; j < 8; ++j) ring[u][j] = *reinterpret_cast<const f32x4*>(rb + j * 256 + lane * 4);
            } else if constexpr (MODE != 0) {
                ld(ring[(u + 3) % 4], c + u + 3);
            }
            if constexpr (MODE == 6) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
            PIN();
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const f32x4& b = (MODE == 1 || MODE == 3 || MODE == 4 || MODE == 5 || MODE == 6) ? ring[u][j] : fixed[j];
                    if constexpr (MODE == 6)
                        asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc[j]) : "a"(b[s]), "v"(a[s]));
                    else
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[s], a[s], acc[j], 0, 0, 0);
                }
            PIN();
            if constexpr (MODE == 2) {
#pragma unroll
                for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(ring[u][j]));
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float sacc = 0;
    for (int j = 0; j < 8; ++j) sacc += acc[j].x + acc[j].y;
    if (sacc == 1234.5f) out[threadIdx.x] = lds[0];
    if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
}

template <int MODE, int NS = 2>
void run(const f32x4* w, float* out, unsigned long long* cyc, const char* name) {
    const int chunks = 68 * 30;
    hipFuncSetAttribute((const void*)&kern<MODE, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL((kern<MODE, NS>), dim3(256), dim3(256), 140 * 1024, 0, w, chunks, out, cyc);
    hipDeviceSynchronize();
    hipLaunchKernelGGL((kern<MODE, NS>), dim3(256), dim3(256), 140 * 1024, 0, w, chunks, out, cyc);
    hipDeviceSynchronize();
    unsigned long long h[1024];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 1024; ++i) s += h[i];
    s /= 1024;
    printf("%-40s cycles/MFMA %.2f  (ideal 32)\n", name, s / (chunks * 32.0));
}

// Wave specialisation probes (512 threads: waves 0-3 = MFMA waves, one per SIMD; waves 4-7 = streamers)
//   SPEC 0: streamers idle                      -> MFMA waves' cycles/MFMA alone
//   SPEC 1: streamers global_load_dwordx4 into a register sink (same byte rate as MODE 1)
//   SPEC 2: streamers global_load_lds_dwordx4 (LDS-DMA) into an LDS ring; MFMA waves ds_read frags
template <int SPEC, int SLEEP>
__global__ void __launch_bounds__(512) spec(const f32x4* __restrict__ w, int chunks, float* out,
                                            unsigned long long* cyc) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int cs = 4 * 8 * 64;
    const int wrap = 68;
    if (wave >= 4) {
        const unsigned long long s0 = __builtin_amdgcn_s_memtime();
        const int sw = wave - 4;
        const f32x4* p = w + sw * 8 * 64 + lane;
        if constexpr (SPEC == 1) {
            f32x4 b[3][8];
            for (int c = 0; c < chunks; c += 3) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(b[q][j]) : "v"(p + (size_t)((c + q) % wrap) * cs + j * 64) : "memory");
                    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
#pragma unroll
                    for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(b[(q + 1) % 3][j]));
                    __builtin_amdgcn_s_sleep(SLEEP);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if constexpr (SPEC == 2) {
            float* wl = lds + 16384 + sw * 3 * 2048;
            const unsigned wl_addr = (unsigned)(size_t)wl;
            for (int c = 0; c < chunks; ++c) {
                const f32x4* src = p + (size_t)(c % wrap) * cs;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    unsigned keep;
                    const unsigned dst = __builtin_amdgcn_readfirstlane(wl_addr + (c % 3) * 8192 + j * 1024);
                    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                                 : "=&s"(keep) : "v"(src + j * 64), "s"(dst) : "memory");
                }
                asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                __builtin_amdgcn_s_sleep(SLEEP);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (lane == 0) cyc[4096 + blockIdx.x * 4 + sw] = __builtin_amdgcn_s_memtime() - s0;
        return;
    }
    f32x4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0, 0, 0, 0};
    f32x4 fixed[8];
    for (int j = 0; j < 8; ++j) fixed[j] = f32x4{1.f * lane, 2.f, 3.f, 4.f};
    f32x4 a = {0.5f, 0.25f, 0.125f, 1.f};
    const float* rb = lds + wave * 2048;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < chunks; ++c) {
        f32x4 b[8];
        if constexpr (SPEC == 2) {
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j] = *reinterpret_cast<const f32x4*>(rb + j * 256 + lane * 4);
        }
        PIN();
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(SPEC == 2 ? b[j][s] : fixed[j][s], a[s], acc[j], 0, 0, 0);
        PIN();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float sacc = 0;
    for (int j = 0; j < 8; ++j) sacc += acc[j].x + acc[j].y;
    if (sacc == 1234.5f) out[threadIdx.x] = lds[0];
    if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
}

template <int SPEC, int SLEEP>
void run_spec(const f32x4* w, float* out, unsigned long long* cyc, const char* name) {
    const int chunks = 68 * 30;
    hipFuncSetAttribute((const void*)&spec<SPEC, SLEEP>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((spec<SPEC, SLEEP>), dim3(256), dim3(512), 140 * 1024, 0, w, chunks, out, cyc);
        hipDeviceSynchronize();
    }
    unsigned long long h[8192];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0, st = 0;
    for (int i = 0; i < 1024; ++i) { s += h[i]; st += h[4096 + i]; }
    s /= 1024;
    st /= 1024;
    printf("%-44s cycles/MFMA %.2f  streamer cycles/chunk %.0f (MFMA chunk %.0f)\n", name, s / (chunks * 32.0),
           st / chunks, s / chunks);
}

// Two waves per SIMD, each with half the tiles (T = 4) and its own weight loads (8 waves / CU):
// per-SIMD MFMA rate when another wave can issue MFMAs while one issues its loads.
template <int NT>
__global__ void __launch_bounds__(64 * 32 / NT) dual(const f32x4* __restrict__ w, int chunks, float* out,
                                            unsigned long long* cyc) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f32x4 acc[NT];
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0, 0, 0, 0};
    f32x4 ring[4][NT];
    const f32x4* p = w + wave * NT * 64 + lane;
    const int cs = 32 * 64;   // one chunk = 32 tiles x 1 KiB, whatever the waves-per-tile split
    const int wrap = 68;
    auto ld = [&](f32x4 (&b)[NT], int g) {
        g = g % wrap;
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = p[(size_t)g * cs + j * 64];
    };
    f32x4 a = {0.5f, 0.25f, 0.125f, 1.f};
    for (int q = 0; q < 3; ++q) ld(ring[q], q);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c = 0; c < chunks; c += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            ld(ring[(u + 3) % 4], c + u + 3);
            PIN();
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ring[u][j][s], a[s], acc[j], 0, 0, 0);
            PIN();
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float sacc = 0;
    for (int j = 0; j < NT; ++j) sacc += acc[j].x + acc[j].y;
    if (sacc == 1234.5f) out[threadIdx.x] = sacc;
    if (lane == 0) cyc[blockIdx.x * (32 / NT) + wave] = t1 - t0;
}

template <int NT>
void run_dual(const f32x4* w, float* out, unsigned long long* cyc, const char* name) {
    const int chunks = 68 * 30;
    const int nw = 32 / NT;                 // waves per workgroup; nw / 4 share each SIMD
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL((dual<NT>), dim3(256), dim3(64 * nw), 0, 0, w, chunks, out, cyc);
        hipDeviceSynchronize();
    }
    static unsigned long long h[256 * 16];
    hipMemcpy(h, cyc, sizeof(unsigned long long) * 256 * nw, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 256 * nw; ++i) s += h[i];
    s /= 256 * nw;
    // nw/4 waves share a SIMD: per-SIMD cycles per MFMA = wave time / ((nw/4) * chunks * 4 * NT)
    printf("%-44s cycles/MFMA per SIMD %.2f  (ideal 32)\n", name, s / ((nw / 4.0) * chunks * 4 * NT));
}

int main() {
    f32x4* w;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&w, 68 * 32768);
    hipMemset(w, 0, 68 * 32768);
    hipMalloc(&out, 4096);
    hipMalloc(&cyc, 8192 * 8);
    run<0>(w, out, cyc, "mfma only");
    run<1>(w, out, cyc, "mfma + global_load stream (dependent)");
    run<2>(w, out, cyc, "mfma + global_load stream (sink)");
    run<3>(w, out, cyc, "mfma + buffer_load stream (dependent)");
    run<4, 2>(w, out, cyc, "mfma + LDS-DMA 2-slot + ds_read frags");
    run<4, 3>(w, out, cyc, "mfma + LDS-DMA 3-slot + ds_read frags");
    run<4, 4>(w, out, cyc, "mfma + LDS-DMA 4-slot + ds_read frags");
    run<5>(w, out, cyc, "mfma + ds_read frags (no global)");
    run<6>(w, out, cyc, "mfma + global_load into AGPRs (dependent)");
    run_spec<0, 0>(w, out, cyc, "spec: mfma waves, streamers idle");
    run_spec<1, 0>(w, out, cyc, "spec: + streamer global_load sink, sleep 0");
    run_spec<1, 4>(w, out, cyc, "spec: + streamer global_load sink, sleep 4");
    run_spec<2, 0>(w, out, cyc, "spec: + streamer LDS-DMA, ds_read, sleep 0");
    run_spec<2, 4>(w, out, cyc, "spec: + streamer LDS-DMA, ds_read, sleep 4");
    run_dual<8>(w, out, cyc, "dual: 1 wave/SIMD x 8 tiles, own loads");
    run_dual<4>(w, out, cyc, "dual: 2 waves/SIMD x 4 tiles, own loads");
    run_dual<2>(w, out, cyc, "dual: 4 waves/SIMD x 2 tiles, own loads");
    return 0;
}
