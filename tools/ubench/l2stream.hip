// Microbenchmark: per-CU throughput of an L2-resident weight stream (the rollout kernel's access
// pattern: every workgroup streams the same 2.2 MB buffer as 1 KiB wave-instructions) as a function
// of waves per workgroup and loads in flight. One workgroup per CU (LDS-forced), 256 workgroups.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NW, int DEPTH>
__global__ void __launch_bounds__(NW * 64) stream_kernel(const f32x4* __restrict__ w, size_t n_frag_per_wave_step,
                                                         int steps, float* out) {
    extern __shared__ float lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f32x4 acc = {0, 0, 0, 0};
    for (int t = 0; t < steps; ++t) {
        const f32x4* p = w + (size_t)wave * 64 + lane;
        for (size_t f = 0; f < n_frag_per_wave_step; f += DEPTH) {
            f32x4 v[DEPTH];
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) v[d] = p[(f + d) * NW * 64];
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) acc += v[d];
        }
    }
    if (acc.x == 1234.5f) out[threadIdx.x] = acc.y + lds[0];
}

template <int NW, int DEPTH>
void run(const f32x4* w, size_t bytes, float* out, int grid = 256) {
    const size_t frags = bytes / 1024 / NW;  // per wave per step
    const int steps = 30;
    hipFuncSetAttribute((const void*)&stream_kernel<NW, DEPTH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL((stream_kernel<NW, DEPTH>), dim3(grid), dim3(NW * 64), 96 * 1024, 0, w, frags, steps, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
    }
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double per_cu = (double)bytes * steps / (ms * 1e-3) / 1e9;
    printf("workgroups %3d  waves/CU %2d  loads-in-flight/wave %2d : %.3f ms  per-CU %.1f GB/s  chip %.2f TB/s\n", grid,
           NW, DEPTH, ms, per_cu, per_cu * grid / 1e3);
}

int main() {
    const size_t bytes = 2228224;  // cheetah step stream (68 chunks x 32 KiB)
    f32x4* w;
    float* out;
    hipMalloc(&w, bytes);
    hipMalloc(&out, 4096 * 4);
    hipMemset(w, 0, bytes);
    run<4, 8>(w, bytes, out);
    run<4, 16>(w, bytes, out);
    run<4, 32>(w, bytes, out);
    run<8, 8>(w, bytes, out);
    run<8, 16>(w, bytes, out);
    run<16, 8>(w, bytes, out);
    run<16, 4>(w, bytes, out);
    // half the CUs streaming (32 candidates per workgroup at N = 4096): per-CU rate when the
    // aggregate L2 bandwidth is not shared by every CU
    run<8, 8>(w, bytes, out, 128);
    run<8, 16>(w, bytes, out, 128);
    run<16, 8>(w, bytes, out, 128);
    run<8, 8>(w, bytes, out, 64);
    return 0;
}
