// Microbenchmark: issue rate of v_mfma_f32_4x4x1_16b_f32 dependency chains on one SIMD.
// NC independent accumulator chains per wave, interleaved (chain c takes every NC-th MFMA), with
// NWS waves per SIMD (workgroup of 4 * NWS waves on one CU). Reports cycles per MFMA per SIMD.
// Decides how many chains a 4-candidate rollout tile needs per SIMD to run at the MFMA issue rate.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NC>
__global__ void kern(int iters, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x & 63;
    f32x4 acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    float a = 1.0f + lane * 1e-3f, b = 0.5f + lane * 1e-4f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 64 / NC; ++u)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[c], 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int NC>
void run(int nws) {
    const int iters = 2000, nwaves = 4 * nws;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 64 * nwaves * 4);
    hipMalloc(&cyc, nwaves * 8);
    hipLaunchKernelGGL(kern<NC>, dim3(1), dim3(64 * nwaves), 0, 0, iters, out, cyc);
    hipLaunchKernelGGL(kern<NC>, dim3(1), dim3(64 * nwaves), 0, 0, iters, out, cyc);
    unsigned long long h[64];
    hipMemcpy(h, cyc, nwaves * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int w = 0; w < nwaves; ++w) mx = h[w] > mx ? h[w] : mx;
    // s_memtime counts at the shader clock; MFMAs per SIMD = nws waves x iters x 64
    const double per = mx / ((double)nws * iters * 64);
    printf("chains/wave %d waves/SIMD %d: %.2f cycles per 4x4x1 MFMA per SIMD (issue-rate bound 8)\n", NC, nws, per);
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int nws = 1; nws <= 2; ++nws) {
        run<1>(nws);
        run<2>(nws);
        run<4>(nws);
        run<8>(nws);
    }
    return 0;
}
