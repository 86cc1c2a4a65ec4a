// Single-trajectory rollout: the predicted states of the final CEM mean (SURVEY.md §8a a11,
// "final mu as actions plus the states of its re-rollout"), one workgroup of 1024 threads per
// ensemble member.
//
// One candidate is a chain of H*(L+1) dependent matrix-vector products: latency- and per-CU
// bandwidth-bound, not FLOP-bound. The 16-row MFMA tile of rollout.hip would spend 15/16 of its
// matrix issue on padding rows, so this kernel uses VALU dot products over plain weight copies
// (written by the pack step next to the fragment stream):
//   * layer 0 / hidden layers: W^T [in][Wpad]; thread (g4, ks) owns 4 consecutive outputs and a
//     K slice -> coalesced 16-byte loads, fixed-order partial sums through LDS;
//   * output layer: row-major [s][W]; one wave per output row, shuffle reduction.
// Semantics per step are DynamicsModel.forward (models.py:13-29) with the GoalStateAgent
// normalisers, exactly as the rollout kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mbrl_internal.h"

namespace mbrl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TRAJ_THREADS = 1024;

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// y[0..Wpad) = relu(W x + b) with W^T [in][Wpad]; x in LDS, part scratch [KS][Wpad].
__device__ __forceinline__ void traj_dense_relu(const float* __restrict__ wt, const float* __restrict__ bias,
                                                int in, int Wpad, const float* x, float* part, float* y) {
    const int G4 = Wpad / 4;
    const int KS = TRAJ_THREADS / G4;            // Wpad <= 1024 -> KS >= 4
    const int tid = threadIdx.x;
    const int g4 = tid % G4, ks = tid / G4;
    const int per = (in + KS - 1) / KS;
    const int k0 = ks * per, k1 = min(in, k0 + per);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const f32x4* w4 = reinterpret_cast<const f32x4*>(wt) + g4;
#pragma unroll 8
    for (int k = k0; k < k1; ++k) {
        const f32x4 w = w4[(size_t)k * G4];
        const float xv = x[k];
        acc += xv * w;
    }
    *reinterpret_cast<f32x4*>(part + ks * Wpad + 4 * g4) = acc;
    __syncthreads();
    for (int n = tid; n < Wpad; n += TRAJ_THREADS) {
        float v = bias[n];
        for (int j = 0; j < KS; ++j) v += part[j * Wpad + n];
        y[n] = fmaxf(v, 0.0f);
    }
    __syncthreads();
}

__global__ void __launch_bounds__(TRAJ_THREADS) traj_kernel(const TrajArgs A) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int e = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int K0 = A.s + A.a;
    const int xdim = K0 > A.Wpad ? K0 : A.Wpad;
    float* x = smem;                       // layer input  [xdim]
    float* y = x + ((xdim + 3) & ~3);      // layer output [Wpad]
    float* part = y + A.Wpad;              // [4096]
    float* out = part + 4096;              // output layer result [s]
    const float* member = A.packed + (size_t)e * A.member_stride;
    const float* bias = member + A.bias_off;
    const float* tw = member + A.tw_base;

    for (int d = tid; d < A.s; d += TRAJ_THREADS) {
        const float sv = A.s0[d];
        x[d] = A.norm_s ? (sv - A.obs_mean[d]) / A.obs_std[d] : sv;
    }
    for (int t = 0; t < A.H; ++t) {
        for (int d = tid; d < A.a; d += TRAJ_THREADS) {
            const float av = A.actions[t * A.a + d];
            x[A.s + d] = A.norm_a ? (av - A.act_mean[d]) / A.act_std[d] : av;
        }
        __syncthreads();
        traj_dense_relu(tw + A.tw_off[0], bias, K0, A.Wpad, x, part, y);
        float* cur = y;
        float* nxt = x;
        for (int l = 1; l < A.L; ++l) {
            traj_dense_relu(tw + A.tw_off[l], bias + l * A.Wpad, A.W, A.Wpad, cur, part, nxt);
            float* tmp = cur; cur = nxt; nxt = tmp;
        }
        // output layer: one wave per row n, W row-major
        const float* wo = tw + A.tw_off[A.L];
        const float* bo = bias + A.L * A.Wpad;
        for (int n = wave; n < A.s; n += TRAJ_THREADS / 64) {
            float v = 0.f;
            for (int k = lane; k < A.W; k += 64) v += wo[(size_t)n * A.W + k] * cur[k];
            v = wave_sum64(v);
            if (lane == 0) out[n] = v + bo[n];
        }
        __syncthreads();
        for (int d = tid; d < A.s; d += TRAJ_THREADS) {
            const float sn = A.unnorm_s ? out[d] * A.obs_std[d] + A.obs_mean[d] : out[d];
            A.states_out[((size_t)e * A.H + t) * A.s + d] = sn;
            x[d] = A.norm_s ? (sn - A.obs_mean[d]) / A.obs_std[d] : sn;
        }
        // x[s..s+a) is rewritten at the top of the next step; cur/nxt never alias x's state part
        // before that barrier.
    }
}

hipError_t launch_traj(const TrajArgs& A, int E, hipStream_t stream) {
    const int K0 = A.s + A.a;
    const int xdim = K0 > A.Wpad ? K0 : A.Wpad;
    const size_t lds = ((size_t)((xdim + 3) & ~3) + A.Wpad + 4096 + ((A.s + 3) & ~3)) * sizeof(float);
    hipLaunchKernelGGL(traj_kernel, dim3(E), dim3(TRAJ_THREADS), lds, stream, A);
    return hipGetLastError();
}

}  // namespace mbrl
