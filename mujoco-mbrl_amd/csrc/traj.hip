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

namespace mbrl {

// ------------------------------------------------------------------------------------------------
// Cooperative single-trajectory rollout (see mbrl_internal.h). Hand-off protocol: R2 granules of
// cdna_hip_programming.md §6 Guideline 16 -- each value travels as ONE aligned 8-byte
// {tag = epoch, value} agent-scope atomic store; the consumer wave re-reads (agent-scope atomic
// loads, L1-bypassing) until every tag equals the epoch. epoch = phase + 1, phase = t*(L-1) + l-1;
// two buffers by phase parity (a workgroup cannot be two phases ahead of a reader: it must first
// gather the phase in between, which needs everyone's publish that follows their read).
// Every spin is bounded (s_memrealtime, 100 MHz); on timeout `status` is set and the kernel exits.
// ------------------------------------------------------------------------------------------------
constexpr int COOP_THREADS = 256;
constexpr int COOP_ROWS = 16;  // hidden units per workgroup per layer

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;

__device__ __forceinline__ float rowsum16_t(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x122, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x121, 0xF, 0xF, false));
    return v;
}

__global__ void __launch_bounds__(COOP_THREADS) traj_coop_kernel(const TrajArgs A, u64* __restrict__ xchg_all,
                                                                  unsigned* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int p = blockIdx.x, P = gridDim.x, e = blockIdx.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int Wp = A.Wpad, K0 = A.s + A.a;
    float* slices = smem;                                      // [(L-1)][16][W]
    float* x0 = slices + (size_t)(A.L - 1) * COOP_ROWS * A.W;  // [K0 padded to 4]
    float* hA = x0 + ((K0 + 3) & ~3);                          // [Wp]
    float* hB = hA + Wp;                                       // [Wp]
    float* out = hB + Wp;                                      // [s rounded up to 4]
    int& abort_flag = *reinterpret_cast<int*>(out + ((A.s + 3) & ~3));  // dynamic region (G17)
    const float* member = A.packed + (size_t)e * A.member_stride;
    const float* bias = member + A.bias_off;
    const float* tw = member + A.tw_base;
    u64* xchg = xchg_all + (size_t)e * 2 * Wp;

    if (tid == 0) abort_flag = 0;
    // this workgroup's rows of every hidden W -> W layer: W_l[n][k] = W^T_l[k][n] (plain region);
    // 16 consecutive threads read one 64-byte run of a W^T row
    for (int l = 1; l < A.L; ++l) {
        const float* wt = tw + A.tw_off[l];
        float* dst = slices + (size_t)(l - 1) * COOP_ROWS * A.W;
        for (int i = tid; i < COOP_ROWS * A.W; i += COOP_THREADS) {
            const int k = i >> 4, o = i & 15;
            dst[o * A.W + k] = wt[(size_t)k * Wp + p * COOP_ROWS + o];
        }
    }
    for (int d = tid; d < A.s; d += COOP_THREADS) {
        const float sv = A.s0[d];
        x0[d] = A.norm_s ? (sv - A.obs_mean[d]) / A.obs_std[d] : sv;
    }
    __syncthreads();

    int phase = 0;
    for (int t = 0; t < A.H; ++t) {
        for (int d = tid; d < A.a; d += COOP_THREADS) {
            const float av = A.actions[t * A.a + d];
            x0[A.s + d] = A.norm_a ? (av - A.act_mean[d]) / A.act_std[d] : av;
        }
        __syncthreads();
        // layer 0, all Wp units (redundant in every workgroup): W^T_0 [K0][Wp], coalesced over n
        for (int n = tid; n < Wp; n += COOP_THREADS) {
            const float* w0 = tw + A.tw_off[0] + n;
            float v = bias[n];
            for (int k = 0; k < K0; ++k) v += w0[(size_t)k * Wp] * x0[k];
            hA[n] = fmaxf(v, 0.0f);
        }
        __syncthreads();
        float* cur = hA;
        float* nxt = hB;
        for (int l = 1; l < A.L; ++l, ++phase) {
            // my 16 units: row o = tid >> 4, lanes j = tid & 15 split K
            const int o = tid >> 4, j = tid & 15;
            const float* ws = slices + (size_t)(l - 1) * COOP_ROWS * A.W + (size_t)o * A.W;
            float v = 0.f;
            for (int k = j; k < A.W; k += 16) v += ws[k] * cur[k];
            v = rowsum16_t(v);
            const unsigned epoch = (unsigned)phase + 1u;
            u64* buf = xchg + (size_t)(phase & 1) * Wp;
            if (j == 0) {
                const int n = p * COOP_ROWS + o;
                const float y = fmaxf(v + bias[(size_t)l * Wp + n], 0.0f);
                __hip_atomic_store(&buf[n], ((u64)epoch << 32) | __float_as_uint(y), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            // gather all P slices: wave 0 sweeps the granules until every tag matches
            if (wave == 0) {
                const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    bool ok = true;
                    for (int n = lane; n < P * COOP_ROWS; n += 64) {
                        const u64 g = __hip_atomic_load(&buf[n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok &= (unsigned)(g >> 32) == epoch;
                        nxt[n] = __uint_as_float((unsigned)g);
                    }
                    if (__all(ok)) break;
                    if (__builtin_amdgcn_s_memrealtime() - t_start > 20000000ull) {  // 200 ms
                        if (lane == 0) {
                            abort_flag = 1;
                            atomicOr(status, 1u);
                        }
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __syncthreads();
            if (abort_flag) return;
            float* tmp = cur; cur = nxt; nxt = tmp;
        }
        // output layer (redundant): 16 lanes per output row, Wout row-major [s][W]
        const float* wo = tw + A.tw_off[A.L];
        const float* bo = bias + (size_t)A.L * Wp;
        for (int base = 0; base < A.s; base += COOP_THREADS / 16) {
            const int o = base + (tid >> 4), j = tid & 15;
            float v = 0.f;
            if (o < A.s)
                for (int k = j; k < A.W; k += 16) v += wo[(size_t)o * A.W + k] * cur[k];
            v = rowsum16_t(v);
            if (j == 0 && o < A.s) out[o] = v + bo[o];
        }
        __syncthreads();
        for (int d = tid; d < A.s; d += COOP_THREADS) {
            const float sn = A.unnorm_s ? out[d] * A.obs_std[d] + A.obs_mean[d] : out[d];
            if (p == 0) A.states_out[((size_t)e * A.H + t) * A.s + d] = sn;
            x0[d] = A.norm_s ? (sn - A.obs_mean[d]) / A.obs_std[d] : sn;
        }
        // x0[s..s+a) is rewritten before the barrier at the top of the next step
    }
}

bool traj_coop_supported(const TrajArgs& A, int E) {
    const int P = A.Wpad / COOP_ROWS;
    const size_t lds = ((size_t)(A.L - 1) * COOP_ROWS * A.W + ((A.s + A.a + 3) & ~3) + 2 * A.Wpad +
                        ((A.s + 3) & ~3) + 4) * 4;
    return A.L >= 2 && A.W == A.Wpad && P * E <= 256 && lds <= 150 * 1024;
}

size_t traj_coop_xchg_bytes(const TrajArgs& A, int E) { return (size_t)E * 2 * A.Wpad * sizeof(u64); }

hipError_t launch_traj_coop(const TrajArgs& A, int E, unsigned long long* xchg, unsigned* status,
                            hipStream_t stream) {
    const int P = A.Wpad / COOP_ROWS;
    const size_t lds = ((size_t)(A.L - 1) * COOP_ROWS * A.W + ((A.s + A.a + 3) & ~3) + 2 * A.Wpad +
                        ((A.s + 3) & ~3) + 4) * 4;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(&traj_coop_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (err != hipSuccess) return err;
        attr_set = true;
    }
    hipError_t err = hipMemsetAsync(xchg, 0, traj_coop_xchg_bytes(A, E), stream);
    if (err != hipSuccess) return err;
    err = hipMemsetAsync(status, 0, sizeof(unsigned), stream);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(traj_coop_kernel, dim3(P, E), dim3(COOP_THREADS), lds, stream, A, xchg, status);
    return hipGetLastError();
}

}  // namespace mbrl
