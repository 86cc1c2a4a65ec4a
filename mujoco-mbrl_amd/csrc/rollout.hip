// Persistent H-step candidate rollout + goal-state cost, fp32 MFMA, one launch per CEM iteration.
//
// Replaces the reference's hot loop (planners.py:199-210): for t in H: state_list[t] =
// model(states, actions) with DynamicsModel.forward (models.py:13-29) wired through the
// GoalStateAgent normalisers (agents.py:219-230), then cost = SmoothAbsLoss(s_{t+1}) +
// CoshLoss(a_t) (agents.py:182-183) summed over t.
//
// Mapping:
//   * one workgroup = 4 waves = M = 16*R candidates of one ensemble member, for all H steps; the
//     candidates' activations live in LDS for the whole horizon (never touch HBM).
//   * every Linear is a chain of v_mfma_f32_16x16x4_f32 (exact fp32): wave w owns output columns
//     [w*W/4, (w+1)*W/4) of each hidden layer (T = W/64 16-column tiles); the output layer splits
//     K over the 4 waves and reduces through LDS.
//   * weights are pre-packed (pack kernels in cem.hip) into the exact fragment order each wave
//     consumes: one global_load_dwordx4 per lane = one 1 KiB coalesced B fragment. The per-step
//     stream (~2.2 MB for 3x512) stays resident in every XCD's 4 MB L2; each wave streams its
//     slice with a register double buffer that runs ahead across layer and step boundaries.
//   * the step epilogue (unnormalise, goal cost, renormalise, next proposal draw from the Philox
//     counter RNG) runs on the VALU from LDS; the per-candidate return is a register of thread m.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mbrl_internal.h"
#include "mbrl_rng.h"

namespace mbrl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int T>
__device__ __forceinline__ void load_chunk(f32x4 (&b)[T], const f32x4* __restrict__ p) {
#pragma unroll
    for (int j = 0; j < T; ++j) b[j] = p[j * 64];
}

// Hidden-type chunk: one 16-deep K slice x T output tiles.
template <int T, int R>
__device__ __forceinline__ void mma_hidden(f32x4 (&acc)[R][T], const f32x4 (&b)[T], const float* act,
                                           int lda, int kc, int lane) {
    f32x4 a[R];
#pragma unroll
    for (int r = 0; r < R; ++r)
        a[r] = *reinterpret_cast<const f32x4*>(act + (16 * r + (lane & 15)) * lda + 16 * kc + 4 * (lane >> 4));
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < T; ++j)
#pragma unroll
            for (int r = 0; r < R; ++r)
                acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[r][s], b[j][s], acc[r][j], 0, 0, 0);
}

// Output-type chunk: one 16-column output tile over this wave's W/4-deep K range.
template <int T, int R>
__device__ __forceinline__ void mma_out(const f32x4 (&aout)[R][T], const f32x4 (&b)[T], float* part,
                                        int pw, int tile, int lane) {
    f32x4 o0[R], o1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) { o0[r] = f32x4{0.f, 0.f, 0.f, 0.f}; o1[r] = o0[r]; }
#pragma unroll
    for (int kc = 0; kc < T; ++kc)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            o0[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(aout[r][kc][0], b[kc][0], o0[r], 0, 0, 0);
            o1[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(aout[r][kc][1], b[kc][1], o1[r], 0, 0, 0);
            o0[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(aout[r][kc][2], b[kc][2], o0[r], 0, 0, 0);
            o1[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(aout[r][kc][3], b[kc][3], o1[r], 0, 0, 0);
        }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i)
            part[(16 * r + 4 * (lane >> 4) + i) * pw + 16 * tile + (lane & 15)] = o0[r][i] + o1[r][i];
}

template <int T, int R>
__device__ __forceinline__ void hidden_epilogue(f32x4 (&acc)[R][T], float* act, int lda, const float* hb,
                                                int wave, int lane) {
    __syncthreads();  // every wave has finished reading this layer's input
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int col = wave * 16 * T + 16 * j + (lane & 15);
            const float bias = hb[col];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = 16 * r + 4 * (lane >> 4) + i;
                act[row * lda + col] = fmaxf(acc[r][j][i] + bias, 0.0f);
            }
        }
    __syncthreads();
}

template <int T, int R>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[R][T]) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < T; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Draw (or read) a_t for this tile's candidates, write the normalised action into the MLP input,
// and stage its CoshLoss terms.  Threads 64..64+M*G (waves 1..3) so it overlaps phase B on wave 0.
template <int R>
__device__ __forceinline__ void stage_actions(const RolloutArgs& A, const LdsMap& L, int tile, int t) {
    constexpr int M = 16 * R;
    const int G = (A.a + 3) >> 2;
    const int idx = (int)threadIdx.x - 64;
    if (idx < 0 || idx >= M * G) return;
    const int m = idx / G, g = idx - (idx / G) * G;
    const int n = tile * M + m;
    const bool valid = n < A.N;
    float z[4] = {0.f, 0.f, 0.f, 0.f};
    if (A.actions == nullptr)
        cem_normal4(A.seed, (uint32_t)(A.n_offset + n), (uint32_t)t, (uint32_t)A.iteration, (uint32_t)g, z);
    float* aterm = L.aterm + (t & 1) * M * A.a;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int d = 4 * g + j;
        if (d >= A.a) break;
        float av;
        if (A.actions == nullptr)
            av = cem_action(L.mu[t * A.a + d], L.sigma[t * A.a + d], z[j], A.lo, A.hi);
        else
            av = valid ? A.actions[((size_t)t * A.N + n) * A.a + d] : 0.0f;
        L.act[m * A.lda + A.s + d] = A.norm_a ? (av - L.act_mean[d]) / L.act_std[d] : av;
        aterm[m * A.a + d] = A.has_ac ? coshf(av / A.alpha_a) - 1.0f : 0.0f;
        if (A.actions_out != nullptr && valid) A.actions_out[((size_t)t * A.N + n) * A.a + d] = av;
    }
}

template <int T, int R>
__global__ void __launch_bounds__(256, 1) rollout_kernel(const RolloutArgs A) {
    constexpr int M = 16 * R;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const LdsMap L = lds_map(A, smem, M);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int tile = blockIdx.x, e = blockIdx.y;
    const float* member = A.packed + (size_t)e * A.member_stride;

    // ---- prologue: parameters into LDS, s0 into the MLP input
    for (int i = tid; i < A.s; i += 256) {
        L.obs_mean[i] = A.obs_mean ? A.obs_mean[i] : 0.f;
        L.obs_std[i] = A.obs_std ? A.obs_std[i] : 1.f;
        L.goal[i] = A.goal ? A.goal[i] : 0.f;
        L.cw[i] = A.cw ? A.cw[i] : 0.f;
    }
    for (int i = tid; i < A.a; i += 256) {
        L.act_mean[i] = A.act_mean ? A.act_mean[i] : 0.f;
        L.act_std[i] = A.act_std ? A.act_std[i] : 1.f;
    }
    const float* bias_src = member + A.stream_floats;
    for (int i = tid; i < A.L * A.Wpad + 16 * A.NOT; i += 256) L.hbias[i] = bias_src[i];
    if (A.actions == nullptr)
        for (int i = tid; i < A.H * A.a; i += 256) { L.mu[i] = A.mu[i]; L.sigma[i] = A.sigma[i]; }
    __syncthreads();
    for (int i = tid; i < M * A.s; i += 256) {
        const int m = i / A.s, d = i - (i / A.s) * A.s;
        const int n = min(tile * M + m, A.N - 1);
        const float sv = A.s0_per_cand ? A.s0[(size_t)n * A.s + d] : A.s0[d];
        L.act[m * A.lda + d] = A.norm_s ? (sv - L.obs_mean[d]) / L.obs_std[d] : sv;
    }
    for (int i = tid; i < M * A.k0pad_extra; i += 256) {
        const int m = i / A.k0pad_extra, j = i - (i / A.k0pad_extra) * A.k0pad_extra;
        L.act[m * A.lda + A.s + A.a + j] = 0.f;
    }
    stage_actions<R>(A, L, tile, 0);
    __syncthreads();

    // ---- weight stream: this wave's slice of chunk g is at wb + g * cs (f32x4 units)
    const f32x4* wb = reinterpret_cast<const f32x4*>(member) + wave * T * 64 + lane;
    const int cs = 4 * T * 64;
    const int C = A.chunks_per_step;
    auto chunk_ptr = [&](int g) { return wb + (size_t)(g < C ? g : g - C) * cs; };

    f32x4 bA[T], bB[T];
    f32x4 acc[R][T];
    load_chunk<T>(bA, wb);
    float total = 0.f;
    const int KH = 4 * T;  // K chunks of a hidden (W -> W) layer

    for (int t = 0; t < A.H; ++t) {
        int g = 0;
        // ---- layer 0: [s | a | 0-pad] -> W
        zero_acc<T, R>(acc);
        for (int kc = 0; kc < A.K0C; kc += 2) {
            load_chunk<T>(bB, chunk_ptr(g + 1));
            mma_hidden<T, R>(acc, bA, L.act, A.lda, kc, lane);
            load_chunk<T>(bA, chunk_ptr(g + 2));
            mma_hidden<T, R>(acc, bB, L.act, A.lda, kc + 1, lane);
            g += 2;
        }
        hidden_epilogue<T, R>(acc, L.act, A.lda, L.hbias, wave, lane);
        // ---- hidden layers 1..L-1: W -> W
        for (int l = 1; l < A.L; ++l) {
            zero_acc<T, R>(acc);
            for (int kc = 0; kc < KH; kc += 2) {
                load_chunk<T>(bB, chunk_ptr(g + 1));
                mma_hidden<T, R>(acc, bA, L.act, A.lda, kc, lane);
                load_chunk<T>(bA, chunk_ptr(g + 2));
                mma_hidden<T, R>(acc, bB, L.act, A.lda, kc + 1, lane);
                g += 2;
            }
            hidden_epilogue<T, R>(acc, L.act, A.lda, L.hbias + l * A.Wpad, wave, lane);
        }
        // ---- output layer: W -> s, K split over the 4 waves, partials through LDS
        {
            f32x4 aout[R][T];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int kc = 0; kc < T; ++kc)
                    aout[r][kc] = *reinterpret_cast<const f32x4*>(
                        L.act + (16 * r + (lane & 15)) * A.lda + wave * 16 * T + 16 * kc + 4 * (lane >> 4));
            float* part = L.part + wave * M * A.pw;
            for (int j = 0; j < A.NOT; j += 2) {
                load_chunk<T>(bB, chunk_ptr(g + 1));
                mma_out<T, R>(aout, bA, part, A.pw, j, lane);
                load_chunk<T>(bA, chunk_ptr(g + 2));
                mma_out<T, R>(aout, bB, part, A.pw, j + 1, lane);
                g += 2;
            }
        }
        __syncthreads();

        // ---- phase A: s_{t+1} = unnormalize(out), state-cost terms, next MLP input
        const float* bout = L.hbias + A.L * A.Wpad;
        for (int i = tid; i < M * A.s; i += 256) {
            const int m = i / A.s, d = i - (i / A.s) * A.s;
            const int ro = m * A.pw + d;
            const int ws = M * A.pw;
            const float o = L.part[ro] + L.part[ws + ro] + L.part[2 * ws + ro] + L.part[3 * ws + ro] + bout[d];
            const float sn = A.unnorm_s ? o * L.obs_std[d] + L.obs_mean[d] : o;
            float term = 0.f;
            if (A.has_sc) {
                const float x = (sn - L.goal[d]) * L.cw[d];
                term = sqrtf(x * x + A.alpha_s2) - A.alpha_s;
            }
            L.sterm[m * A.s + d] = term;
            L.act[m * A.lda + d] = A.norm_s ? (sn - L.obs_mean[d]) / L.obs_std[d] : sn;
            const int n = tile * M + m;
            if (A.states_out != nullptr && n < A.N)
                A.states_out[(((size_t)e * A.H + t) * A.N + n) * A.s + d] = sn;
        }
        for (int i = tid; i < M * A.k0pad_extra; i += 256) {
            const int m = i / A.k0pad_extra, j = i - (i / A.k0pad_extra) * A.k0pad_extra;
            L.act[m * A.lda + A.s + A.a + j] = 0.f;
        }
        __syncthreads();
        // ---- phase B (wave 0): per-candidate step cost, sequential return; phase C (waves 1-3): a_{t+1}
        if (tid < M) {
            float sc = 0.f, ac = 0.f;
            for (int d = 0; d < A.s; ++d) sc += L.sterm[tid * A.s + d];
            const float* aterm = L.aterm + (t & 1) * M * A.a;
            for (int d = 0; d < A.a; ++d) ac += aterm[tid * A.a + d];
            ac = A.alpha_a2 * (ac / (float)A.a);
            total += sc + ac;
        }
        if (t + 1 < A.H) stage_actions<R>(A, L, tile, t + 1);
        __syncthreads();
    }
    if (tid < M) {
        const int n = tile * M + tid;
        if (n < A.N) A.costs[(size_t)e * A.N + n] = total;
    }
}

template <int T, int R>
static hipError_t launch_rollout_tr(const RolloutArgs& A, hipStream_t stream) {
    const int M = 16 * R;
    dim3 grid((A.N + M - 1) / M, A.E);
    const size_t lds = rollout_lds_bytes(A, M);
    static bool attr_set = false;  // raise the dynamic-LDS cap once per instantiation
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&rollout_kernel<T, R>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL((rollout_kernel<T, R>), grid, dim3(256), lds, stream, A);
    return hipGetLastError();
}

hipError_t launch_rollout(const RolloutArgs& A, int T, int R, hipStream_t stream) {
#define MBRL_CASE(TT, RR) \
    if (T == TT && R == RR) return launch_rollout_tr<TT, RR>(A, stream);
    MBRL_CASE(1, 1) MBRL_CASE(2, 1) MBRL_CASE(4, 1) MBRL_CASE(8, 1) MBRL_CASE(16, 1)
    MBRL_CASE(1, 2) MBRL_CASE(2, 2) MBRL_CASE(4, 2) MBRL_CASE(8, 2)
#undef MBRL_CASE
    return hipErrorInvalidValue;
}

}  // namespace mbrl
