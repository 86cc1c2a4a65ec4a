// Persistent H-step candidate rollout + goal-state cost, fp32 MFMA, one launch per CEM iteration.
//
// Replaces the reference's hot loop (planners.py:199-210): for t in H: state_list[t] =
// model(states, actions) with DynamicsModel.forward (models.py:13-29) wired through the
// GoalStateAgent normalisers (agents.py:219-230), then cost = SmoothAbsLoss(s_{t+1}) +
// CoshLoss(a_t) (agents.py:182-183) summed over t.
//
// Mapping:
//   * one workgroup = M = 16*R candidates of one ensemble member, for all H steps (8 candidates in
//     rollout_m8_kernel at the end of this file); 8 waves (two per
//     SIMD) for R = 1, 4 for R = 2. The candidates' activations live in LDS for the whole horizon
//     (ping-pong buffers, never HBM).
//   * every Linear is a chain of v_mfma_f32_16x16x4_f32 (exact fp32) with the weights as the A
//     operand: wave w owns output columns [w*W/NW, (w+1)*W/NW) of each hidden layer; the output
//     layer splits K over the waves (each wave's own columns, straight from its accumulators) and
//     reduces through LDS.
//   * weights are pre-packed (pack kernels in cem.hip) into the exact fragment order each wave
//     consumes: one buffer_load_dwordx4 per lane = one 1 KiB coalesced fragment. The per-step
//     stream (~2.2 MB for 3x512) stays resident in every XCD's 4 MB L2; each wave streams its
//     slice through a 4-deep register ring that runs 3 chunks ahead across layer and step
//     boundaries. sched_barrier pins the issue order so hipcc cannot sink the prefetch next to its
//     use (it did: the unpinned build drained vmcnt(0) every chunk).
//   * the activation fragments are read from LDS one chunk ahead as well.
//   * candidate actions come from HBM ([H][N][a], written by the proposal kernel or given by the
//     caller); a_{t+1} is loaded at the start of step t so its latency hides under the MFMAs.
//   * the step epilogue (unnormalise, goal cost, renormalise) runs on the VALU out of LDS, waves 0-3
//     for the state and waves 4-7 for the actions; per-row sums are DPP row reductions; the return
//     is a register of the reducing lane.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "mbrl_internal.h"

// Waves per workgroup for the rollout: 8 (two per SIMD, T/2 tiles each) for R = 1, and for R = 2 where
// the aliased output partials fit LDS; else 4. The weight stream goes through buffer_load (SGPR
// descriptor + 32-bit offsets). Measured on cheetah, rollout ms (r01; the other forms were removed in
// r06): global 4 waves 1.083 | buffer 4 waves 1.044 | global 8 waves 1.171 | buffer 8 waves 1.035
// State slots per lane (ceil(s / 16)) up to which the 8/16-candidate epilogues keep their per-lane
// parameter copies in registers; wider states read them from LDS (the copies spilled on humanoid).
#ifndef MBRL_EPI_REG_SLOTS
#define MBRL_EPI_REG_SLOTS 2
#endif
// Timing ablation only (results are garbage): -DMBRL_PAIR_DIAG=1 keeps the column-split pairs' LDS
// hand-off flow but drops every cross-workgroup store, poll and load.
#ifndef MBRL_PAIR_DIAG
#define MBRL_PAIR_DIAG 0
#endif

namespace mbrl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MBRL_PIN() __builtin_amdgcn_sched_barrier(0)

// Diagnostic build only (make diag, -DMBRL_STAMPS): per-wave s_memtime sums per kernel segment,
// written to a buffer set by mbrl_diag_set_stamps(). The timed kernel never contains stamps.
#ifdef MBRL_STAMPS
constexpr int NSEG = 8;
__device__ unsigned long long* g_mbrl_stamps;
#define STAMP(k)                                                   \
    do {                                                           \
        MBRL_PIN();                                                \
        const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
        seg[k] += _t - tprev;                                      \
        tprev = _t;                                                \
        MBRL_PIN();                                                \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif

// The weight stream through buffer_load_dwordx4 (SGPR descriptor, 32-bit per-lane offsets: one VGPR of
// address per load instead of a global_load's two).
template <int T>
__device__ __forceinline__ void load_chunk_buf(f32x4 (&b)[T], __amdgpu_buffer_rsrc_t rsrc, unsigned voff) {
#ifdef MBRL_DIAG_NOLOAD  // timing ablation only: no weight stream (results are garbage)
    (void)rsrc;
    (void)voff;
#pragma unroll
    for (int j = 0; j < T; ++j) asm volatile("" : "+v"(b[j]));
#else
#pragma unroll
    for (int j = 0; j < T; ++j)
        b[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + (unsigned)(j * 64 * 16), 0, 0));
#endif
}

template <int R>
__device__ __forceinline__ void read_a(f32x4 (&a)[R], const float* act, int lda, int kc, int lane) {
#pragma unroll
    for (int r = 0; r < R; ++r)
        a[r] = *reinterpret_cast<const f32x4*>(act + (16 * r + (lane & 15)) * lda + 16 * kc + 4 * (lane >> 4));
}

// Hidden-type chunk: one 16-deep K slice x T output tiles (MFMAs on independent accumulators).
// Weights are the A operand and activations the B operand (Y^T = W X^T), so lane l ends up with
// 4 consecutive output features n0 + 4(l>>4) + i of candidate 16r + (l&15): a float4 row store.
template <int T, int R>
__device__ __forceinline__ void mma_hidden(f32x4 (&acc)[R][T], const f32x4 (&a)[R], const f32x4 (&b)[T]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < T; ++j)
#pragma unroll
            for (int r = 0; r < R; ++r)
                acc[r][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j][s], a[r][s], acc[r][j], 0, 0, 0);
}

// Output-type chunk: one 16-column output tile over this wave's own K range; four accumulator
// chains so consecutive MFMAs never wait on each other.
// Canonical output sum (the same bits for every tile height, wave count and shard size): the hidden
// features split into 8 "halves" of T/2 tiles each (NW = 8: one per wave; NW = 4, T >= 2: two per
// wave, NH = 2); a half is four chains (k = 16 kc + 4 s + i, chain s) closed as (c0 + c1) + (c2 + c3);
// the output is ((h0 + h1) + (h2 + h3)) + ((h4 + h5) + (h6 + h7)) -- sum_partials below. A 4-wave
// workgroup stores (h_2w + h_2w+1) per wave, which is exactly the inner pair of that tree.
template <int T, int R, int NH>
__device__ __forceinline__ void mma_out(const f32x4 (&aout)[R][T], const f32x4 (&b)[T], float* part, int pw,
                                        int tile, int lane) {
    static_assert(NH == 1 || (NH == 2 && T % 2 == 0), "halves");
    constexpr int TH = T / NH;
    f32x4 o[NH][R][4];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int s = 0; s < 4; ++s) o[h][r][s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < T; ++kc)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int r = 0; r < R; ++r)
                o[kc / TH][r][s] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[kc][s], aout[r][kc][s], o[kc / TH][r][s], 0, 0, 0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        f32x4 v = (o[0][r][0] + o[0][r][1]) + (o[0][r][2] + o[0][r][3]);
        if constexpr (NH == 2) v = v + ((o[1][r][0] + o[1][r][1]) + (o[1][r][2] + o[1][r][3]));
        *reinterpret_cast<f32x4*>(part + (16 * r + (lane & 15)) * pw + 16 * tile + 4 * (lane >> 4)) = v;
    }
}

// acc + bias -> ReLU -> next activation buffer (float4 row stores); one barrier (ping-pong buffers).
// T here is the tiles per wave (TW): wave w owns columns [16 T w, 16 T (w + 1)).
template <int T, int R>
__device__ __forceinline__ void hidden_store(const f32x4 (&acc)[R][T], const f32x4 (&bias)[T], float* out,
                                             int lda, int wave, int lane) {
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < T; ++j) {
            f32x4 v = acc[r][j] + bias[j];
            v = __builtin_elementwise_max(v, zero);
            *reinterpret_cast<f32x4*>(out + (16 * r + (lane & 15)) * lda + wave * 16 * T + 16 * j + 4 * (lane >> 4)) = v;
        }
    __syncthreads();
}

// hidden_store without the barrier (the column-split pairs' first of two layer-0 stores)
template <int T, int R>
__device__ __forceinline__ void hidden_store_nobar(const f32x4 (&acc)[R][T], const f32x4 (&bias)[T], float* out,
                                                   int lda, int wave, int lane) {
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < T; ++j) {
            f32x4 v = acc[r][j] + bias[j];
            v = __builtin_elementwise_max(v, zero);
            *reinterpret_cast<f32x4*>(out + (16 * r + (lane & 15)) * lda + wave * 16 * T + 16 * j + 4 * (lane >> 4)) = v;
        }
}

template <int T>
__device__ __forceinline__ void load_bias(f32x4 (&bias)[T], const float* hb, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < T; ++j)
        bias[j] = *reinterpret_cast<const f32x4*>(hb + wave * 16 * T + 16 * j + 4 * (lane >> 4));
}

template <int T, int R>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[R][T]) {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < T; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Sum over the 16 lanes of a DPP row (row_ror 8, 4, 2, 1): every lane of the row gets the total.
__device__ __forceinline__ float rowsum16(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x122, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x121, 0xF, 0xF, false));
    return v;
}

// Epilogue mapping: lane l of wave w owns candidate row m = 16r + 4w + (l >> 4) and the feature
// slots d = (l & 15) + 16k of that row, so per-row reductions are one DPP row sum.
constexpr int MAX_A_PER_LANE = 3;  // action_dim <= 48

__device__ __forceinline__ int epi_row(int r, int wave, int lane) { return 16 * r + 4 * wave + (lane >> 4); }

// a_t for this lane's (row, slots), loaded early and unconditionally (clamped indices) so hipcc
// emits no branch-around-load with its vmcnt(0) (cdna_hip_programming.md §5, trap (c)).
template <int R>
__device__ __forceinline__ void fetch_actions(const RolloutArgs& A, int tile, int t, int wave, int lane,
                                              float (&av)[R][MAX_A_PER_LANE]) {
    constexpr int M = 16 * R;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int n = min(tile * M + epi_row(r, wave, lane), A.N - 1);
        const float* src = A.actions + ((size_t)t * A.N + n) * A.a;
#pragma unroll
        for (int k = 0; k < MAX_A_PER_LANE; ++k) av[r][k] = src[min((lane & 15) + 16 * k, A.a - 1)];
    }
}

// Per-lane copies of the step-invariant epilogue operands (this lane's feature slots d = (l&15) +
// 16k), loaded once so the per-step epilogue issues no LDS parameter reads.
template <int SS>
struct EpiParams {
    float om[SS], os[SS], goal[SS], cw[SS], bo[SS];   // state slots
    float am[MAX_A_PER_LANE], as[MAX_A_PER_LANE];    // action slots
};

template <int SS>
__device__ __forceinline__ void load_epi_params(const RolloutArgs& A, const LdsMap& L, int lane, EpiParams<SS>& P) {
    const float* bout = L.hbias + A.L * A.Wpad;
#pragma unroll
    for (int k = 0; k < SS; ++k) {
        const int d = min((lane & 15) + 16 * k, A.s - 1);
        P.om[k] = L.obs_mean[d]; P.os[k] = L.obs_std[d]; P.goal[k] = L.goal[d]; P.cw[k] = L.cw[d]; P.bo[k] = bout[d];
    }
#pragma unroll
    for (int k = 0; k < MAX_A_PER_LANE; ++k) {
        const int d = min((lane & 15) + 16 * k, A.a - 1);
        P.am[k] = L.act_mean[d]; P.as[k] = L.act_std[d];
    }
}

// a_t -> normalised MLP input columns [s, s+a); returns this lane's share of sum_d (cosh(a_d/alpha)-1).
template <int R, int SS, bool REG = (SS <= MBRL_EPI_REG_SLOTS)>
__device__ __forceinline__ void stage_actions(const RolloutArgs& A, const EpiParams<SS>& P, const LdsMap& L, float* act,
                                              int wave, int lane, const float (&av)[R][MAX_A_PER_LANE],
                                              float (&acp)[R], int lda) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int m = epi_row(r, wave, lane);
        float c = 0.f;
#pragma unroll
        for (int k = 0; k < MAX_A_PER_LANE; ++k) {
            const int d = (lane & 15) + 16 * k;
            if (d < A.a) {
                const float x = av[r][k];
                // wide states keep no per-lane copies (see MBRL_EPI_REG_SLOTS): same values from LDS
                const float am = REG ? P.am[k] : L.act_mean[d];
                const float as = REG ? P.as[k] : L.act_std[d];
                const float xn = A.norm_a ? (x - am) / as : x;
                act[m * lda + A.s + d] = xn;
                if (A.reward) L.aterm[m * A.a + d] = xn;   // the state pass re-reads a_t
                if (A.has_ac) c += coshf(x / A.alpha_a) - 1.0f;
            }
        }
        acp[r] = c;
    }
}

// ---- column-split pairs (rollout_kernel PAIR) --------------------------------------------------
// Two workgroups share one 16-candidate tile. Half h computes the columns of virtual waves 4h..4h+3
// of the 8-wave layout (its 4 compute waves), so every accumulator runs the 8-wave kernel's chains in
// the canonical K order, and the output layer's four partials of half h are exactly halves 4h..4h+3
// of the canonical sum: ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)) = S_0 + S_1. With two
// layer-0 chunks both halves compute all of layer 0 (the partner's columns with the partner's exact
// MFMA sequence), so a step has L - 1 hand-offs. The other 4
// waves move the halves (MI355X_MICROARCH.md sc1 hand-off table, first row): after each layer barrier
// every hand-off wave stores its compute wave's columns write-through (16-byte sc1 buffer stores),
// drains them, and the last of the four (an LDS arrival counter) sets the workgroup's flag; one wave
// polls the partner's flag (sc1 loads), the others wait on an LDS word it sets, and all four load the
// partner's columns with sc1 loads into LDS, then count themselves into an LDS word the compute waves
// wait on before their first read of partner columns. Half 0 owns the first K half of every layer,
// so it starts on its own columns while the partner's arrive; half 1 trails it by one hand-off.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;
constexpr int PAIR_SC1 = 16;   // buffer-op aux bit: sc1 (write-through stores, L1-bypassing loads)

// Bounded poll of a partner's flag (relaxed agent-scope loads = sc1): false after ~200 ms, with the
// status word raised to this launch's epoch, so a broken hand-off ends the launch instead of hanging
// the GPU (and the gated redo launch behind it recomputes the candidates).
__device__ __forceinline__ void pair_fail(gu32* status, unsigned epoch) {
    __hip_atomic_fetch_max(status, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool pair_poll(gu32* flag, unsigned want, gu32* status, unsigned epoch) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
            pair_fail(status, epoch);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

typedef __attribute__((address_space(3))) uint32_t lu32;   // LDS words: ds_read / ds_write, not flat

__device__ __forceinline__ void lds_wait_ge(const uint32_t* w, uint32_t need) {
    while (*(const volatile lu32*)(w) < need) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// This hand-off wave's stores are drained; count it in (LDS word arr, the ns-th signal of the launch)
// and let the last of the four set the workgroup's flag to `value` (l2: both halves on one XCD, an
// L2-resident store; else sc1).
__device__ __forceinline__ void pair_signal(uint32_t* arr, gu32* flag, unsigned value, unsigned ns, int lane, bool l2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned old = 0;
    if (lane == 0) old = atomicAdd(arr, 1u);
    old = (unsigned)__shfl((int)old, 0, 64);
    if (old == 4 * ns + 3 && lane == 0) {
        if (l2)
            __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
            __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Buffer stores of the hand-off payload: sc0 (the line stays in the XCD's L2) when both halves share
// that L2, else sc1 (written through). The cache-policy operand must be an immediate.
__device__ __forceinline__ void pair_store_b128(u32x4 v, __amdgpu_buffer_rsrc_t r, unsigned off, bool l2) {
    if (l2) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 1);
    else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
// A tagged 8-byte granule {value, tag}: one store, read untorn (MI355X_MICROARCH.md, granules), so a
// reader that sees the tag holds the value and needs no flag.
__device__ __forceinline__ void pair_store_b64(u32x2 v, __amdgpu_buffer_rsrc_t r, unsigned off, bool l2) {
    if (l2) __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 1);
    else __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 16);
}

// Wait until the partner's flag reads base + q + 1: hand-off wave 0 polls it and publishes the match
// in LDS (word go: q + 1); the other three wait on that word.
__device__ __forceinline__ void pair_await(gu32* pflag, uint32_t* go, unsigned base, unsigned q, int hw, int lane,
                                           gu32* status, unsigned epoch) {
    if (hw == 0) {
        pair_poll(pflag, base + q + 1, status, epoch);
        if (lane == 0) *(volatile lu32*)(go) = q + 1;
    } else {
        lds_wait_ge(go, q + 1);
    }
}

// K0C / NOT > 0: compile-time layer-0 / output chunk counts, enabling a 4-deep weight ring with
// static register slots (three chunks = ~3000 MFMA cycles of load cover). K0C == 0: runtime counts,
// 2-deep ring (any shape).
// NW = 4 or 8 waves per workgroup; each wave owns TW = 4T/NW 16-column tiles of every layer. With
// NW = 8 two waves share a SIMD: while one issues its weight loads the other keeps the matrix pipe
// busy (a wave's own VMEM issue otherwise stalls its MFMA stream ~10 %: tools/ubench). The epilogue
// (per-candidate VALU work) runs on waves 0-3.
template <int T, int R, int K0C_T, int NOT_T, int NW, bool PAIR = false>
__global__ void __launch_bounds__(64 * NW, 1) rollout_kernel(const RolloutArgs A) {
    constexpr int M = 16 * R;
    constexpr int TW = 4 * T / NW;
    constexpr int NHO = (NW == 4 && TW >= 2) ? 2 : 1;   // output halves per wave (mma_out)
    constexpr int NT = 64 * NW;
    static_assert(TW >= 1 && TW * NW == 4 * T, "tiles per wave");
    constexpr bool RING = K0C_T > 0;
    constexpr int NB = RING ? 4 : 2;        // weight ring slots: 3 chunks ahead (2 slots: 0.5-1.2 % slower, r03)
    constexpr int SS = RING ? NOT_T : 1;    // register state slots per lane (ceil(s / 16) <= NOT); generic: LDS
    // per-lane epilogue parameter copies in registers (else the same values from LDS): not at 32
    // candidates x 8 waves, whose MFMA loop already takes the whole 256-VGPR budget
    constexpr bool EREG = SS <= MBRL_EPI_REG_SLOTS && !(R == 2 && NW == 8);
    static_assert(!RING || ((K0C_T + NOT_T) % NB == 0 && K0C_T % 2 == 0 && NOT_T % 2 == 0), "ring layout");
    static_assert(!PAIR || (NW == 8 && R == 1 && RING && T % 2 == 0), "column-split pairs: 8 waves, 16 rows");
    constexpr bool L0DUP = PAIR && K0C_T == 2;   // PAIR: layer 0 computed by both halves (below)
    // LDS row strides: compile-time for the ring instances (make_geometry: lda = max(Wpad, 16 K0C) + 4,
    // pw = 16 NOT + 4; the launcher checks them), so every LDS address of a row block, partial or
    // slot is one base register plus an immediate offset. With runtime strides hipcc hoisted one
    // address register per (row, slot, partial) out of the step loop and spilled them on the
    // 32-candidate kernel (76 B/lane of scratch, ~18 MB of scratch write-back per walker launch).
    constexpr int LDAC = (64 * T > 16 * K0C_T ? 64 * T : 16 * K0C_T) + 4;
    constexpr int PWC = 16 * NOT_T + 4;
    const int lda = RING ? LDAC : A.lda;
    const int pw = RING ? PWC : A.pw;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const LdsMap L = lds_map(A, smem, M);
    uint32_t* const lflag = L.lflag;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int ntiles = (A.N + M - 1) / M;
    int tile, e;
    int half = 0;          // PAIR: which column half of the tile this workgroup computes
    if constexpr (PAIR) {
        // pairs (u, u + 8) of each 16-id group: the same XCD under round-robin dispatch
        const int u = blockIdx.x;
        tile = (u >> 4) * 8 + (u & 7);
        half = (u >> 3) & 1;
        e = blockIdx.y;
        if (tile >= ntiles) return;   // both halves of a padding pair leave together
        if (A.debug_abort) {          // test hook: behave as a timed-out hand-off (the redo launch runs)
            if (tid == 0) pair_fail((gu32*)(A.pair_flags) + (size_t)2 * ntiles * A.E * 32, A.pair_epoch);
            return;
        }
    } else {
        // the redo behind a column-split pair launch: runs only if one of its hand-offs timed out
        if (A.gate != nullptr && *A.gate < A.gate_epoch) return;
        xcd_unit(A.xcd_map, ntiles, tile, e);
    }
    const int cw = PAIR ? 4 * half + wave : wave;   // the 8-wave layout's wave whose columns this one computes
    // half-rotated K order of the W->W layers (cem.hip rot_chunk): a wave whose columns lie in the
    // second half reads K chunk (kc + 2T) mod 4T at position kc; rof = that offset in floats
    const int rof = 2 * cw >= NW ? 16 * 2 * T : 0;
    if (A.redo) {
        // F16X3 redo pass (rollout_f16x3.hip): run only where the split kernel left MBRL_REDO_MARK
        bool any = false;
        for (int m = 0; m < M; ++m) {
            const int n = tile * M + m;
            if (n < A.N && __float_as_uint(A.costs[(size_t)e * A.N + n]) == MBRL_REDO_MARK) any = true;
        }
        if (!any) return;
    }
    const float* member = A.packed + (size_t)e * A.member_stride;
    float* const actX = L.act;   // step input (layer 0) and every even layer's input
    float* const actY = L.act2;

    const bool epi = wave < 4;   // epilogue waves
    // 8 waves, goal-state cost: waves 4-7 own the actions (fetch, normalise, CoshLoss) for the rows
    // of wave w-4, in parallel with waves 0-3's state epilogue; the per-row action cost crosses
    // through LDS (acs[t & 1][m]), so the return still accumulates sc_t + ac_t in t order.
    const bool split = NW == 8 && !A.reward;
    const bool actw = split ? (wave >= 4 && wave < 8) : epi;    // waves holding the action registers
    const int awave = split ? wave - 4 : wave;     // their row mapping (epi_row of wave w - 4)
    float* acs = L.aterm;                          // [2][M] per-row action cost (split mode)
    // ---- prologue: parameters into LDS, s0 and a_0 into the MLP input
    float av[R][MAX_A_PER_LANE];
    float acp[R];  // this lane's share of the current step's CoshLoss sum, per row
    if (actw) fetch_actions<R>(A, tile, 0, awave, lane, av);
    for (int i = tid; i < A.s; i += NT) {
        L.obs_mean[i] = A.obs_mean ? A.obs_mean[i] : 0.f;
        L.obs_std[i] = A.obs_std ? A.obs_std[i] : 1.f;
        L.goal[i] = A.goal ? A.goal[i] : 0.f;
        L.cw[i] = A.cw ? A.cw[i] : 0.f;
    }
    for (int i = tid; i < A.a; i += NT) {
        L.act_mean[i] = A.act_mean ? A.act_mean[i] : 0.f;
        L.act_std[i] = A.act_std ? A.act_std[i] : 1.f;
    }
    const float* bias_src = member + A.stream_floats;
    for (int i = tid; i < A.L * A.Wpad + 16 * A.NOT; i += NT) L.hbias[i] = bias_src[i];
    __syncthreads();
    for (int i = tid; i < M * A.s; i += NT) {
        const int m = i / A.s, d = i - (i / A.s) * A.s;
        const int n = min(tile * M + m, A.N - 1);
        const float sv = A.s0_per_cand ? A.s0[(size_t)n * A.s + d] : A.s0[d];
        actX[m * lda + d] = A.norm_s ? (sv - L.obs_mean[d]) / L.obs_std[d] : sv;
    }
    for (int i = tid; i < M * A.k0pad_extra; i += NT) {
        const int m = i / A.k0pad_extra, j = i - (i / A.k0pad_extra) * A.k0pad_extra;
        actX[m * lda + A.s + A.a + j] = 0.f;
    }
    EpiParams<SS> P;
    load_epi_params<SS>(A, L, lane, P);
    if (actw) {
        stage_actions<R, SS, EREG>(A, P, L, actX, awave, lane, av, acp, lda);
        if (split)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const float v = rowsum16(acp[r]);      // all 16 lanes of the row take part in the DPP sum
                if ((lane & 15) == 0) acs[epi_row(r, awave, lane)] = v;
            }
    }
    // reward-head models: two MLP passes per step (state pass on (s_t, a_t), reward pass on
    // (s_{t+1}, a_t)); the normalised s_{t+1} and a_t are kept in LDS across the passes
    const int npass = A.reward ? 2 : 1;
    const float rmean = (A.reward && A.unnorm_r) ? A.rew_mean[0] : 0.f;
    const float rstd = (A.reward && A.unnorm_r) ? A.rew_std[0] : 1.f;
    if (tid < NW) lflag[tid] = 0;
    __syncthreads();

    // PAIR: lflag[0] counts the hand-off waves' finished partner copies (the compute waves wait on it),
    // lflag[1] their drained publishes, lflag[2] the partner flag value seen by hand-off wave 0.
    // Both halves run their own K half first (the half-rotated K order, cem.hip rot_chunk): the
    // partner's columns are K positions [2T, 4T) of every hidden layer for either half.
    [[maybe_unused]] const int pwait = PAIR ? 2 * T : -1;   // first K position of the partner's columns
    [[maybe_unused]] uint32_t xneed = 0;                                   // hand-offs consumed so far
    if constexpr (PAIR) {
        if (wave >= 4) {
            // ---- hand-off waves: per step the same barriers as the compute waves, and after each one
            // the hand-off of what the compute waves stored before it
            const int hw = wave - 4;
            const int sid = (e * ntiles + tile) * 2 + half;
            // pair_data (pair_layout): every workgroup's granules (2 parities x 16 pw), then every
            // workgroup's layer columns (2 parities x 16 x Wpad / 2 floats)
            const size_t nwg = (size_t)2 * ntiles * A.E;
            const size_t gper = (size_t)2 * 16 * pw;             // granules per workgroup
            const size_t lper = (size_t)16 * A.Wpad;               // layer floats per workgroup
            const size_t gbytes = nwg * gper * 8;
            gu32* const flags = (gu32*)(A.pair_flags);
            gu32* const status = flags + nwg * 32;
            gu32* const myflag = flags + (size_t)sid * 32;
            gu32* const pflag = flags + (size_t)(sid ^ 1) * 32;
            const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
                A.pair_data, 0, (int)(gbytes + nwg * lper * sizeof(float)), 0x00020000);
            const unsigned mine = (unsigned)(gbytes + (size_t)sid * lper * sizeof(float));
            const unsigned theirs = (unsigned)(gbytes + (size_t)(sid ^ 1) * lper * sizeof(float));
            const unsigned gmine = (unsigned)((size_t)sid * gper * 8);
            const unsigned gtheirs = (unsigned)((size_t)(sid ^ 1) * gper * 8);
            const int ocw = 4 * (half ^ 1) + hw;   // the partner's compute wave paired with this one
            unsigned q = 0;    // hand-offs so far (layer columns and output half sums)
            unsigned ns = 0;   // flag signals so far (layer columns only)
            // roll call (A.pair_l2): each half writes its XCD (16 epoch + XCC_ID + 1) to word 1 of its flag
            // line and reads the partner's; on one XCD the halves share an L2, and every hand-off then
            // travels as L2-resident (sc0) stores read by sc1 loads, else as written-through sc1 stores.
            // Hand-off wave 0 decides for the workgroup (LDS word lflag[3]: 2 = one XCD, 1 = not).
            const unsigned epoch = A.pair_epoch, fbase = A.pair_base;
            bool l2 = false;
            if (A.pair_l2 && !MBRL_PAIR_DIAG) {
                if (hw == 0) {
                    unsigned xcc;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
                    const unsigned me = 16u * epoch + xcc + 1;
                    if (lane == 0) __hip_atomic_store(myflag + 1, me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    unsigned px = 0;
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    while ((px = __hip_atomic_load(pflag + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < 16u * epoch) {
                        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
                            pair_fail(status, epoch);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                    if (lane == 0) *(volatile lu32*)(lflag + 3) = px == me ? 2u : 1u;
                }
                lds_wait_ge(lflag + 3, 1);
                l2 = *(volatile lu32*)(lflag + 3) == 2u;
            }
            // layer columns: publish this half's cw = 4 half + hw slice of buffer `buf`, copy the partner's in
            auto layer = [&](float* buf) {
                const unsigned slot = (unsigned)((((q & 1) * 4 + hw) * TW * 64 + lane) * 16);
                const int row = (lane & 15) * lda + 4 * (lane >> 4);
                f32x4 v[TW];
#pragma unroll
                for (int j = 0; j < TW; ++j) v[j] = *reinterpret_cast<const f32x4*>(buf + row + (4 * half + hw) * 16 * TW + 16 * j);
                if constexpr (!MBRL_PAIR_DIAG) {
#pragma unroll
                    for (int j = 0; j < TW; ++j) pair_store_b128(__builtin_bit_cast(u32x4, v[j]), xr, mine + slot + j * 1024, l2);
                    pair_signal(lflag + 1, myflag, fbase + q + 1, ns++, lane, l2);
                    pair_await(pflag, lflag + 2, fbase, q, hw, lane, status, epoch);
#pragma unroll
                    for (int j = 0; j < TW; ++j)
                        v[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, theirs + slot + j * 1024, 0, PAIR_SC1));
                }
#pragma unroll
                for (int j = 0; j < TW; ++j) *reinterpret_cast<f32x4*>(buf + row + ocw * 16 * TW + 16 * j) = v[j];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane == 0) atomicAdd(lflag, 1u);
                ++q;
            };
            // output layer: this half's sum of its four partials, then S_0 + S_1 into partial slot 0. The
            // half sums cross as tagged granules (tag = the flag value this hand-off would carry, unique
            // within the plan; the granules are zeroed with the flags): each lane stores its own and
            // polls the partner's at the same index -- one fabric round trip where a flag costs a drain,
            // the flag store, its poll and then the payload load (MI355X_MICROARCH.md handoff-1to1 vs
            // handoff-flag).
            auto partials = [&]() {
                const int ws = M * pw, nel = M * A.s;
                const unsigned gslot = (unsigned)((q & 1) * 16 * pw * 8);
                const unsigned tag = fbase + q + 1;
                float so[NOT_T], sp[NOT_T];
                unsigned need = 0;
#pragma unroll
                for (int i = 0; i < NOT_T; ++i) {
                    const int idx = 256 * i + 64 * hw + lane;
                    so[i] = 0.f;
                    sp[i] = 0.f;
                    if (idx < nel) {
                        const int m = idx / A.s, ro = m * pw + (idx - m * A.s);
                        so[i] = (L.part[ro] + L.part[ws + ro]) + (L.part[2 * ws + ro] + L.part[3 * ws + ro]);
                        if constexpr (!MBRL_PAIR_DIAG)
                            pair_store_b64(u32x2{__float_as_uint(so[i]), tag}, xr, gmine + gslot + idx * 8, l2);
                        need |= 1u << i;
                    }
                }
                if constexpr (!MBRL_PAIR_DIAG) {
                    unsigned got = 0;
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    while (true) {
                        u32x2 v[NOT_T];
#pragma unroll
                        for (int i = 0; i < NOT_T; ++i) {   // every load in flight before the first compare
                            const int idx = min(256 * i + 64 * hw + lane, nel - 1);
                            v[i] = __builtin_amdgcn_raw_buffer_load_b64(xr, gtheirs + gslot + idx * 8, 0, PAIR_SC1);
                        }
#pragma unroll
                        for (int i = 0; i < NOT_T; ++i)
                            if ((need >> i) & 1u && !((got >> i) & 1u) && v[i].y == tag) {
                                sp[i] = __uint_as_float(v[i].x);
                                got |= 1u << i;
                            }
                        if (got == need) break;
                        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
                            pair_fail(status, epoch);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
#pragma unroll
                for (int i = 0; i < NOT_T; ++i) {
                    const int idx = 256 * i + 64 * hw + lane;
                    if (idx < nel) {
                        const int m = idx / A.s, ro = m * pw + (idx - m * A.s);
                        L.part[ro] = so[i] + sp[i];    // S_0 + S_1 (exactly commutative)
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane == 0) atomicAdd(lflag, 1u);
                ++q;
            };
            for (int t = 0; t < A.H; ++t) {
                if (t + 1 < A.H) fetch_actions<R>(A, tile, t + 1, awave, lane, av);
                if (A.L > 1) {
                    __syncthreads();     // layer 0 stored (actY)
                    if constexpr (!L0DUP) layer(actY);   // L0DUP: both halves computed all of layer 0
                }
                for (int l = 1; l + 1 < A.L; ++l) {
                    __syncthreads();     // hidden layer l stored (odd l: actX)
                    layer((l & 1) ? actX : actY);
                }
                __syncthreads();         // output partials stored
                partials();
                if (t + 1 < A.H) {
                    stage_actions<R, SS, EREG>(A, P, L, actX, awave, lane, av, acp, lda);
                    const float v = rowsum16(acp[0]);
                    if ((lane & 15) == 0) acs[((t + 1) & 1) * M + epi_row(0, awave, lane)] = v;
                }
                __syncthreads();         // epilogue done
            }
            return;
        }
    }

    // ---- weight stream: this wave's slice of chunk g is at wb + g * cs (f32x4 units)
    const f32x4* wb = reinterpret_cast<const f32x4*>(member) + cw * TW * 64 + lane;
    const int cs = 4 * T * 64;
    const int C = A.chunks_per_step;
    (void)wb;
    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(member), 0, (int)(A.stream_floats * sizeof(float)), 0x00020000);
    const unsigned lane_off = (unsigned)((cw * TW * 64 + lane) * 16);
#ifdef MBRL_DIAG_SAMECHUNK  // timing ablation only: every load re-reads chunk 0 (L1 hits; results garbage)
    (void)C;
#define MBRL_LOAD_CHUNK(DST, G) load_chunk_buf<TW>(DST, wrsrc, lane_off + 0u * (unsigned)(G))
#else
#define MBRL_LOAD_CHUNK(DST, G) \
    load_chunk_buf<TW>(DST, wrsrc, lane_off + (unsigned)(((G) < C ? (G) : (G) - C) * cs * 16))
#endif

    f32x4 ring[NB][TW];
    f32x4 aAB[2][R];  // A fragments of chunks with even / odd index within the layer
    f32x4 acc[R][TW];
    f32x4 bias[TW];
#pragma unroll
    for (int q = 0; q < NB - 1; ++q) MBRL_LOAD_CHUNK(ring[q], q);
    // PAIR with two layer-0 chunks: this wave also computes the partner half's layer-0 columns (the
    // partner wave's exact MFMA sequence, weights held in registers for the launch), so hidden
    // layer 1 starts without a hand-off
    [[maybe_unused]] const int ocw0 = PAIR ? 4 * (half ^ 1) + wave : 0;
    [[maybe_unused]] f32x4 w0p[L0DUP ? K0C_T : 1][TW];
    if constexpr (L0DUP) {
        const unsigned poff = (unsigned)((ocw0 * TW * 64 + lane) * 16);
#pragma unroll
        for (int kc = 0; kc < K0C_T; ++kc) load_chunk_buf<TW>(w0p[kc], wrsrc, poff + (unsigned)(kc * cs * 16));
    }
    int pwl = -1;   // PAIR: first partner K chunk of the current hidden layer (-1: no hand-off to wait for)
    float total[R];  // return of row epi_row(r, wave, lane), held by the 16 lanes of that row
#pragma unroll
    for (int r = 0; r < R; ++r) total[r] = 0.f;
#ifdef MBRL_STAMPS
    unsigned long long seg[NSEG] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tprev = __builtin_amdgcn_s_memtime();
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz: seg[7] -> clock
#endif

// One chunk of a hidden-type layer: refill the slot chunk (c-1) vacated with chunk c+NB-1, read the
// next A fragment, then the MFMAs of chunk c. SLOT must fold to a constant (unrolled loops).
#define MBRL_HIDDEN_CHUNK(SLOT, KC, NK, IN)                                          \
    do {                                                                             \
        MBRL_LOAD_CHUNK(ring[((SLOT) + NB - 1) % NB], g + NB - 1);                   \
        if (PAIR && (KC) + 1 == pwl) lds_wait_ge(lflag, 4 * ++xneed);               \
        if ((KC) + 1 < (NK)) read_a<R>(aAB[((KC) + 1) & 1], IN, lda, (KC) + 1, lane); \
        mma_hidden<TW, R>(acc, aAB[(KC) & 1], ring[SLOT]);                           \
        MBRL_PIN();                                                                  \
        ++g;                                                                         \
    } while (0)

    for (int tp = 0; tp < A.H * npass; ++tp) {
        const int t = A.reward ? (tp >> 1) : tp;
        const int pass = A.reward ? (tp & 1) : 0;
        int g = 0;
        // a_{t+1} from HBM now; consumed in this step's (last) epilogue
        if (actw && pass == 0 && t + 1 < A.H) fetch_actions<R>(A, tile, t + 1, awave, lane, av);
        // ---- layer 0: actX [s | a | 0-pad] -> actY (W)
        zero_acc<TW, R>(acc);
        load_bias<TW>(bias, L.hbias, cw, lane);
        read_a<R>(aAB[0], actX, lda, 0, lane);
        if constexpr (RING) {
            // a chunk whose 16 inputs are all zero padding (k >= s + a) is skipped: the accumulator starts
            // at +0 and a round-to-nearest sum never turns +0 into -0, so adding exact zero products
            // leaves it unchanged and the bits match (rollout_m8_kernel's K0L does it per MFMA).
#pragma unroll
            for (int kc = 0; kc < K0C_T; ++kc) {
                MBRL_LOAD_CHUNK(ring[((kc % NB) + NB - 1) % NB], g + NB - 1);
                if (kc + 1 < K0C_T) read_a<R>(aAB[(kc + 1) & 1], actX, lda, kc + 1, lane);
                if (16 * kc < A.s + A.a) mma_hidden<TW, R>(acc, aAB[kc & 1], ring[kc % NB]);
                MBRL_PIN();
                ++g;
            }
        } else {
            for (int kc = 0; kc < A.K0C; kc += 2) {
                MBRL_HIDDEN_CHUNK(0, 0, 2, actX + 16 * kc);
                MBRL_HIDDEN_CHUNK(1, 1, 2, actX + 16 * kc);
                if (kc + 2 < A.K0C) read_a<R>(aAB[0], actX, lda, kc + 2, lane);
            }
        }
        STAMP(0);
        // The last hidden layer's activations stay in registers: the output layer splits K by wave,
        // so wave w only needs the columns it produced itself, in exactly the accumulator layout
        // (lane: 4 consecutive units of candidate lane & 15). No LDS store, barrier or re-read.
        if (A.L > 1) {
            if constexpr (L0DUP) {
                hidden_store_nobar<TW, R>(acc, bias, actY, lda, cw, lane);
                zero_acc<TW, R>(acc);
                load_bias<TW>(bias, L.hbias, ocw0, lane);
#pragma unroll
                for (int kc = 0; kc < K0C_T; ++kc)
                    if (16 * kc < A.s + A.a) mma_hidden<TW, R>(acc, aAB[kc & 1], w0p[kc]);
                hidden_store<TW, R>(acc, bias, actY, lda, ocw0, lane);
            } else {
                hidden_store<TW, R>(acc, bias, actY, lda, cw, lane);
            }
        }
        STAMP(1);
        // ---- hidden layers 1..L-1 (W -> W), alternating Y->X->Y...
        float* in = actY;
        float* out = actX;
        for (int l = 1; l < A.L; ++l) {
            zero_acc<TW, R>(acc);
            load_bias<TW>(bias, L.hbias + l * A.Wpad, cw, lane);
            constexpr int KH = 4 * T;  // 4T % NB == 0: every hidden layer starts on the same slot
            constexpr int S0 = RING ? K0C_T % NB : 0;
            pwl = (L0DUP && l == 1) ? -1 : pwait;                   // layer 0's partner columns are local
            // K position kc reads chunk kc + rof/16 (kc < 2T) or kc - rof/16 (kc >= 2T): two bases
            const float* const inLo = in + rof;
            const float* const inHi = in - rof;
            read_a<R>(aAB[0], inLo, lda, 0, lane);
#pragma unroll
            for (int kc = 0; kc < KH; ++kc) MBRL_HIDDEN_CHUNK((S0 + kc) % NB, kc, KH, (kc + 1 < KH / 2 ? inLo : inHi));
            STAMP(2);
            if (l + 1 < A.L) hidden_store<TW, R>(acc, bias, out, lda, cw, lane);
            STAMP(3);
            float* tmp = in; in = out; out = tmp;
        }
        // ---- output layer: W -> s, K split over the 4 waves, partials through LDS
        {
            f32x4 aout[R][TW];
            const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int kc = 0; kc < TW; ++kc) aout[r][kc] = __builtin_elementwise_max(acc[r][kc] + bias[kc], zero4);
            float* part = L.part + wave * M * pw;
#define MBRL_OUT_CHUNK(SLOT, J)                                                   \
    do {                                                                          \
        MBRL_LOAD_CHUNK(ring[((SLOT) + NB - 1) % NB], g + NB - 1);                \
        MBRL_PIN();                                                               \
        mma_out<TW, R, NHO>(aout, ring[SLOT], part, pw, J, lane);               \
        MBRL_PIN();                                                               \
        ++g;                                                                      \
    } while (0)
            if constexpr (RING) {
                constexpr int S0 = K0C_T % NB;
#pragma unroll
                for (int j = 0; j < NOT_T; ++j) MBRL_OUT_CHUNK((S0 + j) % NB, j);
            } else {
                for (int j = 0; j < A.NOT; j += 2) {
                    MBRL_OUT_CHUNK(0, j);
                    MBRL_OUT_CHUNK(1, j + 1);
                }
            }
#undef MBRL_OUT_CHUNK
        }
        STAMP(4);
        __syncthreads();
        STAMP(5);

        // ---- epilogue (one pass, no cross-wave traffic): s_{t+1} = unnormalize(out), goal cost of
        // (s_{t+1}, a_t), next MLP input [norm(s_{t+1}) | norm(a_{t+1}) | 0-pad] into actX
        if (epi && A.reward) {
            // reward-head model. State pass: s_{t+1} -> states_out, next input [norm(s_{t+1}) | norm(a_t)].
            // Reward pass: cost_t = unnormalize_reward(reward head), next input [norm(s_{t+1}) | norm(a_{t+1})].
            const float* bout = L.hbias + A.L * A.Wpad;
            const int ws = M * pw;
            const int j = lane & 15;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int m = epi_row(r, wave, lane);
                const int n = tile * M + m;
                float rc = 0.f;
                for (int d = j; d <= A.s; d += 16) {
                    const int ro = m * pw + d;
                    float o = 0.f;
                    if (pass == 0 || d == A.s) {
                        o = sum_partials<NW>(L.part, ws, ro) + bout[d];
                    }
                    if (d < A.s) {
                        float xn;
                        if (pass == 0) {
                            const float sn = A.unnorm_s ? o * L.obs_std[d] + L.obs_mean[d] : o;
                            if (A.states_out != nullptr && n < A.N)
                                A.states_out[(((size_t)e * A.H + t) * A.N + n) * A.s + d] = sn;
                            xn = A.norm_s ? (sn - L.obs_mean[d]) / L.obs_std[d] : sn;
                            L.sterm[m * A.s + d] = xn;
                        } else {
                            xn = L.sterm[m * A.s + d];
                        }
                        actX[m * lda + d] = xn;
                    } else if (pass == 1) {
                        rc = A.unnorm_r ? o * rstd + rmean : o;
                    }
                }
                for (int d = A.s + A.a + j; d < A.s + A.a + A.k0pad_extra; d += 16) actX[m * lda + d] = 0.f;
                if (pass == 0) {
                    for (int d = j; d < A.a; d += 16) actX[m * lda + A.s + d] = L.aterm[m * A.a + d];
                } else {
                    total[r] += rowsum16(rc);
                }
            }
            if (pass == 1 && t + 1 < A.H) stage_actions<R, SS, EREG>(A, P, L, actX, wave, lane, av, acp, lda);
        } else if (epi) {
            const float* bout = L.hbias + A.L * A.Wpad;
            const int ws = M * pw;
            const int j = lane & 15;
            if constexpr (PAIR) lds_wait_ge(lflag, 4 * ++xneed);   // S_0 + S_1 in partial slot 0
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int m = epi_row(r, wave, lane);
                const int n = tile * M + m;
                float sc = 0.f;
                auto slot = [&](int d, float om, float os, float goal, float cwt, float bo) {
                    const int ro = m * pw + d;
                    float o = PAIR ? L.part[ro] : sum_partials<NW>(L.part, ws, ro);
                    o = o + bo;
                    const float sn = A.unnorm_s ? o * os + om : o;
                    if (A.has_sc) {
                        const float x = (sn - goal) * cwt;
                        sc += sqrtf(x * x + A.alpha_s2) - A.alpha_s;
                    }
                    actX[m * lda + d] = A.norm_s ? (sn - om) / os : sn;
                    if (A.states_out != nullptr && n < A.N && (!PAIR || half == 0))
                        A.states_out[(((size_t)e * A.H + t) * A.N + n) * A.s + d] = sn;
                };
                if constexpr (RING && EREG) {
#pragma unroll
                    for (int k = 0; k < SS; ++k)
                        if (j + 16 * k < A.s) slot(j + 16 * k, P.om[k], P.os[k], P.goal[k], P.cw[k], P.bo[k]);
                } else if constexpr (RING) {
                    // wide states: the 5 SS per-lane copies would spill; same values from LDS, same order
#pragma unroll
                    for (int k = 0; k < SS; ++k) {
                        const int d = j + 16 * k;
                        if (d < A.s) slot(d, L.obs_mean[d], L.obs_std[d], L.goal[d], L.cw[d], bout[d]);
                    }
                } else {
                    for (int d = j; d < A.s; d += 16)
                        slot(d, L.obs_mean[d], L.obs_std[d], L.goal[d], L.cw[d], bout[d]);
                }
                for (int d = A.s + A.a + j; d < A.s + A.a + A.k0pad_extra; d += 16) actX[m * lda + d] = 0.f;
                sc = rowsum16(sc);
                const float ac = split ? acs[(t & 1) * M + m] : rowsum16(acp[r]);
                total[r] += sc + A.alpha_a2 * (ac / (float)A.a);
            }
            if (!split && t + 1 < A.H) stage_actions<R, SS, EREG>(A, P, L, actX, wave, lane, av, acp, lda);
        } else if (split && actw && t + 1 < A.H) {
            // waves 4-7, concurrently: a_{t+1} into the next MLP input, its CoshLoss row sum into LDS
            stage_actions<R, SS, EREG>(A, P, L, actX, awave, lane, av, acp, lda);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const float v = rowsum16(acp[r]);
                if ((lane & 15) == 0) acs[((t + 1) & 1) * M + epi_row(r, awave, lane)] = v;
            }
        }
        __syncthreads();
        STAMP(6);
    }
#undef MBRL_HIDDEN_CHUNK
#undef MBRL_LOAD_CHUNK
#ifdef MBRL_STAMPS
    seg[NSEG - 1] = __builtin_amdgcn_s_memrealtime() - rt0;
    if (lane == 0 && g_mbrl_stamps != nullptr) {
        unsigned long long* dst = g_mbrl_stamps + (((size_t)e * ntiles + tile) * NW + wave) * NSEG;
#pragma unroll
        for (int k = 0; k < NSEG; ++k) dst[k] = seg[k];
    }
#endif
    if (epi && (lane & 15) == 0 && (!PAIR || half == 0)) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int n = tile * M + epi_row(r, wave, lane);
            if (n < A.N) A.costs[(size_t)e * A.N + n] = total[r];
        }
    }
}

// The ring instances compile the LDS row strides in (rollout_kernel LDAC / PWC): the geometry must
// agree (make_geometry computes the same two numbers).
template <int T, int K0C_T, int NOT_T>
static bool ring_strides_ok(const RolloutArgs& A) {
    if constexpr (K0C_T == 0) return true;
    else return A.lda == (64 * T > 16 * K0C_T ? 64 * T : 16 * K0C_T) + 4 && A.pw == 16 * NOT_T + 4;
}

template <int T, int R, int K0C_T, int NOT_T, int NW>
static hipError_t launch_rollout_tr(const RolloutArgs& A_in, hipStream_t stream) {
    RolloutArgs A = A_in;
    A.nw = NW;
    if (!ring_strides_ok<T, K0C_T, NOT_T>(A)) return hipErrorInvalidValue;
    const int M = 16 * R;
    const int ntiles = (A.N + M - 1) / M;
    const dim3 grid = A.xcd_map ? dim3(ntiles * A.E) : dim3(ntiles, A.E);
    const size_t lds = rollout_lds_bytes(A, M);
    hipError_t e = ensure_dynamic_lds(reinterpret_cast<const void*>(&rollout_kernel<T, R, K0C_T, NOT_T, NW>),
                                      160 * 1024);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((rollout_kernel<T, R, K0C_T, NOT_T, NW>), grid, dim3(64 * NW), lds, stream, A);
    return hipGetLastError();
}

template <int T, int R, int NW>
static hipError_t launch_rollout_tn(const RolloutArgs& A, hipStream_t stream) {
    if constexpr (4 * T / NW <= 8) {  // the 4-deep ring needs 4*TW*4 VGPRs
        if (A.K0C == 2 && A.NOT == 2) return launch_rollout_tr<T, R, 2, 2, NW>(A, stream);
        if (A.K0C == 6 && A.NOT == 6) return launch_rollout_tr<T, R, 6, 6, NW>(A, stream);
        if (A.K0C == 2 && A.NOT == 6) return launch_rollout_tr<T, R, 2, 6, NW>(A, stream);
        if (A.K0C == 6 && A.NOT == 2) return launch_rollout_tr<T, R, 6, 2, NW>(A, stream);
    }
    return launch_rollout_tr<T, R, 0, 0, NW>(A, stream);
}

template <int T, int R>
static hipError_t launch_rollout_t(const RolloutArgs& A, hipStream_t stream) {
    // two waves per SIMD (8 waves, T/2 tiles each) where the tile count and LDS allow it: always for
    // R = 1; for R = 2 when the launcher asks (A.nw == 8: the aliased partials fit LDS)
    // (16 waves, T/4 tiles each, measured 8 % slower than 8: the 128-VGPR budget spills)
    if constexpr (R == 2 && T >= 2) {
        if (A.nw == 8) return launch_rollout_tn<T, R, 8>(A, stream);
    }
    constexpr int NW = (T >= 2 && R == 1) ? 8 : 4;
    return launch_rollout_tn<T, R, NW>(A, stream);
}

hipError_t launch_rollout(const RolloutArgs& A, int T, int R, hipStream_t stream) {
#define MBRL_CASE(TT, RR) \
    if (T == TT && R == RR) return launch_rollout_t<TT, RR>(A, stream);
    MBRL_CASE(1, 1) MBRL_CASE(2, 1) MBRL_CASE(4, 1) MBRL_CASE(8, 1) MBRL_CASE(16, 1)
    MBRL_CASE(1, 2) MBRL_CASE(2, 2) MBRL_CASE(4, 2) MBRL_CASE(8, 2)
#undef MBRL_CASE
    return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------------
// Column-split pairs: rollout_kernel<T, 1, K0C, NOT, 8, true>, 2 ceil(N / 16) E
// workgroups, all co-resident (checked; a hand-off never waits on an undispatched workgroup).
bool rollout_pair_supported(const RolloutArgs& A, int T) {
    if (A.reward || A.redo || !A.pair_data || !A.pair_flags || T != 8) return false;
    if (!((A.K0C == 2 || A.K0C == 6) && (A.NOT == 2 || A.NOT == 6))) return false;
    RolloutArgs X = A;
    X.nw = 8;
    X.part_alias = 0;
    return rollout_lds_bytes(X, 16) <= 160 * 1024;
}

template <int T, int K0C_T, int NOT_T>
static hipError_t launch_pair_tr(const RolloutArgs& A_in, hipStream_t stream) {
    RolloutArgs A = A_in;
    A.nw = 8;
    A.part_alias = 0;
    if (!ring_strides_ok<T, K0C_T, NOT_T>(A)) return hipErrorInvalidValue;
    const int ntiles = (A.N + 15) / 16;
    const dim3 grid(16 * ((ntiles + 7) / 8), A.E);
    const size_t lds = rollout_lds_bytes(A, 16);
    const auto fn = &rollout_kernel<T, 1, K0C_T, NOT_T, 8, true>;
    hipError_t e = ensure_dynamic_lds(reinterpret_cast<const void*>(fn), 160 * 1024);
    if (e != hipSuccess) return e;
    if (!grid_fits(reinterpret_cast<const void*>(fn), 512, lds, (int)(grid.x * grid.y)))
        return hipErrorCooperativeLaunchTooLarge;
    // every polled word (flags, status) zero before the first launch of its epochs: the plan's first
    // launch cleared them (cem_init_kernel), else one memset node here (a lone rollout, epoch 1)
    if (!A.pair_prezeroed) {
        e = hipMemsetAsync(A.pair_flags, 0, pair_layout(A.Wpad, A.pw, ntiles, A.E).zero_bytes, stream);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(fn, grid, dim3(512), lds, stream, A);
    return hipGetLastError();
}

hipError_t launch_rollout_pair(const RolloutArgs& A, int T, hipStream_t stream) {
    if (T != 8) return hipErrorInvalidValue;
    if (A.K0C == 2 && A.NOT == 2) return launch_pair_tr<8, 2, 2>(A, stream);
    if (A.K0C == 6 && A.NOT == 6) return launch_pair_tr<8, 6, 6>(A, stream);
    if (A.K0C == 2 && A.NOT == 6) return launch_pair_tr<8, 2, 6>(A, stream);
    if (A.K0C == 6 && A.NOT == 2) return launch_pair_tr<8, 6, 2>(A, stream);
    return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------------
// 8-candidate tiles (DESIGN.md §3 "rollout_m8_kernel"): v_mfma_f32_4x4x1_16b_f32.
//
// A shard of N <= 2048 candidates fills at most 128 workgroups of 16, half the chip. The 4x4x1
// MFMA runs at the same f32 rate as 16x16x4 but needs only 4 columns per block, so a workgroup can
// own 8 candidates with no idle MFMA lanes, and twice as many CUs work. Its 16 blocks (b = l >> 2)
// are 8 row groups x 2 candidate groups: A broadcast within block pairs (CBSZ = 1) lets ONE weight
// register carry two 32-row tiles, even blocks tile 0 (ABID 0), odd blocks tile 1 (ABID 1):
//   A (lane l): W[32 tile + 4 (l >> 3) + (l & 3)][k]     B (lane l): X[k][cand l & 7]
//   D (lane l, v): row 32 tile + 4 (l >> 3) + v of cand l & 7 -> one float4 row store
// (tools/ubench/mfma4x4.hip checks the layout on the GPU). Every accumulator consumes its k in the
// 16-candidate kernel's order (16-deep chunk kc, step s, then q: k = 16 kc + 4 q + s): 16x16x4 is
// an fmaf chain over its 4 k (same microtest), so both kernels give bit-identical sums, and a plan
// does not depend on which tile height its shard size picked. The output layer mirrors the 8-wave
// kernel's K split (one partial per 16 T/2 features, four chains (c0 + c1) + (c2 + c3)) and its
// epilogue, operation for operation.
// Wave w owns hidden features [64 w, 64 w + 64) (two 32-row tiles); T = Wpad / 64 waves. In KP mode
// (below) wave w owns [32 w, 32 w + 32) of 8 waves.
// Weight stream (packed by pack_m8_*_kernel in cem.hip): per 16-deep chunk, per wave, 4 x 64 lanes
// x float4 (load s holds q = 0..3); chunks per step = K0C + (L-1) 4T + NOC (output: 2 K-chunk pairs
// of the one 32-row tile, or own 4 K chunks x 2-tile pairs), plus DUM ring-alignment slots that
// reload the last chunk (L2 hits; none for the BASELINE shapes).
// KP mode (Wpad 256 with one 32-row output tile, e.g. cartpole): 8 waves of ONE 32-row tile each,
// so two waves share every SIMD, and a weight register carries two consecutive k of that tile
// (even blocks position 2i, odd blocks 2i + 1 of the chunk's order; ABID 0 / 1). Otherwise wave w
// owns two tiles (ABID 0 / 1) and T = Wpad / 64 waves run (one per SIMD at Wpad 256).
constexpr bool m8_kp(int T, int NOT) { return T == 4 && NOT == 2; }
constexpr int m8_waves(int T, int NOT) { return m8_kp(T, NOT) ? 8 : T; }

// K0L > 0 (compile time): every real input index k = s + a is below K0L, so layer-0 MFMAs whose k is
// >= K0L (zero padding: weight and activation both +0) are not issued -- bit-identical, since the
// accumulator starts at +0 and a round-to-nearest sum never turns +0 into -0. Instantiated for
// cartpole's KP shape (6 inputs: 8 of 32 dependent layer-0 MFMAs per wave remain).
template <int T, int K0C_T, int NOT_T, int K0L = 0>
__global__ void __launch_bounds__(64 * m8_waves(T, NOT_T), 1) rollout_m8_kernel(const RolloutArgs A) {
    constexpr int M = 8;
    // compile-time LDS row strides (rollout_kernel LDAC / PWC; the launcher checks the geometry)
    const int lda = (64 * T > 16 * K0C_T ? 64 * T : 16 * K0C_T) + 4;
    const int pw = 16 * NOT_T + 4;
    constexpr bool KP = m8_kp(T, NOT_T);
    constexpr int NW = m8_waves(T, NOT_T);
    constexpr int TPW = KP ? 1 : 2;          // 32-row tiles per wave
    constexpr int FPW = 32 * TPW;            // hidden features per wave
    constexpr int RSL = KP ? 2 : 4;          // float4 loads per lane per ring slot
    constexpr int NT = 64 * NW;
    constexpr int KH = 4 * T;
    constexpr int NOT8 = NOT_T / 2;          // 32-row output tiles
    constexpr int NOP = (NOT8 + 1) / 2;      // pairs of them (one weight register each)
    // output chunks: one 32-row tile (s <= 32) pairs two own K chunks in one register (even blocks
    // chunk 2o, odd blocks 2o + 1: no idle half); wider outputs pair two tiles per K chunk
    constexpr bool KPAIR = NOT8 == 1;
    constexpr int NOC = KPAIR ? 2 : 4 * NOP;
    constexpr int NB = 4;                    // ring slots (16 VGPRs each), 3 chunks ahead: 1 % faster than 8
                                             // (walker 2048-candidate shard, tools/ab.sh, r01)
    constexpr int DUM = (NB - (K0C_T + NOC) % NB) % NB;
    constexpr int TW16 = T / 2;              // the 16-candidate kernel's K chunks per output partial
    constexpr int NPW = (FPW / 16) / TW16;   // its partials inside this wave's own chunks
    constexpr int SS = NOT_T;
    static_assert(KH % NB == 0 && (T == 4 || T == 8), "m8 geometry");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const LdsMap L = lds_map(A, smem, M);
    uint32_t* const lflag = L.lflag;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int ntiles = (A.N + M - 1) / M;
    int tile, e;
    if (A.gate != nullptr && *A.gate < A.gate_epoch) return;   // redo behind a pair launch (rollout_kernel)
    xcd_unit(A.xcd_map, ntiles, tile, e);
    const float* member = A.packed + (size_t)e * A.member_stride;
    float* const actX = L.act;
    float* const actY = L.act2;
    // epilogue roles as the 8-wave kernel's split mode: waves 0-1 the state rows (4 each), waves 2-3
    // the actions of the same rows
    const bool epi = wave < 2;
    const bool actw = wave >= 2 && wave < 4;
    const int awave = wave - 2;
    float* acs = L.aterm;
    const int cand = lane & 7;
    // the half-rotated K order of the W->W layers (rollout_kernel): waves whose features lie in the
    // second half start at chunk KH / 2
    const int rofc = 2 * FPW * wave >= 64 * T ? KH / 2 : 0;
    float av[1][MAX_A_PER_LANE];
    float acp[1];
    auto fetch_a = [&](int t) {
        const int n = min(tile * M + epi_row(0, awave, lane), A.N - 1);
        const float* src = A.actions + ((size_t)t * A.N + n) * A.a;
#pragma unroll
        for (int k = 0; k < MAX_A_PER_LANE; ++k) av[0][k] = src[min((lane & 15) + 16 * k, A.a - 1)];
    };
    if (actw) fetch_a(0);
    for (int i = tid; i < A.s; i += NT) {
        L.obs_mean[i] = A.obs_mean ? A.obs_mean[i] : 0.f;
        L.obs_std[i] = A.obs_std ? A.obs_std[i] : 1.f;
        L.goal[i] = A.goal ? A.goal[i] : 0.f;
        L.cw[i] = A.cw ? A.cw[i] : 0.f;
    }
    for (int i = tid; i < A.a; i += NT) {
        L.act_mean[i] = A.act_mean ? A.act_mean[i] : 0.f;
        L.act_std[i] = A.act_std ? A.act_std[i] : 1.f;
    }
    const float* bias_src = member + A.stream_floats;
    for (int i = tid; i < A.L * A.Wpad + 16 * A.NOT; i += NT) L.hbias[i] = bias_src[i];
    __syncthreads();
    for (int i = tid; i < M * A.s; i += NT) {
        const int m = i / A.s, d = i - (i / A.s) * A.s;
        const int n = min(tile * M + m, A.N - 1);
        const float sv = A.s0_per_cand ? A.s0[(size_t)n * A.s + d] : A.s0[d];
        actX[m * lda + d] = A.norm_s ? (sv - L.obs_mean[d]) / L.obs_std[d] : sv;
    }
    for (int i = tid; i < M * A.k0pad_extra; i += NT) {
        const int m = i / A.k0pad_extra, j = i - (i / A.k0pad_extra) * A.k0pad_extra;
        actX[m * lda + A.s + A.a + j] = 0.f;
    }
    EpiParams<SS> P;
    load_epi_params<SS>(A, L, lane, P);
    if (actw) {
        stage_actions<1, SS>(A, P, L, actX, awave, lane, av, acp, lda);
        const float v = rowsum16(acp[0]);
        if ((lane & 15) == 0) acs[epi_row(0, awave, lane)] = v;
    }
    if (tid < NW) lflag[tid] = 0;
    __syncthreads();

    // ---- weight stream: chunk g of this wave at byte (g T + wave) 4096 + s 1024 + lane 16
    const int C8 = A.C8;
    const int CSQ = C8 + DUM;
    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(member + A.m8_off), 0, (int)((size_t)C8 * 4096 * T), 0x00020000);
    const unsigned lane_off = (unsigned)(wave * RSL * 1024 + lane * 16);
    f32x4 ring[NB][RSL];
#define M8_LOAD(SLOT, G)                                                                          \
    do {                                                                                          \
        int gg_ = (G);                                                                            \
        if (gg_ >= CSQ) gg_ -= CSQ;                                                               \
        gg_ = gg_ < C8 ? gg_ : C8 - 1;                                                            \
        const int so_ = gg_ * (4096 * T);                                                         \
        _Pragma("unroll") for (int s_ = 0; s_ < RSL; ++s_) ring[SLOT][s_] = __builtin_bit_cast(   \
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, lane_off + s_ * 1024, so_, 0));   \
    } while (0)
#pragma unroll
    for (int q = 0; q < NB - 1; ++q) M8_LOAD(q, q);
    f32x4 bb[2][4];     // B: X[cand][16 kc + 4 q' .. +3], double-buffered over chunks
    f32x4 acc[TPW];
    f32x4 bias[TPW];
    float total = 0.f;
#ifdef MBRL_STAMPS
    unsigned long long seg[NSEG] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tprev = __builtin_amdgcn_s_memtime();
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz: seg[7] -> clock
#endif
    auto read_b = [&](f32x4 (&b)[4], const float* in, int col) {
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = *reinterpret_cast<const f32x4*>(in + cand * lda + col + 4 * q);
    };
    auto mma_pair = [&](const f32x4 (&w)[RSL], const f32x4 (&b)[4]) {
        if constexpr (KP) {
            // pair i: chunk positions 2i (ABID 0) and 2i + 1 (ABID 1), position p = 4 s + q
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float a = w[i >> 2][i & 3];
                acc[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b[(2 * i) & 3][(2 * i) >> 2], acc[0], 1, 0, 0);
                acc[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b[(2 * i + 1) & 3][(2 * i + 1) >> 2], acc[0], 1, 1, 0);
            }
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    acc[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[s][q], b[q][s], acc[0], 1, 0, 0);
                    acc[TPW - 1] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[s][q], b[q][s], acc[TPW - 1], 1, 1, 0);
                }
        }
    };
    auto mma_pair_l0 = [&](const f32x4 (&w)[RSL], const f32x4 (&b)[4], auto kcc) {
        constexpr int kc = decltype(kcc)::value;
        if constexpr (KP) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float a = w[i >> 2][i & 3];
                const int p0 = 2 * i, p1 = 2 * i + 1;    // position p = 4 s + q, k = 16 kc + 4 q + s
                if (16 * kc + 4 * (p0 & 3) + (p0 >> 2) < K0L)
                    acc[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b[p0 & 3][p0 >> 2], acc[0], 1, 0, 0);
                if (16 * kc + 4 * (p1 & 3) + (p1 >> 2) < K0L)
                    acc[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b[p1 & 3][p1 >> 2], acc[0], 1, 1, 0);
            }
        } else {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (16 * kc + 4 * q + s < K0L) {
                        acc[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[s][q], b[q][s], acc[0], 1, 0, 0);
                        acc[TPW - 1] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[s][q], b[q][s], acc[TPW - 1], 1, 1, 0);
                    }
        }
    };
    auto store_layer = [&](float* out) {
        const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            f32x4 v = acc[u] + bias[u];
            v = __builtin_elementwise_max(v, zero);
            *reinterpret_cast<f32x4*>(out + cand * lda + FPW * wave + 32 * u + 4 * (lane >> 3)) = v;
        }
    };
    // a stored layer another wave reads: wait for every wave (barrier)
    auto publish_layer = [&]() { __syncthreads(); };
    auto load_bias8 = [&](const float* hb) {
#pragma unroll
        for (int u = 0; u < TPW; ++u)
            bias[u] = *reinterpret_cast<const f32x4*>(hb + FPW * wave + 32 * u + 4 * (lane >> 3));
    };
    auto zero_acc8 = [&]() {
#pragma unroll
        for (int u = 0; u < TPW; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
// one hidden-type chunk: refill the slot chunk c-1 vacated, read the next chunk's B, MFMAs of chunk c
#define M8_CHUNK(SLOT, KC, NK, IN)                                          \
    do {                                                                    \
        M8_LOAD(((SLOT) + NB - 1) % NB, g + NB - 1);                         \
        if ((KC) + 1 < (NK)) read_b(bb[((KC) + 1) & 1], IN, 16 * ((KC) + 1)); \
        mma_pair(ring[SLOT], bb[(KC) & 1]);                                 \
        MBRL_PIN();                                                         \
        ++g;                                                                \
    } while (0)

    for (int t = 0; t < A.H; ++t) {
        int g = 0;
        if (actw && t + 1 < A.H) fetch_a(t + 1);
        // ---- layer 0: actX [s | a | 0-pad] -> actY
        zero_acc8();
        load_bias8(L.hbias);
        read_b(bb[0], actX, 0);
        if constexpr (K0L > 0) {
            static_assert(K0C_T == 2, "K0L instance");
            M8_LOAD((0 + NB - 1) % NB, g + NB - 1);
            read_b(bb[1], actX, 16);
            mma_pair_l0(ring[0], bb[0], std::integral_constant<int, 0>());
            MBRL_PIN();
            ++g;
            M8_LOAD((1 + NB - 1) % NB, g + NB - 1);
            mma_pair_l0(ring[1], bb[1], std::integral_constant<int, 1>());
            MBRL_PIN();
            ++g;
        } else {
#pragma unroll
            for (int kc = 0; kc < K0C_T; ++kc) M8_CHUNK(kc % NB, kc, K0C_T, actX);
        }
        STAMP(0);
        store_layer(actY);
        if (A.L > 1) publish_layer();
        STAMP(1);
        float* in = actY;
        float* out = actX;
        for (int l = 1; l < A.L; ++l) {
            zero_acc8();
            load_bias8(L.hbias + l * A.Wpad);
            // the half-rotated K order (rollout_kernel): position kc reads chunk (kc + rofc) mod KH
            const float* const inLo = in + 16 * rofc;
            const float* const inHi = in - 16 * rofc;
            read_b(bb[0], inLo, 0);
#pragma unroll
            for (int kc = 0; kc < KH; ++kc) M8_CHUNK((K0C_T + kc) % NB, kc, KH, (kc + 1 < KH / 2 ? inLo : inHi));
            STAMP(2);
            store_layer(out);
            if (l + 1 < A.L) publish_layer();   // the last hidden layer is read back by its own wave only
            STAMP(3);
            float* tmp = in; in = out; out = tmp;
        }
        // ---- output layer over this wave's own 64 features (from LDS: its own stores, in order)
        {
            f32x4 ch[NPW][NOT8][4];
#pragma unroll
            for (int j = 0; j < NPW; ++j)
#pragma unroll
                for (int u = 0; u < NOT8; ++u)
#pragma unroll
                    for (int s = 0; s < 4; ++s) ch[j][u][s] = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (KP) {
                // own 32 features = two K chunks, each a chunk of k pairs; chain s takes the pairs
                // whose positions carry step s (both positions of pair i do: s = i >> 1)
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    f32x4 b[4];
                    read_b(b, in, 32 * wave + 16 * o);
                    constexpr int base = K0C_T;
                    M8_LOAD((base + o + NB - 1) % NB, g + NB - 1);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const float a = ring[(base + o) % NB][i >> 2][i & 3];
                        const int sc = i >> 1;
                        ch[0][0][sc] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b[(2 * i) & 3][(2 * i) >> 2], ch[0][0][sc],
                                                                          1, 0, 0);
                        ch[0][0][sc] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b[(2 * i + 1) & 3][(2 * i + 1) >> 2],
                                                                          ch[0][0][sc], 1, 1, 0);
                    }
                    MBRL_PIN();
                    ++g;
                }
            } else if constexpr (KPAIR) {
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    f32x4 b0[4], b1[4];
                    read_b(b0, in, FPW * wave + 32 * o);
                    read_b(b1, in, FPW * wave + 32 * o + 16);
                    constexpr int base = K0C_T;
                    M8_LOAD((base + o + NB - 1) % NB, g + NB - 1);
                    const int j0 = (2 * o) / TW16, j1 = (2 * o + 1) / TW16;
                    // chain s: chunk 2o (q = 0..3, ABID 0), then chunk 2o + 1 (ABID 1) -- the
                    // 16-candidate kernel's kc-then-q order
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            ch[j0][0][s] = __builtin_amdgcn_mfma_f32_4x4x1f32(ring[(base + o) % NB][s][q], b0[q][s],
                                                                              ch[j0][0][s], 1, 0, 0);
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            ch[j1][0][s] = __builtin_amdgcn_mfma_f32_4x4x1f32(ring[(base + o) % NB][s][q], b1[q][s],
                                                                              ch[j1][0][s], 1, 1, 0);
                    }
                    MBRL_PIN();
                    ++g;
                }
            } else {
#pragma unroll
            for (int kc = 0; kc < 4; ++kc) {
                f32x4 b[4];
                read_b(b, in, FPW * wave + 16 * kc);
#pragma unroll
                for (int p = 0; p < NOP; ++p) {
                    constexpr int base = K0C_T;   // slots fold: kc, p are unrolled
                    M8_LOAD(((base + kc * NOP + p) + NB - 1) % NB, g + NB - 1);
                    const int j = kc / TW16;
#pragma unroll
                    for (int s = 0; s < 4; ++s)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float w = ring[(base + kc * NOP + p) % NB][s][q];
                            ch[j][2 * p][s] = __builtin_amdgcn_mfma_f32_4x4x1f32(w, b[q][s], ch[j][2 * p][s], 1, 0, 0);
                            if (2 * p + 1 < NOT8)
                                ch[j][2 * p + 1][s] =
                                    __builtin_amdgcn_mfma_f32_4x4x1f32(w, b[q][s], ch[j][2 * p + 1][s], 1, 1, 0);
                        }
                    MBRL_PIN();
                    ++g;
                }
            }
            }
#pragma unroll
            for (int d = 0; d < DUM; ++d) {
                M8_LOAD((K0C_T + NOC + d + NB - 1) % NB, g + NB - 1);
                ++g;
            }
#pragma unroll
            for (int j = 0; j < NPW; ++j)
#pragma unroll
                for (int u = 0; u < NOT8; ++u) {
                    const f32x4 v = (ch[j][u][0] + ch[j][u][1]) + (ch[j][u][2] + ch[j][u][3]);
                    *reinterpret_cast<f32x4*>(L.part + (wave * NPW + j) * (M * pw) + cand * pw + 32 * u +
                                              4 * (lane >> 3)) = v;
                }
        }
        STAMP(4);
        __syncthreads();
        STAMP(5);
        // ---- epilogue: the 8-wave kernel's split-mode goal-state epilogue for rows 0..7
        if (epi) {
            const int ws = M * pw;
            const int j = lane & 15;
            const int m = epi_row(0, wave, lane);
            const int n = tile * M + m;
            float sc = 0.f;
            auto slot = [&](int d, float om, float os, float goal, float cw, float bo) {
                const int ro = m * pw + d;
                float o = sum_partials<8>(L.part, ws, ro);
                o = o + bo;
                const float sn = A.unnorm_s ? o * os + om : o;
                if (A.has_sc) {
                    const float x = (sn - goal) * cw;
                    sc += sqrtf(x * x + A.alpha_s2) - A.alpha_s;
                }
                actX[m * lda + d] = A.norm_s ? (sn - om) / os : sn;
                if (A.states_out != nullptr && n < A.N)
                    A.states_out[(((size_t)e * A.H + t) * A.N + n) * A.s + d] = sn;
            };
            if constexpr (SS <= MBRL_EPI_REG_SLOTS) {
#pragma unroll
                for (int k = 0; k < SS; ++k)
                    if (j + 16 * k < A.s) slot(j + 16 * k, P.om[k], P.os[k], P.goal[k], P.cw[k], P.bo[k]);
            } else {
                // wide states: the same values from LDS, in the same order (as the 16-candidate kernel)
                const float* bout = L.hbias + A.L * A.Wpad;
#pragma unroll
                for (int k = 0; k < SS; ++k) {
                    const int d = j + 16 * k;
                    if (d < A.s) slot(d, L.obs_mean[d], L.obs_std[d], L.goal[d], L.cw[d], bout[d]);
                }
            }
            for (int d = A.s + A.a + j; d < A.s + A.a + A.k0pad_extra; d += 16) actX[m * lda + d] = 0.f;
            sc = rowsum16(sc);
            const float ac = acs[(t & 1) * M + m];
            total += sc + A.alpha_a2 * (ac / (float)A.a);
        } else if (actw && t + 1 < A.H) {
            stage_actions<1, SS>(A, P, L, actX, awave, lane, av, acp, lda);
            const float v = rowsum16(acp[0]);
            if ((lane & 15) == 0) acs[((t + 1) & 1) * M + epi_row(0, awave, lane)] = v;
        }
        __syncthreads();
        STAMP(6);
    }
#ifdef MBRL_STAMPS
    seg[NSEG - 1] = __builtin_amdgcn_s_memrealtime() - rt0;
    if (lane == 0 && g_mbrl_stamps != nullptr) {
        unsigned long long* dst = g_mbrl_stamps + (((size_t)e * ntiles + tile) * 8 + wave) * NSEG;
#pragma unroll
        for (int k = 0; k < NSEG; ++k) dst[k] = seg[k];
    }
#endif
#undef M8_CHUNK
#undef M8_LOAD
    if (epi && (lane & 15) == 0) {
        const int n = tile * M + epi_row(0, wave, lane);
        if (n < A.N) A.costs[(size_t)e * A.N + n] = total;
    }
}

bool rollout_m8_supported(const RolloutArgs& A, int T) {
    if (A.reward || A.redo || A.m8_off == 0) return false;
    if (T != 4 && T != 8) return false;
    return (A.K0C == 2 || A.K0C == 6) && (A.NOT == 2 || A.NOT == 6) && rollout_lds_bytes(A, 8) <= 160 * 1024;
}

template <int T, int K0C_T, int NOT_T, int K0L = 0>
static hipError_t launch_m8_tr(const RolloutArgs& A_in, hipStream_t stream) {
    RolloutArgs A = A_in;
    A.nw = 8;   // output partials: the 8-wave kernel's count
    if (!ring_strides_ok<T, K0C_T, NOT_T>(A)) return hipErrorInvalidValue;
    const dim3 grid = A.xcd_map ? dim3((A.N + 7) / 8 * A.E) : dim3((A.N + 7) / 8, A.E);
    const size_t lds = rollout_lds_bytes(A, 8);
    const auto fn = &rollout_m8_kernel<T, K0C_T, NOT_T, K0L>;
    hipError_t e = ensure_dynamic_lds(reinterpret_cast<const void*>(fn), 160 * 1024);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fn, grid, dim3(64 * m8_waves(T, NOT_T)), lds, stream, A);
    return hipGetLastError();
}

template <int T>
static hipError_t launch_m8_t(const RolloutArgs& A, hipStream_t stream) {
    if constexpr (T == 4)   // cartpole-sized inputs in KP mode: padded layer-0 MFMAs not issued
        if (A.K0C == 2 && A.NOT == 2 && A.s + A.a <= 8) return launch_m8_tr<T, 2, 2, 8>(A, stream);
    if (A.K0C == 2 && A.NOT == 2) return launch_m8_tr<T, 2, 2>(A, stream);
    if (A.K0C == 6 && A.NOT == 6) return launch_m8_tr<T, 6, 6>(A, stream);
    if (A.K0C == 2 && A.NOT == 6) return launch_m8_tr<T, 2, 6>(A, stream);
    if (A.K0C == 6 && A.NOT == 2) return launch_m8_tr<T, 6, 2>(A, stream);
    return hipErrorInvalidValue;
}

hipError_t launch_rollout_m8(const RolloutArgs& A, int T, hipStream_t stream) {
    if (T == 4) return launch_m8_t<4>(A, stream);
    if (T == 8) return launch_m8_t<8>(A, stream);
    return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------------
// 4-candidate tiles (DESIGN.md §3 "rollout_m4_kernel"): v_mfma_f32_4x4x1_16b_f32 without A broadcast.
//
// A plan of N <= 1024 candidates fills at most 128 CUs with 8-candidate tiles. Here each workgroup
// owns 4 candidates and every 4x4x1 block a distinct 4-row group: wave w (T waves, T = Wpad / 64)
// owns hidden rows [64 w, 64 w + 64) of every layer as ONE accumulator chain, fed by the 8-candidate
// weight stream without KP pairing (lane l: row 64 w + 32 ((l >> 2) & 1) + 4 (l >> 3) + (l & 3)):
//   A (lane l): W[row(l)][k]   B (lane l): X[k][cand l & 3]   D (lane l, v): row(4 (l >> 2) + v), cand l & 3
// Every accumulator consumes its k in the canonical order (16-deep chunk kc, step s, then q: k =
// 16 kc + 4 q + s), so sums equal the 8/16/32-candidate kernels' bit for bit
// (tools/ubench/mfma4x4_chain.hip: one chain per SIMD issues every 12.3 cycles against 8 for two;
// at Wpad 256 that single chain still beats two waves x two 32-row tiles of 8 candidates).
// Output layer: the canonical chains of mma_out -- per half of T/2 16-feature tiles, four chains
// c (k = 16 kc + 4 q + c) -- as 4x4x1 blocks: block b = 4 (l >> 4) + chain, rows 16 g + 4 (l >> 4) + v
// of output group g, B = the chain's own k of the wave's own features (from LDS), then the chains
// close as (c0 + c1) + (c2 + c3) through two lane swaps (exactly commutative) and each half's partial
// goes to LDS for the canonical 8-partial sum of the epilogue (sum_partials<8>).
template <int T, int K0C_T, int NG, int K0L = 0>
__global__ void __launch_bounds__(64 * T, 1) rollout_m4_kernel(const RolloutArgs A) {
    constexpr int M = 4;
    // compile-time LDS row strides (rollout_kernel LDAC / PWC; the launcher checks the geometry)
    const int lda = (64 * T > 16 * K0C_T ? 64 * T : 16 * K0C_T) + 4;
    const int pw = 16 * ((NG + 1) & ~1) + 4;
    constexpr int NW = T;
    constexpr int NT = 64 * NW;
    constexpr int KH = 4 * T;
    constexpr int NB = 4;                    // ring slots of 4 float4 per lane, 3 chunks ahead
    constexpr int NOC = 4;                   // output chunks: the wave's own 4 K chunks
    constexpr int DUM = (NB - (K0C_T + NOC) % NB) % NB;
    constexpr int NHW = 8 / T;               // canonical output halves per wave (T / 2 tiles each)
    constexpr int KPH = 4 / NHW;             // own K chunks per half
    constexpr int SS = NG;                   // state slots per epilogue lane (ceil(s / 16) <= NG)
    static_assert((T == 4 || T == 8) && NG >= 1 && NG <= 4 && KH % NB == 0, "m4 geometry");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const LdsMap L = lds_map(A, smem, M);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int ntiles = (A.N + M - 1) / M;
    int tile, e;
    xcd_unit(A.xcd_map, ntiles, tile, e);
    const float* member = A.packed + (size_t)e * A.member_stride;
    float* const actX = L.act;
    float* const actY = L.act2;
    // epilogue roles: wave 0 the state rows of the 4 candidates, wave 1 their actions
    const bool epi = wave == 0;
    const bool actw = wave == 1;
    const int awave = 0;
    float* acs = L.aterm;
    const int cand = lane & 3;
    float av[1][MAX_A_PER_LANE];
    float acp[1];
    auto fetch_a = [&](int t) {
        const int n = min(tile * M + epi_row(0, awave, lane), A.N - 1);
        const float* src = A.actions + ((size_t)t * A.N + n) * A.a;
#pragma unroll
        for (int k = 0; k < MAX_A_PER_LANE; ++k) av[0][k] = src[min((lane & 15) + 16 * k, A.a - 1)];
    };
    if (actw) fetch_a(0);
    for (int i = tid; i < A.s; i += NT) {
        L.obs_mean[i] = A.obs_mean ? A.obs_mean[i] : 0.f;
        L.obs_std[i] = A.obs_std ? A.obs_std[i] : 1.f;
        L.goal[i] = A.goal ? A.goal[i] : 0.f;
        L.cw[i] = A.cw ? A.cw[i] : 0.f;
    }
    for (int i = tid; i < A.a; i += NT) {
        L.act_mean[i] = A.act_mean ? A.act_mean[i] : 0.f;
        L.act_std[i] = A.act_std ? A.act_std[i] : 1.f;
    }
    const float* bias_src = member + A.stream_floats;
    for (int i = tid; i < A.L * A.Wpad + 16 * A.NOT; i += NT) L.hbias[i] = bias_src[i];
    __syncthreads();
    for (int i = tid; i < M * A.s; i += NT) {
        const int m = i / A.s, d = i - (i / A.s) * A.s;
        const int n = min(tile * M + m, A.N - 1);
        const float sv = A.s0_per_cand ? A.s0[(size_t)n * A.s + d] : A.s0[d];
        actX[m * lda + d] = A.norm_s ? (sv - L.obs_mean[d]) / L.obs_std[d] : sv;
    }
    for (int i = tid; i < M * A.k0pad_extra; i += NT) {
        const int m = i / A.k0pad_extra, j = i - (i / A.k0pad_extra) * A.k0pad_extra;
        actX[m * lda + A.s + A.a + j] = 0.f;
    }
    EpiParams<SS> P;
    load_epi_params<SS>(A, L, lane, P);
    if (actw) {
        stage_actions<1, SS>(A, P, L, actX, awave, lane, av, acp, lda);
        const float v = rowsum16(acp[0]);
        if ((lane & 15) == 0) acs[epi_row(0, awave, lane)] = v;
    }
    __syncthreads();

    // ---- weight stream: chunk g of this wave at byte (g T + wave) 4096 + slot 1024 + lane 16
    const int C4 = A.C4;
    const int CSQ = C4 + DUM;
    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(member + A.m4_off), 0, (int)((size_t)C4 * 4096 * T), 0x00020000);
    const unsigned lane_off = (unsigned)(wave * 4 * 1024 + lane * 16);
    f32x4 ring[NB][4];
#define M4_LOAD(SLOT, G)                                                                          \
    do {                                                                                          \
        int gg_ = (G);                                                                            \
        if (gg_ >= CSQ) gg_ -= CSQ;                                                               \
        gg_ = gg_ < C4 ? gg_ : C4 - 1;                                                            \
        const int so_ = gg_ * (4096 * T);                                                         \
        _Pragma("unroll") for (int s_ = 0; s_ < 4; ++s_) ring[SLOT][s_] = __builtin_bit_cast(     \
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, lane_off + s_ * 1024, so_, 0));   \
    } while (0)
#pragma unroll
    for (int q = 0; q < NB - 1; ++q) M4_LOAD(q, q);
    f32x4 bb[2][4];     // B: X[cand][16 kc + 4 q' .. +3], double-buffered over chunks
    f32x4 acc;
    f32x4 bias;
    float total = 0.f;
    const int row0 = 64 * wave + 32 * ((lane >> 2) & 1) + 4 * (lane >> 3);   // this lane's 4 D rows
    auto read_b = [&](f32x4 (&b)[4], const float* in, int col) {
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = *reinterpret_cast<const f32x4*>(in + cand * lda + col + 4 * q);
    };
    auto mma_chunk = [&](const f32x4 (&w)[4], const f32x4 (&b)[4]) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(w[s][q], b[q][s], acc, 0, 0, 0);
    };
    auto mma_chunk_l0 = [&](const f32x4 (&w)[4], const f32x4 (&b)[4], auto kcc) {
        constexpr int kc = decltype(kcc)::value;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (16 * kc + 4 * q + s < K0L) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(w[s][q], b[q][s], acc, 0, 0, 0);
    };
    auto store_layer = [&](float* out) {
        f32x4 v = acc + bias;
        v = __builtin_elementwise_max(v, f32x4{0.f, 0.f, 0.f, 0.f});
        *reinterpret_cast<f32x4*>(out + cand * lda + row0) = v;
    };
#define M4_CHUNK(SLOT, KC, NK, IN)                                          \
    do {                                                                    \
        M4_LOAD(((SLOT) + NB - 1) % NB, g + NB - 1);                         \
        if ((KC) + 1 < (NK)) read_b(bb[((KC) + 1) & 1], IN, 16 * ((KC) + 1)); \
        mma_chunk(ring[SLOT], bb[(KC) & 1]);                                \
        MBRL_PIN();                                                         \
        ++g;                                                                \
    } while (0)

    for (int t = 0; t < A.H; ++t) {
        int g = 0;
        if (actw && t + 1 < A.H) fetch_a(t + 1);
        // ---- layer 0: actX [s | a | 0-pad] -> actY
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
        bias = *reinterpret_cast<const f32x4*>(L.hbias + row0);
        read_b(bb[0], actX, 0);
        if constexpr (K0L > 0) {
            static_assert(K0C_T == 2, "K0L instance");
            M4_LOAD((0 + NB - 1) % NB, g + NB - 1);
            read_b(bb[1], actX, 16);
            mma_chunk_l0(ring[0], bb[0], std::integral_constant<int, 0>());
            MBRL_PIN();
            ++g;
            M4_LOAD((1 + NB - 1) % NB, g + NB - 1);
            mma_chunk_l0(ring[1], bb[1], std::integral_constant<int, 1>());
            MBRL_PIN();
            ++g;
        } else {
#pragma unroll
            for (int kc = 0; kc < K0C_T; ++kc) M4_CHUNK(kc % NB, kc, K0C_T, actX);
        }
        store_layer(actY);
        if (A.L > 1) __syncthreads();
        float* in = actY;
        float* out = actX;
        for (int l = 1; l < A.L; ++l) {
            acc = f32x4{0.f, 0.f, 0.f, 0.f};
            bias = *reinterpret_cast<const f32x4*>(L.hbias + l * A.Wpad + row0);
            // the half-rotated K order (rollout_kernel): second-half rows start at chunk KH / 2
            const int rof = 2 * wave >= T ? 16 * (KH / 2) : 0;
            const float* const inLo = in + rof;
            const float* const inHi = in - rof;
            read_b(bb[0], inLo, 0);
#pragma unroll
            for (int kc = 0; kc < KH; ++kc) M4_CHUNK((K0C_T + kc) % NB, kc, KH, (kc + 1 < KH / 2 ? inLo : inHi));
            store_layer(out);
            if (l + 1 < A.L) __syncthreads();   // the last hidden layer is read back by its own wave only
            float* tmp = in; in = out; out = tmp;
        }
        // ---- output layer over this wave's own 64 features (its own LDS stores, in order)
        {
            const int chain = (lane >> 2) & 3;
            f32x4 ch[NHW][NG];
#pragma unroll
            for (int h = 0; h < NHW; ++h)
#pragma unroll
                for (int gr = 0; gr < NG; ++gr) ch[h][gr] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int o = 0; o < NOC; ++o) {
                f32x4 hq[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    hq[q] = *reinterpret_cast<const f32x4*>(in + cand * lda + 64 * wave + 16 * o + 4 * q);
                constexpr int base = K0C_T;   // output chunk o sits in slot (K0C + KH + o) % NB
                M4_LOAD(((base + o) + NB - 1) % NB, g + NB - 1);
                const int h = o / KPH;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float b = chain == 0 ? hq[q][0] : chain == 1 ? hq[q][1] : chain == 2 ? hq[q][2] : hq[q][3];
#pragma unroll
                    for (int gr = 0; gr < NG; ++gr)
                        ch[h][gr] = __builtin_amdgcn_mfma_f32_4x4x1f32(ring[(base + o) % NB][gr][q], b, ch[h][gr], 0, 0, 0);
                }
                MBRL_PIN();
                ++g;
            }
#pragma unroll
            for (int d = 0; d < DUM; ++d) {
                M4_LOAD((K0C_T + NOC + d + NB - 1) % NB, g + NB - 1);
                ++g;
            }
            // (c0 + c1) + (c2 + c3): chains c ^ 1 / c ^ 2 sit 4 / 8 lanes away
#pragma unroll
            for (int h = 0; h < NHW; ++h)
#pragma unroll
                for (int gr = 0; gr < NG; ++gr) {
                    f32x4 x, y;
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[i] = ch[h][gr][i] + __shfl_xor(ch[h][gr][i], 4);
#pragma unroll
                    for (int i = 0; i < 4; ++i) y[i] = x[i] + __shfl_xor(x[i], 8);
                    if (chain == 0)
                        *reinterpret_cast<f32x4*>(L.part + (wave * NHW + h) * (M * pw) + cand * pw + 16 * gr +
                                                  4 * (lane >> 4)) = y;
                }
        }
        __syncthreads();
        // ---- epilogue: the 8-wave kernel's split-mode goal-state epilogue for rows 0..3
        if (epi) {
            const int ws = M * pw;
            const int j = lane & 15;
            const int m = epi_row(0, 0, lane);
            const int n = tile * M + m;
            float sc = 0.f;
            auto slot = [&](int d, float om, float os, float goal, float cw, float bo) {
                const int ro = m * pw + d;
                float o = sum_partials<8>(L.part, ws, ro);
                o = o + bo;
                const float sn = A.unnorm_s ? o * os + om : o;
                if (A.has_sc) {
                    const float x = (sn - goal) * cw;
                    sc += sqrtf(x * x + A.alpha_s2) - A.alpha_s;
                }
                actX[m * lda + d] = A.norm_s ? (sn - om) / os : sn;
                if (A.states_out != nullptr && n < A.N)
                    A.states_out[(((size_t)e * A.H + t) * A.N + n) * A.s + d] = sn;
            };
            if constexpr (SS <= MBRL_EPI_REG_SLOTS) {
#pragma unroll
                for (int k = 0; k < SS; ++k)
                    if (j + 16 * k < A.s) slot(j + 16 * k, P.om[k], P.os[k], P.goal[k], P.cw[k], P.bo[k]);
            } else {
                const float* bout = L.hbias + A.L * A.Wpad;
#pragma unroll
                for (int k = 0; k < SS; ++k) {
                    const int d = j + 16 * k;
                    if (d < A.s) slot(d, L.obs_mean[d], L.obs_std[d], L.goal[d], L.cw[d], bout[d]);
                }
            }
            for (int d = A.s + A.a + j; d < A.s + A.a + A.k0pad_extra; d += 16) actX[m * lda + d] = 0.f;
            sc = rowsum16(sc);
            const float ac = acs[(t & 1) * M + m];
            total += sc + A.alpha_a2 * (ac / (float)A.a);
        } else if (actw && t + 1 < A.H) {
            stage_actions<1, SS>(A, P, L, actX, awave, lane, av, acp, lda);
            const float v = rowsum16(acp[0]);
            if ((lane & 15) == 0) acs[((t + 1) & 1) * M + epi_row(0, awave, lane)] = v;
        }
        __syncthreads();
    }
#undef M4_CHUNK
#undef M4_LOAD
    if (epi && (lane & 15) == 0) {
        const int n = tile * M + epi_row(0, 0, lane);
        if (n < A.N) A.costs[(size_t)e * A.N + n] = total;
    }
}

bool rollout_m4_supported(const RolloutArgs& A, int T, int NG) {
    if (A.reward || A.redo || A.m4_off == 0) return false;
    if ((T != 4 && T != 8) || NG < 1 || NG > 4) return false;
    return (A.K0C == 2 || A.K0C == 6) && rollout_lds_bytes(A, 4) <= 160 * 1024;
}

template <int T, int K0C_T, int NG, int K0L = 0>
static hipError_t launch_m4_tr(const RolloutArgs& A_in, hipStream_t stream) {
    RolloutArgs A = A_in;
    A.nw = 8;   // output partials: the canonical 8
    if (!ring_strides_ok<T, K0C_T, (NG + 1) & ~1>(A)) return hipErrorInvalidValue;
    const int ntiles = (A.N + 3) / 4;
    const dim3 grid = A.xcd_map ? dim3(ntiles * A.E) : dim3(ntiles, A.E);
    const size_t lds = rollout_lds_bytes(A, 4);
    const auto fn = &rollout_m4_kernel<T, K0C_T, NG, K0L>;
    hipError_t e = ensure_dynamic_lds(reinterpret_cast<const void*>(fn), 160 * 1024);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fn, grid, dim3(64 * T), lds, stream, A);
    return hipGetLastError();
}

template <int T, int K0C_T>
static hipError_t launch_m4_tk(const RolloutArgs& A, int NG, hipStream_t stream) {
    if (NG == 1) return launch_m4_tr<T, K0C_T, 1>(A, stream);
    if (NG == 2) return launch_m4_tr<T, K0C_T, 2>(A, stream);
    return launch_m4_tr<T, K0C_T, 4>(A, stream);   // NG 3: one all-zero group more
}

hipError_t launch_rollout_m4(const RolloutArgs& A, int T, int NG, hipStream_t stream) {
    if (T == 4 && A.K0C == 2 && NG == 1 && A.s + A.a <= 8)   // cartpole-sized inputs: padded MFMAs skipped
        return launch_m4_tr<4, 2, 1, 8>(A, stream);
    if (T == 4) return A.K0C == 2 ? launch_m4_tk<4, 2>(A, NG, stream) : launch_m4_tk<4, 6>(A, NG, stream);
    if (T == 8) return A.K0C == 2 ? launch_m4_tk<8, 2>(A, NG, stream) : launch_m4_tk<8, 6>(A, NG, stream);
    return hipErrorInvalidValue;
}

}  // namespace mbrl

#ifdef MBRL_STAMPS
extern "C" int mbrl_diag_set_stamps(void* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mbrl::g_mbrl_stamps), &buf, sizeof(buf));
}
#endif
