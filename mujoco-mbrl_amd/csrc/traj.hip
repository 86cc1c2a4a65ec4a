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
    // fallback behind the cooperative kernel: only when that one gave up (status word set)
    if (A.gate != nullptr && *A.gate == 0u) return;
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
// Cooperative single-trajectory rollout (see mbrl_internal.h).
//
// P = Wpad/16 workgroups per member, 512 threads each. Workgroup p owns hidden units
// [16p, 16p+16) of every W -> W layer (those 16 rows LDS-resident, row stride W+32 so the two
// half-waves of a wave read disjoint bank halves). Layer 0 and the output layer are computed
// redundantly by every workgroup from REGISTER-resident weights (loaded once): thread u holds column
// u of W0^T (K0 <= K0R values); thread (g = tid>>5, c = tid&31) holds Wout[g+16m][c+32i]. Every
// step-invariant operand (normalised actions for all H steps, biases, normaliser statistics) is
// staged in LDS at the start, so a step issues no global load except the hand-off sweeps.
//
// Hand-off: R2 granules of cdna_hip_programming.md §6 Guideline 16 -- each value travels as ONE
// aligned 8-byte {tag = epoch, value} agent-scope atomic store to global memory; one wave re-reads
// (agent-scope atomic loads, L1-bypassing) until every tag equals the epoch. epoch = phase + 1,
// phase = t*(L-1) + l-1; two buffers by phase parity (a workgroup cannot be two phases ahead of a
// reader: it must first gather the phase in between, which needs everyone's publish that follows
// their read). Every spin is bounded (s_memrealtime, 100 MHz); on timeout `status` is set and the
// kernel exits.
// ------------------------------------------------------------------------------------------------
constexpr int COOP_THREADS = 512;
constexpr int COOP_ROWS = 16;  // hidden units per workgroup per layer
constexpr int COOP_MAX_W = 512;

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;

// Diagnostic build only (-DMBRL_STAMPS): per-workgroup s_memrealtime sums (10 ns ticks) of the
// coop kernel's segments, written to a buffer set by mbrl_diag_set_traj_stamps().
#ifdef MBRL_STAMPS
constexpr int TRAJ_NSEG = 4;
__device__ unsigned long long* g_mbrl_traj_stamps;
#define TSTAMP(k)                                                      \
    do {                                                               \
        const unsigned long long _t = __builtin_amdgcn_s_memrealtime(); \
        tseg[k] += _t - tprev;                                         \
        tprev = _t;                                                    \
    } while (0)
#else
#define TSTAMP(k) \
    do {          \
    } while (0)
#endif

// sum over the 32 lanes of a half-wave, fixed butterfly order (identical result in every lane)
__device__ __forceinline__ float halfwave_sum(float v) {
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// halfwave_sum_hi and CoopDot: mbrl_internal.h (shared with gd.hip)

struct CoopLds {
    int rs;                         // slice row stride (floats)
    size_t slices, x0, hA, hB, out, acts, hb, ob, om, os, flag, total;
};

__host__ __device__ inline CoopLds coop_lds(int s, int a, int W, int Wp, int L, int H, int K0R) {
    CoopLds m;
    auto al4 = [](size_t n) { return (n + 3) & ~(size_t)3; };
    m.rs = W + 32;
    size_t o = 0;
    m.slices = o; o += (size_t)(L - 1) * COOP_ROWS * m.rs;
    m.x0 = o;     o += al4(K0R > s + a ? K0R : s + a);
    m.hA = o;     o += Wp;
    m.hB = o;     o += Wp;
    m.out = o;    o += al4(s);
    m.acts = o;   o += al4((size_t)H * a);       // normalised actions, [H][a]
    m.hb = o;     o += al4((size_t)(L - 1) * COOP_ROWS);  // my hidden biases
    m.ob = o;     o += al4(s);                    // output bias
    m.om = o;     o += al4(s);                    // obs mean
    m.os = o;     o += al4(s);                    // obs std
    m.flag = o;   o += 4;
    m.total = o * sizeof(float);
    return m;
}

// K0R: layer-0 inputs held per thread (>= s + a); SM: output rows per half-wave (16 SM >= s);
// WI = W / 32: columns per lane of a 16-row dot (W == Wpad). All loops are unguarded: operands past
// the real sizes are zero (weights) or finite zeros (x0 padding), so LDS reads issue in batches.
template <int K0R, int SM, int WI>
__global__ void __launch_bounds__(COOP_THREADS) traj_coop_kernel(const TrajArgs A, u64* __restrict__ xchg_all,
                                                                  unsigned* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // hop_mode >= 1: member e's workgroups are blocks e, e + 8, e + 16, ... (one XCD under round-robin
    // dispatch: speed only, the granule protocol below holds on any placement)
    const bool xgrid = A.hop_mode >= 1;
    const int p = xgrid ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    const int e = xgrid ? (int)(blockIdx.x & 7) : (int)blockIdx.y;
    if (e >= A.E) return;                      // the XCD slots past the ensemble
    [[maybe_unused]] const int P = xgrid ? (int)(gridDim.x >> 3) : (int)gridDim.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int s = A.s, a = A.a, W = A.W, Wp = A.Wpad, K0 = s + a;
    const CoopLds m = coop_lds(s, a, W, Wp, A.L, A.H, K0R);
    float* slices = smem + m.slices;
    float* x0 = smem + m.x0;
    float* acts = smem + m.acts;
    float* hb = smem + m.hb;
    float* ob = smem + m.ob;
    float* om = smem + m.om;
    float* os = smem + m.os;
    int& abort_flag = *reinterpret_cast<int*>(smem + m.flag);
    const float* member = A.packed + (size_t)e * A.member_stride;
    const float* bias = member + A.bias_off;
    const float* tw = member + A.tw_base;
    gu64* xchg = (gu64*)(xchg_all + (size_t)e * 2 * Wp);

    if (A.debug_abort) {                       // test hook: behave as a timed-out hand-off
        if (tid == 0) atomicOr(status, 1u);
        return;
    }
    // ---- one-time staging ----------------------------------------------------------------------
    if (tid == 0) abort_flag = 0;
    for (int k = tid; k < K0R; k += COOP_THREADS) x0[k] = 0.0f;
    __syncthreads();
    for (int l = 1; l < A.L; ++l) {      // my rows of W_l: W_l[n][k] = W^T_l[k][n]
        const float* wt = tw + A.tw_off[l];
        float* dst = slices + (size_t)(l - 1) * COOP_ROWS * m.rs;
        for (int i = tid; i < COOP_ROWS * W; i += COOP_THREADS) {
            const int k = i >> 4, o = i & 15;
            dst[o * m.rs + k] = wt[(size_t)k * Wp + p * COOP_ROWS + o];
        }
    }
    for (int i = tid; i < A.H * a; i += COOP_THREADS) {
        const int d = i % a;
        const float av = A.actions[i];
        acts[i] = A.norm_a ? (av - A.act_mean[d]) / A.act_std[d] : av;
    }
    for (int i = tid; i < (A.L - 1) * COOP_ROWS; i += COOP_THREADS)
        hb[i] = bias[(size_t)(1 + i / COOP_ROWS) * Wp + p * COOP_ROWS + (i % COOP_ROWS)];
    for (int d = tid; d < s; d += COOP_THREADS) {
        ob[d] = bias[(size_t)A.L * Wp + d];
        om[d] = A.obs_mean[d];
        os[d] = A.obs_std[d];
        const float sv = A.s0[d];
        x0[d] = A.norm_s ? (sv - A.obs_mean[d]) / A.obs_std[d] : sv;
    }
    // layer-0 column of unit u = tid (W^T_0 [K0][Wp]), zero past K0
    float w0r[K0R];
    const bool has_unit = tid < Wp;
    const float b0 = has_unit ? bias[tid] : 0.0f;
#pragma unroll
    for (int k = 0; k < K0R; ++k)
        w0r[k] = (has_unit && k < K0) ? tw[A.tw_off[0] + (size_t)k * Wp + tid] : 0.0f;
    // output rows d = g + 16 mm, columns CoopDot<WI>::col(c, i) (Wout row-major [s][W]), zero past s / W
    const int g = tid >> 5, c = tid & 31;
    using Dot = CoopDot<WI>;
    float wor[SM][WI];
#pragma unroll
    for (int mm = 0; mm < SM; ++mm)
#pragma unroll
        for (int i = 0; i < WI; ++i) {
            const int d = g + 16 * mm, k = Dot::col(c, i);
            wor[mm][i] = (d < s && k < W) ? tw[A.tw_off[A.L] + (size_t)d * W + k] : 0.0f;
        }
    __syncthreads();

    // hop_mode 2: roll call. Each workgroup publishes its XCD (XCC_ID) as a granule in the parity-1
    // buffer (first used by phase 1, which no workgroup can publish before every workgroup has read
    // the roll call: phase 1 follows the gather of phase 0). If all P share one XCD they share its L2,
    // and the granules travel as L2-resident stores (kept in the XCD's L2) read by sc1 loads; else as
    // sc1 stores (written through) as on any placement.
    int& l2_flag = *(reinterpret_cast<int*>(smem + m.flag) + 1);
    if (A.hop_mode == 2) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        gu64* roll = xchg + Wp;
        constexpr unsigned RTAG = 0xFFFFFFFFu;
        if (tid == 0)
            __hip_atomic_store(&roll[p], ((u64)RTAG << 32) | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (wave == 0) {
            const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
            bool same = true;
            for (;;) {
                u64 gv = lane < P ? __hip_atomic_load(&roll[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : (((u64)RTAG << 32) | xcc);
                if (__all((unsigned)(gv >> 32) == RTAG)) {
                    same = __all((unsigned)gv == xcc);
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t_start > 20000000ull) {  // 200 ms
                    if (lane == 0) {
                        abort_flag = 1;
                        atomicOr(status, 1u);
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0) l2_flag = same ? 1 : 0;
        }
        __syncthreads();
        if (abort_flag) return;
    } else if (tid == 0) {
        l2_flag = 0;
    }
    __syncthreads();
    const bool l2 = l2_flag != 0;
#ifdef MBRL_STAMPS
    unsigned long long tseg[TRAJ_NSEG] = {0, 0, 0, 0};
    unsigned long long tprev = __builtin_amdgcn_s_memrealtime();
#endif
    int phase = 0;
    for (int t = 0; t < A.H; ++t) {
        // x0 = (normalised s_t written by the last step's output lanes, normalised a_t)
        for (int d = tid; d < a; d += COOP_THREADS) x0[s + d] = acts[t * a + d];
        __syncthreads();
        float* cur = smem + m.hA;
        float* nxt = smem + m.hB;
        if (has_unit) {                                 // layer 0 (redundant in every workgroup)
            float v = b0;
#pragma unroll
            for (int k = 0; k < K0R; ++k) v = fmaf(w0r[k], x0[k], v);
            cur[tid] = fmaxf(v, 0.0f);
        }
        __syncthreads();
        TSTAMP(0);
        for (int l = 1; l < A.L; ++l, ++phase) {
            // my 16 units: row g (half-wave), lanes c split K; the sum lands in lane c == 16
            const float* ws = slices + (size_t)(l - 1) * COOP_ROWS * m.rs + (size_t)g * m.rs;
            const float v = halfwave_sum_hi(Dot::lds(ws, cur, c));
            const unsigned epoch = (unsigned)phase + 1u;
            gu64* buf = xchg + (size_t)(phase & 1) * Wp;
            if (c == 16) {
                const float y = fmaxf(v + hb[(l - 1) * COOP_ROWS + g], 0.0f);
                const u64 gr = ((u64)epoch << 32) | __float_as_uint(y);
                if (l2)   // every reader shares this L2: a store that keeps the line there (sc0)
                    __hip_atomic_store(&buf[p * COOP_ROWS + g], gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    __hip_atomic_store(&buf[p * COOP_ROWS + g], gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            TSTAMP(1);
            // gather all P slices: wave 0 sweeps the granules until every tag matches
            if (wave == 0) {
                const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
                constexpr int GR = WI / 2;         // granules per lane: P * 16 = Wp = 32 WI
                for (;;) {
                    u64 gv[GR];
#pragma unroll
                    for (int q = 0; q < GR; ++q)    // all loads in flight before the first compare
                        gv[q] = __hip_atomic_load(&buf[lane + 64 * q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bool ok = true;
#pragma unroll
                    for (int q = 0; q < GR; ++q) {
                        ok &= (unsigned)(gv[q] >> 32) == epoch;
                        nxt[lane + 64 * q] = __uint_as_float((unsigned)gv[q]);
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
            TSTAMP(2);
            if (abort_flag) return;
            float* tmp = cur; cur = nxt; nxt = tmp;
        }
        // output layer (redundant): half-wave g owns rows g + 16 mm; the lane holding a row's sum
        // unnormalises it, stores the state and writes the next step's normalised input (x0 and cur
        // are read / rewritten only after the barrier at the top of the next step)
#pragma unroll
        for (int mm = 0; mm < SM; ++mm) {
            const float v = halfwave_sum_hi(Dot::reg(wor[mm], cur, c));
            const int d = g + 16 * mm;
            if (c == 16 && d < s) {
                const float o = v + ob[d];
                const float sn = A.unnorm_s ? o * os[d] + om[d] : o;
                if (p == 0) A.states_out[((size_t)e * A.H + t) * s + d] = sn;
                x0[d] = A.norm_s ? (sn - om[d]) / os[d] : sn;
            }
        }
        TSTAMP(3);
    }
#ifdef MBRL_STAMPS
    if (tid == 0 && g_mbrl_traj_stamps != nullptr)
        for (int k = 0; k < TRAJ_NSEG; ++k)
            g_mbrl_traj_stamps[((size_t)e * P + p) * TRAJ_NSEG + k] = tseg[k];
#endif
}

// register budgets: (K0 <= 32, s <= 32) for cartpole / cheetah / walker, (K0 <= 96, s <= 80) humanoid
static int coop_k0r(const TrajArgs& A) {
    const int K0 = A.s + A.a;
    if (K0 <= 32 && A.s <= 32) return 32;
    if (K0 <= 96 && A.s <= 80) return 96;
    return 0;
}

bool traj_coop_supported(const TrajArgs& A, int E) {
    const int P = A.Wpad / COOP_ROWS;
    const int k0r = coop_k0r(A);
    // P * E workgroups must be co-resident: launch_coop_variant checks the device's occupancy
    if (k0r == 0 || A.L < 2 || A.W != A.Wpad || A.Wpad > COOP_MAX_W || P * E > 1024) return false;
    return coop_lds(A.s, A.a, A.W, A.Wpad, A.L, A.H, k0r).total <= 150 * 1024;
}

size_t traj_coop_xchg_bytes(const TrajArgs& A, int E) { return (size_t)E * 2 * A.Wpad * sizeof(u64); }

template <int K0R, int SM, int WI>
static hipError_t launch_coop_variant(const TrajArgs& A_in, int E, u64* xchg, unsigned* status, hipStream_t stream) {
    hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(&traj_coop_kernel<K0R, SM, WI>), 160 * 1024);
    if (err != hipSuccess) return err;
    const size_t lds = coop_lds(A_in.s, A_in.a, A_in.W, A_in.Wpad, A_in.L, A_in.H, K0R).total;
    const int P = A_in.Wpad / COOP_ROWS;
    if (!grid_fits(reinterpret_cast<const void*>(&traj_coop_kernel<K0R, SM, WI>), COOP_THREADS, lds, P * E))
        return hipErrorCooperativeLaunchTooLarge;
    TrajArgs A = A_in;
    A.E = E;
    // the per-XCD grid puts each member's P workgroups on one XCD: P must fit an eighth of the capacity
    const bool xcd_fits = grid_fits(reinterpret_cast<const void*>(&traj_coop_kernel<K0R, SM, WI>), COOP_THREADS, lds, 8 * P);
    if (A.hop_mode >= 1 && E <= 8 && xcd_fits) {
        hipLaunchKernelGGL((traj_coop_kernel<K0R, SM, WI>), dim3(8 * P), dim3(COOP_THREADS), lds, stream, A, xchg,
                           status);
    } else {
        A.hop_mode = 0;
        hipLaunchKernelGGL((traj_coop_kernel<K0R, SM, WI>), dim3(P, E), dim3(COOP_THREADS), lds, stream, A, xchg,
                           status);
    }
    return hipGetLastError();
}

template <int K0R, int SM>
static hipError_t launch_coop_width(const TrajArgs& A, int E, u64* xchg, unsigned* status, hipStream_t stream) {
    switch (A.Wpad) {
        case 64: return launch_coop_variant<K0R, SM, 2>(A, E, xchg, status, stream);
        case 128: return launch_coop_variant<K0R, SM, 4>(A, E, xchg, status, stream);
        case 256: return launch_coop_variant<K0R, SM, 8>(A, E, xchg, status, stream);
        case 512: return launch_coop_variant<K0R, SM, 16>(A, E, xchg, status, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_traj_coop(const TrajArgs& A, int E, unsigned long long* xchg, unsigned* status,
                            hipStream_t stream) {
    // one memset when the status word directly follows the granules (the workspaces lay them out so);
    // none when the plan's first launch zeroed both (cem_init_kernel)
    if (!A.prezeroed) {
        const size_t xb = traj_coop_xchg_bytes(A, E);
        const bool adjacent = reinterpret_cast<char*>(status) == reinterpret_cast<char*>(xchg) + xb;
        hipError_t err = hipMemsetAsync(xchg, 0, adjacent ? xb + 16 : xb, stream);
        if (err != hipSuccess) return err;
        if (!adjacent) {
            err = hipMemsetAsync(status, 0, sizeof(unsigned), stream);
            if (err != hipSuccess) return err;
        }
    }
    return coop_k0r(A) == 32 ? launch_coop_width<32, 2>(A, E, xchg, status, stream)
                             : launch_coop_width<96, 5>(A, E, xchg, status, stream);
}

// ------------------------------------------------------------------------------------------------
// Register-resident single-trajectory rollout for narrow models (Wpad <= 256: cartpole's 2x256, the
// reference's default widths 50 / 200): one workgroup of 1024 threads per member holds EVERY weight
// in registers for the whole horizon -- W0 and the hidden W_l rows split over TPR = 1024 / Wpad threads
// (K0J / KPT columns each; hidden columns in float4 groups k = 4 (q + TPR j) + i, so that a wave's LDS
// reads of the input vector are 16-byte broadcasts), Wout one row per wave. A step is four barriers and
// no global load (no cross-workgroup hop, no hand-off memset, no fallback launch): ~1 us per step
// where traj_coop_kernel pays a ~3.4 us hop per hidden layer.
// ------------------------------------------------------------------------------------------------
constexpr int REG_THREADS = 1024;

__host__ __device__ inline int reg_max_hidden(int Wp) { return Wp <= 64 ? 3 : (Wp <= 128 ? 3 : (Wp <= 256 ? 1 : 0)); }

template <int WP, int NHL, int K0R>
__global__ void __launch_bounds__(REG_THREADS) traj_reg_kernel(const TrajArgs A) {
    constexpr int TPR = REG_THREADS / WP;   // threads per hidden row
    constexpr int KPT = WP / TPR;           // columns per thread (a multiple of 4)
    static_assert(KPT % 4 == 0, "float4 column groups");
    constexpr int OI = WP / 64;             // output-layer columns per lane
    constexpr int SM = 2;                   // output rows per wave (s <= 32)
    constexpr int K0J = (K0R + TPR - 1) / TPR;   // layer-0 columns per thread
    static_assert(K0J * TPR <= 32, "x0 holds 32 inputs");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int e = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int r = tid / TPR, q = tid - (tid / TPR) * TPR;
    const int s = A.s, a = A.a, W = A.W, Wp = A.Wpad, K0 = s + a;
    float* x0 = smem;                        // [32]
    float* hA = x0 + 32;                     // [WP]
    float* hB = hA + WP;                     // [WP]
    float* out = hB + WP;                    // [32]
    float* prm = out + 32;                   // [4][32]: output bias, obs mean, obs std, (pad)
    float* acts = prm + 128;                 // [H][a] normalised actions
    const float* member = A.packed + (size_t)e * A.member_stride;
    const float* bias = member + A.bias_off;
    const float* tw = member + A.tw_base;

    for (int k = tid; k < 32; k += REG_THREADS) {
        float v = 0.f;
        if (k < s) {
            const float sv = A.s0[k];
            v = A.norm_s ? (sv - A.obs_mean[k]) / A.obs_std[k] : sv;
        }
        x0[k] = v;
    }
    for (int d = tid; d < s; d += REG_THREADS) {
        prm[d] = bias[(size_t)A.L * Wp + d];
        prm[32 + d] = A.obs_mean ? A.obs_mean[d] : 0.f;
        prm[64 + d] = A.obs_std ? A.obs_std[d] : 1.f;
    }
    for (int i = tid; i < A.H * a; i += REG_THREADS) {
        const int d = i % a;
        const float av = A.actions[i];
        acts[i] = A.norm_a ? (av - A.act_mean[d]) / A.act_std[d] : av;
    }
    // weights into registers (zero past the real sizes)
    float w0r[K0J];                                      // W0[r][q + TPR j] (W^T_0 [K0][Wpad])
    const float b0 = r < W ? bias[r] : 0.f;
#pragma unroll
    for (int j = 0; j < K0J; ++j) {
        const int k = q + TPR * j;
        w0r[j] = (r < W && k < K0) ? tw[A.tw_off[0] + (size_t)k * Wp + r] : 0.f;
    }
    float wh[NHL > 0 ? NHL : 1][KPT];
    float bh[NHL > 0 ? NHL : 1];
#pragma unroll
    for (int l = 0; l < NHL; ++l) {
        const float* wt = tw + A.tw_off[l + 1];          // W^T_l [W][Wpad]: W_l[r][k] = wt[k * Wpad + r]
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const int k = 4 * (q + TPR * (j >> 2)) + (j & 3);
            wh[l][j] = (r < W && k < W) ? wt[(size_t)k * Wp + r] : 0.f;
        }
        bh[l] = r < W ? bias[(size_t)(l + 1) * Wp + r] : 0.f;
    }
    float wor[SM][OI];
    const float* wo = tw + A.tw_off[A.L];               // Wout row-major [so][W]
#pragma unroll
    for (int m = 0; m < SM; ++m)
#pragma unroll
        for (int i = 0; i < OI; ++i) {
            const int d = wave + 16 * m, k = lane + 64 * i;
            wor[m][i] = (d < s && k < W) ? wo[(size_t)d * W + k] : 0.f;
        }
    __syncthreads();

    for (int t = 0; t < A.H; ++t) {
        for (int d = tid; d < a; d += REG_THREADS) x0[s + d] = acts[t * a + d];
        __syncthreads();
        float* cur = hA;
        float* nxt = hB;
        {                                                // layer 0: row r over TPR lanes
            float v = 0.f;
#pragma unroll
            for (int j = 0; j < K0J; ++j) v += w0r[j] * x0[q + TPR * j];
#pragma unroll
            for (int o = TPR / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
            if (q == 0) cur[r] = fmaxf(v + b0, 0.f);
        }
        __syncthreads();
#pragma unroll
        for (int l = 0; l < NHL; ++l) {                  // W -> W: row r over TPR lanes, fixed butterfly
            float v = 0.f;
#pragma unroll
            for (int j4 = 0; j4 < KPT / 4; ++j4) {
                const f32x4 x = *reinterpret_cast<const f32x4*>(cur + 4 * (q + TPR * j4));
#pragma unroll
                for (int i = 0; i < 4; ++i) v += wh[l][4 * j4 + i] * x[i];
            }
#pragma unroll
            for (int o = TPR / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
            if (q == 0) nxt[r] = fmaxf(v + bh[l], 0.f);
            __syncthreads();
            float* tmp = cur; cur = nxt; nxt = tmp;
        }
#pragma unroll
        for (int m = 0; m < SM; ++m) {                   // output rows wave + 16 m
            float v = 0.f;
#pragma unroll
            for (int i = 0; i < OI; ++i) v += wor[m][i] * cur[lane + 64 * i];
            v = wave_sum64(v);
            const int d = wave + 16 * m;
            if (lane == 0 && d < s) out[d] = v + prm[d];
        }
        __syncthreads();
        for (int d = tid; d < s; d += REG_THREADS) {
            const float sn = A.unnorm_s ? out[d] * prm[64 + d] + prm[32 + d] : out[d];
            A.states_out[((size_t)e * A.H + t) * s + d] = sn;
            x0[d] = A.norm_s ? (sn - prm[32 + d]) / prm[64 + d] : sn;
        }
        // x0 and out are next touched after the barrier at the top of the next step
    }
}

bool traj_reg_supported(const TrajArgs& A) {
    const int K0 = A.s + A.a;
    if (A.Wpad > 256 || A.L - 1 > reg_max_hidden(A.Wpad) || K0 > 32 || A.s > 32) return false;
    return (size_t)(32 + 2 * A.Wpad + 32 + 128 + A.H * A.a) * sizeof(float) <= 64 * 1024;
}

template <int WP, int NHL>
static hipError_t launch_reg_k0(const TrajArgs& A, int E, hipStream_t stream) {
    const int K0 = A.s + A.a;
    const size_t lds = (size_t)(32 + 2 * WP + 32 + 128 + A.H * A.a) * sizeof(float);
    if (K0 <= 8)
        hipLaunchKernelGGL((traj_reg_kernel<WP, NHL, 8>), dim3(E), dim3(REG_THREADS), lds, stream, A);
    else
        hipLaunchKernelGGL((traj_reg_kernel<WP, NHL, 32>), dim3(E), dim3(REG_THREADS), lds, stream, A);
    return hipGetLastError();
}

template <int WP>
static hipError_t launch_reg_w(const TrajArgs& A, int E, hipStream_t stream) {
    switch (A.L - 1) {
        case 0: return launch_reg_k0<WP, 0>(A, E, stream);
        case 1: return launch_reg_k0<WP, 1>(A, E, stream);
        case 2: if constexpr (WP <= 128) return launch_reg_k0<WP, 2>(A, E, stream); else return hipErrorInvalidValue;
        case 3: if constexpr (WP <= 128) return launch_reg_k0<WP, 3>(A, E, stream); else return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_traj_reg(const TrajArgs& A, int E, hipStream_t stream) {
    switch (A.Wpad) {
        case 64: return launch_reg_w<64>(A, E, stream);
        case 128: return launch_reg_w<128>(A, E, stream);
        case 256: return launch_reg_w<256>(A, E, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mbrl

#ifdef MBRL_STAMPS
extern "C" int mbrl_diag_set_traj_stamps(void* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mbrl::g_mbrl_traj_stamps), &buf, sizeof(buf));
}
#endif
