// The model-training optimizer step: torch.optim.Adam's step for fp32
// parameter groups as ONE launch over every tensor of the group (include/mbrl_cem.h
// mbrl_adam_step).
//
// torch.optim.Adam (foreach path, capturable = False: the default for CUDA/HIP parameters, and what
// the reference's experiment.py:55-62 builds) runs a chain of multi-tensor kernels per step, each a
// full pass over the group's state: lerp_ (exp_avg), mul_ + addcmul_ (exp_avg_sq), sqrt, div_,
// add_ (denominator), addcdiv_ (param) -- plus an add for weight decay. Every one of those rounds to
// fp32 once per element. This kernel applies the same element-wise chain with the same roundings in
// one pass (param, grad, exp_avg, exp_avg_sq read once, three arrays written once), so the
// parameters and optimizer state it leaves are bit-identical to torch's: the file is built with
// -ffp-contract=off and every fused multiply-add torch's own build forms is spelled out as fmaf()
// (AdamArith; pinned on the MI355X by tests/test_gpu_train_adam.py against torch.optim.Adam).
// Per-tensor scalars (bias corrections of that tensor's step count) come from the host, computed
// in double exactly as adam.py does and rounded to float as the multi-tensor kernels round them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "../../include/mbrl_cem.h"
#include "mbrl_internal.h"

namespace mbrl {

constexpr int ADAM_THREADS = 256;
constexpr int ADAM_CHUNK = ADAM_THREADS * 4;   // elements per workgroup (one float4 per lane)

struct AdamLaunch {
    mbrl_adam_tensor t[ADAM_MAX_TENSORS];
    int first_block[ADAM_MAX_TENSORS + 1];      // workgroup prefix over the tensors' chunks
    int count;
    mbrl_adam_hparams hp;
    int arith;                                  // AdamArith bits
};

// One element of the chain. Bits of `arith` select which of torch's expressions were contracted to
// a fused multiply-add by the compiler that built torch (ForeachFunctors.cuh / Lerp.h):
//   ADAM_FMA_WD      grad + wd * param                        (_foreach_add(grads, params, alpha=wd))
//   ADAM_FMA_LERP    exp_avg + w * (grad - exp_avg)           (_foreach_lerp_, w < 0.5; else
//                    grad - (grad - exp_avg) * (1 - w))
//   ADAM_FMA_ADDCMUL exp_avg_sq + (1 - beta2) * (grad * grad) (_foreach_addcmul_)
//   ADAM_FMA_ADDCDIV param + step_size * (exp_avg / denom)    (_foreach_addcdiv_)
__device__ __forceinline__ void adam_element(float& p, float g, float& m, float& v, float step_size, float bc2,
                                             const mbrl_adam_hparams& hp, int arith) {
    if (hp.weight_decay != 0.0f)
        g = (arith & ADAM_FMA_WD) ? fmaf(hp.weight_decay, p, g) : g + hp.weight_decay * p;
    const float w = hp.lerp_weight;
    if (fabsf(w) < 0.5f) {
        const float d = g - m;
        m = (arith & ADAM_FMA_LERP) ? fmaf(w, d, m) : m + w * d;
    } else {
        const float d = g - m, omw = 1.0f - w;
        m = (arith & ADAM_FMA_LERP) ? fmaf(-d, omw, g) : g - d * omw;
    }
    v = v * hp.beta2;
    const float gg = g * g;
    v = (arith & ADAM_FMA_ADDCMUL) ? fmaf(hp.one_minus_beta2, gg, v) : v + hp.one_minus_beta2 * gg;
    float den = sqrtf(v);
    den = den / bc2;
    den = den + hp.eps;
    const float q = m / den;
    p = (arith & ADAM_FMA_ADDCDIV) ? fmaf(step_size, q, p) : p + step_size * q;
}

__global__ __launch_bounds__(ADAM_THREADS) void adam_step_kernel(const AdamLaunch L) {
    const int blk = blockIdx.x;
    int ti = 0;
    while (ti + 1 < L.count && blk >= L.first_block[ti + 1]) ++ti;
    const mbrl_adam_tensor& T = L.t[ti];
    const int64_t base = (int64_t)(blk - L.first_block[ti]) * ADAM_CHUNK;
    const int64_t i0 = base + 4 * (int64_t)threadIdx.x;
    if (i0 >= T.numel) return;
    const float ss = T.step_size, bc2 = T.bc2_sqrt;
    const bool vec = i0 + 4 <= T.numel &&
                     ((reinterpret_cast<uintptr_t>(T.param) | reinterpret_cast<uintptr_t>(T.grad) |
                       reinterpret_cast<uintptr_t>(T.exp_avg) | reinterpret_cast<uintptr_t>(T.exp_avg_sq)) & 15) == 0;
    if (vec) {
        float4 p = *reinterpret_cast<const float4*>(T.param + i0);
        const float4 g = *reinterpret_cast<const float4*>(T.grad + i0);
        float4 m = *reinterpret_cast<const float4*>(T.exp_avg + i0);
        float4 v = *reinterpret_cast<const float4*>(T.exp_avg_sq + i0);
        adam_element(p.x, g.x, m.x, v.x, ss, bc2, L.hp, L.arith);
        adam_element(p.y, g.y, m.y, v.y, ss, bc2, L.hp, L.arith);
        adam_element(p.z, g.z, m.z, v.z, ss, bc2, L.hp, L.arith);
        adam_element(p.w, g.w, m.w, v.w, ss, bc2, L.hp, L.arith);
        *reinterpret_cast<float4*>(T.param + i0) = p;
        *reinterpret_cast<float4*>(T.exp_avg + i0) = m;
        *reinterpret_cast<float4*>(T.exp_avg_sq + i0) = v;
        return;
    }
    for (int64_t i = i0; i < i0 + 4 && i < T.numel; ++i) {
        float p = T.param[i], m = T.exp_avg[i], v = T.exp_avg_sq[i];
        adam_element(p, T.grad[i], m, v, ss, bc2, L.hp, L.arith);
        T.param[i] = p;
        T.exp_avg[i] = m;
        T.exp_avg_sq[i] = v;
    }
}

hipError_t launch_adam_step(const mbrl_adam_tensor* tensors, int count, const mbrl_adam_hparams& hp, int arith,
                            hipStream_t stream) {
    AdamLaunch L{};
    L.hp = hp;
    L.arith = arith;
    int blocks = 0;
    for (int i = 0; i <= count; ++i) {
        // launch when the table is full or the tensors are exhausted
        if (L.count == ADAM_MAX_TENSORS || (i == count && L.count > 0)) {
            L.first_block[L.count] = blocks;
            hipLaunchKernelGGL(adam_step_kernel, dim3(blocks), dim3(ADAM_THREADS), 0, stream, L);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
            L.count = 0;
            blocks = 0;
        }
        if (i == count || tensors[i].numel <= 0) continue;
        L.t[L.count] = tensors[i];
        L.first_block[L.count] = blocks;
        blocks += (int)((tensors[i].numel + ADAM_CHUNK - 1) / ADAM_CHUNK);
        ++L.count;
    }
    return hipSuccess;
}

// ================================================================================================
// Model training forward + backward (mbrl_train_grads): the gradient of the reference's per-batch
// loss (models.py:65-85 / 188-207: MSELoss of the predicted next state, plus the reward head's for
// ModelWithReward, summed over the horizon steps) with respect to every Linear of the MLP, as
// n_hidden + 2 launches of one tiled fp32 MFMA kernel instead of autograd's chain of library GEMMs,
// elementwise kernels and reductions.
//
// Every launch computes one or two products C = A . B^T over 32 x 32 tiles of C, one tile per
// workgroup: 4 or 16 waves split K, each accumulating a 32 x 32 partial with v_mfma_f32_16x16x4f32
// (lane l feeds A(m0 + l%16, k) and B(n0 + l%16, k) for k = kb + 4(l/16) + s, s = 0..3, so a lane's
// four k are consecutive and one float4 load serves four MFMAs when the operand is k-contiguous).
// The partials meet in LDS, summed in wave order, and the epilogue fuses what follows the product:
//   forward        H_l = relu(A W_l^T + b_l)                                  (EPI_ACT)
//   output layer   Y = H W_out^T + b_out;  dY = (Y - target) * 2 / numel, loss partials (EPI_LOSS)
//   backward dX    dH_{l-1} = (dH_l W_l) * (H_{l-1} > 0)                        (EPI_MASK)
//   backward dW    dW_l = dH_l^T H_{l-1}, db_l from column sums the dH / dY launch left per
//                  row tile                                                     (EPI_GRAD)
// The batch is gathered on the fly from the stacked transitions through the batch's row indices
// (no materialised input), and the state and reward heads are one output layer of s + 1 rows.
// Arithmetic is fp32 with fp32 accumulation; the summation order differs from autograd's, so the
// gradients agree with torch's to rounding (tests/test_gpu_train_native.py), not bit for bit.

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Diagnostic build only (-DMBRL_STAMPS): s_memrealtime (100 MHz) at fixed points of the first and
// the last workgroup of each launch, 8 slots per launch, into the buffer set by
// mbrl_diag_set_train_stamps() (tools/train_stamps.py).
#ifdef MBRL_STAMPS
__device__ unsigned long long* g_train_stamps;
#define TSTAMP(k)                                                                                    \
    do {                                                                                             \
        const unsigned probe_ = L.nd > 1 ? (unsigned)L.d[0].tiles : gridDim.x - 1;                 \
        if (g_train_stamps && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == probe_))        \
            g_train_stamps[L.slot * 8 + (blockIdx.x == 0 ? 0 : 4) + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// the fused kernels: slot `slot_`, first workgroup and the last
#define FSTAMP(slot_, k)                                                                             \
    do {                                                                                             \
        if (g_train_stamps && threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1)) \
            g_train_stamps[(slot_) * 8 + (blockIdx.x == 0 ? 0 : 4) + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define TSTAMP(k) \
    do {          \
    } while (0)
#define FSTAMP(slot_, k) \
    do {                 \
    } while (0)
#endif

enum { OP_DIRECT = 0, OP_TRANS = 1, OP_GATHER = 2 };
enum { EPI_ACT = 0, EPI_LOSS = 1, EPI_MASK = 2, EPI_GRAD = 3 };
constexpr int TT = 32;              // C tile edge
constexpr int ADAM_FUSED_MAX = 4;   // tensors per fused Adam role (a layer's weight and bias, or both heads')
constexpr int FOLD_K0MAX = 64;      // the dW_0 fold stages its tile's input rows in LDS up to this K0

// Logical operand X(i, k), i < rows, k < K, over a row-major storage matrix S whose rows below
// `split` live at p0 and the rest at p1 (the state and reward heads as one matrix).
struct Operand {
    const float* p0;
    const float* p1;
    int split, ld;
    int kind;          // OP_DIRECT: X(i,k) = S[i][k]   OP_TRANS: X(i,k) = S[k][i]   OP_GATHER: batch input
    int rows;          // extent of i (including the ones row)
    int ones_row;      // i == ones_row reads 1 (the bias-gradient column); -1: none
    int gather_trans;  // OP_GATHER: 0: X(i,k) = input[row i][col k]; 1: X(i,k) = input[row k][col i]
    int vec;           // OP_DIRECT: rows 16-byte aligned (float4 loads)
};

struct Output {
    int mode;
    float* c0;
    float* c1;
    int split, ldc;           // C[m][n]: m < split -> c0[m*ldc + n], else c1[(m - split)*ldc + n]
    const float* b0;          // EPI_ACT / EPI_LOSS bias by column: n < bsplit ? b0[n] : b1[n - bsplit]
    const float* b1;
    int bsplit;
    int relu;
    const float* mask;        // EPI_MASK: C *= (mask[m*ldm + n] > 0)
    int ldm;
    float* g0;                // EPI_GRAD: the bias gradient, g0[m] / g1[m - split], from colsum_in
    float* g1;
    const float* colsum_in;   // EPI_GRAD: [colsum_tiles][M] column sums of this layer's output gradient
                              // (NULL: the bias gradient is finished elsewhere -- the fused step's O)
    int colsum_tiles;
    float* colsum_out;        // EPI_MASK / EPI_LOSS: [row tile][N] column sums of the stored C
    int adam;                 // EPI_GRAD: also take this layer's Adam step in place (nothing reads it
                              // in this launch): weight at aw (= c0 layout), bias at ab
    mbrl_adam_tensor aw, ab;
    // EPI_GRAD with adam, fused step: this launch's dH tiles read the weight block being stepped; the
    // tile waits until wait_ticket[n0 / 32] (their arrivals per column block) reaches wait_count.
    // Those tiles have lower workgroup ids, so they were dispatched first and always finish; the
    // bounded spin only guards against a hang (bit 0 of wait_status on timeout).
    const unsigned* wait_ticket;
    unsigned wait_count;
    unsigned* wait_status;
    unsigned* arrive_ticket;  // EPI_MASK, fused step: one add per tile to [n0 / 32] once its K loop (every
                              // read of the weight block) is done -- what wait_ticket counts
    // EPI_MASK of dH_0 with fold (launch_train_grads): the tile also yields the layer-0 weight
    // gradient's partial over each of its 32-row blocks -- exactly what wave tr of the separate dW_0
    // launch summed -- as tagged granules (fold_gran below); the dW_1 tiles of row block 0 add them
    // in wave order into dW_0 / db_0 and take layer 0's Adam step (fold_sum)
    int fold, fold_k0, fold_nw;         // input columns K0, the separate launch's wave count
    const float* fold_x;                // the gathered input [R][K0] (xbuf, written by the forward)
    float *fold_dw, *fold_db;           // dW_0 [W][K0], db_0 [W]
    int fold_cs_tiles;                  // 32-row tiles of the column sums (colsum_out of this product)
    int fold_adam;
    mbrl_adam_tensor fold_aw, fold_ab;
    // the fold's hand-off as tagged granules {value, tag} (8-byte stores, read untorn): the partials
    // [tr][W][K0] and the column sums [tr][W] of dH_0, tag = the step's serial (*fold_serial, raised
    // by the step's first launch); the dW_1 tiles of row block 0 (fold_sum) poll them and finish
    // dW_0 / db_0 and layer 0's Adam step. No drain, ticket or last arriver on the producers' side.
    unsigned long long *fold_gran, *cs_gran;
    const unsigned* fold_serial;
    unsigned* fold_status;              // bit 0: a bounded wait timed out
    int fold_sum;                       // EPI_GRAD (dW_1): row block 0's tiles run fold_sum
    float scale_s, scale_r;   // EPI_LOSS: dY scale of the state / reward columns (2 / numel)
    float inv_s, inv_r;       // EPI_LOSS: loss weight of the state / reward columns (1 / numel)
    int s;                    // EPI_LOSS: state columns (n >= s: the reward column)
    float* loss_part;         // EPI_LOSS: [tile][2] partial losses (state, reward)
};

struct GemmDesc {
    Operand A, B;
    Output out;
    int M, N, K, tiles_n, tiles;
};

struct GemmLaunch {
    GemmDesc d[2];
    int nd;
    // the batch: row r of the logical input is transition idx[r / H], horizon step r % H
    const int64_t* idx;
    const float* gs;    // stacked states      [T][H][s]
    const float* ga;    // stacked actions     [T][H][a]
    const float* gns;   // stacked next states [T][H][s]
    const float* grw;   // stacked rewards     [T][H]
    int H, s, a;
    float* xstore;      // [rows][s + a]: the gathered input, written by the layer-0 forward launch
    int slot;           // launch index within the step (diagnostic stamps)
    // loss: one extra workgroup sums the partials (fixed order) into loss_out[0..2]
    const float* loss_part;
    int loss_parts;
    float* loss_out;
    // fused Adam (mbrl_train_epoch): the step of a layer whose gradient the previous launch finished,
    // as extra workgroups after the products' tiles (ADAM_FUSED_CHUNK elements each)
    int adam_count, adam_blocks, adam_chunk;   // adam_chunk: elements per Adam workgroup
    mbrl_adam_tensor adam_t[ADAM_FUSED_MAX];
    unsigned* zero_words;   // workgroup 0 zeroes zero_n words first (the fold's tickets; forward launch)
    int zero_n;
    unsigned* serial;       // workgroup 0 raises the step's serial (the fold's granule tag; forward launch)
    int adam_first[ADAM_FUSED_MAX + 1];
    mbrl_adam_hparams hp;
    int arith;
    // product 0's tiles in XCD order (MBRL_OPT_TRAIN_XCD): every 64-row band of the batch on XCD
    // (band % 8) in every launch, so a launch reads the rows the previous launch wrote on its own XCD
    int xcd;
};

__device__ __forceinline__ int64_t batch_row(const GemmLaunch& L, int r) {
    return L.idx[r / L.H] * L.H + r % L.H;
}

__device__ __forceinline__ float input_at(const GemmLaunch& L, int r, int c) {
    const int64_t src = batch_row(L, r);
    return c < L.s ? L.gs[src * L.s + c] : L.ga[src * L.a + (c - L.s)];
}

__device__ __forceinline__ const float* storage_row(const Operand& o, int row) {
    return row < o.split ? o.p0 + (int64_t)row * o.ld : o.p1 + (int64_t)(row - o.split) * o.ld;
}

template <int KIND>
__device__ __forceinline__ f32x4 load_operand(const GemmLaunch& L, const Operand& o, int i, int k0, int K) {
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
    if (i >= o.rows) return v;
    if (i == o.ones_row) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = k0 + e < K ? 1.0f : 0.0f;
        return v;
    }
    if constexpr (KIND == OP_DIRECT) {
        const float* row = storage_row(o, i);
        if (o.vec && k0 + 3 < K) return *reinterpret_cast<const f32x4*>(row + k0);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (k0 + e < K) v[e] = row[k0 + e];
    } else if constexpr (KIND == OP_TRANS) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (k0 + e < K) v[e] = storage_row(o, k0 + e)[i];
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (k0 + e < K) v[e] = o.gather_trans ? input_at(L, k0 + e, i) : input_at(L, i, k0 + e);
    }
    return v;
}

// Whether a lane's 4 columns of chunk kb lie inside K on a row-contiguous operand: one 16-byte load.
template <int KIND>
__device__ __forceinline__ bool staged_vec(const Operand& o, int kb, int K) {
    return KIND == OP_DIRECT && o.vec && kb + 16 <= K;
}

// Branch-free operand loads (OP_DIRECT / OP_TRANS): every lane loads from a valid address -- its own
// element, or the operand's first element where it has none -- and the value is masked once all of
// the chunk's loads are in flight (mask_raw). load_operand's guarded loads compile to divergent
// branches, and hipcc closes each join with vmcnt(0): one memory round trip per fragment.
template <int KIND>
__device__ __forceinline__ f32x4 load_raw(const Operand& o, int i, int kb, int k0, int K) {
    const bool row_ok = i < o.rows && i != o.ones_row;
    if (staged_vec<KIND>(o, kb, K)) {
        const float* g = row_ok ? storage_row(o, i) + k0 : o.p0;
        return *reinterpret_cast<const f32x4*>(g);
    }
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float* g = o.p0;
        if (row_ok && k0 + e < K) {
            if constexpr (KIND == OP_DIRECT) g = storage_row(o, i) + k0 + e;
            else g = storage_row(o, k0 + e) + i;
        }
        v[e] = *g;
    }
    return v;
}

template <int KIND>
__device__ __forceinline__ f32x4 mask_raw(const Operand& o, int i, int kb, int k0, int K, f32x4 v) {
    if (i >= o.rows) return f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (i == o.ones_row) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = k0 + e < K ? 1.0f : 0.0f;
        return v;
    }
    if (!staged_vec<KIND>(o, kb, K))
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (!(k0 + e < K)) v[e] = 0.0f;
    return v;
}

// The gathered batch input, kept for the layer-0 weight gradient (fwd0 writes it as it loads it).
__device__ __forceinline__ void stash_input(const GemmLaunch& L, const GemmDesc& D, const f32x4& v, int m, int k0) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (m < D.M && k0 + e < D.K) L.xstore[(int64_t)m * D.K + k0 + e] = v[e];
}

template <int NW, int TMX, int DI>
__device__ __forceinline__ void fold_dw0(const GemmLaunch& L, int tm, int n0, float (*red)[TT * TMX][TT + 1],
                                         const float (*xs)[FOLD_K0MAX]);
template <int NW>
__device__ __forceinline__ void fold_sum(const GemmLaunch& L, int n0);

// A tagged granule {value, tag}: one 8-byte store, read untorn (MI355X_MICROARCH.md, granules)
__device__ __forceinline__ unsigned long long granule(float v, unsigned tag) {
    return ((unsigned long long)tag << 32) | __float_as_uint(v);
}

// p[0] + p[stride] + ... + p[(n - 1) stride], summed in index order like a plain loop, with the loads
// of each 16 terms in flight together (a loop that loads one term per iteration pays the memory
// latency n times: ~10 us for the 16 row tiles of a bias gradient). SC1: agent-scope (sc1) loads.
template <bool SC1>
__device__ __forceinline__ float ordered_sum(const float* p, int64_t stride, int n) {
    float g = 0.0f;
    for (int i0 = 0; i0 < n; i0 += 16) {
        float t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const float* a = p + (int64_t)(i0 + u) * stride;
            t[u] = i0 + u >= n ? 0.0f
                   : SC1       ? __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : *a;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (i0 + u < n) g = i0 + u == 0 ? t[u] : g + t[u];
    }
    return g;
}

// One lane polls an arrival counter (sc1 loads) until it reaches `need`, then the workgroup goes on.
// Used only where the awaited workgroups have lower ids than the waiter (dispatched before it), so the
// wait always ends; the 1 s bound (s_memrealtime, 100 MHz) turns a broken assumption into bit 0 of
// *status instead of a hang.
__device__ __forceinline__ void wait_arrivals(const unsigned* counter, unsigned need, unsigned* status) {
    if (threadIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
                if (status) atomicOr(status, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

// TMX = 1: 32 x 32 C tiles; TMX = 2: 64 x 32 (the W x W backward products, so that a launch's tiles
// fit one round of the CUs). Each element's K order is the same for both (the K split over the waves
// depends on K and NW only), so the tile height never changes a bit of the result.
// DI: which of the launch's products, a constant index into the kernel arguments. Always inlined: a
// call that is not would take the argument block's address, and the compiler copies the whole block
// (1.5 KB) to scratch per lane for that (the 4-wave backward launch did until r04).
template <int NW, int AK, int BK, int TMX, int DI>
__device__ __forceinline__ void gemm_tile(const GemmLaunch& L, int tile, float (*red)[TT * TMX][TT + 1],
                                          float (*xs)[FOLD_K0MAX]) {
    const GemmDesc& D = L.d[DI];
    constexpr int NT = 64 * NW;
    constexpr int TM = TT * TMX;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4, c = lane & 15;
    const int tm = tile / D.tiles_n, m0 = tm * TM, n0 = (tile % D.tiles_n) * TT;
    const bool stash = AK == OP_GATHER && L.xstore != nullptr && n0 == 0;
    // wave w takes the w-th of NW contiguous K ranges (in 16-deep chunks): a few chunks per wave, so
    // the loads' latency is paid about once per wave instead of once per chunk
    const int chunks = (D.K + 15) >> 4, per = (chunks + NW - 1) / NW;
    const int kb0 = wave * per * 16, kb1 = min(D.K, (wave + 1) * per * 16);
    f32x4 acc[2 * TMX][2];
#pragma unroll
    for (int x = 0; x < 2 * TMX; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // the epilogue's own operands (bias, ReLU mask, loss targets) are fetched before the K loop so
    // their latency overlaps the products'
    const Output& O = D.out;
    constexpr int EPT = TM * TT / NT;       // C elements per thread in the epilogue
    float pre[EPT], ap[EPT], am[EPT], av[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const int e = tid + j * NT, m = m0 + (e >> 5), n = n0 + (e & 31);
        pre[j] = ap[j] = am[j] = av[j] = 0.0f;
        if (m >= D.M || n >= D.N) continue;
        if (O.mode == EPI_ACT) pre[j] = n < O.bsplit ? O.b0[n] : O.b1[n - O.bsplit];
        else if (O.mode == EPI_MASK) pre[j] = O.mask[(int64_t)m * O.ldm + n];
        else if (O.mode == EPI_GRAD && O.adam) {   // the in-place Adam step's operands (only this tile
            const int64_t i = (int64_t)m * O.ldc + n;   // writes them; the weight is only read by others)
            ap[j] = O.aw.param[i];
            am[j] = O.aw.exp_avg[i];
            av[j] = O.aw.exp_avg_sq[i];
        }
        else if (O.mode == EPI_LOSS) {
            const int64_t src = batch_row(L, m);
            const float t = n < O.s ? L.gns[src * O.s + n] : L.grw[src];
            pre[j] = t - (n < O.bsplit ? O.b0[n] : O.b1[n - O.bsplit]);   // y - t = acc - (t - bias)
        }
    }
    // the dW_0 fold's operand, the tile's rows of the gathered input: loaded now, into LDS after the
    // K loop (its latency then hides behind the products')
    constexpr int XPT = TM * FOLD_K0MAX / NT;
    float xv[XPT];
    const bool xstage = O.mode == EPI_MASK && O.fold && O.fold_k0 <= FOLD_K0MAX;
    if (xstage) {
#pragma unroll
        for (int j = 0; j < XPT; ++j) {
            const int e = tid + j * NT, r = e / FOLD_K0MAX, k = e % FOLD_K0MAX;
            xv[j] = (k < O.fold_k0 && m0 + r < D.M) ? O.fold_x[(int64_t)(m0 + r) * O.fold_k0 + k] : 0.0f;
        }
    }
    // (stamp slots: 0 entry, 1 K loop done, 2 after the reduction barrier / arrival wait, 3 exit)
    // up to GROUP chunks' operands in flight at once, then their MFMAs: with the usual 1-4 chunks
    // per wave the loads' latency is paid once
    constexpr int GROUP = NW == 16 ? (TMX == 2 ? 1 : 2) : NW == 8 ? 2 : 4;   // TMX 2 at 16 waves: the 128-VGPR budget
    int g0 = kb0;
    constexpr bool RAW = AK != OP_GATHER && BK != OP_GATHER;   // branch-free loads (load_raw / mask_raw)
    for (; g0 < kb1; g0 += 16 * GROUP) {
        f32x4 a[GROUP][2 * TMX], b[GROUP][2];
#pragma unroll
        for (int u = 0; u < GROUP; ++u) {
            const int kb = g0 + 16 * u;
            if (kb >= kb1) break;
            if constexpr (RAW) {
#pragma unroll
                for (int x = 0; x < 2 * TMX; ++x) a[u][x] = load_raw<AK>(D.A, m0 + 16 * x + c, kb, kb + 4 * q, D.K);
#pragma unroll
                for (int y = 0; y < 2; ++y) b[u][y] = load_raw<BK>(D.B, n0 + 16 * y + c, kb, kb + 4 * q, D.K);
            } else {
#pragma unroll
                for (int x = 0; x < 2 * TMX; ++x) {
                    a[u][x] = load_operand<AK>(L, D.A, m0 + 16 * x + c, kb + 4 * q, D.K);
                    if (stash) stash_input(L, D, a[u][x], m0 + 16 * x + c, kb + 4 * q);
                }
#pragma unroll
                for (int y = 0; y < 2; ++y) b[u][y] = load_operand<BK>(L, D.B, n0 + 16 * y + c, kb + 4 * q, D.K);
            }
        }
        if constexpr (RAW) {
#pragma unroll
            for (int u = 0; u < GROUP; ++u) {   // the masks, once every load of the group is in flight
                const int kb = g0 + 16 * u;
                if (kb >= kb1) break;
#pragma unroll
                for (int x = 0; x < 2 * TMX; ++x) a[u][x] = mask_raw<AK>(D.A, m0 + 16 * x + c, kb, kb + 4 * q, D.K, a[u][x]);
#pragma unroll
                for (int y = 0; y < 2; ++y) b[u][y] = mask_raw<BK>(D.B, n0 + 16 * y + c, kb, kb + 4 * q, D.K, b[u][y]);
            }
        }
#pragma unroll
        for (int u = 0; u < GROUP; ++u) {
            if (g0 + 16 * u >= kb1) break;
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int x = 0; x < 2 * TMX; ++x)
#pragma unroll
                    for (int y = 0; y < 2; ++y)
                        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][x][s], b[u][y][s], acc[x][y], 0, 0, 0);
        }
    }
    TSTAMP(1);
    // lane l holds C rows 16x + 4q + v, column 16y + c
#pragma unroll
    for (int x = 0; x < 2 * TMX; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int v = 0; v < 4; ++v) red[wave][16 * x + 4 * q + v][16 * y + c] = acc[x][y][v];
    if (xstage) {
#pragma unroll
        for (int j = 0; j < XPT; ++j) {
            const int e = tid + j * NT;
            xs[e / FOLD_K0MAX][e % FOLD_K0MAX] = xv[j];
        }
    }
    __syncthreads();
    // every wave's K loop is done: this tile no longer reads the weight block (its loads were consumed)
    if (O.mode == EPI_MASK && O.arrive_ticket && tid == 0)
        __hip_atomic_fetch_add(O.arrive_ticket + n0 / TT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    if (O.mode == EPI_GRAD && O.adam && O.wait_ticket)
        wait_arrivals(O.wait_ticket + n0 / TT, O.wait_count, O.wait_status);
    TSTAMP(2);

    // the fused epilogue, EPT C elements per thread; each element sums the waves' partials in wave
    // order. Elements of this tile that feed the next layer's bias gradient (EPI_MASK, EPI_LOSS)
    // are kept for the column sums below.
    float loss_s = 0.0f, loss_r = 0.0f;
    float keep[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const int e = tid + j * NT, row = e >> 5, col = e & 31, m = m0 + row, n = n0 + col;
        keep[j] = 0.0f;
        if (m >= D.M || n >= D.N) continue;
        float v = red[0][row][col];
#pragma unroll
        for (int w = 1; w < NW; ++w) v = v + red[w][row][col];
        if (O.mode == EPI_ACT) v = v + pre[j];
        if (O.mode == EPI_ACT && O.relu) v = v > 0.0f ? v : 0.0f;
        if (O.mode == EPI_MASK && !(pre[j] > 0.0f)) v = 0.0f;
        if (O.mode == EPI_LOSS) {
            const float d = v - pre[j];
            if (n < O.s) loss_s = loss_s + d * d * O.inv_s;
            else loss_r = loss_r + d * d * O.inv_r;
            v = d * (n < O.s ? O.scale_s : O.scale_r);
        }
        keep[j] = v;
        // (with the dW_0 fold nothing reads dH_0 after this launch: its tiles keep it in LDS only)
        if (!(O.mode == EPI_MASK && O.fold)) {
            float* dst = m < O.split ? O.c0 + (int64_t)m * O.ldc : O.c1 + (int64_t)(m - O.split) * O.ldc;
            dst[n] = v;
        }
        if (O.mode == EPI_GRAD && O.adam) {
            const int64_t i = (int64_t)m * O.ldc + n;
            adam_element(ap[j], v, am[j], av[j], O.aw.step_size, O.aw.bc2_sqrt, L.hp, L.arith);
            O.aw.param[i] = ap[j];
            O.aw.exp_avg[i] = am[j];
            O.aw.exp_avg_sq[i] = av[j];
        }
    }
    // EPI_GRAD: the first column tile also finishes the bias gradient of each row m from the column
    // sums the launch that produced this layer's output gradient left per row tile
    if (O.mode == EPI_GRAD && O.colsum_in && n0 == 0 && tid < TM && m0 + tid < D.M) {
        const int m = m0 + tid;
        const float g = ordered_sum<false>(O.colsum_in + m, D.M, O.colsum_tiles);
        (m < O.split ? O.g0[m] : O.g1[m - O.split]) = g;
        if (O.adam)
            adam_element(O.ab.param[m], g, O.ab.exp_avg[m], O.ab.exp_avg_sq[m], O.ab.step_size, O.ab.bc2_sqrt, L.hp,
                         L.arith);
    }
    if (O.mode == EPI_MASK || O.mode == EPI_LOSS) {   // per-32-row-tile column sums (the next bias gradient)
        __syncthreads();
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = tid + j * NT;
            red[0][e >> 5][e & 31] = keep[j];
        }
        __syncthreads();
        const int sub = tid / TT, col = tid - (tid / TT) * TT;
        if (tid < TM && n0 + col < D.N && m0 + TT * sub < D.M) {
            float t = red[0][TT * sub][col];
            for (int r = 1; r < TT; ++r) t = t + red[0][TT * sub + r][col];
            const int64_t di = (int64_t)(tm * TMX + sub) * D.N + n0 + col;
            if (O.fold)   // read by fold_sum (dW_1 tile (0, n0 / 32)) as a tagged granule
                __hip_atomic_store(O.cs_gran + di, granule(t, *O.fold_serial), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            else
                O.colsum_out[di] = t;
        }
        if (O.mode == EPI_MASK && O.fold) fold_dw0<NW, TMX, DI>(L, tm, n0, red, xs);
    }
    if (O.mode == EPI_GRAD && O.fold_sum && tm == 0) fold_sum<NW>(L, n0);
    if (O.mode == EPI_LOSS) {   // the tile's loss: a butterfly per wave, then the waves in order
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            loss_s += __shfl_xor(loss_s, o);
            loss_r += __shfl_xor(loss_r, o);
        }
        __syncthreads();        // red is reused
        float* sl = &red[1][0][0];
        if (lane == 0) {
            sl[2 * wave] = loss_s;
            sl[2 * wave + 1] = loss_r;
        }
        __syncthreads();
        if (tid < 2) {
            float t = sl[tid];
            for (int w = 1; w < NW; ++w) t = t + sl[2 * w + tid];
            O.loss_part[tile * 2 + tid] = t;
        }
    }
    TSTAMP(3);
}

// The layer-0 weight gradient folded into the dH_0 launch (Output.fold). red[0] holds this tile's
// dH_0 rows [m0, m0 + TM) x columns [n0, n0 + 32) (the EPI_MASK column-sum staging). The separate
// dW_0 launch (M = W, N = K0, K = R, fold_nw waves of 32 rows each) computed, per wave tr, one 32 x 32
// block of dW_0 over rows [32 tr, 32 tr + 32) with acc[x][y] over 16-row chunks u, k = 4 q + s: the
// same loads and MFMAs in the same order run here per 32-row half of the tile, so every partial is
// the same float; they leave as tagged granules, and fold_sum (a dW_1 tile of the same launch) adds
// them in wave order with the empty waves' +0 -- the separate launch's result bit for bit.
template <int NW, int TMX, int DI>
__device__ __forceinline__ void fold_dw0(const GemmLaunch& L, int tm, int n0, float (*red)[TT * TMX][TT + 1],
                                         const float (*xs)[FOLD_K0MAX]) {
    const GemmDesc& D = L.d[DI];
    constexpr int TM = TT * TMX;
    (void)TM;
    const Output& O = D.out;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
    const int R = D.M, W = D.N, K0 = O.fold_k0, m0 = tm * TT * TMX;
    const int kt = (K0 + TT - 1) / TT;
    const unsigned tag = *O.fold_serial;
    for (int task = wave; task < TMX * kt; task += NW) {
        const int h = task / kt, kb = task - (task / kt) * kt;
        const int r0 = m0 + TT * h;
        if (r0 >= R) continue;
        const int r1 = min(R, r0 + TT);
        f32x4 acc[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k0 = r0 + 16 * u;
            if (k0 >= r1) break;
            f32x4 a[2], b[2];
#pragma unroll
            for (int x = 0; x < 2; ++x) {          // A(i = j, k = r) = dH_0[r][j]
                const int j = 16 * x + c;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = k0 + 4 * q + e;
                    a[x][e] = (n0 + j < W && r < R) ? red[0][r - m0][j] : 0.0f;
                }
            }
#pragma unroll
            for (int y = 0; y < 2; ++y) {          // B(i = k, k = r) = X[r][k]
                const int kk = TT * kb + 16 * y + c;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = k0 + 4 * q + e;
                    b[y][e] = (kk < K0 && r < R) ? (K0 <= FOLD_K0MAX ? xs[r - m0][kk] : O.fold_x[(int64_t)r * K0 + kk])
                                                 : 0.0f;
                }
            }
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int x = 0; x < 2; ++x)
#pragma unroll
                    for (int y = 0; y < 2; ++y)
                        acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x][s], b[y][s], acc[x][y], 0, 0, 0);
        }
        const int tr = r0 / TT;
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int j = n0 + 16 * x + 4 * q + v, kk = TT * kb + 16 * y + c;
                    if (j < W && kk < K0)    // read by fold_sum as a tagged granule: nothing to drain
                        __hip_atomic_store(O.fold_gran + ((int64_t)tr * W + j) * K0 + kk, granule(acc[x][y][v], tag),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
    }
}

// The fold's sums, in the dW_1 tile (0, n0 / 32) of the same launch (higher workgroup ids than every
// dH_0 tile, so those were dispatched first and always finish): the column block's per-32-row partials
// added in wave order with the empty waves' +0 -- the separate dW_0 launch's sum, bit for bit -- and
// db_0 from the column sums over the 32-row tiles, then layer 0's Adam step. Each lane loads all of its
// granules at once and reloads the ones whose tag is not yet this step's (bounded: 1 s, then bit 0 of
// the status word).
template <int NW>
__device__ __forceinline__ bool poll_granules(const unsigned long long* const* p, int n, unsigned tag, float* out,
                                              unsigned* status) {
    unsigned long long g[16];
    unsigned need = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        out[i] = 0.0f;
        if (i < n) need |= 1u << i;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (need) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            g[i] = ((need >> i) & 1u) ? __hip_atomic_load(p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (((need >> i) & 1u) && (unsigned)(g[i] >> 32) == tag) {
                out[i] = __uint_as_float((unsigned)g[i]);
                need &= ~(1u << i);
            }
        if (!need) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
            if (status) atomicOr(status, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

template <int NW>
__device__ __forceinline__ void fold_sum(const GemmLaunch& L, int n0) {
    const GemmDesc& D = L.d[0];
    const Output& O = D.out;
    const int tid = threadIdx.x;
    const int R = D.M, W = D.N, K0 = O.fold_k0;
    const int ntr = (R + TT - 1) / TT;      // non-empty waves of the separate launch
    const unsigned tag = *O.fold_serial;
    constexpr int NT = 64 * NW;
    const bool dbt = tid < TT && n0 + tid < W;
    // the Adam operands of this column block first: their latency overlaps the polls
    float bp = 0.0f, bm = 0.0f, bv = 0.0f;
    if (O.fold_adam && dbt) {
        bp = O.fold_ab.param[n0 + tid];
        bm = O.fold_ab.exp_avg[n0 + tid];
        bv = O.fold_ab.exp_avg_sq[n0 + tid];
    }
    for (int e0 = 0; e0 < TT * K0; e0 += NT) {
        const int e = e0 + tid, j = n0 + e / K0, kk = e - (e / K0) * K0;
        const bool in = e < TT * K0 && j < W;
        const int64_t i = (int64_t)j * K0 + kk;
        float fp = 0.0f, fm = 0.0f, fv = 0.0f;
        if (in && O.fold_adam) {
            fp = O.fold_aw.param[i];
            fm = O.fold_aw.exp_avg[i];
            fv = O.fold_aw.exp_avg_sq[i];
        }
        const unsigned long long* ptr[16];
        const int np = in ? min(ntr, O.fold_nw) : 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) ptr[w] = O.fold_gran + ((int64_t)min(w, max(np - 1, 0)) * W + j) * K0 + kk;
        float p[16];
        poll_granules<NW>(ptr, np, tag, p, O.fold_status);
        if (!in) continue;
        float v = p[0];
#pragma unroll
        for (int w = 1; w < 16; ++w)
            if (w < O.fold_nw) v = v + p[w];
        O.fold_dw[i] = v;
        if (O.fold_adam) {
            adam_element(fp, v, fm, fv, O.fold_aw.step_size, O.fold_aw.bc2_sqrt, L.hp, L.arith);
            O.fold_aw.param[i] = fp;
            O.fold_aw.exp_avg[i] = fm;
            O.fold_aw.exp_avg_sq[i] = fv;
        }
    }
    if (tid < 64) {                          // db_0: the column sums of dH_0 over the 32-row tiles
        const int j = n0 + tid;
        const unsigned long long* ptr[16];
        const int np = dbt ? min(O.fold_cs_tiles, 16) : 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) ptr[i] = O.cs_gran + (int64_t)min(i, max(np - 1, 0)) * W + min(j, W - 1);
        float cs[16];
        poll_granules<NW>(ptr, np, tag, cs, O.fold_status);
        if (dbt) {
            float g = cs[0];
#pragma unroll
            for (int i = 1; i < 16; ++i)
                if (i < O.fold_cs_tiles) g = g + cs[i];
            O.fold_db[j] = g;
            if (O.fold_adam) {
                adam_element(bp, g, bm, bv, O.fold_ab.step_size, O.fold_ab.bc2_sqrt, L.hp, L.arith);
                O.fold_ab.param[j] = bp;
                O.fold_ab.exp_avg[j] = bm;
                O.fold_ab.exp_avg_sq[j] = bv;
            }
        }
    }
}

// NW waves per workgroup; A0/B0 (A1/B1): operand kinds of the launch's first (second) product, fixed
// at compile time so each instantiation carries only its own load paths.
template <int NW, int A0, int B0, int A1, int B1, int TMX>
__global__ __launch_bounds__(64 * NW) void train_gemm_kernel(const GemmLaunch L) {
    __shared__ __attribute__((aligned(16))) float red[NW][TT * TMX][TT + 1];   // (16-B: the staged chunk's slots)
    __shared__ float xs[TT * TMX][FOLD_K0MAX];   // the dW_0 fold's input rows (dH_0 launches only)
    TSTAMP(0);
    // (constant indices only: a dynamic index into the kernel arguments would copy them to scratch)
    const int b = blockIdx.x;
    if (b == 0 && L.zero_words)
        for (int i = threadIdx.x; i < L.zero_n; i += 64 * NW) L.zero_words[i] = 0u;
    if (b == 0 && L.serial && threadIdx.x == 0) *L.serial = *L.serial + 1u;
    if (b < L.d[0].tiles) {
        int tile = b;
        if (L.xcd) {   // block b on XCD b % 8 (round-robin dispatch) takes a tile of a 64-row band of that XCD
            constexpr int G = 2 / TMX;                    // tile rows per 64-row band
            const int tn_all = L.d[0].tiles_n, per = G * tn_all, x = b & 7, j = b >> 3;
            const int u = j / per, r = j - u * per;
            tile = ((x + 8 * u) * G + r / tn_all) * tn_all + r % tn_all;
        }
        gemm_tile<NW, A0, B0, TMX, 0>(L, tile, red, xs);
        return;
    }
    int r = b - L.d[0].tiles;
    if constexpr (A1 >= 0) {
        if (L.nd > 1 && r < L.d[1].tiles) {
            gemm_tile<NW, A1, B1, TMX, 1>(L, r, red, xs);
            return;
        }
        if (L.nd > 1) r -= L.d[1].tiles;
    }
    if (r < L.adam_blocks) {    // fused Adam: ADAM_FUSED_CHUNK elements of one tensor per workgroup
        int ti = 0;
        while (ti + 1 < L.adam_count && r >= L.adam_first[ti + 1]) ++ti;
        const mbrl_adam_tensor& T = L.adam_t[ti];
        const int64_t base = (int64_t)(r - L.adam_first[ti]) * L.adam_chunk;
        for (int64_t i = base + threadIdx.x; i < T.numel && i < base + L.adam_chunk; i += 64 * NW)
            adam_element(T.param[i], T.grad[i], T.exp_avg[i], T.exp_avg_sq[i], T.step_size, T.bc2_sqrt, L.hp,
                         L.arith);
        return;
    }
    // the loss workgroup: partials of the output-layer launch, summed in tile order
    if (threadIdx.x < 2 && L.loss_out) {   // (loads 16 at a time in flight, sums in the same order)
        float t = 0.0f, u = 0.0f;
        for (int i0 = 0; i0 < L.loss_parts; i0 += 16) {
            float ps[16], pr[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const bool in = i0 + k < L.loss_parts;
                ps[k] = in ? L.loss_part[(i0 + k) * 2] : 0.0f;
                pr[k] = in ? L.loss_part[(i0 + k) * 2 + 1] : 0.0f;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (i0 + k < L.loss_parts) {
                    t = t + (threadIdx.x == 0 ? ps[k] : pr[k]);
                    u = u + ps[k] + pr[k];
                }
        }
        L.loss_out[1 + threadIdx.x] = t;
        if (threadIdx.x == 0) L.loss_out[0] = u;
    }
}

// ================================================================================================
// The fused step for two hidden layers (the reference's Model / ModelWithReward, models.py:97-132):
// three launches per batch instead of five. Every product is the same MFMA chains over the same K
// ranges as in the five-launch layout, and every sum of partials runs in the same order, so the
// gradients, losses and Adam steps are the same floats (tests/test_gpu_train_native.py pins it):
//   F  train_fused_fwd_kernel: per 32 x 32 tile of H_1, the tile's 32 rows of H_0 are recomputed into
//      LDS (K0 = s + a is small: the layer-0 launch's 4-wave K split, summed in its wave order), then
//      the H_1 tile is the layer-1 launch's tile with its A operand from LDS. Removes a launch and
//      the H_0 round trip through memory before the layer-1 products. The first column tiles also
//      gather the batch's targets for O; in mbrl_train_epoch the second column tiles gather the next
//      batch's rows and targets into the other gather slot.
//   O  train_fused_out_kernel: per 32 x 32 tile of dH_1, the tile's 32 rows of dY (the output-layer
//      launch's tile: loss partials and dY column sums from the first column tile), dH_1 =
//      (dY W_out) * (H_1 > 0), and the output layer's weight-gradient partial over the tile's 32 rows
//      -- exactly wave tm of the separate dW_out product -- summed in wave order by the column block's
//      last arriver (an sc1 hand-off), which also finishes db_out, db_1 and b_1's Adam step.
//      Removes a launch and the dY round trip.
//   B  launch_gemm: dH_0 with the folded dW_0 and its Adam step, dW_1 -- whose tiles step W_1 in place
//      once the dH_0 tiles of their column block have read it -- and the output layer's Adam step as
//      extra workgroups. No Adam step is deferred to the next batch.
constexpr int FUSED_WMAX = 512;    // H_0 rows of the tile in LDS: 32 x (W + 4) floats
constexpr int FUSED_K0MAX = 64;    // s + a: one 16-deep chunk per wave of the layer-0 launch's split

struct FusedArgs {
    const int64_t* idx;
    const float *gs, *ga, *gns, *grw;   // stacked transitions (GemmLaunch's meaning)
    int H, s, a;
    int R, W, K0, J, tiles_n, tiles_r;
    int nwb;                            // waves of the separate backward launches (K = R): the dH_1 split
    const float *w0, *b0, *w1, *b1;
    const float *wo, *wo_r, *bo, *bo_r; // output layer: state rows from wo / bo, the reward row from *_r
    float *act0, *act1, *xstore;
    float* tgt;                         // [R][J] the batch's targets, gathered by F's first column tiles for O
    int pre_rows;                       // 1: xstore / tgt already hold this batch (the previous F gathered it)
    const int64_t* idx_next;            // non-NULL: F's second column tiles gather the next batch's rows
    int R_next;                         //   (R_next of them) into xnext / tnext
    float *xnext, *tnext;
    float *dh1, *cs_dh1, *cs_dy, *loss_part, *out_part;
    float *dwo, *dwo_r, *dbo, *dbo_r;
    unsigned* out_ticket;               // [tiles_n] arrivals per column block of dH_1 tiles (O)
    float* db1;                         // O's last arrivers: db_1 from dH_1's column sums (+ b_1's Adam step)
    int adam;
    mbrl_adam_tensor ab1;
    mbrl_adam_hparams hp;
    int arith;
    unsigned* zero_words;               // F's workgroup 0 zeroes zero_n words (the tickets of later launches)
    int zero_n;
    unsigned* serial;                   // F's workgroup 0 raises the step's serial (B's granule tag)
    float scale_s, scale_r, inv_s, inv_r;
    // F and O in one launch (train_fused_fo_kernel): per 32-row band of the batch a counter (own 128-B
    // line) that the band's F tiles add to once their H_1 columns are written through; each O tile
    // waits for all tiles_n, then adds again, and the last add of the band resets it (zero between
    // launches, as the caller's once-zeroed workspace starts). status: bit 0 = a bounded wait timed out.
    unsigned* band;
    unsigned* status;
};

constexpr int TRAIN_SC1 = 16;   // buffer-op aux bit: sc1 (write-through stores, L1-bypassing loads)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// A wave's K range in a launch of nw waves (gemm_tile's split: contiguous 16-deep chunks).
__device__ __forceinline__ void wave_k_range(int K, int nw, int w, int& kb0, int& kb1) {
    const int chunks = (K + 15) >> 4, per = (chunks + nw - 1) / nw;
    kb0 = w * per * 16;
    kb1 = min(K, (w + 1) * per * 16);
}

// Four consecutive k of one row of a row-major matrix (row stride ld), zero past K or for an absent
// row: load_operand<OP_DIRECT>'s values (float4 when aligned, else element by element).
// (The guarded loads here measured faster than load_raw's branch-free form in F and O: 49.2-49.3
// against 50.0 us per step, late r05 -- unlike the backward launch's K loop, where the branch-free
// form saves 3.6 us.)
__device__ __forceinline__ f32x4 row4(const float* row, bool valid, int k0, int K, bool vec) {
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
    if (!valid) return v;
    if (vec && k0 + 3 < K) return *reinterpret_cast<const f32x4*>(row + k0);
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (k0 + e < K) v[e] = row[k0 + e];
    return v;
}

constexpr int FUSED_HLD = FUSED_WMAX + 4, FUSED_XLD = FUSED_K0MAX + 4;

// F's body. KCH: 16-deep chunks of K0 (2: K0 <= 32, 4: K0 <= 64), one per wave of the layer-0 launch
// (4 waves). FO (one launch with O): the batch's targets and the H_1 tile leave as write-through (sc1)
// stores, the tile also stays in LDS (hm: O's ReLU mask and dW_out operand), and the workgroup then
// adds to its band's counter.
template <int NW, int KCH, bool FO>
__device__ __forceinline__ void fused_fwd(const FusedArgs& F, float (*red)[TT][TT + 1], float (*h0)[FUSED_HLD],
                                          float (*xr)[FUSED_XLD], float (*hm)[TT + 1]) {
    constexpr int NT = 64 * NW, EPT = TT * TT / NT, MAXPER = NW == 16 ? 2 : 4, MAXY = NW == 16 ? 2 : 4;
    constexpr int NW0 = 4;   // the layer-0 launch's waves (K0 < 256)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4, c = lane & 15;
    const int tm = blockIdx.x / F.tiles_n, tn = blockIdx.x - tm * F.tiles_n, m0 = tm * TT, n0 = tn * TT;
    const int W = F.W, K0 = F.K0, R = F.R;
    FSTAMP(0, 0);
    if (blockIdx.x == 0 && F.zero_words)
        for (int i = tid; i < F.zero_n; i += NT) F.zero_words[i] = 0u;
    if (blockIdx.x == 0 && F.serial && tid == 0) *F.serial = *F.serial + 1u;
    // the batch's 32 input rows are gathered through the row indices: the indices, the rows, then every
    // weight operand of the launch (in-order vmcnt: a wait for the rows then waits for nothing issued
    // after them, and the weights travel while the rows do)
    constexpr int GPT = TT * 16 * KCH / NT;      // gathered elements per thread (k0pad <= 16 KCH)
    const int k0pad = (K0 + 15) & ~15;
    const bool nx = F.idx_next != nullptr && tn == 1;   // the second column tiles gather the next batch
    int64_t gi[GPT], gn[GPT];
#pragma unroll
    for (int j = 0; j < GPT; ++j) {
        const int e = tid + j * NT, r = e / k0pad, k = e - r * k0pad, m = m0 + r;
        gi[j] = (r < TT && m < R && k < K0) ? (F.pre_rows ? 0 : F.idx[m / F.H]) : -1;
        gn[j] = (nx && r < TT && m < F.R_next && k < K0) ? F.idx_next[m / F.H] : -1;
    }
    // the first column tiles also gather the targets O's loss epilogue needs (J <= 32: 32 x 32 slots)
    constexpr int TPT = TT * TT / NT;
    float tv[TPT];
    int64_t tsrc[TPT];
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
        const int e = tid + j * NT, r = e >> 5, o = e & 31, m = m0 + r;
        tsrc[j] = -1;
        if (!F.pre_rows && tn == 0 && o < F.J && m < R) tsrc[j] = F.idx[m / F.H] * F.H + m % F.H;
        if (nx && o < F.J && m < F.R_next) tsrc[j] = F.idx_next[m / F.H] * F.H + m % F.H;
    }
    // the rows (zero past K0 to the chunk end); the first column tile keeps them for the layer-0 weight
    // gradient, as the layer-0 launch did
    float gv[GPT];
#pragma unroll
    for (int j = 0; j < GPT; ++j) {
        const int e = tid + j * NT, r = e / k0pad, k = e - r * k0pad, m = m0 + r;
        gv[j] = 0.0f;
        if (gi[j] >= 0) {
            if (F.pre_rows) {
                gv[j] = F.xstore[(int64_t)m * K0 + k];
            } else {
                const int64_t src = gi[j] * F.H + m % F.H;
                gv[j] = k < F.s ? F.gs[src * F.s + k] : F.ga[src * F.a + (k - F.s)];
            }
        }
    }
    float gx[GPT];
#pragma unroll
    for (int j = 0; j < GPT; ++j) {
        const int e = tid + j * NT, r = e / k0pad, k = e - r * k0pad, m = m0 + r;
        const int64_t src = gn[j] * F.H + m % F.H;
        gx[j] = gn[j] < 0 ? 0.0f : k < F.s ? F.gs[src * F.s + k] : F.ga[src * F.a + (k - F.s)];
    }
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
        const int o = (tid + j * NT) & 31;
        tv[j] = tsrc[j] < 0 ? 0.0f : o < F.s ? F.gns[tsrc[j] * F.s + o] : F.grw[tsrc[j]];
    }
    // the layer-1 operands (this wave's K range of W_1's rows n0..n0+31, and the bias), issued behind
    // the rows: their latency overlaps the rows' and the H_0 recompute
    int kb0, kb1;
    wave_k_range(W, NW, wave, kb0, kb1);
    const bool vec1 = (W % 4 == 0) && (reinterpret_cast<uintptr_t>(F.w1) & 15) == 0;
    f32x4 bw[MAXPER][2];
#pragma unroll
    for (int u = 0; u < MAXPER; ++u)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int n = n0 + 16 * y + c, kb = kb0 + 16 * u;
            bw[u][y] = row4(F.w1 + (int64_t)min(n, W - 1) * W, n < W && kb < kb1, kb + 4 * q, W, vec1);
        }
    float pre[FO ? 1 : EPT];
    f32x4 pre4 = {0.0f, 0.0f, 0.0f, 0.0f};   // FO: thread t < 256 finishes 4 consecutive columns
    if constexpr (FO) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = n0 + (tid & 7) * 4 + i;
            pre4[i] = (tid < TT * TT / 4 && n < W) ? F.b1[n] : 0.0f;
        }
    } else {
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = tid + j * NT, n = n0 + (e & 31);
            pre[j] = n < W ? F.b1[n] : 0.0f;
        }
    }
    // W_0's rows for this wave's 16-column blocks of H_0 (y = wave, wave + NW, ...), every chunk
    const int ny = (W + 15) >> 4, nch0 = (K0 + 15) >> 4;
    const bool vec0 = (K0 % 4 == 0) && (reinterpret_cast<uintptr_t>(F.w0) & 15) == 0;
    f32x4 w0r[MAXY][KCH];
    float b0r[MAXY];
#pragma unroll
    for (int yy = 0; yy < MAXY; ++yy) {
        const int n = 16 * (wave + yy * NW) + c;
        b0r[yy] = n < W ? F.b0[n] : 0.0f;
#pragma unroll
        for (int ch = 0; ch < KCH; ++ch)
            w0r[yy][ch] = row4(F.w0 + (int64_t)min(n, W - 1) * K0, n < W && ch < nch0, 16 * ch + 4 * q, K0, vec0);
    }
#pragma unroll
    for (int j = 0; j < GPT; ++j) {
        const int e = tid + j * NT, r = e / k0pad, k = e - r * k0pad, m = m0 + r;
        if (r < TT) xr[r][k] = gv[j];
        if (gi[j] >= 0 && tn == 0 && !F.pre_rows) F.xstore[(int64_t)m * K0 + k] = gv[j];
        if (gn[j] >= 0) F.xnext[(int64_t)m * K0 + k] = gx[j];
    }
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
        const int e = tid + j * NT, r = e >> 5, o = e & 31;
        if (tsrc[j] < 0) continue;
        float* dst = (nx ? F.tnext : F.tgt) + (int64_t)(m0 + r) * F.J + o;
        if (FO && !nx) __hip_atomic_store(dst, tv[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // O reads it
        else *dst = tv[j];
    }
    __syncthreads();
    FSTAMP(0, 1);
    // H_0 rows m0..m0+31, all W columns: wave w takes the 16-column blocks y = w, w + NW, ...; each
    // 16 x 16 block is the sum, in wave order, of the layer-0 launch's per-wave chains (NW0 waves,
    // empty ones adding +0), then bias and ReLU -- that launch's epilogue
#pragma unroll
    for (int yy = 0; yy < MAXY; ++yy) {
        const int y = wave + yy * NW, n = 16 * y + c;
        if (y >= ny) break;
        f32x4 tot[2];
#pragma unroll
        for (int vw = 0; vw < NW0; ++vw) {      // wave vw of the layer-0 launch: chunk vw (or nothing)
            f32x4 p[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
            if (vw < KCH && vw < nch0) {
                f32x4 a[2];
#pragma unroll
                for (int x = 0; x < 2; ++x) a[x] = *reinterpret_cast<const f32x4*>(&xr[16 * x + c][16 * vw + 4 * q]);
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int x = 0; x < 2; ++x)
                        p[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x][s], w0r[yy][vw < KCH ? vw : 0][s], p[x], 0, 0, 0);
            }
#pragma unroll
            for (int x = 0; x < 2; ++x) tot[x] = vw == 0 ? p[x] : tot[x] + p[x];
        }
        const float bias = b0r[yy];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int row = 16 * x + 4 * q + v;
                float h = tot[x][v] + bias;
                h = h > 0.0f ? h : 0.0f;
                h0[row][n] = (n < W && m0 + row < R) ? h : 0.0f;
            }
    }
    __syncthreads();
    FSTAMP(0, 2);
    // this tile's columns of H_0 (every element stored by exactly one workgroup)
    for (int e = tid; e < TT * TT; e += NT) {
        const int r = e >> 5, col = e & 31, m = m0 + r, n = n0 + col;
        if (m < R && n < W) F.act0[(int64_t)m * W + n] = h0[r][n];
    }
    // the H_1 tile: the layer-1 launch's chains with the A operand from LDS
    f32x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < MAXPER; ++u) {
        const int kb = kb0 + 16 * u;
        if (kb >= kb1) break;
        f32x4 a[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) a[x] = *reinterpret_cast<const f32x4*>(&h0[16 * x + c][kb + 4 * q]);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x][s], bw[u][y][s], acc[x][y], 0, 0, 0);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int v = 0; v < 4; ++v) red[wave][16 * x + 4 * q + v][16 * y + c] = acc[x][y][v];
    __syncthreads();
    if constexpr (!FO) {
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = tid + j * NT, row = e >> 5, col = e & 31, m = m0 + row, n = n0 + col;
            if (m >= R || n >= W) continue;
            float v = red[0][row][col];
#pragma unroll
            for (int w = 1; w < NW; ++w) v = v + red[w][row][col];
            v = v + pre[j];
            F.act1[(int64_t)m * W + n] = v > 0.0f ? v : 0.0f;
        }
    } else {
        // the same sums, 4 columns per thread: one 16-byte write-through store (4-byte ones at a ragged
        // or unaligned edge), and the tile into hm
        if (tid < TT * TT / 4) {
            const int row = tid >> 3, c4 = (tid & 7) * 4, m = m0 + row;
            f32x4 h;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v = red[0][row][c4 + i];
#pragma unroll
                for (int w = 1; w < NW; ++w) v = v + red[w][row][c4 + i];
                v = v + pre4[i];
                h[i] = (m < R && n0 + c4 + i < W) ? (v > 0.0f ? v : 0.0f) : 0.0f;
                hm[row][c4 + i] = h[i];
            }
            if (m < R) {
                const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
                    F.act1, 0, (int)((int64_t)R * W * sizeof(float)), 0x00020000);
                const unsigned off = (unsigned)(((int64_t)m * W + n0 + c4) * sizeof(float));
                if ((W & 3) == 0 && (reinterpret_cast<uintptr_t>(F.act1) & 15) == 0 && n0 + c4 + 3 < W) {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, h), ar, off, 0, TRAIN_SC1);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (n0 + c4 + i < W)
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, (float)h[i]), ar, off + 4 * i, 0,
                                                                  TRAIN_SC1);
                }
            }
        }
        // every storing wave drains its stores, then one lane signals for the workgroup
        // (MI355X_MICROARCH.md, the first row of the sc1 hand-off table)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(F.band + tm * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    FSTAMP(0, 3);
}

// KCH: as fused_fwd
template <int NW, int KCH>
__global__ __launch_bounds__(64 * NW) void train_fused_fwd_kernel(const FusedArgs F) {
    __shared__ float red[NW][TT][TT + 1];
    __shared__ __attribute__((aligned(16))) float h0[TT][FUSED_HLD];
    __shared__ __attribute__((aligned(16))) float xr[TT][FUSED_XLD];
    fused_fwd<NW, KCH, false>(F, red, h0, xr, nullptr);
}

// Four consecutive k of an H_1 row handed over in this launch: sc1 buffer loads (the row's byte
// offset `row_off`; row4's zero fill and element fallback)
__device__ __forceinline__ f32x4 row4_sc1(__amdgpu_buffer_rsrc_t r, unsigned row_off, bool valid, int k0, int K,
                                          bool vec) {
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
    if (!valid) return v;
    if (vec && k0 + 3 < K)
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, row_off + 4u * k0, 0, TRAIN_SC1));
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (k0 + e < K)
            v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, row_off + 4u * (k0 + e), 0, TRAIN_SC1));
    return v;
}

// FO: wait until every F tile of band tm has written its H_1 columns (one lane polls, sc1 loads; a
// 1 s bound sets bit 0 of *status instead of hanging), then count this tile as past the wait; the
// band's last such add resets the counter for the next launch. The band's tiles are consecutive
// workgroup ids, so with in-order dispatch the earliest unfinished band is always fully resident.
__device__ __forceinline__ void band_wait(const FusedArgs& F, int tm) {
    if (threadIdx.x == 0) {
        unsigned* c = F.band + tm * 32;
        const unsigned need = (unsigned)F.tiles_n;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
                atomicOr(F.status, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == 2 * need)
            __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
}

// O's body. dy: the tile's 32 rows of dY (columns past J zero); hm: H_1 of the tile (the ReLU mask and
// the dW_out operand). FO (one launch with F): hm is already there, W_out's rows are loaded before
// the band wait and the band's H_1 rows and targets after it, with sc1 loads.
template <int NW, bool FO>
__device__ __forceinline__ void fused_out(const FusedArgs& F, float (*red)[TT][TT + 1], float (*dy)[TT + 1],
                                          float (*hm)[TT + 1], unsigned& last) {
    constexpr int NT = 64 * NW, EPT = TT * TT / NT, MAXPER = NW == 16 ? 2 : 4;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4, c = lane & 15;
    const int tm = blockIdx.x / F.tiles_n, tn = blockIdx.x - tm * F.tiles_n, m0 = tm * TT, n0 = tn * TT;
    const int W = F.W, J = F.J, R = F.R, S = F.s;
    FSTAMP(1, 0);
    // b_1's Adam operands for this column block (threads 64-95), for the last arriver's tail
    const bool b1t = tid >= 64 && tid < 64 + TT && n0 + tid - 64 < W;
    float b1p = 0.0f, b1m = 0.0f, b1v = 0.0f;
    if (F.adam && b1t) {
        b1p = F.ab1.param[n0 + tid - 64];
        b1m = F.ab1.exp_avg[n0 + tid - 64];
        b1v = F.ab1.exp_avg_sq[n0 + tid - 64];
    }
    // ---- the output-layer tile (tm, 0): Y = H_1 W_out^T + b_out over this wave's K range
    int kb0, kb1;
    wave_k_range(W, NW, wave, kb0, kb1);
    const bool veca = (W % 4 == 0) && (reinterpret_cast<uintptr_t>(F.act1) & 15) == 0;
    const bool vecb = (W % 4 == 0) && ((reinterpret_cast<uintptr_t>(F.wo) | reinterpret_cast<uintptr_t>(F.wo_r)) & 15) == 0;
    f32x4 av[MAXPER][2], bv[MAXPER][2];
#pragma unroll
    for (int u = 0; u < MAXPER; ++u) {
        const int kb = kb0 + 16 * u;
#pragma unroll
        for (int y = 0; y < 2; ++y) {
            const int o = 16 * y + c;
            const float* row = o < S ? F.wo + (int64_t)o * W : F.wo_r;
            bv[u][y] = row4(row, o < J && kb < kb1, kb + 4 * q, W, vecb);
        }
    }
    if constexpr (FO) {
        band_wait(F, tm);
        const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
            F.act1, 0, (int)((int64_t)R * W * sizeof(float)), 0x00020000);
#pragma unroll
        for (int u = 0; u < MAXPER; ++u) {
            const int kb = kb0 + 16 * u;
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                const int m = m0 + 16 * x + c;
                av[u][x] = row4_sc1(ar, (unsigned)((int64_t)min(m, R - 1) * W * sizeof(float)), m < R && kb < kb1,
                                    kb + 4 * q, W, veca);
            }
        }
    } else {
#pragma unroll
        for (int u = 0; u < MAXPER; ++u) {
            const int kb = kb0 + 16 * u;
#pragma unroll
            for (int x = 0; x < 2; ++x) {
                const int m = m0 + 16 * x + c;
                av[u][x] = row4(F.act1 + (int64_t)min(m, R - 1) * W, m < R && kb < kb1, kb + 4 * q, W, veca);
            }
        }
    }
    // the loss epilogue's y - t = acc - (t - bias), and the tile's H_1 block (mask, dW_out operand)
    float pre[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const int e = tid + j * NT, m = m0 + (e >> 5), o = e & 31;
        pre[j] = 0.0f;
        if (m >= R || o >= J) continue;
        const float* tg = F.tgt + (int64_t)m * J + o;
        pre[j] = (FO ? __hip_atomic_load(tg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *tg) -
                 (o < S ? F.bo[o] : F.bo_r[o - S]);
    }
    if constexpr (!FO)
        for (int e = tid; e < TT * TT; e += NT) {
            const int r = e >> 5, col = e & 31, m = m0 + r, n = n0 + col;
            hm[r][col] = (m < R && n < W) ? F.act1[(int64_t)m * W + n] : 0.0f;
        }
    f32x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < MAXPER; ++u) {
        if (kb0 + 16 * u >= kb1) break;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][x][s], bv[u][y][s], acc[x][y], 0, 0, 0);
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int v = 0; v < 4; ++v) red[wave][16 * x + 4 * q + v][16 * y + c] = acc[x][y][v];
    __syncthreads();
    // the output-layer launch's EPI_LOSS epilogue: dY = (Y - T) * 2 / numel, the loss terms
    float loss_s = 0.0f, loss_r = 0.0f;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
        const int e = tid + j * NT, row = e >> 5, col = e & 31, m = m0 + row;
        float v = 0.0f;
        if (m < R && col < J) {
            v = red[0][row][col];
#pragma unroll
            for (int w = 1; w < NW; ++w) v = v + red[w][row][col];
            const float d = v - pre[j];
            if (col < S) loss_s = loss_s + d * d * F.inv_s;
            else loss_r = loss_r + d * d * F.inv_r;
            v = d * (col < S ? F.scale_s : F.scale_r);
        }
        dy[row][col] = v;
    }
    __syncthreads();
    FSTAMP(1, 1);
    if (tn == 0) {
        // dY's column sums over the tile's rows (db_out), read back by this launch's last arriver
        if (tid < TT && tid < J) {
            float t = dy[0][tid];
            for (int r = 1; r < TT; ++r) t = t + dy[r][tid];
            __hip_atomic_store(F.cs_dy + (int64_t)tm * J + tid, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            loss_s += __shfl_xor(loss_s, o);
            loss_r += __shfl_xor(loss_r, o);
        }
        float* sl = &red[1][0][0];      // red[1] is free: every wave's partials were summed above
        if (lane == 0) {
            sl[2 * wave] = loss_s;
            sl[2 * wave + 1] = loss_r;
        }
        __syncthreads();
        if (tid < 2) {
            float t = sl[tid];
            for (int w = 1; w < NW; ++w) t = t + sl[2 * w + tid];
            F.loss_part[tm * 2 + tid] = t;
        }
    }
    // ---- tasks 0-3: the dH_1 tile, K = J (the [dH_1 + dW_out] launch's split over nwb waves: one
    // 16-deep chunk per wave, the rest adding +0), masked by H_1 > 0. Tasks 4-7: the dW_out partial
    // over rows m0..m0+31 (that launch's wave tm: its two 16-row chunks, M = J, N = this column block)
    for (int task = wave; task < 8; task += NW) {   // (4 waves: each takes one block of both)
      if (task < 4) {
        const int x = task >> 1, y = task & 1, n = n0 + 16 * y + c;
        f32x4 tot = {0.0f, 0.0f, 0.0f, 0.0f};
        const int nch = (J + 15) >> 4;
        for (int ch = 0; ch < nch; ++ch) {
            f32x4 a, b, p = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = 16 * ch + 4 * q + s;     // an output unit o
                a[s] = dy[16 * x + c][k];
                b[s] = (k < J && n < W) ? (k < S ? F.wo[(int64_t)k * W + n] : F.wo_r[(int64_t)(k - S) * W + n]) : 0.0f;
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) p = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], p, 0, 0, 0);
            tot = ch == 0 ? p : tot + p;
        }
        for (int w = nch; w < F.nwb; ++w) tot = tot + f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int row = 16 * x + 4 * q + v, m = m0 + row;
            const float g = hm[row][16 * y + c] > 0.0f ? tot[v] : 0.0f;
            const float keep = (m < R && n < W) ? g : 0.0f;
            if (m < R && n < W) F.dh1[(int64_t)m * W + n] = g;
            red[0][row][16 * y + c] = keep;
        }
      } else {
        const int x = (task - 4) >> 1, y = (task - 4) & 1;
        f32x4 p = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f32x4 a, b;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int r = 16 * u + 4 * q + s;      // a row of the batch tile (K of this product)
                a[s] = dy[r][16 * x + c];
                b[s] = hm[r][16 * y + c];
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) p = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], p, 0, 0, 0);
        }
        const int i = n0 + 16 * y + c;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int o = 16 * x + 4 * q + v;
            if (o < J && i < W)    // sc1 (write-through) stores, read back by the last arriver
                __hip_atomic_store(F.out_part + ((int64_t)tm * J + o) * W + i, p[v], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __syncthreads();
    // dH_1's column sums over the tile's 32 rows, in row order (db_1: this column block's last arriver)
    if (tid < TT && n0 + tid < W) {
        float t = red[0][0][tid];
        for (int r = 1; r < TT; ++r) t = t + red[0][r][tid];
        __hip_atomic_store(F.cs_dh1 + (int64_t)tm * W + n0 + tid, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    FSTAMP(1, 2);
    // the column block's last arriver sums the dW_out partials in wave order (row tiles past the
    // batch: the empty waves' +0), and the first column block's also db_out from dY's column sums
    if (tid == 0) {
        const unsigned t = __hip_atomic_fetch_add(&F.out_ticket[tn], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (t + 1 == (unsigned)F.tiles_r) ? 1u : 0u;
        // every arrival is in: reset the ticket for the next launch (in one launch with F, nothing
        // zeroes it at the start)
        if (last) __hip_atomic_store(&F.out_ticket[tn], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    FSTAMP(1, 3);
    if (!last) return;
    // every load of the tail first (db_out's and db_1's column sums, then the partials): one round trip
    const bool dyt = tn == 0 && tid < J, tfast = F.tiles_r <= 16;
    float cs[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const float* src = dyt ? F.cs_dy + (int64_t)i * J + tid : F.cs_dh1 + (int64_t)i * W + n0 + tid - 64;
        cs[i] = ((dyt || b1t) && tfast && i < F.tiles_r)
                    ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
    }
    for (int e = tid; e < J * TT; e += NT) {
        const int o = e / TT, i = n0 + (e - o * TT);
        if (i >= W) continue;
        float p[16];
#pragma unroll
        for (int w = 0; w < 16; ++w)
            p[w] = (w < F.tiles_r && w < F.nwb)
                       ? __hip_atomic_load(F.out_part + ((int64_t)w * J + o) * W + i, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)
                       : 0.0f;
        float v = p[0];
#pragma unroll
        for (int w = 1; w < 16; ++w)
            if (w < F.nwb) v = v + p[w];
        if (o < S) F.dwo[(int64_t)o * W + i] = v;
        else F.dwo_r[(int64_t)(o - S) * W + i] = v;
    }
    if (dyt || b1t) {
        float g = cs[0];
#pragma unroll
        for (int i = 1; i < 16; ++i)
            if (i < F.tiles_r) g = g + cs[i];
        if (dyt) {              // db_out
            if (!tfast) g = ordered_sum<true>(F.cs_dy + tid, J, F.tiles_r);
            if (tid < S) F.dbo[tid] = g;
            else F.dbo_r[tid - S] = g;
        } else {                // db_1 (the five-launch layout's dW_1 launch summed the same column sums in
            const int n = n0 + tid - 64;   // the same order) and b_1's Adam step: nothing reads b_1 before
            if (!tfast) g = ordered_sum<true>(F.cs_dh1 + n, W, F.tiles_r);   // the next batch's F
            F.db1[n] = g;
            if (F.adam) {
                adam_element(b1p, g, b1m, b1v, F.ab1.step_size, F.ab1.bc2_sqrt, F.hp, F.arith);
                F.ab1.param[n] = b1p;
                F.ab1.exp_avg[n] = b1m;
                F.ab1.exp_avg_sq[n] = b1v;
            }
        }
    }
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void train_fused_out_kernel(const FusedArgs F) {
    __shared__ float red[NW][TT][TT + 1];
    __shared__ float dy[TT][TT + 1];
    __shared__ float hm[TT][TT + 1];
    __shared__ unsigned last;
    fused_out<NW, false>(F, red, dy, hm, last);
}

// F and O as one launch: the O tiles of a 32-row band wait (band_wait) for that band's F tiles only,
// instead of the whole grid at a kernel boundary, and W_out's rows load during the wait. The same
// bodies, so the same bits as the two launches (MBRL_OPT_TRAIN_FO = 1 keeps them apart).
template <int NW, int KCH>
__global__ __launch_bounds__(64 * NW) void train_fused_fo_kernel(const FusedArgs F) {
    __shared__ float red[NW][TT][TT + 1];
    __shared__ __attribute__((aligned(16))) float h0[TT][FUSED_HLD];
    __shared__ __attribute__((aligned(16))) float xr[TT][FUSED_XLD];
    __shared__ unsigned last;
    // hm and dy alias h0, which F no longer reads once its H_1 products are in red
    float(*hm)[TT + 1] = reinterpret_cast<float(*)[TT + 1]>(&h0[0][0]);
    float(*dy)[TT + 1] = hm + TT;
    fused_fwd<NW, KCH, true>(F, red, h0, xr, hm);
    fused_out<NW, true>(F, red, dy, hm, last);
}

static Operand direct(const float* p0, const float* p1, int split, int ld, int rows) {
    Operand o{};
    o.p0 = p0; o.p1 = p1 ? p1 : p0; o.split = p1 ? split : rows; o.ld = ld; o.kind = OP_DIRECT; o.rows = rows;
    o.ones_row = -1;
    o.vec = (ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(p0) | reinterpret_cast<uintptr_t>(o.p1)) & 15) == 0;
    return o;
}

static Operand transposed(const float* p0, const float* p1, int split, int ld, int rows, int ones_row) {
    Operand o{};
    o.p0 = p0; o.p1 = p1 ? p1 : p0; o.split = p1 ? split : (1 << 30); o.ld = ld; o.kind = OP_TRANS; o.rows = rows;
    o.ones_row = ones_row;
    return o;
}

static void finish(GemmDesc& D, int M, int N, int K, int tmx = 1) {
    D.M = M; D.N = N; D.K = K;
    D.tiles_n = (N + TT - 1) / TT;
    D.tiles = ((M + TT * tmx - 1) / (TT * tmx)) * D.tiles_n;
}

// 16 waves split a long K (the hidden layers, every weight gradient); 4 suffice for short ones; 8 where
// the longest K is a weight gradient's batch rows in (128, 256) -- each wave then sums 32 rows, the
// row tile of the fused step's folds (launch_waves; fold_waves follows the same rule).
// TMX: the C tile height of every product of the launch (finish() with the same tmx).
static int launch_waves(const GemmLaunch& L) {
    int kmax = 0;
    bool grad_rows = false;
    for (int i = 0; i < L.nd; ++i) kmax = max(kmax, L.d[i].K);
    for (int i = 0; i < L.nd; ++i) grad_rows = grad_rows || (L.d[i].out.mode == EPI_GRAD && L.d[i].K == kmax);
    return kmax >= 256 ? 16 : (kmax > 128 && grad_rows) ? 8 : 4;
}

template <int A0, int B0, int A1 = -1, int B1 = -1, int TMX = 1>
static hipError_t launch_gemm(GemmLaunch& L, bool loss_wg, hipStream_t stream) {
    int blocks = loss_wg ? 1 : 0;
    for (int i = 0; i < L.nd; ++i) blocks += L.d[i].tiles;
    const int nw = launch_waves(L);
    // fused Adam blocks: chunks of 4 elements per thread of the launch's workgroup size
    const int chunk = 64 * nw * 4;
    L.adam_chunk = chunk;
    L.adam_blocks = 0;
    for (int i = 0; i < L.adam_count; ++i) {
        L.adam_first[i] = L.adam_blocks;
        L.adam_blocks += (int)((L.adam_t[i].numel + chunk - 1) / chunk);
    }
    L.adam_first[L.adam_count] = L.adam_blocks;
    blocks += L.adam_blocks;
    if (!loss_wg) L.loss_out = nullptr;
    ++L.slot;
    // XCD order needs whole groups of 8 64-row bands (a bijection of the tiles)
    const int tiles_m0 = L.d[0].tiles / L.d[0].tiles_n;
    L.xcd = L.xcd && (tiles_m0 % (8 * (2 / TMX)) == 0);
    if constexpr (TMX == 2) {   // chosen only for long K (launch_train_grads): 16 waves
        if (nw != 16) return hipErrorInvalidValue;
        hipLaunchKernelGGL((train_gemm_kernel<16, A0, B0, A1, B1, TMX>), dim3(blocks), dim3(64 * 16), 0, stream, L);
    } else if (nw == 16) {
        hipLaunchKernelGGL((train_gemm_kernel<16, A0, B0, A1, B1, TMX>), dim3(blocks), dim3(64 * 16), 0, stream, L);
    } else if (nw == 8) {
        hipLaunchKernelGGL((train_gemm_kernel<8, A0, B0, A1, B1, TMX>), dim3(blocks), dim3(64 * 8), 0, stream, L);
    } else {
        hipLaunchKernelGGL((train_gemm_kernel<4, A0, B0, A1, B1, TMX>), dim3(blocks), dim3(64 * 4), 0, stream, L);
    }
    return hipGetLastError();
}

// Workspace (floats, each piece 256-byte aligned): hidden activations H_0..H_{L-1} [R][W], two
// backward buffers dH [R][W], dY [R][J], loss partials, the gathered input [R][s + a], and the
// per-row-tile column sums of dY [tiles][J] and of the two dH [tiles][W].
struct TrainWs {
    float* act[MBRL_TRAIN_MAX_LAYERS];
    float *dh[2], *dy, *loss_part, *xbuf, *cs_dy, *cs_dh[2];
    float *xbuf2, *tgt2;  // the fused step's second gather slot (the next batch's rows and targets)
    float* out_part;      // fused step: the output layer's weight-gradient partials [row tile][J][W]
    float* tgt;           // fused step: the batch's targets [R][J] (F gathers, O reads)
    unsigned* tickets;    // [ceil(W / 32)] each: (unused: the dW_0 fold's before its granules), the fused
                          // dH_0 tiles' W_1-read arrivals, the fused dW_out fold's
    unsigned* status;     // fused step: bit 0 = a bounded wait timed out (never expected)
    unsigned* bands;      // fused step, F and O in one launch: [row tiles][32] band counters (one line each)
    unsigned* serial;     // the step's serial: the dW_0 fold's granule tag (raised by each step's first launch)
    unsigned long long *fold_gran, *cs_gran;   // the fold's tagged partials [tr][W][K0] and column sums [tr][W]
    size_t floats;
};

// The fused step needs the dW_0 fold, whose 32-row waves bound its rows: R <= 512, 16 bands of 32.
constexpr int FUSED_MAX_BANDS = 16;

static TrainWs train_ws(const TrainShape& t, int batch, float* base) {
    const size_t R = (size_t)batch * t.H, J = t.s + (t.reward ? 1 : 0), W = t.W, tiles_r = (R + TT - 1) / TT;
    const size_t tiles_out = tiles_r * ((J + TT - 1) / TT);
    auto up = [](size_t x) { return (x + 63) & ~(size_t)63; };
    TrainWs w{};
    size_t off = 0;
    auto take = [&](size_t n) { float* p = base ? base + off : nullptr; off += up(n); return p; };
    // the control words first, at offsets that depend on the model only: every batch of an epoch
    // (the short last one lays out its data areas for its own size) finds the tickets, the sticky
    // status word and the band counters where the others left them, zero between launches; the band
    // counters sized for the fused step's largest batch (FUSED_MAX_BANDS)
    // (tickets and band counters first: every training call zeroes them in one memset on entry, see
    // train_counter_bytes; the status word and the serial behind them keep their values)
    w.tickets = reinterpret_cast<unsigned*>(take(3 * ((W + TT - 1) / TT)));
    w.bands = reinterpret_cast<unsigned*>(take(32 * FUSED_MAX_BANDS));
    w.status = reinterpret_cast<unsigned*>(take(1));
    w.serial = reinterpret_cast<unsigned*>(take(1));
    for (int l = 0; l < t.L; ++l) w.act[l] = take(R * W);
    w.dh[0] = take(R * W);
    w.dh[1] = take(R * W);
    w.dy = take(R * J);
    w.loss_part = take(tiles_out * 2);
    w.xbuf = take(R * (t.s + t.a));
    w.cs_dy = take(tiles_r * J);
    w.cs_dh[0] = take(tiles_r * W);
    w.cs_dh[1] = take(tiles_r * W);
    w.out_part = take(tiles_r * J * W);
    w.tgt = take(R * J);
    w.xbuf2 = take(R * (t.s + t.a));
    w.tgt2 = take(R * J);
    w.fold_gran = reinterpret_cast<unsigned long long*>(take(2 * tiles_r * W * (size_t)(t.s + t.a)));
    w.cs_gran = reinterpret_cast<unsigned long long*>(take(2 * tiles_r * W));
    w.floats = off;
    return w;
}

size_t train_ws_floats(const TrainShape& t, int batch) { return train_ws(t, batch, nullptr).floats; }

// Bytes at the start of the workspace holding the fused step's arrival tickets and band counters. Their
// protocol leaves them zero between launches, but a workspace that was never zeroed, or a step whose
// bounded wait timed out, would leave counts behind: mbrl_train_grads / mbrl_train_epoch clear them
// once per call. The sticky status word and the fold's serial lie behind them and are kept.
size_t train_counter_bytes(const TrainShape& t, int batch) {
    float* base = reinterpret_cast<float*>(static_cast<uintptr_t>(64));
    return (size_t)(reinterpret_cast<char*>(train_ws(t, batch, base).status) - reinterpret_cast<char*>(base));
}

size_t train_status_offset(const TrainShape& t, int batch) {
    float* base = reinterpret_cast<float*>(static_cast<uintptr_t>(64));   // any aligned base: offsets only
    return (size_t)(reinterpret_cast<char*>(train_ws(t, batch, base).status) - reinterpret_cast<char*>(base));
}

// Whether the layer-0 weight gradient folds into the dH_0 launch bit-identically: its separate launch
// (M = W, K = R) gives each of its waves one 32-row block of the batch (16 waves at R >= 256, 8 in
// (128, 256), else 4: launch_waves).
static int fold_waves(const TrainShape& t, int R) {
    if (t.fold == 0 || t.L < 1) return 0;
    const int nw = R >= 256 ? 16 : R > 128 ? 8 : 4, chunks = (R + 15) / 16, per = (chunks + nw - 1) / nw;
    return per == 2 ? nw : 0;
}

// Whether the fused three-launch step applies (train_fused_*_kernel): two hidden layers, the dW_0
// fold (its 32-row waves are also the dW_out partials' row tiles), dY within one 32-column tile, the
// layer-0 input within one chunk per wave of its launch, H_0's tile rows within LDS.
static bool fused_step(const TrainShape& t, int fold_nw) {
    const int J = t.s + (t.reward ? 1 : 0), K0 = t.s + t.a;
    return t.split == 0 && t.L == 2 && fold_nw > 0 && J <= TT && K0 <= FUSED_K0MAX && t.W <= FUSED_WMAX;
}
static bool fused_step(const TrainShape& t, int fold_nw, int R) {
    return fused_step(t, fold_nw) && (R + TT - 1) / TT <= FUSED_MAX_BANDS;   // (fold_nw > 0 implies it)
}

bool train_fused_applies(const TrainShape& t, int batch) {
    return fused_step(t, fold_waves(t, batch * t.H), batch * t.H);
}

hipError_t launch_train_grads(const TrainShape& t, const TrainTensors& w, const int64_t* idx, int batch,
                              float* loss_out, float* ws, hipStream_t stream, const mbrl_adam_tensor* adam,
                              const mbrl_adam_hparams* hp, int arith, const mbrl_adam_tensor* prior, int prior_n,
                              mbrl_adam_tensor* pending, int* pending_n, const TrainGather* gather) {
    const int R = batch * t.H, W = t.W, K0 = t.s + t.a, J = t.s + (t.reward ? 1 : 0), L = t.L;
    const int tiles_r = (R + TT - 1) / TT;
    const int fold_nw = fold_waves(t, R);
    const bool fused = fused_step(t, fold_nw, R);
    if (pending_n) *pending_n = 0;
    if ((prior_n > 0 && !prior) || prior_n > ADAM_FUSED_MAX || (adam && fold_nw && (!pending || !pending_n)))
        return hipErrorInvalidValue;
    TrainWs B = train_ws(t, batch, ws);
    // the fused step's gather slot: the caller alternates them when F gathers the next batch
    float *xnext = B.xbuf2, *tnext = B.tgt2;
    if (fused && gather && gather->slot) {
        std::swap(B.xbuf, B.xbuf2);
        std::swap(B.tgt, B.tgt2);
        xnext = B.xbuf2;
        tnext = B.tgt2;
    }
    const float* wo_r = t.reward ? w.weight[L + 1] : nullptr;
    const float* bo_r = t.reward ? w.bias[L + 1] : w.bias[L];

    GemmLaunch G{};
    G.idx = idx; G.gs = w.states; G.ga = w.actions; G.gns = w.next_states; G.grw = w.rewards;
    const int xcd_opt = t.xcd;
    G.H = t.H; G.s = t.s; G.a = t.a;
    G.xstore = B.xbuf;
    G.slot = fused ? 1 : -1;   // diagnostic stamps: the fused step's F and O are slots 0 and 1
    if (adam) {
        G.hp = *hp;
        G.arith = arith;
    }
    hipError_t e;
    const int tiles_n = (W + TT - 1) / TT;
    if (fused) {   // F and O (train_fused_*_kernel); the backward launch below is B
        // a step the five-launch layout deferred (a smaller batch before this one): F reads W_1
        if (prior_n > 0 && (e = launch_adam_step(prior, prior_n, *hp, arith, stream)) != hipSuccess) return e;
        FusedArgs F{};
        F.idx = idx; F.gs = w.states; F.ga = w.actions; F.gns = w.next_states; F.grw = w.rewards;
        F.H = t.H; F.s = t.s; F.a = t.a;
        F.R = R; F.W = W; F.K0 = K0; F.J = J; F.tiles_n = tiles_n; F.tiles_r = tiles_r;
        F.nwb = fold_nw;
        F.w0 = w.weight[0]; F.b0 = w.bias[0]; F.w1 = w.weight[1]; F.b1 = w.bias[1];
        F.wo = w.weight[L]; F.wo_r = wo_r; F.bo = w.bias[L]; F.bo_r = bo_r;
        F.act0 = B.act[0]; F.act1 = B.act[1]; F.xstore = B.xbuf; F.tgt = B.tgt;
        if (gather) {   // (the workspace layout depends on the batch size: only equal batches hand over)
            F.pre_rows = gather->pre_rows;
            if (gather->idx_next && gather->batch_next == batch && tiles_n > 1) {
                F.idx_next = gather->idx_next;
                F.R_next = gather->batch_next * t.H;
                F.xnext = xnext;
                F.tnext = tnext;
            }
        }
        F.dh1 = B.dh[1]; F.cs_dh1 = B.cs_dh[1]; F.cs_dy = B.cs_dy; F.loss_part = B.loss_part;
        F.out_part = B.out_part;
        F.dwo = w.weight_grad[L]; F.dwo_r = t.reward ? w.weight_grad[L + 1] : w.weight_grad[L];
        F.dbo = w.bias_grad[L]; F.dbo_r = t.reward ? w.bias_grad[L + 1] : w.bias_grad[L];
        F.out_ticket = B.tickets + 2 * tiles_n;
        F.band = B.bands; F.status = B.status;
        F.db1 = w.bias_grad[1];
        if (adam) {
            F.adam = 1; F.ab1 = adam[3]; F.hp = *hp; F.arith = arith;
        }
        // F zeroes the later launches' tickets (in one launch with O, not O's own: its last arrivers
        // reset them)
        const bool fo = t.fo_split == 0;
        F.zero_words = B.tickets; F.zero_n = (fo ? 2 : 3) * tiles_n;
        F.serial = B.serial;
        F.scale_s = 2.0f / (float)((int64_t)batch * t.s); F.scale_r = 2.0f / (float)batch;
        F.inv_s = 1.0f / (float)((int64_t)batch * t.s); F.inv_r = 1.0f / (float)batch;
        const dim3 grid(tiles_r * tiles_n);
        // the wave count of the separate launches whose K is W; K0's chunks
        if (fo && W >= 256) {
            if (K0 <= 32) hipLaunchKernelGGL((train_fused_fo_kernel<16, 2>), grid, dim3(64 * 16), 0, stream, F);
            else hipLaunchKernelGGL((train_fused_fo_kernel<16, 4>), grid, dim3(64 * 16), 0, stream, F);
        } else if (fo) {
            if (K0 <= 32) hipLaunchKernelGGL((train_fused_fo_kernel<4, 2>), grid, dim3(64 * 4), 0, stream, F);
            else hipLaunchKernelGGL((train_fused_fo_kernel<4, 4>), grid, dim3(64 * 4), 0, stream, F);
        } else if (W >= 256) {
            if (K0 <= 32) hipLaunchKernelGGL((train_fused_fwd_kernel<16, 2>), grid, dim3(64 * 16), 0, stream, F);
            else hipLaunchKernelGGL((train_fused_fwd_kernel<16, 4>), grid, dim3(64 * 16), 0, stream, F);
            hipLaunchKernelGGL(train_fused_out_kernel<16>, grid, dim3(64 * 16), 0, stream, F);
        } else {
            if (K0 <= 32) hipLaunchKernelGGL((train_fused_fwd_kernel<4, 2>), grid, dim3(64 * 4), 0, stream, F);
            else hipLaunchKernelGGL((train_fused_fwd_kernel<4, 4>), grid, dim3(64 * 4), 0, stream, F);
            hipLaunchKernelGGL(train_fused_out_kernel<4>, grid, dim3(64 * 4), 0, stream, F);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // forward through the hidden layers
    for (int l = 0; l < (fused ? 0 : L); ++l) {
        GemmDesc& D = G.d[0];
        D = GemmDesc{};
        if (l == 0) {
            D.A = Operand{};
            D.A.kind = OP_GATHER; D.A.rows = R; D.A.ones_row = -1; D.A.gather_trans = 0;
        } else {
            D.A = direct(B.act[l - 1], nullptr, 0, W, R);
        }
        D.B = direct(w.weight[l], nullptr, 0, l == 0 ? K0 : W, W);
        D.out.mode = EPI_ACT; D.out.c0 = D.out.c1 = B.act[l]; D.out.split = R; D.out.ldc = W;
        D.out.b0 = D.out.b1 = w.bias[l]; D.out.bsplit = W; D.out.relu = 1;
        finish(D, R, W, l == 0 ? K0 : W);
        G.nd = 1;
        if (l == 0) {
            // the forward launch raises the step's serial (the fold's granule tag) and takes the
            // previous step's deferred Adam step (a layer nothing before this step's second forward
            // launch reads)
            G.serial = fold_nw ? B.serial : nullptr;
            G.adam_count = 0;
            for (int i = 0; i < prior_n; ++i) G.adam_t[G.adam_count++] = prior[i];
        }
        G.xcd = xcd_opt;
        e = l == 0 ? launch_gemm<OP_GATHER, OP_DIRECT>(G, false, stream) : launch_gemm<OP_DIRECT, OP_DIRECT>(G, false, stream);
        G.zero_words = nullptr;
        G.serial = nullptr;
        G.adam_count = 0;
        if (e != hipSuccess) return e;
    }
    // output layer (state head, reward head) + the loss gradient dY and its column sums
    if (!fused) {
        GemmDesc& D = G.d[0];
        D = GemmDesc{};
        D.A = direct(B.act[L - 1], nullptr, 0, W, R);
        D.B = direct(w.weight[L], wo_r, t.s, W, J);
        Output& O = D.out;
        O.mode = EPI_LOSS; O.c0 = O.c1 = B.dy; O.split = R; O.ldc = J;
        O.b0 = w.bias[L]; O.b1 = bo_r; O.bsplit = t.s;
        O.scale_s = 2.0f / (float)((int64_t)batch * t.s); O.scale_r = 2.0f / (float)batch;
        O.inv_s = 1.0f / (float)((int64_t)batch * t.s); O.inv_r = 1.0f / (float)batch;
        O.s = t.s; O.loss_part = B.loss_part; O.colsum_out = B.cs_dy;
        finish(D, R, J, W);
        G.nd = 1;
        G.xcd = xcd_opt;
        if ((e = launch_gemm<OP_DIRECT, OP_DIRECT>(G, false, stream)) != hipSuccess) return e;
    }
    const int loss_parts = fused ? tiles_r : G.d[0].tiles;
    // backward: layer l = L (output) .. 0; launch l: dH_{l-1} (l >= 1) and dW_l, db_l. With the fold
    // (fold_waves) launch 1 also finishes dW_0 / db_0 and launch 0 does not exist.
    const int l_end = fold_nw ? 1 : 0;
    for (int l = fused ? L - 1 : L; l >= l_end; --l) {
        const bool out_layer = l == L;
        const float* g_in = out_layer ? B.dy : B.dh[l % 2];   // dL/d(pre-activation of layer l), [R][n_out]
        const float* cs_in = out_layer ? B.cs_dy : B.cs_dh[l % 2];
        const int n_out = out_layer ? J : W, n_in = l == 0 ? K0 : W;
        // 64-row tiles when the launch's 32 x 32 tiles would need a second round of the CUs
        // (2 x 512: dH_0 and dW_1 are 256 tiles each); the tile height changes no bit
        const int tiles32 = (l >= 1 ? tiles_r * ((W + TT - 1) / TT) : 0) +
                            ((n_out + TT - 1) / TT) * ((n_in + TT - 1) / TT);
        int tmx = (l >= 1 && tiles32 > device_cu_count() && (n_out >= 256 || R >= 256)) ? 2 : 1;
        if (t.tile == 32 || (t.tile == 64 && l >= 1 && (n_out >= 256 || R >= 256))) tmx = t.tile / 32;
        G.nd = 0;
        if (l >= 1) {           // dH_{l-1} = (g_in W_l) * (H_{l-1} > 0), and its column sums
            GemmDesc& D = G.d[G.nd++];
            D = GemmDesc{};
            D.A = direct(g_in, nullptr, 0, n_out, R);
            D.B = out_layer ? transposed(w.weight[L], wo_r, t.s, W, W, -1) : transposed(w.weight[l], nullptr, 0, W, W, -1);
            D.out.mode = EPI_MASK; D.out.c0 = D.out.c1 = B.dh[(l - 1) % 2]; D.out.split = R; D.out.ldc = W;
            D.out.mask = B.act[l - 1]; D.out.ldm = W; D.out.colsum_out = B.cs_dh[(l - 1) % 2];
            finish(D, R, W, n_out, tmx);
            if (l == 1 && fold_nw) {
                Output& O = D.out;
                O.fold = 1; O.fold_k0 = K0; O.fold_nw = fold_nw; O.fold_x = B.xbuf;
                O.fold_dw = w.weight_grad[0]; O.fold_db = w.bias_grad[0];
                O.fold_cs_tiles = tiles_r;   // <= 16: the fold's 32-row waves bound R by 512 (fold_waves)
                O.fold_gran = B.fold_gran; O.cs_gran = B.cs_gran; O.fold_serial = B.serial; O.fold_status = B.status;
                if (adam) {          // nothing in this launch reads layer 0's parameters
                    O.fold_adam = 1; O.fold_aw = adam[0]; O.fold_ab = adam[1];
                }
            }
        }
        {                       // dW_l = g_in^T X_l; db_l = the column sums of g_in over the row tiles
            GemmDesc& D = G.d[G.nd++];
            D = GemmDesc{};
            D.A = transposed(g_in, nullptr, 0, n_out, n_out, -1);
            D.B = l == 0 ? transposed(B.xbuf, nullptr, 0, K0, n_in, -1) : transposed(B.act[l - 1], nullptr, 0, W, n_in, -1);
            Output& O = D.out;
            O.mode = EPI_GRAD; O.ldc = n_in; O.colsum_in = cs_in; O.colsum_tiles = tiles_r;
            if (fused) O.colsum_in = nullptr;   // db_1 (and b_1's Adam step) came from O's last arrivers
            if (out_layer) {
                O.c0 = w.weight_grad[L]; O.c1 = t.reward ? w.weight_grad[L + 1] : w.weight_grad[L];
                O.split = t.reward ? t.s : J;
                O.g0 = w.bias_grad[L]; O.g1 = t.reward ? w.bias_grad[L + 1] : w.bias_grad[L];
            } else {
                O.c0 = O.c1 = w.weight_grad[l]; O.split = n_out;
                O.g0 = O.g1 = w.bias_grad[l];
            }
            finish(D, n_out, n_in, R, tmx);
            if (l == 1 && fold_nw) O.fold_sum = 1;   // row block 0's tiles finish dW_0 / db_0 (fold_sum)
        }
        if (adam && l == 0) {   // nothing in this launch reads layer 0's parameters: step them in place
            G.d[G.nd - 1].out.adam = 1;
            G.d[G.nd - 1].out.aw = adam[0];
            G.d[G.nd - 1].out.ab = adam[1];
        }
        if (adam && fused && l == 1) {
            // the dH_0 tiles of a column block read that block of W_1: the dW_1 tiles step it in place
            // once those tiles' K loops are done (dH_0 tiles have the lower ids)
            Output& O = G.d[G.nd - 1].out;
            O.adam = 1; O.aw = adam[2];
            O.wait_ticket = B.tickets + tiles_n;
            O.wait_count = (unsigned)((R + TT * tmx - 1) / (TT * tmx));
            O.wait_status = B.status;
            G.d[0].out.arrive_ticket = B.tickets + tiles_n;
        }
        // layer l + 1's gradient is complete (previous launch) and this launch does not read its
        // parameters: its Adam step rides along (with the reward head when l + 1 is the output layer)
        G.adam_count = 0;
        if (adam && l + 1 <= L) {
            const int first = 2 * (l + 1), n = (l + 1 == L && t.reward) ? 4 : 2;
            for (int i = 0; i < n; ++i) G.adam_t[G.adam_count++] = adam[first + i];
        }
        G.loss_part = B.loss_part; G.loss_parts = loss_parts; G.loss_out = loss_out;
        const bool loss_wg = l == l_end && loss_out != nullptr;
        G.xcd = xcd_opt;
        e = l == 0    ? launch_gemm<OP_TRANS, OP_TRANS>(G, loss_wg, stream)
            : tmx == 2 ? launch_gemm<OP_DIRECT, OP_TRANS, OP_TRANS, OP_TRANS, 2>(G, loss_wg, stream)
                       : launch_gemm<OP_DIRECT, OP_TRANS, OP_TRANS, OP_TRANS>(G, loss_wg, stream);
        if (e != hipSuccess) return e;
    }
    if (adam && fold_nw && !fused) {   // layer 1's step (launch 0's passenger before the fold): the next forward launch's
        const int n = (L == 1 && t.reward) ? 4 : 2;
        for (int i = 0; i < n; ++i) pending[i] = adam[2 + i];
        *pending_n = n;
    }
    return hipSuccess;
}

}  // namespace mbrl

#ifdef MBRL_STAMPS
extern "C" int mbrl_diag_set_train_stamps(void* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mbrl::g_train_stamps), &buf, sizeof(buf));
}
#endif
