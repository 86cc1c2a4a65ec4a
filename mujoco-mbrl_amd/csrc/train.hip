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
// workgroup: 4 waves split K, each accumulating a 32 x 32 partial with v_mfma_f32_16x16x4f32
// (lane l feeds A(m0 + l%16, k) and B(n0 + l%16, k) for k = kb + 4(l/16) + s, s = 0..3, so a lane's
// four k are consecutive and one float4 load serves four MFMAs when the operand is k-contiguous).
// The partials meet in LDS, summed in wave order, and the epilogue fuses what follows the product:
//   forward        H_l = relu(A W_l^T + b_l)                                  (EPI_ACT)
//   output layer   Y = H W_out^T + b_out;  dY = (Y - target) * 2 / numel, loss partials (EPI_LOSS)
//   backward dX    dH_{l-1} = (dH_l W_l) * (H_{l-1} > 0)                        (EPI_MASK)
//   backward dW    dW_l = dH_l^T H_{l-1}, db_l from a virtual ones column        (EPI_GRAD)
// The batch is gathered on the fly from the stacked transitions through the batch's row indices
// (no materialised input), and the state and reward heads are one output layer of s + 1 rows.
// Arithmetic is fp32 with fp32 accumulation; the summation order differs from autograd's, so the
// gradients agree with torch's to rounding (tests/test_gpu_train_native.py), not bit for bit.

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { OP_DIRECT = 0, OP_TRANS = 1, OP_GATHER = 2 };
enum { EPI_ACT = 0, EPI_LOSS = 1, EPI_MASK = 2, EPI_GRAD = 3 };
constexpr int TT = 32;              // C tile edge
constexpr int GEMM_THREADS = 256;   // 4 waves

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
    float* g0;                // EPI_GRAD: column bias_col is the bias gradient, g0[m] / g1[m - split]
    float* g1;
    int bias_col;
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
    // loss: one extra workgroup sums the partials (fixed order) into loss_out[0..2]
    const float* loss_part;
    int loss_parts;
    float* loss_out;
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

__device__ __forceinline__ f32x4 load_operand(const GemmLaunch& L, const Operand& o, int i, int k0, int K) {
    f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
    if (i >= o.rows) return v;
    if (i == o.ones_row) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = k0 + e < K ? 1.0f : 0.0f;
        return v;
    }
    if (o.kind == OP_DIRECT) {
        const float* row = storage_row(o, i);
        if (o.vec && k0 + 3 < K) return *reinterpret_cast<const f32x4*>(row + k0);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (k0 + e < K) v[e] = row[k0 + e];
    } else if (o.kind == OP_TRANS) {
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

__device__ void gemm_tile(const GemmLaunch& L, const GemmDesc& D, int tile, float (*red)[TT][TT + 1]) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, q = lane >> 4, c = lane & 15;
    const int m0 = (tile / D.tiles_n) * TT, n0 = (tile % D.tiles_n) * TT;
    // wave w takes the w-th quarter of K (in 16-deep chunks)
    const int chunks = (D.K + 15) >> 4, per = (chunks + 3) >> 2;
    const int kb0 = wave * per * 16, kb1 = min(D.K, (wave + 1) * per * 16);
    f32x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    f32x4 a[2], b[2];
    if (kb0 < kb1) {
#pragma unroll
        for (int x = 0; x < 2; ++x) a[x] = load_operand(L, D.A, m0 + 16 * x + c, kb0 + 4 * q, D.K);
#pragma unroll
        for (int y = 0; y < 2; ++y) b[y] = load_operand(L, D.B, n0 + 16 * y + c, kb0 + 4 * q, D.K);
    }
    for (int kb = kb0; kb < kb1; kb += 16) {
        f32x4 an[2], bn[2];
        const bool more = kb + 16 < kb1;
        if (more) {             // next chunk's operands in flight while this chunk's MFMAs issue
#pragma unroll
            for (int x = 0; x < 2; ++x) an[x] = load_operand(L, D.A, m0 + 16 * x + c, kb + 16 + 4 * q, D.K);
#pragma unroll
            for (int y = 0; y < 2; ++y) bn[y] = load_operand(L, D.B, n0 + 16 * y + c, kb + 16 + 4 * q, D.K);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
                    acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x][s], b[y][s], acc[x][y], 0, 0, 0);
        if (more) {
#pragma unroll
            for (int x = 0; x < 2; ++x) a[x] = an[x];
#pragma unroll
            for (int y = 0; y < 2; ++y) b[y] = bn[y];
        }
    }
    // lane l holds C rows 16x + 4q + v, column 16y + c
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int v = 0; v < 4; ++v) red[wave][16 * x + 4 * q + v][16 * y + c] = acc[x][y][v];
    __syncthreads();

    const Output& O = D.out;
    const int row = tid >> 3, col0 = (tid & 7) * 4, m = m0 + row;
    float loss_s = 0.0f, loss_r = 0.0f;
    if (m < D.M) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int n = n0 + col0 + e;
            if (n >= D.N) break;
            float v = red[0][row][col0 + e];
            v = v + red[1][row][col0 + e];
            v = v + red[2][row][col0 + e];
            v = v + red[3][row][col0 + e];
            if (O.mode == EPI_GRAD && n == O.bias_col) {
                (m < O.split ? O.g0[m] : O.g1[m - O.split]) = v;
                continue;
            }
            if (O.mode == EPI_ACT || O.mode == EPI_LOSS) v = v + (n < O.bsplit ? O.b0[n] : O.b1[n - O.bsplit]);
            if (O.mode == EPI_ACT && O.relu) v = v > 0.0f ? v : 0.0f;
            if (O.mode == EPI_MASK && !(O.mask[(int64_t)m * O.ldm + n] > 0.0f)) v = 0.0f;
            if (O.mode == EPI_LOSS) {
                const int64_t src = batch_row(L, m);
                const float t = n < O.s ? L.gns[src * O.s + n] : L.grw[src];
                const float d = v - t;
                if (n < O.s) loss_s += d * d * O.inv_s;
                else loss_r += d * d * O.inv_r;
                v = d * (n < O.s ? O.scale_s : O.scale_r);
            }
            float* dst = m < O.split ? O.c0 + (int64_t)m * O.ldc : O.c1 + (int64_t)(m - O.split) * O.ldc;
            dst[n] = v;
        }
    }
    if (O.mode == EPI_LOSS) {
        __syncthreads();        // red is reused for the partial-loss reduction
        float* sl = &red[0][0][0];
        sl[tid] = loss_s;
        sl[GEMM_THREADS + tid] = loss_r;
        __syncthreads();
        if (tid < 2) {
            float t = 0.0f;
            for (int i = 0; i < GEMM_THREADS; ++i) t = t + sl[tid * GEMM_THREADS + i];
            O.loss_part[tile * 2 + tid] = t;
        }
    }
}

__global__ __launch_bounds__(GEMM_THREADS) void train_gemm_kernel(const GemmLaunch L) {
    __shared__ float red[4][TT][TT + 1];
    int b = blockIdx.x;
    for (int i = 0; i < L.nd; ++i) {
        if (b < L.d[i].tiles) {
            gemm_tile(L, L.d[i], b, red);
            return;
        }
        b -= L.d[i].tiles;
    }
    // the loss workgroup: partials of the output-layer launch, summed in tile order
    if (threadIdx.x < 2 && L.loss_out) {
        float t = 0.0f;
        for (int i = 0; i < L.loss_parts; ++i) t = t + L.loss_part[i * 2 + threadIdx.x];
        L.loss_out[1 + threadIdx.x] = t;
        if (threadIdx.x == 0) {
            float u = 0.0f;
            for (int i = 0; i < L.loss_parts; ++i) u = u + L.loss_part[i * 2] + L.loss_part[i * 2 + 1];
            L.loss_out[0] = u;
        }
    }
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

static void finish(GemmDesc& D, int M, int N, int K) {
    D.M = M; D.N = N; D.K = K;
    D.tiles_n = (N + TT - 1) / TT;
    D.tiles = ((M + TT - 1) / TT) * D.tiles_n;
}

static hipError_t launch_gemm(GemmLaunch& L, bool loss_wg, hipStream_t stream) {
    int blocks = loss_wg ? 1 : 0;
    for (int i = 0; i < L.nd; ++i) blocks += L.d[i].tiles;
    if (!loss_wg) L.loss_out = nullptr;
    hipLaunchKernelGGL(train_gemm_kernel, dim3(blocks), dim3(GEMM_THREADS), 0, stream, L);
    return hipGetLastError();
}

size_t train_ws_floats(const TrainShape& t, int batch) {
    const size_t R = (size_t)batch * t.H, J = t.s + (t.reward ? 1 : 0);
    const size_t tiles_out = ((R + TT - 1) / TT) * ((J + TT - 1) / TT);
    auto up = [](size_t x) { return (x + 63) & ~(size_t)63; };
    return up(R * t.W) * (t.L + 2) + up(R * J) + up(tiles_out * 2);
}

hipError_t launch_train_grads(const TrainShape& t, const TrainTensors& w, const int64_t* idx, int batch,
                              float* loss_out, float* ws, hipStream_t stream) {
    const int R = batch * t.H, W = t.W, K0 = t.s + t.a, J = t.s + (t.reward ? 1 : 0), L = t.L;
    auto up = [](size_t x) { return (x + 63) & ~(size_t)63; };
    float* act[MBRL_TRAIN_MAX_LAYERS];
    for (int l = 0; l < L; ++l) act[l] = ws + up((size_t)R * W) * l;
    float* dh[2] = {ws + up((size_t)R * W) * L, ws + up((size_t)R * W) * (L + 1)};
    float* dy = ws + up((size_t)R * W) * (L + 2);
    float* loss_part = dy + up((size_t)R * J);
    const float* wo_r = t.reward ? w.weight[L + 1] : nullptr;
    const float* bo_r = t.reward ? w.bias[L + 1] : w.bias[L];

    GemmLaunch G{};
    G.idx = idx; G.gs = w.states; G.ga = w.actions; G.gns = w.next_states; G.grw = w.rewards;
    G.H = t.H; G.s = t.s; G.a = t.a;
    hipError_t e;
    // forward through the hidden layers
    for (int l = 0; l < L; ++l) {
        GemmDesc& D = G.d[0];
        D = GemmDesc{};
        if (l == 0) {
            D.A = Operand{};
            D.A.kind = OP_GATHER; D.A.rows = R; D.A.ones_row = -1; D.A.gather_trans = 0;
        } else {
            D.A = direct(act[l - 1], nullptr, 0, W, R);
        }
        D.B = direct(w.weight[l], nullptr, 0, l == 0 ? K0 : W, W);
        D.out.mode = EPI_ACT; D.out.c0 = D.out.c1 = act[l]; D.out.split = R; D.out.ldc = W;
        D.out.b0 = D.out.b1 = w.bias[l]; D.out.bsplit = W; D.out.relu = 1;
        finish(D, R, W, l == 0 ? K0 : W);
        G.nd = 1;
        if ((e = launch_gemm(G, false, stream)) != hipSuccess) return e;
    }
    // output layer (state head, reward head) + the loss gradient
    {
        GemmDesc& D = G.d[0];
        D = GemmDesc{};
        D.A = direct(act[L - 1], nullptr, 0, W, R);
        D.B = direct(w.weight[L], wo_r, t.s, W, J);
        Output& O = D.out;
        O.mode = EPI_LOSS; O.c0 = O.c1 = dy; O.split = R; O.ldc = J;
        O.b0 = w.bias[L]; O.b1 = bo_r; O.bsplit = t.s;
        O.scale_s = 2.0f / (float)((int64_t)batch * t.s); O.scale_r = 2.0f / (float)batch;
        O.inv_s = 1.0f / (float)((int64_t)batch * t.s); O.inv_r = 1.0f / (float)batch;
        O.s = t.s; O.loss_part = loss_part;
        finish(D, R, J, W);
        G.nd = 1;
        G.loss_part = loss_part; G.loss_parts = D.tiles;
        if ((e = launch_gemm(G, false, stream)) != hipSuccess) return e;
    }
    const int loss_parts = G.d[0].tiles;
    // backward: layer l = L (output) .. 0; launch l: dH_{l-1} (l >= 1) and dW_l, db_l
    for (int l = L; l >= 0; --l) {
        const bool out_layer = l == L;
        const float* g_in = out_layer ? dy : dh[l % 2];   // dL/d(pre-activation of layer l), [R][n_out]
        const int n_out = out_layer ? J : W, n_in = l == 0 ? K0 : W;
        G.nd = 0;
        if (l >= 1) {           // dH_{l-1} = (g_in W_l) * (H_{l-1} > 0)
            GemmDesc& D = G.d[G.nd++];
            D = GemmDesc{};
            D.A = direct(g_in, nullptr, 0, n_out, R);
            D.B = out_layer ? transposed(w.weight[L], wo_r, t.s, W, W, -1) : transposed(w.weight[l], nullptr, 0, W, W, -1);
            D.out.mode = EPI_MASK; D.out.c0 = D.out.c1 = dh[(l - 1) % 2]; D.out.split = R; D.out.ldc = W;
            D.out.mask = act[l - 1]; D.out.ldm = W;
            finish(D, R, W, n_out);
        }
        {                       // dW_l = g_in^T X_l, db_l = column sums of g_in (the ones column)
            GemmDesc& D = G.d[G.nd++];
            D = GemmDesc{};
            D.A = transposed(g_in, nullptr, 0, n_out, n_out, -1);
            if (l == 0) {
                D.B = Operand{};
                D.B.kind = OP_GATHER; D.B.rows = n_in + 1; D.B.ones_row = n_in; D.B.gather_trans = 1;
            } else {
                D.B = transposed(act[l - 1], nullptr, 0, W, n_in + 1, n_in);
            }
            Output& O = D.out;
            O.mode = EPI_GRAD; O.ldc = n_in; O.bias_col = n_in;
            if (out_layer) {
                O.c0 = w.weight_grad[L]; O.c1 = t.reward ? w.weight_grad[L + 1] : w.weight_grad[L]; O.split = t.s;
                O.g0 = w.bias_grad[L]; O.g1 = t.reward ? w.bias_grad[L + 1] : w.bias_grad[L];
                if (!t.reward) O.split = J;
            } else {
                O.c0 = O.c1 = w.weight_grad[l]; O.split = n_out;
                O.g0 = O.g1 = w.bias_grad[l];
            }
            finish(D, n_out, n_in + 1, R);
        }
        G.loss_part = loss_part; G.loss_parts = loss_parts; G.loss_out = loss_out;
        if ((e = launch_gemm(G, l == 0 && loss_out != nullptr, stream)) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace mbrl
