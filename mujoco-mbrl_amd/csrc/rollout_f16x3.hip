// Split-operand persistent rollout: the rollout_kernel (rollout.hip) schedule with every Linear
// emulating fp32 on the f16 matrix cores (mbrl_cem.h, MBRL_PRECISION_F16X3 / MBRL_PRECISION_F16X6).
//
// Why. The fp32 kernel is MFMA-bound: v_mfma_f32_16x16x4_f32 gives 32 MAC/clk/SIMD, and with
// 16 candidates per CU (N = 4096 over 256 CUs) every step re-streams the whole weight set (2.2 MB
// for 3x512) from L2 at ~65 GB/s per CU. v_mfma_f32_16x16x32_f16 gives 512 MAC/clk/SIMD, so
// the split products of each fp32 product cost 3/16 (F16X3) or 6/16 (F16X6) of the fp32
// instruction, and the step becomes bound by the L2 weight stream instead (~125 GB/s per CU when
// every CU streams, ~153 GB/s when half do: tools/ubench/l2stream.hip).
//
// Split into P pieces. An operand is scaled by an exact power of two (activations 2^4, weights
// 2^8) and split as x = x0 + x1 (+ x2) + r, x0 = f16(x), x1 = f16(x - x0), x2 = f16(x - x0 - x1):
// every difference is exact in fp32 and each piece keeps 11 more bits, so |r| <= 2^-22 |x| (P = 2)
// or 2^-33 |x| (P = 3) while the last piece is a normal f16 (P = 2: |x| >= 2^-6 activations,
// 2^-10 weights; P = 3: |x| >= 2^4 and 2^0); below that the error is absolute, under 2^-29
// (activations) and 2^-33 (weights). The kept products are every x_i w_j with i + j < P:
//   P = 2 (F16X3): x0w0 + x0w1 + x1w0; the dropped x1w1 is 2^-22 relative;
//   P = 3 (F16X6): x0w0 + x0w1 + x1w0 + x0w2 + x1w1 + x2w0; dropped terms <= 2^-33 relative.
// All into ONE fp32 accumulator (every product is at scale 2^12); the layer output is acc * 2^-12
// (exact). F16X6 thus carries operands to 33 significant bits (fp32: 24), forms the partial products
// exactly and accumulates in fp32. Scaled operands with |x| >= 32768 (activations >= 2048, weights
// >= 128) would not split: the workgroup then marks its candidates (MBRL_REDO_MARK) and the fp32
// kernel's redo pass recomputes them.
//
// Operand layouts for v_mfma_f32_16x16x32_f16 (cdna_hip_programming.md §3): lane l holds
// A[row l&15][k = 8(l>>4) + e] and B[k = 8(l>>4) + e][col l&15], e = 0..7; C as the f32 form.
// Weights are A (Y^T = W X^T, as rollout.hip), activations are B, so the accumulator of tile j
// holds units 16j + 4(l>>4) + v of candidate l&15.
//   * hidden-type layers (layer 0, W -> W): B comes from LDS, rows [x0: kmax | x1: kmax (| x2)]
//     per candidate; chunk kc covers K rows 32kc .. 32kc + 31 in natural order.
//   * output layer: K split over the 8 waves and fed from registers. A K-chunk pairs two of the
//     wave's own tiles (2kk, 2kk+1): lane group g's eight k are units {4g..4g+3} of each, exactly
//     what its accumulators hold; the weight pack uses the same permutation (cem.hip).
// One workgroup = 8 waves = 16 R candidates of one member for all H steps; wave w owns units
// [w W/8, (w+1) W/8) of every hidden layer (TW = T/2 tiles). Per chunk a wave loads TW P fragments
// (TW tiles x P pieces, 1 KiB each) through a register ring of 4 slots of TS tiles (TS P fragments),
// 3 slots ahead across layers and steps.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mbrl_internal.h"

namespace mbrl {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int SW = 8;       // waves per workgroup
constexpr int SNB = 4;      // weight ring depth (chunks)
constexpr int SMAXA = 3;    // action slots per lane (a <= 48)
// Operand scaling (exact powers of two, mbrl_internal.h): activations x 2^4, weights x 2^8, so the
// residual pieces stay normal f16 for |x| >= 2^-6 and |w| >= 2^-10 (smaller operands keep an
// absolute error below 2^-29 and 2^-33); every product lands at 2^12 and is unscaled once.
constexpr float X_SCALE = MBRL_SPLIT_X_SCALE;
constexpr float OUT_UNSCALE = 1.0f / (MBRL_SPLIT_X_SCALE * MBRL_SPLIT_W_SCALE);
constexpr float SPLIT_LIMIT = 32768.0f;     // |scaled operand| past this: redo in fp32

#define SPIN() __builtin_amdgcn_sched_barrier(0)

struct SplitLds {
    _Float16 *x, *y;   // activation rows [x0: kmax | x1: kmax (| x2)]; y == x without ping-pong (R = 2)
    float *part, *acs, *obs_mean, *obs_std, *act_mean, *act_std, *goal, *cw, *hbias;
    int* flag;
    size_t bytes;
};

__host__ __device__ inline int split_kmax(const RolloutArgs& A) {
    const int k0 = 32 * A.K0S;
    return A.Wpad > k0 ? A.Wpad : k0;
}

// R = 1: ping-pong activation buffers (one barrier per layer); R = 2: one buffer, written after a
// second barrier, so that 32 candidates fit the 160 KiB
__host__ __device__ inline SplitLds split_lds(const RolloutArgs& A, int R, void* base) {
    SplitLds L;
    size_t o = 0;
    char* b = static_cast<char*>(base);
    auto take = [&](size_t bytes) {
        void* p = b ? b + o : nullptr;
        o += (bytes + 15) & ~(size_t)15;
        return p;
    };
    const size_t M = 16 * (size_t)R;
    L.x = static_cast<_Float16*>(take(M * A.sr * 2));
    L.y = R == 1 ? static_cast<_Float16*>(take(M * A.sr * 2)) : L.x;
    L.part = static_cast<float*>(take((size_t)SW * M * A.pw * 4));
    L.acs = static_cast<float*>(take(2 * M * 4));
    L.obs_mean = static_cast<float*>(take(A.s * 4));
    L.obs_std = static_cast<float*>(take(A.s * 4));
    L.act_mean = static_cast<float*>(take(A.a * 4));
    L.act_std = static_cast<float*>(take(A.a * 4));
    L.goal = static_cast<float*>(take(A.s * 4));
    L.cw = static_cast<float*>(take(A.s * 4));
    L.hbias = static_cast<float*>(take(((size_t)A.L * A.Wpad + 16 * (size_t)A.NOT) * 4));
    L.flag = static_cast<int*>(take(16));
    L.bytes = o;
    return L;
}

// x -> P f16 pieces (scaled by X_SCALE); flags an operand outside the split range
template <int P>
__device__ __forceinline__ void split4(const f32x4 x0, f16x4 (&pc)[P], bool& ovf) {
    f32x4 x = x0 * X_SCALE;
    const f32x4 ax = __builtin_elementwise_abs(x);
    ovf |= (ax.x >= SPLIT_LIMIT) | (ax.y >= SPLIT_LIMIT) | (ax.z >= SPLIT_LIMIT) | (ax.w >= SPLIT_LIMIT);
#pragma unroll
    for (int q = 0; q < P; ++q) {
        pc[q] = __builtin_convertvector(x, f16x4);
        if (q + 1 < P) x = x - __builtin_convertvector(pc[q], f32x4);
    }
}

template <int P>
__device__ __forceinline__ void split_store1(float x0, _Float16* row, int kmax, int d, bool& ovf) {
    float x = x0 * X_SCALE;
    ovf |= fabsf(x) >= SPLIT_LIMIT;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        const _Float16 h = (_Float16)x;
        row[q * kmax + d] = h;
        if (q + 1 < P) x = x - (float)h;
    }
}

__device__ __forceinline__ f32x4 mfma16(const f32x4 a_raw, const f16x8 b, const f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a_raw), b, c, 0, 0, 0);
}

template <int FR>
__device__ __forceinline__ void sload(f32x4 (&dst)[FR], __amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned soff) {
#pragma unroll
    for (int f = 0; f < FR; ++f)
        dst[f] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + (unsigned)(f * 1024), soff, 0));
}

template <int P>
__device__ __forceinline__ void read_b(f16x8 (&b)[P], const _Float16* act, int sr, int kmax, int kc, int lane, int r) {
    const _Float16* row = act + (16 * r + (lane & 15)) * sr + 32 * kc + 8 * (lane >> 4);
#pragma unroll
    for (int q = 0; q < P; ++q) b[q] = *reinterpret_cast<const f16x8*>(row + q * kmax);
}

// acc += sum over i + j < P of x_i w_j (w: this tile's P fragments)
template <int P>
__device__ __forceinline__ f32x4 split_mma(const f32x4* w, const f16x8 (&x)[P], f32x4 acc) {
#pragma unroll
    for (int d = 0; d < P; ++d)          // order: by significance, x0w0 first
#pragma unroll
        for (int i = 0; i <= d; ++i) acc = mfma16(w[d - i], x[i], acc);
    return acc;
}

template <int TW>
__device__ __forceinline__ f32x4 layer_out(const f32x4 (&acc)[TW], const float* hb, int wave, int j, int lane) {
    const f32x4 bias = *reinterpret_cast<const f32x4*>(hb + wave * 16 * TW + 16 * j + 4 * (lane >> 4));
    const f32x4 v = acc[j] * OUT_UNSCALE + bias;
    return __builtin_elementwise_max(v, f32x4{0.f, 0.f, 0.f, 0.f});
}

__device__ __forceinline__ float rowsum16(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x122, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x121, 0xF, 0xF, false));
    return v;
}

template <int T, int R, int P, int TS, int K0S, int NOS>
struct SplitRollout {
    static constexpr int M = 16 * R;        // candidates per workgroup (R 16-column B tiles)
    static constexpr bool PP = R == 1;      // ping-pong activation buffers (split_lds)
    static constexpr int TW = T / 2;        // tiles per wave per hidden layer
    static constexpr int FR = TW * P;       // fragments per wave per chunk (TW tiles x P pieces)
    static constexpr int FS = TS * P;       // fragments per ring slot
    static constexpr int SUB = TW / TS;     // ring slots per chunk
    static constexpr int KH = 2 * T;        // chunks per hidden layer
    static constexpr int SS = 2 * NOS;      // state slots per lane (ceil(s / 16) <= NOT)
    static constexpr int SHIFT = ((K0S + NOS) * SUB) % SNB;
    static_assert(TW % 2 == 0 && TW % TS == 0 && (KH * SUB) % SNB == 0 && (SHIFT == 0 || 2 * SHIFT == SNB),
                  "ring phases");

    const RolloutArgs& A;
    const SplitLds& L;
    const int wave, lane, tile, e, kmax;
    const bool epi, actw;
    __amdgpu_buffer_rsrc_t rsrc;
    unsigned voff;
    f32x4 ring[SNB][FS];
    f32x4 acc[R][TW];
    float av[R][SMAXA];
    float total[R];
    bool ovf = false;
    int g = 0;                      // ring-slot index within the step

    __device__ SplitRollout(const RolloutArgs& A_, const SplitLds& L_, int wave_, int lane_, int tile_, int e_,
                            const float* member)
        : A(A_), L(L_), wave(wave_), lane(lane_), tile(tile_), e(e_), kmax(split_kmax(A_)), epi(wave_ < 4),
          actw(wave_ >= 4) {
        rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(member + A.split_off), 0,
                                                 (int)((size_t)A.CS * SW * FR * 1024), 0x00020000);
        voff = (unsigned)((wave * FR * 64 + lane) * 16);
#pragma unroll
        for (int r = 0; r < R; ++r) total[r] = 0.f;
    }

    // epilogue / action row of this lane in candidate tile r: 16 r + 4 (wave & 3) + (lane >> 4)
    __device__ __forceinline__ int row_of(int r) const { return 16 * r + 4 * (wave & 3) + (lane >> 4); }

    // ring slot G of the step sequence (wrapping into the next step): chunk G / SUB, fragments
    // [FS (G % SUB), FS (G % SUB + 1)) of this wave's slice
    __device__ __forceinline__ void load_slot(f32x4 (&dst)[FS], int G) {
        const int css = A.CS * SUB;
        const int gp = G < css ? G : G - css;
        const unsigned soff = (unsigned)(gp / SUB) * (unsigned)(SW * FR * 1024) + (unsigned)((gp % SUB) * FS * 1024);
        sload<FS>(dst, rsrc, voff, soff);
    }

    __device__ __forceinline__ void fetch_actions(int t) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int n = min(tile * M + row_of(r), A.N - 1);
            const float* src = A.actions + ((size_t)t * A.N + n) * A.a;
#pragma unroll
            for (int k = 0; k < SMAXA; ++k) av[r][k] = src[min((lane & 15) + 16 * k, A.a - 1)];
        }
    }

    // a_t -> normalised, split MLP input columns [s, s + a); CoshLoss row sums -> acs[slot]
    __device__ __forceinline__ void stage_actions(int slot) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int m = row_of(r);
            _Float16* row = L.x + m * A.sr;
            float c = 0.f;
#pragma unroll
            for (int k = 0; k < SMAXA; ++k) {
                const int d = (lane & 15) + 16 * k;
                if (d < A.a) {
                    const float x = av[r][k];
                    split_store1<P>(A.norm_a ? (x - L.act_mean[d]) / L.act_std[d] : x, row, kmax, A.s + d, ovf);
                    if (A.has_ac) c += coshf(x / A.alpha_a) - 1.0f;
                }
            }
            c = rowsum16(c);
            if ((lane & 15) == 0) L.acs[slot * M + m] = c;
        }
    }

    __device__ __forceinline__ void zero_pad() {
        const int k0 = A.s + A.a, k1 = 32 * A.K0S;
        for (int i = threadIdx.x; i < M * (k1 - k0); i += 64 * SW) {
            const int m = i / (k1 - k0), d = k0 + i - (i / (k1 - k0)) * (k1 - k0);
#pragma unroll
            for (int q = 0; q < P; ++q) L.x[m * A.sr + q * kmax + d] = (_Float16)0.f;
        }
    }

    __device__ void prologue() {
        for (int i = threadIdx.x; i < A.s; i += 64 * SW) {
            L.obs_mean[i] = A.obs_mean ? A.obs_mean[i] : 0.f;
            L.obs_std[i] = A.obs_std ? A.obs_std[i] : 1.f;
            L.goal[i] = A.goal ? A.goal[i] : 0.f;
            L.cw[i] = A.cw ? A.cw[i] : 0.f;
        }
        for (int i = threadIdx.x; i < A.a; i += 64 * SW) {
            L.act_mean[i] = A.act_mean ? A.act_mean[i] : 0.f;
            L.act_std[i] = A.act_std ? A.act_std[i] : 1.f;
        }
        const float* bias_src = A.packed + (size_t)e * A.member_stride + A.stream_floats;
        for (int i = threadIdx.x; i < A.L * A.Wpad + 16 * A.NOT; i += 64 * SW) L.hbias[i] = bias_src[i];
        if (threadIdx.x == 0) L.flag[0] = 0;
        if (actw) fetch_actions(0);
        __syncthreads();
        for (int i = threadIdx.x; i < M * A.s; i += 64 * SW) {
            const int m = i / A.s, d = i - (i / A.s) * A.s;
            const int n = min(tile * M + m, A.N - 1);
            const float sv = A.s0_per_cand ? A.s0[(size_t)n * A.s + d] : A.s0[d];
            split_store1<P>(A.norm_s ? (sv - L.obs_mean[d]) / L.obs_std[d] : sv, L.x + m * A.sr, kmax, d, ovf);
        }
        zero_pad();
        if (actw) stage_actions(0);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < SNB - 1; ++q) load_slot(ring[q], q);
    }

    // refill the slot that slot g-1 vacated with slot g+SNB-1; `slot` folds to a constant once the
    // chunk loops are unrolled (the ring must stay in registers)
    __device__ __forceinline__ void prefetch(int slot) {
        load_slot(ring[(slot + SNB - 1) % SNB], g + SNB - 1);
    }

    __device__ __forceinline__ void zero_acc() {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < TW; ++j) acc[r][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // Hidden-type layer over NK chunks (NK * SUB ring slots from slot S0), B rows from `in`. The B
    // fragments of chunk kc + 1 are read one chunk ahead when R = 1; at R = 2 (twice the B and
    // accumulator registers) they are read at the head of their own chunk, behind its first
    // slot's weight prefetch.
    template <int S0, int NK>
    __device__ __forceinline__ void hidden_layer(const _Float16* in) {
        constexpr int NBB = R == 1 ? 2 : 1;
        zero_acc();
        f16x8 bx[NBB][R][P];
        if (NBB == 2)
#pragma unroll
            for (int r = 0; r < R; ++r) read_b<P>(bx[0][r], in, A.sr, kmax, 0, lane, r);
#pragma unroll
        for (int kc = 0; kc < NK; ++kc) {
#pragma unroll
            for (int h = 0; h < SUB; ++h) {
                const int slot = (S0 + kc * SUB + h) % SNB;
                prefetch(slot);
                const int b = NBB == 2 ? (kc & 1) : 0;
                if (h == 0) {
                    if (NBB == 2) {
                        if (kc + 1 < NK)
#pragma unroll
                            for (int r = 0; r < R; ++r) read_b<P>(bx[(kc + 1) & 1][r], in, A.sr, kmax, kc + 1, lane, r);
                    } else {
#pragma unroll
                        for (int r = 0; r < R; ++r) read_b<P>(bx[0][r], in, A.sr, kmax, kc, lane, r);
                    }
                }
                const f32x4(&w)[FS] = ring[slot];
                // significance-ordered products, interleaved over this slot's tiles and the R tiles
#pragma unroll
                for (int d = 0; d < P; ++d)
#pragma unroll
                    for (int i = 0; i <= d; ++i)
#pragma unroll
                        for (int j = 0; j < TS; ++j)
#pragma unroll
                            for (int r = 0; r < R; ++r)
                                acc[r][TS * h + j] = mfma16(w[P * j + d - i], bx[b][r][i], acc[r][TS * h + j]);
                SPIN();
                ++g;
            }
        }
    }

    // bias + ReLU + split of this wave's tiles into the next layer's B rows. Without ping-pong the
    // input rows are overwritten, so every wave must be done reading them first.
    __device__ __forceinline__ void produce(const float* hb, _Float16* out) {
        if (!PP) __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < TW; ++j) {
                f16x4 pc[P];
                split4<P>(layer_out<TW>(acc[r], hb, wave, j, lane), pc, ovf);
                _Float16* row = out + (16 * r + (lane & 15)) * A.sr + 16 * (wave * TW + j) + 4 * (lane >> 4);
#pragma unroll
                for (int q = 0; q < P; ++q) *reinterpret_cast<f16x4*>(row + q * kmax) = pc[q];
            }
        __syncthreads();
    }

    // Output layer (K split over the waves, B from this wave's last hidden tiles) -> part[wave].
    // Output chunk q pairs tiles 2q + u (u = 0, 1); its fragments are (u TW/2 + kk) P + piece, so
    // ring slot h of the chunk holds the (u, kk) pairs [h TS, (h + 1) TS).
    template <int S0>
    __device__ __forceinline__ void output_layer(const float* hb) {
        constexpr int KK = TW / 2;
        f16x8 ox[R][KK][P];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
                f16x4 p0[P], p1[P];
                split4<P>(layer_out<TW>(acc[r], hb, wave, 2 * kk, lane), p0, ovf);
                split4<P>(layer_out<TW>(acc[r], hb, wave, 2 * kk + 1, lane), p1, ovf);
#pragma unroll
                for (int q = 0; q < P; ++q) ox[r][kk][q] = __builtin_shufflevector(p0[q], p1[q], 0, 1, 2, 3, 4, 5, 6, 7);
            }
        float* part = L.part + wave * M * A.pw + (lane & 15) * A.pw + 4 * (lane >> 4);
#pragma unroll
        for (int q = 0; q < NOS; ++q) {
            f32x4 o[2][R];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < R; ++r) o[u][r] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int h = 0; h < SUB; ++h) {
                const int slot = (S0 + q * SUB + h) % SNB;
                prefetch(slot);
                const f32x4(&w)[FS] = ring[slot];
#pragma unroll
                for (int d = 0; d < P; ++d)
#pragma unroll
                    for (int i = 0; i <= d; ++i)
#pragma unroll
                        for (int jj = 0; jj < TS; ++jj) {
                            const int pair = TS * h + jj, u = pair / KK, kk = pair % KK;
#pragma unroll
                            for (int r = 0; r < R; ++r) o[u][r] = mfma16(w[P * jj + d - i], ox[r][kk][i], o[u][r]);
                        }
                SPIN();
                ++g;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < R; ++r)
                    *reinterpret_cast<f32x4*>(part + 16 * r * A.pw + 16 * (2 * q + u)) = o[u][r] * OUT_UNSCALE;
        }
    }

    // Goal-state epilogue of step t on waves 0-3 (R rows per lane group), actions a_{t+1} on 4-7.
    __device__ __forceinline__ void epilogue(int t) {
        if (epi) {
            const int ws = M * A.pw;
            const int j = lane & 15;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int m = row_of(r);
                const int n = tile * M + m;
                _Float16* row = L.x + m * A.sr;
                float sc = 0.f;
#pragma unroll
                for (int k = 0; k < SS; ++k) {
                    const int d = j + 16 * k;
                    if (d < A.s) {
                        const int ro = m * A.pw + d;
                        float o = sum_partials<8>(L.part, ws, ro);
                        const float om = L.obs_mean[d], os = L.obs_std[d];
                        o = o + L.hbias[A.L * A.Wpad + d];
                        const float sn = A.unnorm_s ? o * os + om : o;
                        if (A.has_sc) {
                            const float x = (sn - L.goal[d]) * L.cw[d];
                            sc += sqrtf(x * x + A.alpha_s2) - A.alpha_s;
                        }
                        split_store1<P>(A.norm_s ? (sn - om) / os : sn, row, kmax, d, ovf);
                        if (A.states_out != nullptr && n < A.N)
                            A.states_out[(((size_t)e * A.H + t) * A.N + n) * A.s + d] = sn;
                    }
                }
                sc = rowsum16(sc);
                const float ac = L.acs[(t & 1) * M + m];
                total[r] += sc + A.alpha_a2 * (ac / (float)A.a);
            }
        } else if (t + 1 < A.H) {
            stage_actions((t + 1) & 1);
        }
        zero_pad();
        __syncthreads();
    }

    template <int PH>
    __device__ __forceinline__ void step(int t) {
        g = 0;
        if (actw && t + 1 < A.H) fetch_actions(t + 1);
        this->template hidden_layer<PH, K0S>(L.x);
        constexpr int SH = (PH + K0S * SUB) % SNB;
        if (A.L > 1) {
            produce(L.hbias, L.y);
            const _Float16* in = L.y;
            _Float16* out = L.x;
            for (int l = 1; l < A.L; ++l) {
                this->template hidden_layer<SH, KH>(in);
                if (l + 1 < A.L) {
                    produce(L.hbias + l * A.Wpad, out);
                    const _Float16* tmp = in;
                    in = out;
                    out = const_cast<_Float16*>(tmp);
                }
            }
        }
        this->template output_layer<SH>(L.hbias + (A.L - 1) * A.Wpad);
        __syncthreads();
        epilogue(t);
    }

    __device__ void finish() {
        if (__any(ovf) && lane == 0) L.flag[0] = 1;
        __syncthreads();
        const bool redo = L.flag[0] != 0;
        if (epi && (lane & 15) == 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int n = tile * M + row_of(r);
                if (n < A.N) A.costs[(size_t)e * A.N + n] = redo ? __uint_as_float(MBRL_REDO_MARK) : total[r];
            }
        }
    }
};

template <int T, int R, int P, int TS, int K0S, int NOS>
__global__ void __launch_bounds__(64 * SW, 1) rollout_split_kernel(const RolloutArgs A) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int M = 16 * R;
    const SplitLds L = split_lds(A, R, smem);
    const int tid = threadIdx.x;
    const int tile = blockIdx.x, e = blockIdx.y;
    const float* member = A.packed + (size_t)e * A.member_stride;
    // a weight outside the split range (flag word written by the pack): leave it all to the redo pass
    const unsigned bad = *reinterpret_cast<const unsigned*>(member + A.split_off + (size_t)A.CS * 2048 * T * P / 2);
    if (bad != 0u) {
        if (tid < M && tile * M + tid < A.N) A.costs[(size_t)e * A.N + tile * M + tid] = __uint_as_float(MBRL_REDO_MARK);
        return;
    }
    SplitRollout<T, R, P, TS, K0S, NOS> S(A, L, tid >> 6, tid & 63, tile, e, member);
    S.prologue();
    constexpr int SHIFT = SplitRollout<T, R, P, TS, K0S, NOS>::SHIFT;
    for (int t = 0; t < A.H; t += 2) {
        S.template step<0>(t);
        if (t + 1 < A.H) S.template step<SHIFT>(t + 1);
    }
    S.finish();
}

// ring-slot width: 2 tiles, or 1 tile where 2 would not fit the registers without spilling
// (P = 3 at R = 2, or with three layer-0 / output chunks)
template <int R, int P, int K0S, int NOS>
constexpr int split_ts() { return (P == 2 || (R == 1 && K0S <= 2 && NOS <= 2)) ? 2 : 1; }

template <int T, int R, int P, int K0S, int NOS>
hipError_t launch_split_t(const RolloutArgs& A, hipStream_t stream) {
    const auto fn = &rollout_split_kernel<T, R, P, split_ts<R, P, K0S, NOS>(), K0S, NOS>;
    hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(fn), 160 * 1024);
    if (err != hipSuccess) return err;
    dim3 grid((A.N + 16 * R - 1) / (16 * R), A.E);
    hipLaunchKernelGGL(fn, grid, dim3(64 * SW), rollout_split_lds_bytes(A, R), stream, A);
    return hipGetLastError();
}

}  // namespace

size_t rollout_split_lds_bytes(const RolloutArgs& A, int R) {
    const size_t need = split_lds(A, R, nullptr).bytes;
    const size_t floor_bytes = 82 * 1024;   // one workgroup per CU, as rollout_lds_bytes
    return need > floor_bytes ? need : floor_bytes;
}

#define MBRL_SPLIT_SHAPES(X) X(1, 1) X(2, 2) X(3, 1) X(1, 3) X(3, 3)

bool rollout_split_supported(const RolloutArgs& A, int T, int R, int P) {
    if (R != 1 && !(R == 2 && A.NOT == 2)) return false;
    if (P != 2 && P != 3) return false;
    if (A.reward || (T != 4 && T != 8) || A.a > 16 * SMAXA) return false;
    if (A.s > 16 * (A.NOT) || A.NOT != 2 * (A.CS - A.K0S - (A.L - 1) * 2 * T)) return false;
    if (rollout_split_lds_bytes(A, R) > 160 * 1024) return false;
    const int nos = A.NOT / 2;
#define MBRL_SPLIT_OK(K, N) if (A.K0S == K && nos == N) return true;
    MBRL_SPLIT_SHAPES(MBRL_SPLIT_OK)
#undef MBRL_SPLIT_OK
    return false;
}

hipError_t launch_rollout_split(const RolloutArgs& A, int T, int R, int P, hipStream_t stream) {
    const int nos = A.NOT / 2;
    // R = 2 only where its registers fit without spilling (one output chunk: NOS == 1)
#define MBRL_SPLIT_CASE(K, N)                                                                          \
    if (A.K0S == K && nos == N) {                                                                      \
        if (T == 4 && R == 1 && P == 2) return launch_split_t<4, 1, 2, K, N>(A, stream);               \
        if (T == 8 && R == 1 && P == 2) return launch_split_t<8, 1, 2, K, N>(A, stream);               \
        if (T == 4 && R == 1 && P == 3) return launch_split_t<4, 1, 3, K, N>(A, stream);               \
        if (T == 8 && R == 1 && P == 3) return launch_split_t<8, 1, 3, K, N>(A, stream);               \
        if constexpr (N == 1) {                                                                        \
            if (T == 4 && R == 2 && P == 2) return launch_split_t<4, 2, 2, K, N>(A, stream);           \
            if (T == 8 && R == 2 && P == 2) return launch_split_t<8, 2, 2, K, N>(A, stream);           \
            if (T == 4 && R == 2 && P == 3) return launch_split_t<4, 2, 3, K, N>(A, stream);           \
            if (T == 8 && R == 2 && P == 3) return launch_split_t<8, 2, 3, K, N>(A, stream);           \
        }                                                                                              \
    }
    MBRL_SPLIT_SHAPES(MBRL_SPLIT_CASE)
#undef MBRL_SPLIT_CASE
    return hipErrorInvalidValue;
}

}  // namespace mbrl
