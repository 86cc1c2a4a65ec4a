// Weight packing, elite selection, CEM refit, proposal sampling and the extern "C" ABI
// (include/mbrl_cem.h).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <dlfcn.h>

#include <atomic>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>
#include <algorithm>

#include "../../include/mbrl_cem.h"
#include "mbrl_internal.h"
#include <rccl/rccl.h>
#include "mbrl_rng.h"

namespace mbrl {

static thread_local std::string g_err;

// mbrl_set_option switches (include/mbrl_cem.h MBRL_OPT_*); 0 = automatic.
static std::atomic<int> g_opt[MBRL_OPT_COUNT];
// MBRL_OPT_ROLLOUT_PAIR = 0 (auto) takes column-split pairs for small plans (2 = never, the A/B)
static constexpr bool kPairAuto = true;
// traj_coop_kernel hand-off mode under MBRL_OPT_TRAJ_HOP = 0 (TrajArgs.hop_mode)
static constexpr int kTrajHopDefault = 2;

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

static int hip_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return MBRL_OK;
    return fail(MBRL_EHIP, "%s: %s", what, hipGetErrorString(e));
}

// Compute units of the current device (cached per device; 256 on MI355X).
static int device_cus() {
    static std::mutex mu;
    static std::map<int, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
    return n;
}

int device_cu_count() { return device_cus(); }

hipError_t ensure_dynamic_lds(const void* fn, int bytes) {
    static std::mutex mu;
    static std::set<std::tuple<const void*, int, int>> done;
    int dev = 0;
    hipError_t err = hipGetDevice(&dev);
    if (err != hipSuccess) return err;
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({fn, dev, bytes})) return hipSuccess;
    err = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (err == hipSuccess) done.insert({fn, dev, bytes});
    return err;
}

bool grid_fits(const void* fn, int threads, size_t lds, int blocks) {
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, size_t, int>, int> cache;   // -> resident workgroups
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    const auto key = std::make_tuple(fn, threads, lds, dev);
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return blocks <= it->second;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, lds) != hipSuccess) per_cu = 0;
    const int capacity = per_cu * device_cus();
    std::lock_guard<std::mutex> lock(mu);
    cache[key] = capacity;
    return blocks <= capacity;
}

// ------------------------------------------------------------------------------------------------
// Weight packing: nn.Linear [out][in] -> fragment stream (see rollout.hip header)
// ------------------------------------------------------------------------------------------------
// Canonical K order of a W->W layer (r05, DESIGN.md §3 "half-rotated K order"): an output column in
// the second half (n >= Wpad / 2) consumes its K chunks rotated by half, [nkc/2, nkc) then
// [0, nkc/2), so the column half a workgroup owns always starts on the inputs it produced itself
// (the column-split pairs' hand-off then lands behind half a layer of compute). Every fp32 tile
// height packs and reads the same order, so their sums stay bit-identical.
__device__ __forceinline__ int rot_chunk(int kc, int nkc, int n, int Wpad, int rot) {
    return (rot && 2 * n >= Wpad) ? (kc + nkc / 2) % nkc : kc;
}

// Hidden-type layer (layer 0 or W->W): chunk kc holds K rows 16kc..16kc+15 for this wave's T tiles
// (rot: a W->W layer, second-half columns in the rotated order above).
__global__ void pack_hidden_kernel(const float* __restrict__ w, int in_real, int out_real, int nkc, int T,
                                   int rot, float* __restrict__ dst /* chunk base */) {
    const size_t total = (size_t)nkc * 4 * T * 64 * 4;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int s = (int)(i & 3);
        const int lane = (int)((i >> 2) & 63);
        const size_t frag = i >> 8;           // (kc * 4 + wave) * T + j
        const int j = (int)(frag % T);
        const int wave = (int)((frag / T) & 3);
        const int kc = (int)(frag / T / 4);
        const int n = wave * 16 * T + 16 * j + (lane & 15);
        const int k = 16 * rot_chunk(kc, nkc, n, 64 * T, rot) + 4 * (lane >> 4) + s;
        dst[i] = (n < out_real && k < in_real) ? w[(size_t)n * in_real + k] : 0.0f;
    }
}

// Output layer: chunk j = output tile j; fragment kc covers this wave's K rows w*16T + 16kc + ...
// Rows [0, out_real) come from w; with a reward head, row out_real comes from w_r ([1][in]).
__global__ void pack_out_kernel(const float* __restrict__ w, const float* __restrict__ w_r, int in_real,
                                int out_real, int NOT, int T, float* __restrict__ dst) {
    const size_t total = (size_t)NOT * 4 * T * 64 * 4;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int s = (int)(i & 3);
        const int lane = (int)((i >> 2) & 63);
        const size_t frag = i >> 8;           // (j * 4 + wave) * T + kc
        const int kc = (int)(frag % T);
        const int wave = (int)((frag / T) & 3);
        const int j = (int)(frag / T / 4);
        const int n = 16 * j + (lane & 15);
        const int k = wave * 16 * T + 16 * kc + 4 * (lane >> 4) + s;
        float v = 0.0f;
        if (k < in_real) {
            if (n < out_real) v = w[(size_t)n * in_real + k];
            else if (w_r && n == out_real) v = w_r[k];
        }
        dst[i] = v;
    }
}

// 8-candidate stream (rollout.hip rollout_m8_kernel): per 16-deep chunk, per wave (T of them), per
// step s (4), lane l, element q: row 32 (2 pair + ((l >> 2) & 1)) + 4 (l >> 3) + (l & 3) -- the odd
// 4-lane blocks carry the pair's second 32-row tile (ABID 1) -- and k = 16 kc + 4 q + s.
// Hidden-type layers: chunk kc, pair = the wave's own tiles (rows 64 wave + ...).
// KP mode (Wpad 256, one 32-row output tile; rollout.hip m8_kp): 8 waves of one tile, per chunk
// per wave 2 loads x 64 lanes x float4; pair pi = 4 j + e, position p = 2 pi + ((l >> 2) & 1) of
// the chunk order p = 4 s + q, row 32 wave + 4 (l >> 3) + (l & 3).
__device__ __forceinline__ void m8kp_index(size_t i, int& lane, int& wave, size_t& chunk, int& s, int& q) {
    const int e = (int)(i & 3);
    lane = (int)((i >> 2) & 63);
    const int j = (int)((i >> 8) & 1);
    const size_t cw = i >> 9;                 // chunk * 8 + wave
    wave = (int)(cw & 7);
    chunk = cw >> 3;
    const int p = 2 * (4 * j + e) + ((lane >> 2) & 1);
    s = p >> 2;
    q = p & 3;
}

__global__ void pack_m8_hidden_kernel(const float* __restrict__ w, int in_real, int out_real, int nkc, int T,
                                      int kp, int rot, float* __restrict__ dst) {
    const size_t total = (size_t)nkc * T * 1024;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        int n, k;
        if (kp) {
            int lane, wave, s, q;
            size_t kc;
            m8kp_index(i, lane, wave, kc, s, q);
            n = 32 * wave + 4 * (lane >> 3) + (lane & 3);
            k = 16 * rot_chunk((int)kc, nkc, n, 64 * T, rot) + 4 * q + s;
        } else {
            const int q = (int)(i & 3);
            const int lane = (int)((i >> 2) & 63);
            const int s = (int)((i >> 8) & 3);
            const size_t cw = i >> 10;            // kc * T + wave
            const int wave = (int)(cw % T);
            const int kc = (int)(cw / T);
            n = 64 * wave + 32 * ((lane >> 2) & 1) + 4 * (lane >> 3) + (lane & 3);
            k = 16 * rot_chunk(kc, nkc, n, 64 * T, rot) + 4 * q + s;
        }
        dst[i] = (n < out_real && k < in_real) ? w[(size_t)n * in_real + k] : 0.0f;
    }
}

// Output layer over the wave's own K rows 64 wave + 16 kc + ...: with one 32-row tile (kpair) chunk o
// holds own K chunks 2o (even blocks) and 2o + 1 (odd blocks); else chunk o = kc * NOP + pair holds
// output tiles 2 pair (even blocks) and 2 pair + 1 (odd blocks).
__global__ void pack_m8_out_kernel(const float* __restrict__ w, int in_real, int out_real, int NOP, int kpair,
                                   int T, int kp, float* __restrict__ dst) {
    const size_t total = (size_t)(kpair ? 2 : 4 * NOP) * T * 1024;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        if (kp) {   // own K chunk o of the wave's 32 features, one 32-row output tile
            int lane, wave, s, q;
            size_t o;
            m8kp_index(i, lane, wave, o, s, q);
            const int n = 4 * (lane >> 3) + (lane & 3);
            const int k = 32 * wave + 16 * (int)o + 4 * q + s;
            dst[i] = (n < out_real && k < in_real) ? w[(size_t)n * in_real + k] : 0.0f;
            continue;
        }
        const int q = (int)(i & 3);
        const int lane = (int)((i >> 2) & 63);
        const int s = (int)((i >> 8) & 3);
        const size_t cw = i >> 10;            // o * T + wave
        const int wave = (int)(cw % T);
        const int o = (int)(cw / T);
        const int odd = (lane >> 2) & 1;
        const int kc = kpair ? 2 * o + odd : o / NOP;
        const int tile = kpair ? 0 : 2 * (o % NOP) + odd;
        const int n = 32 * tile + 4 * (lane >> 3) + (lane & 3);
        const int k = 64 * wave + 16 * kc + 4 * q + s;
        dst[i] = (n < out_real && k < in_real) ? w[(size_t)n * in_real + k] : 0.0f;
    }
}

// 4-candidate output chunks (rollout_m4_kernel): chunk kc of wave w's own 64 features; float4 s =
// output group g, element q: row n = 16 g + 4 (l >> 4) + (l & 3), k = 64 w + 16 kc + 4 q + chain,
// chain = (l >> 2) & 3 -- the canonical output chains of the 16-candidate kernel (mma_out).
__global__ void pack_m4_out_kernel(const float* __restrict__ w, int in_real, int out_real, int T,
                                   float* __restrict__ dst) {
    const size_t total = (size_t)4 * T * 1024;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int q = (int)(i & 3);
        const int lane = (int)((i >> 2) & 63);
        const int grp = (int)((i >> 8) & 3);
        const size_t cw = i >> 10;            // kc * T + wave
        const int wave = (int)(cw % T);
        const int kc = (int)(cw / T);
        const int n = 16 * grp + 4 * (lane >> 4) + (lane & 3);
        const int k = 64 * wave + 16 * kc + 4 * q + ((lane >> 2) & 3);
        dst[i] = (n < out_real && k < in_real) ? w[(size_t)n * in_real + k] : 0.0f;
    }
}

// Split streams (rollout_f16x3.hip): chunk = 32 K rows; per chunk 8 waves x (T/2 tiles x P pieces)
// fragments of 64 lanes x 8 halves. Fragment f of a hidden-type chunk = tile f / P, piece f % P.
// Lane l, element q: row n = 16 (wave T/2 + tile) + (l & 15), k = 32 kc + 8 (l >> 4) + q.
// Weights are scaled by MBRL_SPLIT_W_SCALE (exact) and split as w0 = f16(w), w1 = f16(w - w0),
// w2 = f16(w - w0 - w1). A scaled weight >= 32768 (|w| >= 128) cannot be split: *bad becomes
// nonzero and every workgroup of the rollout leaves its candidates to the fp32 redo pass.
__device__ __forceinline__ void split_weight(float v0, int P, _Float16* dst, unsigned* bad) {
    float v = v0 * MBRL_SPLIT_W_SCALE;
    if (!(fabsf(v) < 32768.0f)) atomicOr(bad, 1u);
    for (int q = 0; q < P; ++q) {
        const _Float16 h = (_Float16)v;
        dst[q * 512] = h;                 // piece q is fragment f + q: 64 lanes x 8 halves further
        v = v - (float)h;
    }
}

__global__ void pack_split_hidden_kernel(const float* __restrict__ w, int in_real, int out_real, int nkc, int T,
                                         int P, _Float16* __restrict__ dst, unsigned* __restrict__ bad) {
    const int TW = T / 2;
    const size_t total = (size_t)nkc * 8 * TW * 64 * 8;   // (kc, wave, tile, lane, q); all pieces per item
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int q = (int)(i & 7);
        const int lane = (int)((i >> 3) & 63);
        const size_t r = i >> 9;               // (kc * 8 + wave) * TW + tile
        const int tile = (int)(r % TW);
        const int wave = (int)((r / TW) & 7);
        const int kc = (int)(r / TW / 8);
        const int n = 16 * (wave * TW + tile) + (lane & 15);
        const int k = 32 * kc + 8 * (lane >> 4) + q;
        const float v = (n < out_real && k < in_real) ? w[(size_t)n * in_real + k] : 0.0f;
        const size_t frag = ((size_t)kc * 8 + wave) * TW * P + (size_t)tile * P;   // piece 0
        split_weight(v, P, dst + (frag * 64 + lane) * 8 + q, bad);
    }
}

// Output layer: chunk c pairs output tiles 2c, 2c + 1; wave w's K range is units [16 w TW, 16 (w+1) TW)
// taken as K-chunks kk of two tiles (2kk, 2kk+1) in the accumulator order: element q of lane group
// g is unit 16 (w TW + 2kk + (q >> 2)) + 4g + (q & 3). Fragment f = (u TW/2 + kk) P + piece.
__global__ void pack_split_out_kernel(const float* __restrict__ w, const float* __restrict__ w_r, int in_real,
                                      int out_real, int NOS, int T, int P, _Float16* __restrict__ dst,
                                      unsigned* __restrict__ bad) {
    const int TW = T / 2, KK = TW / 2;
    const size_t total = (size_t)NOS * 8 * 2 * KK * 64 * 8;   // (c, wave, u, kk, lane, q)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int q = (int)(i & 7);
        const int lane = (int)((i >> 3) & 63);
        size_t r = i >> 9;
        const int kk = (int)(r % KK); r /= KK;
        const int u = (int)(r % 2); r /= 2;
        const int wave = (int)(r % 8);
        const int c = (int)(r / 8);
        const int n = 16 * (2 * c + u) + (lane & 15);
        const int k = 16 * (wave * TW + 2 * kk + (q >> 2)) + 4 * (lane >> 4) + (q & 3);
        float v = 0.0f;
        if (k < in_real) {
            if (n < out_real) v = w[(size_t)n * in_real + k];
            else if (w_r && n == out_real) v = w_r[k];
        }
        const size_t frag = ((size_t)c * 8 + wave) * TW * P + (size_t)(u * KK + kk) * P;
        split_weight(v, P, dst + (frag * 64 + lane) * 8 + q, bad);
    }
}

// Plain copies for traj.hip: transposed W^T [in][cols] (zero-padded columns) ...
__global__ void pack_transposed_kernel(const float* __restrict__ w, int in_real, int out_real, int cols,
                                       float* __restrict__ dst) {
    const size_t total = (size_t)in_real * cols;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int k = (int)(i / cols), n = (int)(i - (i / cols) * cols);
        dst[i] = n < out_real ? w[(size_t)n * in_real + k] : 0.0f;
    }
}

// ... and a straight copy (the output layer keeps nn.Linear's row-major [out][in]).
__global__ void copy_kernel(const float* __restrict__ src, size_t n, float* __restrict__ dst) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

__global__ void pack_bias_kernel(const float* __restrict__ b, int n_real, int n_pad, float* __restrict__ dst) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_pad; i += gridDim.x * blockDim.x)
        dst[i] = i < n_real ? b[i] : 0.0f;
}

// ------------------------------------------------------------------------------------------------
// Block scan helper (exclusive), blockDim.x multiple of 64, <= 1024
// ------------------------------------------------------------------------------------------------
// Cross-lane moves as DPP operand modifiers (VALU, no LDS round trip as __shfl's ds_bpermute takes).
// Lanes whose source is outside the row, or whose row is not in ROWS, read 0.
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, false);
}

// Inclusive prefix sum over the wave: in-row shifts by 1, 2, 4, 8, then the row broadcasts.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
    x += dpp_u32<0x111>(x);        // row_shr:1
    x += dpp_u32<0x112>(x);        // row_shr:2
    x += dpp_u32<0x114>(x);        // row_shr:4
    x += dpp_u32<0x118>(x);        // row_shr:8
    x += dpp_u32<0x142, 0xA>(x);   // row_bcast:15 (rows 1 and 3)
    x += dpp_u32<0x143, 0xC>(x);   // row_bcast:31 (rows 2 and 3)
    return x;
}

// Wave minimum / maximum: every lane of a row gets the row's (quad swaps, half mirror, mirror), then the
// four rows' through readlane.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    x = min(x, dpp_u32<0xB1>(x));
    x = min(x, dpp_u32<0x4E>(x));
    x = min(x, dpp_u32<0x141>(x));
    x = min(x, dpp_u32<0x140>(x));
    return min(min((uint32_t)__builtin_amdgcn_readlane((int)x, 0), (uint32_t)__builtin_amdgcn_readlane((int)x, 16)),
               min((uint32_t)__builtin_amdgcn_readlane((int)x, 32), (uint32_t)__builtin_amdgcn_readlane((int)x, 48)));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    x = max(x, dpp_u32<0xB1>(x));
    x = max(x, dpp_u32<0x4E>(x));
    x = max(x, dpp_u32<0x141>(x));
    x = max(x, dpp_u32<0x140>(x));
    return max(max((uint32_t)__builtin_amdgcn_readlane((int)x, 0), (uint32_t)__builtin_amdgcn_readlane((int)x, 16)),
               max((uint32_t)__builtin_amdgcn_readlane((int)x, 32), (uint32_t)__builtin_amdgcn_readlane((int)x, 48)));
}

// The lanes' predicate as a 64-bit mask straight from the compare (HIP's __ballot goes through a
// select and a second compare).
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds_waves, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t x = wave_inclusive_scan(v);
    if (lane == 63) lds_waves[wave] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;   // every wave sums the wave totals itself (broadcast reads)
    for (int w = 0; w < nw; ++w) {
        const uint32_t t = lds_waves[w];
        before += w < wave ? t : 0u;
        all += t;
    }
    *total = all;
    __syncthreads();
    return before + x - v;
}

// ------------------------------------------------------------------------------------------------
// Elite selection: returns -> order keys -> radix select of the K-th key -> stable tie break by
// index -> compaction in ascending index order. One workgroup of 1024 threads (N is small:
// 1e3..3e4 candidates; the pass is a few microseconds).
// ------------------------------------------------------------------------------------------------
// Diagnostic build only (-DMBRL_STAMPS): thread 0's s_memrealtime at fixed points of the select
// kernel, written to a buffer set by mbrl_diag_set_cem_stamps() (tools/select_stamps.py).
#ifdef MBRL_STAMPS
__device__ unsigned long long* g_cem_stamps;
#define CSTAMP(k)                                                                      \
    do {                                                                               \
        if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && g_cem_stamps)                \
            g_cem_stamps[k] = __builtin_amdgcn_s_memrealtime();                                       \
    } while (0)
// ... and per workgroup of the split update's two kernels (iteration i, kernel q, workgroup b, point k):
// start, after the selection / the sums, end (mbrl_diag_set_cem_wg_stamps, tools/split_stamps.py).
__device__ unsigned long long* g_cem_wg_stamps;   // [8][2][1024][4]
#define WGSTAMP(q, k)                                                                                     \
    do {                                                                                                  \
        if (threadIdx.x == 0 && blockIdx.x < 1024 && g_cem_wg_stamps)                                     \
            g_cem_wg_stamps[(((U.iteration & 7) * 2 + (q)) * 1024 + blockIdx.x) * 4 + (k)] =              \
                __builtin_amdgcn_s_memrealtime();                                                         \
    } while (0)
#else
#define CSTAMP(k) \
    do {          \
    } while (0)
#define WGSTAMP(q, k) \
    do {              \
    } while (0)
#endif

__device__ __forceinline__ uint32_t order_key(float v, int nan_policy) {
    if (v != v) return nan_policy == MBRL_NAN_LAST ? 0xFFFFFFFFu : 0u;
    if (v == 0.0f) v = 0.0f;  // -0.0 ties with +0.0, as in NumPy's comparisons
    const uint32_t b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__global__ void __launch_bounds__(1024) select_kernel(const float* __restrict__ costs, int E, int N, int K,
                                                      int nan_policy, int64_t* __restrict__ elite_idx,
                                                      float* __restrict__ returns_out, uint32_t* __restrict__ keys,
                                                      int member_stride) {
    costs += (size_t)blockIdx.x * N;                   // segment b (see select_reg_kernel)
    elite_idx += (size_t)blockIdx.x * K;
    if (returns_out) returns_out += (size_t)blockIdx.x * N;
    keys += (size_t)blockIdx.x * N;
    __shared__ uint32_t hist[16][257];   // per-wave rows, padded (no cross-wave bank collisions)
    __shared__ uint32_t scan_ws[16];
    __shared__ uint32_t sel[3];  // prefix, bucket, remaining k
    const int tid = threadIdx.x, nt = blockDim.x, wave = tid >> 6;
    for (int n = tid; n < N; n += nt) {
        float r = costs[n];
        if (E > 1) {
            for (int e = 1; e < E; ++e) r = __fadd_rn(r, costs[(size_t)e * member_stride + n]);
            r = __fdiv_rn(r, (float)E);
        }
        if (returns_out) returns_out[n] = r;
        keys[n] = order_key(r, nan_policy);
    }
    uint32_t prefix = 0, mask = 0, kk = (uint32_t)K;
    __syncthreads();
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = tid; i < 16 * 257; i += nt) (&hist[0][0])[i] = 0;
        __syncthreads();
        for (int n0 = 0; n0 < N; n0 += nt) {        // wave-uniform trip count (ballots below)
            const int n = n0 + tid;
            const uint32_t k = n < N ? keys[n] : 0u;
            const bool pending = n < N && (k & mask) == prefix;
            const uint32_t dig = (k >> shift) & 255u;
            const uint64_t act = __ballot(pending);
            if (act != 0) {
                const int leader = __builtin_ctzll(act);
                const uint32_t d0 = __shfl(dig, leader, 64);
                if (__ballot(pending && dig == d0) == act) {   // clustered: one add per wave
                    if ((tid & 63) == leader) atomicAdd(&hist[wave][d0], (uint32_t)__popcll(act));
                } else if (pending) {
                    atomicAdd(&hist[wave][dig], 1u);
                }
            }
        }
        __syncthreads();
        uint32_t tot;
        uint32_t h = 0;
        if (tid < 256)
            for (int w = 0; w < nt / 64; ++w) h += hist[w][tid];
        const uint32_t before = block_exclusive_scan(h, scan_ws, &tot);
        if (tid < 256 && before < kk && before + h >= kk) { sel[0] = (uint32_t)tid; sel[1] = before; }
        __syncthreads();
        prefix |= sel[0] << shift;
        mask |= 0xFFu << shift;
        kk -= sel[1];
        __syncthreads();
    }
    // prefix = K-th smallest key; kk = how many of the keys equal to it are elites (lowest index first)
    const int seg = (N + nt - 1) / nt;
    const int n0 = tid * seg, n1 = min(N, n0 + seg);
    uint32_t eq = 0;
    for (int n = n0; n < n1; ++n) eq += keys[n] == prefix;
    uint32_t tot;
    uint32_t eq_before = block_exclusive_scan(eq, scan_ws, &tot);
    uint32_t cnt = 0;
    for (int n = n0; n < n1; ++n) {
        const uint32_t k = keys[n];
        if (k < prefix) ++cnt;
        else if (k == prefix) { if (eq_before < kk) ++cnt; ++eq_before; }
    }
    eq_before -= eq;
    uint32_t pos = block_exclusive_scan(cnt, scan_ws, &tot);
    for (int n = n0; n < n1; ++n) {
        const uint32_t k = keys[n];
        bool take = false;
        if (k < prefix) take = true;
        else if (k == prefix) { take = eq_before < kk; ++eq_before; }
        if (take && pos < (uint32_t)K) elite_idx[pos++] = n;
    }
}

// Register-resident selection for N <= 1024 * KPT. Wave w owns candidates [64 KPT w, 64 KPT (w + 1)) and
// every load is coalesced: with 16-byte aligned rows (N and member_stride multiples of 4) lane l holds
// groups of four, group g at 64 KPT w + 256 g + 4 l (one float4 per lane, a contiguous KB per wave load
// instruction), else single keys at 64 KPT w + 64 g + l. A thread's keys are therefore not contiguous;
// the elites' ascending-index positions come from ballots over the lanes (in order) and the waves'
// totals (one barrier), so no key moves between threads.
// Passes: one wide pass over the first SEL_WIDE_BITS bits in which the keys differ (one shared
// histogram), the K-th key's bucket listed in LDS, 8-bit passes over that list (or over every key when
// the bucket is too large to list), then the compaction.
constexpr int SEL_HIST_WORDS = 2 * 16 * 257;   // two buffers of per-wave 8-bit digit histograms
constexpr int SEL_WIDE_BITS = 11, SEL_WIDE_BINS = 1 << SEL_WIDE_BITS;   // the first (wide) pass
constexpr int SEL_LIST = 2048;                  // keys of the wide pass's bucket kept in LDS
// LDS words of the register-resident selection: the histograms, the wide histogram, the list, its count
__host__ __device__ constexpr int sel_words(int) { return SEL_HIST_WORDS + SEL_WIDE_BINS + SEL_LIST + 4; }

// Segmented over blockIdx.x (independent problems of N candidates each, batched planning): segment
// b reads costs[e * member_stride + b * N + n] and writes elite_idx[b * K ..] (local indices) and
// returns_out[b * N ..].
// The body is shared with cem_update_kernel; emit(pos, n) receives each elite with its place in
// ascending candidate order.
template <int KPT, typename Emit>
__device__ __forceinline__ void select_reg_body(const float* __restrict__ costs, int E, int N, int K, int nan_policy,
                                                float* __restrict__ returns_out, int member_stride,
                                                uint32_t* sel_smem, Emit emit) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    uint32_t(*hist)[16][257] = reinterpret_cast<uint32_t(*)[16][257]>(sel_smem);  // [2][16][257]
    __shared__ uint32_t scan_ws[16];
    __shared__ uint32_t sel[3];   // bucket, keys before it, keys in it
    CSTAMP(0);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const bool vec = KPT >= 4 && (N & 3) == 0 && (member_stride & 3) == 0;
    const int lv = 64 * KPT * wave + 4 * lane, ls = 64 * KPT * wave + lane;
    // candidate of this lane's key j (ascending in (wave, j / VW, lane, j % VW): the global order)
    auto idx = [&](int j) { return vec ? lv + 256 * (j >> 2) + (j & 3) : ls + 64 * j; };
    // idx rises with j, so this lane's keys below N are its first nv (one register, not KPT predicates)
    const int nv = vec ? 4 * max(0, min(KPT / 4, (N - lv + 255) / 256)) : max(0, min(KPT, (N - ls + 63) / 64));
    uint32_t key[KPT];
    if (vec && E == 1) {
        // (the plans' usual case) branch-free: every lane loads from a valid address -- its own group,
        // or the row's first where it has none -- and the keys past N are set to all ones by a select
        constexpr int G4 = KPT >= 4 ? KPT / 4 : 1;
        f4 v[G4];
#pragma unroll
        for (int g = 0; g < G4; ++g) v[g] = *reinterpret_cast<const f4*>(costs + (lv + 256 * g < N ? lv + 256 * g : 0));
        if (returns_out) {
#pragma unroll
            for (int g = 0; g < G4; ++g)
                if (lv + 256 * g < N) *reinterpret_cast<f4*>(returns_out + lv + 256 * g) = v[g];
        }
#pragma unroll
        for (int g = 0; g < G4; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) key[4 * g + i] = 4 * g < nv ? order_key(v[g][i], nan_policy) : 0xFFFFFFFFu;
    } else {
        float r[KPT];   // every load in flight before the first use; the member sum keeps its order
        if (vec) {
            constexpr int G4 = KPT >= 4 ? KPT / 4 : 1;
#pragma unroll
            for (int g = 0; g < G4; ++g) {
                const int n = lv + 256 * g;
                const f4 v = n < N ? *reinterpret_cast<const f4*>(costs + n) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < 4; ++i) r[4 * g + i] = v[i];
            }
            for (int e = 1; e < E; ++e)
#pragma unroll
                for (int g = 0; g < G4; ++g) {
                    const int n = lv + 256 * g;
                    if (n < N) {
                        const f4 c = *reinterpret_cast<const f4*>(costs + (size_t)e * member_stride + n);
#pragma unroll
                        for (int i = 0; i < 4; ++i) r[4 * g + i] = __fadd_rn(r[4 * g + i], c[i]);
                    }
                }
#pragma unroll
            for (int g = 0; g < G4; ++g) {
                const int n = lv + 256 * g;
                f4 v;
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = E > 1 ? __fdiv_rn(r[4 * g + i], (float)E) : r[4 * g + i];
                if (returns_out && n < N) *reinterpret_cast<f4*>(returns_out + n) = v;
#pragma unroll
                for (int i = 0; i < 4; ++i) key[4 * g + i] = n < N ? order_key(v[i], nan_policy) : 0xFFFFFFFFu;
            }
        } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const int n = ls + 64 * j;
                r[j] = n < N ? costs[n] : 0.f;
            }
            for (int e = 1; e < E; ++e)
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const int n = ls + 64 * j;
                    if (n < N) r[j] = __fadd_rn(r[j], costs[(size_t)e * member_stride + n]);
                }
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const int n = ls + 64 * j;
                const float v = E > 1 ? __fdiv_rn(r[j], (float)E) : r[j];
                if (returns_out && n < N) returns_out[n] = v;
                key[j] = n < N ? order_key(v, nan_policy) : 0xFFFFFFFFu;
            }
        }
    }
    // leading bits every key shares (block min / max): returns of one plan usually share sign and
    // exponent, so the first digit starts at the first bit in which the keys differ
    // every key of the wave below N (idx rises with the lane): the passes below skip the per-key test
    const bool wfull = __builtin_amdgcn_readlane(nv, 63) == KPT;
    uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
    if (wfull) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) { kmin = min(kmin, key[j]); kmax = max(kmax, key[j]); }
    } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j)
            if (j < nv) { kmin = min(kmin, key[j]); kmax = max(kmax, key[j]); }
    }
    kmin = wave_min_u32(kmin);
    kmax = wave_max_u32(kmax);
    __shared__ uint32_t mm_ws[2][16];
    if (lane == 0) { mm_ws[0][wave] = kmin; mm_ws[1][wave] = kmax; }
    uint32_t* wide = sel_smem + SEL_HIST_WORDS;          // [SEL_WIDE_BINS] the first pass's histogram
    uint32_t* list = wide + SEL_WIDE_BINS;               // [SEL_LIST] its bucket's keys, then
    uint32_t* list_n = list + SEL_LIST;                  // their count
    for (int i = tid; i < SEL_WIDE_BINS; i += 1024) wide[i] = 0;
    for (int i = tid; i < 16 * 257; i += 1024) (&hist[0][0][0])[i] = 0;
    if (tid == 0) *list_n = 0;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 16; ++w) { kmin = min(kmin, mm_ws[0][w]); kmax = max(kmax, mm_ws[1][w]); }
    // keys relative to the smallest (order kept: every key is >= kmin, no wrap): the passes then
    // resolve the bits of (key - kmin), so the wide pass's 2048 bins span [kmin, kmax] whatever bit
    // boundaries the range straddles (plan returns of one binade sit in a few % of its mantissa range:
    // with bins over the bits below the shared ones, walker's K-th bucket held 200-500 keys, now ~10)
#pragma unroll
    for (int j = 0; j < KPT; ++j) key[j] -= kmin;
    const uint32_t kpad = 0xFFFFFFFFu - kmin;            // keys past N (all ones before the shift)
    const uint32_t range = kmax - kmin;
    const int lead = range == 0 ? 32 : __clz(range);     // leading bits every shifted key shares (zero)
    uint32_t mask = lead == 0 ? 0u : (lead >= 32 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> lead));
    uint32_t prefix = 0u, kk = (uint32_t)K;
    uint32_t eqn = (uint32_t)N;                          // keys equal to prefix once it is resolved
    int rem = 32 - lead;                                 // bits below the shared ones still to resolve
    CSTAMP(1);
    // (1) one wide pass over the first SEL_WIDE_BITS differing bits: 2048 bins, one shared histogram
    // (plan returns spread over most of them, so the K-th key's bucket holds a handful of keys)
    bool listed = false;
    if (rem > 0) {
        const int wb = min(SEL_WIDE_BITS, rem), wshift = rem - wb;
        const uint32_t wmask = (1u << wb) - 1u;
        auto wide_count = [&](auto check) {   // (keys past N into a dummy bin: no branch per key)
#pragma unroll
            for (int j = 0; j < KPT; ++j)
                atomicAdd(&wide[(!decltype(check)::value || j < nv) ? (key[j] >> wshift) & wmask
                                                                   : SEL_WIDE_BINS + SEL_LIST + 1], 1u);
        };
        if (wfull) wide_count(std::false_type{});
        else wide_count(std::true_type{});
        __syncthreads();
        const uint32_t h0 = wide[2 * tid], h1 = wide[2 * tid + 1];
        uint32_t tot;
        const uint32_t b0 = block_exclusive_scan(h0 + h1, scan_ws, &tot);
        if (b0 < kk && b0 + h0 >= kk) { sel[0] = 2u * tid; sel[1] = b0; sel[2] = h0; }
        else if (b0 + h0 < kk && b0 + h0 + h1 >= kk) { sel[0] = 2u * tid + 1u; sel[1] = b0 + h0; sel[2] = h1; }
        __syncthreads();
        prefix |= sel[0] << wshift;
        mask |= wmask << wshift;
        kk -= sel[1];
        const uint32_t bsz = sel[2];   // (a register: wave 0 rewrites sel below)
        eqn = bsz;
        rem = wshift;
        CSTAMP(2);
        // (2) the bucket's keys (sel[2] of them) into an LDS list: the later passes read it, not the
        // KPT keys of every thread
        if (rem > 0 && bsz <= (uint32_t)SEL_LIST) {
            auto list_keys = [&](auto check) {
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const bool pend = (!decltype(check)::value || j < nv) && (key[j] & mask) == prefix;
                    const uint64_t act = wave_ballot(pend);
                    if (act != 0) {
                        const int leader = __builtin_ctzll(act);
                        uint32_t base = 0;
                        if (lane == leader) base = atomicAdd(list_n, (uint32_t)__popcll(act));
                        base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
                        const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
                        if (pend) list[base + below] = key[j];
                    }
                }
            };
            if (wfull) list_keys(std::false_type{});
            else list_keys(std::true_type{});
            listed = true;
            __syncthreads();
            // a bucket of at most 64 keys (the usual case): wave 0 ranks them directly -- the kk-th
            // smallest is the key with (keys below it) < kk <= (keys not above it) -- in place of the
            // remaining 8-bit passes and their barriers
            if (bsz <= 64u) {
                const uint32_t nb = (uint32_t)__builtin_amdgcn_readfirstlane((int)bsz);
                if (wave == 0) {
                    const uint32_t x = (uint32_t)lane < nb ? list[lane] : 0xFFFFFFFFu;
                    uint32_t lt = 0, le = 0;
                    for (uint32_t j = 0; j < nb; ++j) {   // key j to every lane (readlane: no LDS trip)
                        const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)x, (int)j);
                        lt += y < x;
                        le += y <= x;
                    }
                    if ((uint32_t)lane < nb && lt < kk && le >= kk) { sel[0] = x; sel[1] = kk - lt; sel[2] = le - lt; }
                }
                __syncthreads();
                prefix = sel[0];
                kk = sel[1];
                eqn = sel[2];
                mask = 0xFFFFFFFFu;
                rem = 0;
            }
        }
        CSTAMP(3);
    }
    // (3) 8-bit radix passes over the remaining bits: over the list (a few keys, at most SEL_LIST / 1024
    // per thread), or over every thread's KPT keys when the bucket was too large to list. Per-wave
    // histograms (rows padded to 257: no cross-wave bank collisions on a shared digit); the buffer of pass
    // p+1 is cleared during pass p; the bucket search is a 256-entry scan by waves 0-3.
    const uint32_t nl = listed ? *list_n : 0u;
    int buf = 0;
    while (rem > 0) {
        const int db = min(8, rem), shift = rem - db;
        const uint32_t dmask = (1u << db) - 1u;
        auto count = [&](uint32_t kv, bool valid) {
            const bool pending = valid && (kv & mask) == prefix;
            const uint32_t dig = (kv >> shift) & dmask;
            const uint64_t act = wave_ballot(pending);
            if (act != 0) {
                const int leader = __builtin_ctzll(act);
                const uint32_t d0 = __shfl(dig, leader, 64);
                if (wave_ballot(pending && dig == d0) == act) {   // clustered: one add per wave
                    if (lane == leader) atomicAdd(&hist[buf][wave][d0], (uint32_t)__popcll(act));
                } else if (pending) {
                    atomicAdd(&hist[buf][wave][dig], 1u);
                }
            }
        };
        if (listed) {
            for (uint32_t i0 = 0; i0 < nl; i0 += 1024)   // block-uniform trip count
                count(i0 + tid < nl ? list[i0 + tid] : 0u, i0 + tid < nl);
        } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) count(key[j], j < nv);
        }
        for (int i = tid; i < 16 * 257; i += 1024) (&hist[buf ^ 1][0][0])[i] = 0;
        __syncthreads();
        uint32_t h = 0, incl = 0;
        if (tid < 256) {
#pragma unroll
            for (int w = 0; w < 16; ++w) h += hist[buf][w][tid];
            incl = wave_inclusive_scan(h);
            if (lane == 63) scan_ws[wave] = incl;
        }
        __syncthreads();
        if (tid < 256) {
            uint32_t before = incl - h;
            for (int w = 0; w < wave; ++w) before += scan_ws[w];
            if (before < kk && before + h >= kk) { sel[0] = (uint32_t)tid; sel[1] = before; sel[2] = h; }
        }
        __syncthreads();
        prefix |= sel[0] << shift;
        mask |= dmask << shift;
        kk -= sel[1];
        eqn = sel[2];
        rem = shift;
        buf ^= 1;
    }
    CSTAMP(4);
    // prefix = the K-th smallest key; the elites are every key below it and the first kk keys equal to
    // it in candidate order.
    // (a) Every key equal to it is an elite (eqn == kk: the K-th key unique, or all its ties taken --
    // the usual case): the elites are the keys <= prefix. Their flags go to an LDS bitmap in candidate
    // order (a lane's four adjacent keys are a nibble, eight lanes' nibbles one word, OR-ed by DPP;
    // or one ballot per key, two words, in the single-key layout), and thread t emits the set bits of
    // word t after a block scan of the words' counts: ~3 VALU ops per key instead of ~20.
    // Keys past N are kpad, the largest shifted key; prefix is not (checked), so they are never flagged.
    // (From KPT = 8: at 4 keys per lane and fewer the scan and barrier of (a) cost more than (b)'s
    // per-key work -- 1.35 against 0.76 us at N = 4096.)
    if (KPT >= 8 && eqn == kk && prefix != kpad) {
        uint32_t* bits = &hist[0][0][0];   // [32 KPT] (the 8-bit passes are done with it)
        auto ballot_words = [&]() {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint64_t m = wave_ballot(key[j] <= prefix);
                if (lane < 2) bits[((ls - lane + 64 * j) >> 5) + lane] = (uint32_t)(m >> (32 * lane));
            }
        };
        if constexpr (KPT >= 4) {
            if (vec) {
#pragma unroll
                for (int g = 0; g < KPT / 4; ++g) {
                    uint32_t nib = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) nib |= (uint32_t)(key[4 * g + i] <= prefix) << i;
                    nib <<= 4 * (lane & 7);
                    nib |= dpp_u32<0xB1>(nib);    // quad_perm [1,0,3,2]
                    nib |= dpp_u32<0x4E>(nib);    // quad_perm [2,3,0,1]
                    nib |= dpp_u32<0x141>(nib);   // row_half_mirror: the other quad of the eight
                    if ((lane & 7) == 0) bits[(lv + 256 * g) >> 5] = nib;
                }
            } else {
                ballot_words();
            }
        } else {
            ballot_words();
        }
        __syncthreads();
        uint32_t m = tid < (N + 31) >> 5 ? bits[tid] : 0u, tot;
        uint32_t pos = block_exclusive_scan((uint32_t)__popc(m), scan_ws, &tot);
        while (m != 0u) {
            emit(pos++, 32 * tid + __builtin_ctz(m));
            m &= m - 1u;
        }
        CSTAMP(5);
        return;
    }
    // (b) Otherwise an elite's place in that order is (keys below it before it) + min(equal
    // keys before it, kk) -- below K by construction. Keys past N are kpad and follow every real key
    // in the order, so they can only tie with a K-th key of kpad after the kk real ones: no validity
    // test is needed here. Counts are packed (below << 16 | equal; N <= 32768, so neither half carries)
    // and kept in VALU registers; one conditional store per key is the only branch (the scalar unit,
    // shared by the CU's 16 waves, was the bottleneck of a ballot-per-key compaction).
    auto below = [&](uint64_t b) {   // set bits of b in lanes before this one
        return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    };
    auto cnt2 = [&](uint32_t k) { return ((uint32_t)(k < prefix) << 16) | (uint32_t)(k == prefix); };
    constexpr int VW = KPT >= 4 ? 4 : 1;   // keys of one lane that are adjacent in the order
    const int vw = vec ? VW : 1;
    {
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < KPT; ++j) c += cnt2(key[j]);
        c = wave_inclusive_scan(c);
        if (lane == 63) scan_ws[wave] = c;   // this wave's keys below / equal to the prefix, packed
    }
    __syncthreads();
    uint32_t run = 0;   // packed counts of the keys before this wave's current group (wave-uniform)
    for (int w = 0; w < wave; ++w) run += scan_ws[w];
#pragma unroll
    for (int g = 0; g < KPT / VW; ++g) {
        // the group's keys in candidate order: lanes ascending, and inside a lane its vw keys (one
        // group of VW keys per lane), or VW groups of single keys (vw = 1)
        if (vw == VW) {
            // counts of the group's keys in lanes before this one: ballots and mbcnt (VALU only)
            uint64_t bl[VW], be[VW], beany = 0;
            uint32_t before = 0, tot = 0;
#pragma unroll
            for (int i = 0; i < VW; ++i) {
                bl[i] = wave_ballot(key[VW * g + i] < prefix);
                be[i] = wave_ballot(key[VW * g + i] == prefix);
                beany |= be[i];
                before += below(bl[i]) << 16;
                tot += (uint32_t)__popcll(bl[i]) << 16;
            }
            if (beany != 0) {   // (rare: keys equal to the K-th in this group)
#pragma unroll
                for (int i = 0; i < VW; ++i) {
                    before += below(be[i]);
                    tot += (uint32_t)__popcll(be[i]);
                }
            }
            uint32_t at = run + before;
#pragma unroll
            for (int i = 0; i < VW; ++i) {
                const uint32_t k = key[VW * g + i];
                const uint32_t lb = at >> 16, eb = at & 0xFFFFu;
                const bool lt = k < prefix, eq = k == prefix;
                const bool take = lt || (eq && eb < kk);
                const uint32_t pos = lb + (lt ? min(eb, kk) : eb);
                if (take) emit(pos, idx(VW * g + i));
                at += cnt2(k);
            }
            run += tot;
        } else {
#pragma unroll
            for (int i = 0; i < VW; ++i) {
                const uint32_t k = key[VW * g + i];
                const bool lt = k < prefix, eq = k == prefix;
                const uint64_t bl = wave_ballot(lt), be = wave_ballot(eq);
                const uint32_t lb = (run >> 16) + below(bl), eb = (run & 0xFFFFu) + below(be);
                const bool take = lt || (eq && eb < kk);
                const uint32_t pos = lb + (lt ? min(eb, kk) : eb);
                if (take) emit(pos, idx(VW * g + i));
                run += ((uint32_t)__popcll(bl) << 16) + (uint32_t)__popcll(be);
            }
        }
    }
    CSTAMP(5);
}

template <int KPT>
__global__ void __launch_bounds__(1024) select_reg_kernel(const float* __restrict__ costs, int E, int N, int K,
                                                          int nan_policy, int64_t* __restrict__ elite_idx,
                                                          float* __restrict__ returns_out, int member_stride) {
    extern __shared__ __attribute__((aligned(16))) uint32_t sel_smem[];
    costs += (size_t)blockIdx.x * N;
    elite_idx += (size_t)blockIdx.x * K;
    if (returns_out) returns_out += (size_t)blockIdx.x * N;
    select_reg_body<KPT>(costs, E, N, K, nan_policy, returns_out, member_stride, sel_smem,
                         [&](uint32_t pos, int n) { elite_idx[pos] = n; });
}

static size_t select_reg_lds(int KPT) { return 4 * (size_t)sel_words(KPT); }

// ------------------------------------------------------------------------------------------------
// CEM refit. gather: regenerate every elite's a_t from the counter RNG into aelite[t][e][a].
// refit: canonical chunked sums (ELITE_CHUNK = 32, oracle/cem.py:chunked_sum) -> mean, population
// variance -> alpha-smoothed mu / sigma. All float ops correctly rounded, no contraction.
// ------------------------------------------------------------------------------------------------
constexpr int ELITE_CHUNK = 32;

__global__ void gather_elites_kernel(uint64_t seed, int iteration, const float* __restrict__ mu,
                                     const float* __restrict__ sigma, float lo, float hi, int a,
                                     const int64_t* __restrict__ elite_idx, int K, float* __restrict__ aelite) {
    const int t = blockIdx.y;
    const int G = (a + 3) >> 2;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= K * G) return;
    const int e = idx / G, g = idx - (idx / G) * G;
    float z[4];
    cem_normal4(seed, (uint32_t)elite_idx[e], (uint32_t)t, (uint32_t)iteration, (uint32_t)g, z);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int d = 4 * g + j;
        if (d < a) aelite[((size_t)t * K + e) * a + d] = cem_action(mu[t * a + d], sigma[t * a + d], z[j], lo, hi);
    }
}

__global__ void refit_kernel(const float* __restrict__ aelite, int a, int K, float alpha, float oma,
                             const float* __restrict__ mu, const float* __restrict__ sigma,
                             float* __restrict__ mu_out, float* __restrict__ sigma_out) {
#pragma clang fp contract(off)
    extern __shared__ float part[];  // [nch][a]
    __shared__ float mean[64];
    const int t = blockIdx.x;
    const int nch = (K + ELITE_CHUNK - 1) / ELITE_CHUNK;
    const float* A = aelite + (size_t)t * K * a;
    for (int pass = 0; pass < 2; ++pass) {
        for (int idx = threadIdx.x; idx < nch * a; idx += blockDim.x) {
            const int c = idx / a, d = idx - (idx / a) * a;
            const int e0 = c * ELITE_CHUNK, e1 = min(K, e0 + ELITE_CHUNK);
            float acc = 0.f;
            for (int e = e0; e < e1; ++e) {
                float v = A[(size_t)e * a + d];
                if (pass == 1) { const float df = __fadd_rn(v, -mean[d]); v = __fmul_rn(df, df); }
                acc = (e == e0) ? v : __fadd_rn(acc, v);
            }
            part[c * a + d] = acc;
        }
        __syncthreads();
        if ((int)threadIdx.x < a) {
            const int d = threadIdx.x;
            float tot = part[d];
            for (int c = 1; c < nch; ++c) tot = __fadd_rn(tot, part[c * a + d]);
            const float m = __fdiv_rn(tot, (float)K);
            if (pass == 0) {
                mean[d] = m;
            } else {
                const float mu0 = mu[t * a + d], s0 = sigma[t * a + d];
                mu_out[t * a + d] = __fadd_rn(__fmul_rn(alpha, mu0), __fmul_rn(oma, mean[d]));
                const float v = __fadd_rn(__fmul_rn(alpha, __fmul_rn(s0, s0)), __fmul_rn(oma, m));
                sigma_out[t * a + d] = exact_sqrt(v);
            }
        }
        __syncthreads();
    }
}

// Fused gather + refit for one timestep per workgroup: the K elites' a_t are regenerated from the
// counter RNG straight into LDS ([K][a], when it fits), then the canonical chunked sums run out of
// LDS. Same operation order as gather_elites_kernel + refit_kernel (bit-identical). With `final`
// set it also writes the plan outputs: mu / sigma copies and actions = clip(mu', lo, hi).
constexpr int REFIT_THREADS = 1024;
constexpr size_t REFIT_LDS_MAX = 96 * 1024;

// The elites' actions in LDS: [K][a] with one spare row after every chunk of ELITE_CHUNK elites, so a
// chunk starts 33 a floats after the previous one and the chunk sums' lanes -- lane (c, d) reads
// elite 32 c + q, dimension d -- fall on consecutive banks (at 32 a they all shared a bank, ~10-way).
// The last chunk is padded to 32 rows of -0.0 (ael_pad): x + (-0.0) == x for every x, so every chunk
// sums 32 values with no per-element predicate and the same bits as a sum over its real elites.
__host__ __device__ inline int ael_pos(int e, int d, int a) { return (e + e / ELITE_CHUNK) * a + d; }
__host__ __device__ inline size_t ael_floats(int a, int K) {
    const size_t nch = (size_t)(K + ELITE_CHUNK - 1) / ELITE_CHUNK;
    return (nch * (ELITE_CHUNK + 1) * a + 3) & ~(size_t)3;
}
__device__ __forceinline__ void ael_pad(float* ael, int a, int K) {
    const int nch = (K + ELITE_CHUNK - 1) / ELITE_CHUNK, np = nch * ELITE_CHUNK - K;
    for (int i = threadIdx.x; i < np * a; i += blockDim.x) ael[ael_pos(K + i / a, i % a, a)] = -0.0f;
}

// LDS floats refit_rows works in: the elite actions (ael_pos), [nch][a] chunk partials, mean, this
// row's mu, sigma.
__host__ __device__ inline size_t refit_rows_floats(int a, int K) {
    const size_t nch = (size_t)(K + ELITE_CHUNK - 1) / ELITE_CHUNK;
    const size_t a4 = ((size_t)a + 3) & ~(size_t)3;
    return ael_floats(a, K) + ((nch * a + 3) & ~(size_t)3) + 3 * a4;
}

// Row t of the refit (mu, sigma, outputs already offset to the problem; NULL outputs are skipped): eidx
// = the K elites' global candidate indices in LDS (visible after refit_rows' first barrier). With
// `next` (LDS [2][a4]) the new mu_t, sigma_t are also left there for the next proposal draw.
// The chunked sums of refit_rows over the elites' actions already in LDS (ael = smem [K][a]) and this
// row's mu, sigma staged in musg: mean, population variance, the alpha-smoothed mu', sigma' and the
// outputs. Ends on a barrier.
__device__ __forceinline__ void refit_sums(int t, float* smem, float lo, float hi, int a, int K, float alpha, float oma,
                                           float* __restrict__ mu_out, float* __restrict__ sigma_out,
                                           float* __restrict__ fin_mu, float* __restrict__ fin_sigma,
                                           float* __restrict__ fin_actions, float* next) {
#pragma clang fp contract(off)
    const int nch = (K + ELITE_CHUNK - 1) / ELITE_CHUNK;
    const int a4 = (a + 3) & ~3;
    float* ael = smem;                                   // ael_pos layout
    float* part = smem + ael_floats(a, K);               // [nch][a]
    float* mean = part + (((size_t)nch * a + 3) & ~(size_t)3);  // [a]
    const float* smu = mean + a4;                               // [2][a]: this step's mu, sigma
    const float* ssg = smu + a4;
    CSTAMP(8);
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {   // (unrolled: each pass's code has no pass test)
        for (int idx = threadIdx.x; idx < nch * a; idx += blockDim.x) {
            const int c = idx / a, d = idx - (idx / a) * a;
            const int e0 = c * ELITE_CHUNK, n = min(K - e0, ELITE_CHUNK);
            const float md = pass == 1 ? mean[d] : 0.f;
            float v[ELITE_CHUNK];
            const float* src = ael + (e0 + c) * a + d;   // ael_pos(e0, d); the chunk's rows a floats apart
#pragma unroll
            for (int q = 0; q < ELITE_CHUNK; ++q) v[q] = src[q * a];   // (padding rows: -0.0)
            if (pass == 1)   // the squared deviations first, off the dependent chain; padding stays -0.0
#pragma unroll
                for (int q = 0; q < ELITE_CHUNK; ++q) {
                    const float df = __fadd_rn(v[q], -md);
                    v[q] = q < n ? __fmul_rn(df, df) : -0.0f;
                }
            float acc = v[0];
#pragma unroll
            for (int q = 1; q < ELITE_CHUNK; ++q) acc = __fadd_rn(acc, v[q]);   // 31 dependent additions
            part[c * a + d] = acc;
        }
        __syncthreads();
        CSTAMP(9 + 2 * pass);
        if ((int)threadIdx.x < a) {
            const int d = threadIdx.x;
            // the chunk partials in sequence, eight LDS reads in flight at a time (the same additions
            // in the same order: a dependent read per partial cost ~2 us per pass at walker's 52 chunks)
            float tot = part[d];
            int c = 1;
            for (; c + 8 <= nch; c += 8) {
                float v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = part[(c + q) * a + d];
#pragma unroll
                for (int q = 0; q < 8; ++q) tot = __fadd_rn(tot, v[q]);
            }
            for (; c < nch; ++c) tot = __fadd_rn(tot, part[c * a + d]);
            const float m = __fdiv_rn(tot, (float)K);
            if (pass == 0) {
                mean[d] = m;
            } else {
                const float mu0 = smu[d], s0 = ssg[d];
                const float mn = __fadd_rn(__fmul_rn(alpha, mu0), __fmul_rn(oma, mean[d]));
                const float v = __fadd_rn(__fmul_rn(alpha, __fmul_rn(s0, s0)), __fmul_rn(oma, m));
                const float sn = exact_sqrt(v);
                if (mu_out) mu_out[t * a + d] = mn;
                if (sigma_out) sigma_out[t * a + d] = sn;
                if (next) { next[d] = mn; next[a4 + d] = sn; }
                if (fin_actions) {
                    if (fin_mu) fin_mu[t * a + d] = mn;
                    if (fin_sigma) fin_sigma[t * a + d] = sn;
                    fin_actions[t * a + d] = fminf(fmaxf(mn, lo), hi);
                }
            }
        }
        __syncthreads();
        CSTAMP(10 + 2 * pass);
    }
}

// Row t's mu, sigma into LDS (musg, behind the mean) -- refit_rows' and the split update's first step.
__device__ __forceinline__ void refit_stage_row(int t, float* smem, const float* __restrict__ mu,
                                                const float* __restrict__ sigma, int a, int K) {
    const int nch = (K + ELITE_CHUNK - 1) / ELITE_CHUNK;
    const int a4 = (a + 3) & ~3;
    float* musg = smem + ael_floats(a, K) + (((size_t)nch * a + 3) & ~(size_t)3) + a4;
    for (int d = threadIdx.x; d < a; d += blockDim.x) {
        musg[d] = mu[t * a + d];
        musg[a4 + d] = sigma[t * a + d];
    }
}

// Elites [e0, e1)'s actions of row t regenerated from the counter RNG (bit-identical to the sampled
// ones): into dst, [e][a] (global: the split update's hand-off) or in the ael_pos layout (LDS, padded).
// smu / ssg: this row's mu, sigma.
__device__ __forceinline__ void regen_elites(int t, const uint32_t* eidx, int e0, int e1, uint64_t seed, int iteration,
                                             const float* smu, const float* ssg, float lo, float hi, int a,
                                             float* __restrict__ dst, bool padded) {
#pragma clang fp contract(off)
    const int G = (a + 3) >> 2;
    for (int idx = threadIdx.x; idx < (e1 - e0) * G; idx += blockDim.x) {
        const int e = e0 + idx / G, g = idx - (idx / G) * G;
        float z[4];
        cem_normal4(seed, eidx[e], (uint32_t)t, (uint32_t)iteration, (uint32_t)g, z);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = 4 * g + j;
            if (d < a) dst[padded ? (size_t)ael_pos(e, d, a) : (size_t)e * a + d] = cem_action(smu[d], ssg[d], z[j], lo, hi);
        }
    }
}

__device__ __forceinline__ void refit_rows(int t, const uint32_t* eidx, float* smem, uint64_t seed, int iteration,
                                           const float* __restrict__ mu, const float* __restrict__ sigma, float lo,
                                           float hi, int a, int K, float alpha, float oma, float* __restrict__ mu_out,
                                           float* __restrict__ sigma_out, float* __restrict__ fin_mu,
                                           float* __restrict__ fin_sigma, float* __restrict__ fin_actions,
                                           float* next) {
    const int nch = (K + ELITE_CHUNK - 1) / ELITE_CHUNK;
    const int a4 = (a + 3) & ~3;
    const float* musg = smem + ael_floats(a, K) + (((size_t)nch * a + 3) & ~(size_t)3) + a4;
    // stage every global operand first (all loads in flight together), then compute from LDS
    refit_stage_row(t, smem, mu, sigma, a, K);
    ael_pad(smem, a, K);
    __syncthreads();
    regen_elites(t, eidx, 0, K, seed, iteration, musg, musg + a4, lo, hi, a, smem, true);
    __syncthreads();
    refit_sums(t, smem, lo, hi, a, K, alpha, oma, mu_out, sigma_out, fin_mu, fin_sigma, fin_actions, next);
}

__global__ void __launch_bounds__(REFIT_THREADS) refit_fused_kernel(
    uint64_t seed, int iteration, const float* __restrict__ mu, const float* __restrict__ sigma, float lo, float hi,
    int a, const int64_t* __restrict__ elite_idx, int K, float alpha, float oma, float* __restrict__ mu_out,
    float* __restrict__ sigma_out, float* __restrict__ fin_mu, float* __restrict__ fin_sigma,
    float* __restrict__ fin_actions, int n_env) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // batched planning: blockIdx.y = problem b, whose [H][a] distribution rows sit at b*H*a, whose
    // K elites (local indices) at b*K, and whose candidates are global n = b*n_env + local
    const int t = blockIdx.x, H = gridDim.x;
    const size_t eo = (size_t)blockIdx.y * H * a;
    const uint32_t nbase = (uint32_t)blockIdx.y * (uint32_t)n_env;
    uint32_t* eidx = reinterpret_cast<uint32_t*>(smem + refit_rows_floats(a, K));   // [K]
    elite_idx += (size_t)blockIdx.y * K;
    for (int e = threadIdx.x; e < K; e += REFIT_THREADS) eidx[e] = nbase + (uint32_t)elite_idx[e];
    refit_rows(t, eidx, smem, seed, iteration, mu + eo, sigma + eo, lo, hi, a, K, alpha, oma, mu_out + eo,
               sigma_out + eo, fin_mu ? fin_mu + eo : nullptr, fin_sigma ? fin_sigma + eo : nullptr,
               fin_actions ? fin_actions + eo : nullptr, nullptr);
}

static size_t refit_fused_lds(int a, int K) { return (refit_rows_floats(a, K) + (size_t)K) * sizeof(float); }

// ------------------------------------------------------------------------------------------------
// One launch per CEM iteration after the rollout (DESIGN.md §3 "update"): workgroup (t * S + j, b)
// selects the elites of problem b (every workgroup of the problem the same, deterministic), refits
// row t, and draws row t of the next iteration's proposals for candidate slice j of S from the new
// mu_t, sigma_t. Bit-identical to select_reg_kernel + refit_fused_kernel + sample_kernel: the same
// bodies in the same order. Three launches and their gaps become one; the selection and the row's
// refit are repeated by the workgroups side by side instead of run once (no longer critical path),
// and the draw -- ~400 VALU ops per Philox block -- is spread over S x H workgroups (~256 CUs).
// ------------------------------------------------------------------------------------------------
struct UpdateArgs {
    const float* costs;
    int E, N, K, member_stride, H, a;
    int64_t* elite_out;          // [B][K] local indices (block t = 0 of each problem writes them), or NULL
    float* returns_out;          // [B][N] member-mean returns (block t = 0), or NULL
    uint64_t seed;
    int iteration;
    const float *mu, *sigma;     // [B][H][a] this iteration's distribution
    float lo, hi, alpha, oma;
    float *mu_out, *sigma_out;   // [B][H][a] the refit
    float *fin_mu, *fin_sigma, *fin_actions;   // last iteration: plan outputs (or NULL)
    float* next_actions;         // [H][B*draw_n][a] proposals of iteration + 1, or NULL
    int draw_off, draw_n;        // problem b draws candidates b*N + draw_off + [0, draw_n) (a plan: 0, N)
    float* ael;                  // split update (B == 1): [H][K][a] the elites' actions between its launches
};

__host__ __device__ inline size_t update_lds_words(int KPT, int a, int K) {
    const size_t sel = (size_t)sel_words(KPT);
    const size_t ref = refit_rows_floats(a, K);
    return (((size_t)K + 3) & ~(size_t)3) + 2 * (((size_t)a + 3) & ~(size_t)3) + (sel > ref ? sel : ref);
}

// Row t of the next iteration's proposals for candidate slice j of S, from mu', sigma' in LDS (next).
__device__ __forceinline__ void update_draw(const UpdateArgs& U, int t, int j, int S, int b, uint32_t nbase,
                                            const float* next) {
    const int a = U.a, a4 = (a + 3) & ~3;
    const int G = (a + 3) >> 2;
    const int Dn = U.draw_n;
    const size_t row = (size_t)gridDim.y * Dn;
    const uint32_t cbase = nbase + (uint32_t)U.draw_off;   // global candidate of local index 0
    const int NS = (Dn + S - 1) / S, n0 = j * NS, n1 = min(Dn, n0 + NS);
    for (int idx = threadIdx.x; idx < (n1 - n0) * G; idx += 1024) {
        const int n = n0 + idx / G, g = idx - (idx / G) * G;
        float z[4];
        cem_normal4(U.seed, cbase + (uint32_t)n, (uint32_t)t, (uint32_t)(U.iteration + 1), (uint32_t)g, z);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int d = 4 * g + q;
            if (d < a)
                U.next_actions[((size_t)t * row + (size_t)b * Dn + n) * a + d] =
                    cem_action(next[d], next[a4 + d], z[q], U.lo, U.hi);
        }
    }
}

template <int KPT>
__global__ void __launch_bounds__(1024) cem_update_kernel(const UpdateArgs U) {
    extern __shared__ __attribute__((aligned(16))) uint32_t usmem[];
    const int S = gridDim.x / U.H;                      // draw slices per row
    const int t = blockIdx.x / S, j = blockIdx.x - (blockIdx.x / S) * S, b = blockIdx.y;
    const bool lead = t == 0 && j == 0;                 // writes the elites and returns
    const int K = U.K, N = U.N, a = U.a, a4 = (a + 3) & ~3;
    uint32_t* eidx = usmem;                                                  // [K] global candidate index
    float* next = reinterpret_cast<float*>(usmem + ((K + 3) & ~3));          // [2][a4] mu', sigma' of row t
    uint32_t* work = usmem + ((K + 3) & ~3) + 2 * a4;                        // select, then refit
    const uint32_t nbase = (uint32_t)b * (uint32_t)N;
    int64_t* eo = (U.elite_out && lead) ? U.elite_out + (size_t)b * K : nullptr;
    float* ro = (U.returns_out && lead) ? U.returns_out + (size_t)b * N : nullptr;
    select_reg_body<KPT>(U.costs + (size_t)b * N, U.E, N, K, MBRL_NAN_LAST, ro, U.member_stride, work,
                         [&](uint32_t pos, int n) {
                             eidx[pos] = nbase + (uint32_t)n;
                             if (eo) eo[pos] = n;
                         });
    __syncthreads();   // eidx complete; the selection's LDS becomes the refit's
    CSTAMP(6);
    const size_t rb = (size_t)b * U.H * a;
    const bool w = j == 0;   // slice 0 of the row writes its refit
    refit_rows(t, eidx, reinterpret_cast<float*>(work), U.seed, U.iteration, U.mu + rb, U.sigma + rb, U.lo, U.hi, a,
               K, U.alpha, U.oma, w ? U.mu_out + rb : nullptr, w ? U.sigma_out + rb : nullptr,
               (w && U.fin_mu) ? U.fin_mu + rb : nullptr, (w && U.fin_sigma) ? U.fin_sigma + rb : nullptr,
               (w && U.fin_actions) ? U.fin_actions + rb : nullptr, U.next_actions ? next : nullptr);
    CSTAMP(7);
    if (U.next_actions) update_draw(U, t, j, S, b, nbase, next);   // refit_rows ended on a barrier
}

// The same update as two launches (the split update): the regeneration of the K elites'
// actions -- K ceil(a / 4) Philox blocks per row, repeated by each of the row's S workgroups in
// cem_update_kernel -- is shared out: launch 1 (select + regenerate) has workgroup (t, j) select, then
// regenerate elites [j K / S, (j + 1) K / S) of row t into U.ael; launch 2 (refit + draw) has every
// workgroup of row t read the row's K elites back, then run the same chunked sums and the draw. The
// kernel boundary is the only hand-off. Bit-identical to cem_update_kernel: the same values in the
// same order.
template <int KPT>
__global__ void __launch_bounds__(1024) cem_select_regen_kernel(const UpdateArgs U) {
    extern __shared__ __attribute__((aligned(16))) uint32_t usmem[];
    const int S = gridDim.x / U.H;
    const int t = blockIdx.x / S, j = blockIdx.x - (blockIdx.x / S) * S;
    const bool lead = t == 0 && j == 0;
    const int K = U.K, N = U.N, a = U.a, a4 = (a + 3) & ~3;
    uint32_t* eidx = usmem;                                                  // [K] global candidate index
    float* row = reinterpret_cast<float*>(usmem + ((K + 3) & ~3));          // [2][a4] mu_t, sigma_t
    uint32_t* work = usmem + ((K + 3) & ~3) + 2 * a4;
    int64_t* eo = (U.elite_out && lead) ? U.elite_out : nullptr;
    float* ro = (U.returns_out && lead) ? U.returns_out : nullptr;
    WGSTAMP(0, 0);
    for (int d = threadIdx.x; d < a; d += 1024) {
        row[d] = U.mu[t * a + d];
        row[a4 + d] = U.sigma[t * a + d];
    }
    select_reg_body<KPT>(U.costs, U.E, N, K, MBRL_NAN_LAST, ro, U.member_stride, work,
                         [&](uint32_t pos, int n) {
                             eidx[pos] = (uint32_t)n;
                             if (eo) eo[pos] = n;
                         });
    __syncthreads();   // eidx complete (and the row staged)
    WGSTAMP(0, 1);
    const int KS = (K + S - 1) / S, e0 = min(K, j * KS), e1 = min(K, e0 + KS);
    regen_elites(t, eidx, e0, e1, U.seed, U.iteration, row, row + a4, U.lo, U.hi, a, U.ael + (size_t)t * K * a, false);
#ifdef MBRL_STAMPS
    __syncthreads();
    WGSTAMP(0, 2);
#endif
}

__global__ void __launch_bounds__(1024) cem_refit_draw_kernel(const UpdateArgs U) {
    extern __shared__ __attribute__((aligned(16))) float fsmem[];
    const int S = gridDim.x / U.H;
    const int t = blockIdx.x / S, j = blockIdx.x - (blockIdx.x / S) * S;
    const int K = U.K, a = U.a, a4 = (a + 3) & ~3;
    float* next = fsmem;                  // [2][a4] mu', sigma' of row t
    float* work = fsmem + 2 * a4;         // refit_rows' layout: [K][a] elites, partials, mean, mu / sigma
    WGSTAMP(1, 0);
    const float* src = U.ael + (size_t)t * K * a;
    const int n = K * a, ca = ELITE_CHUNK * a;   // flat index f = e a + d lands at f + (f / ca) a (ael_pos)
    if ((n & 3) == 0) {
        // 16-byte loads, up to four per thread in flight before the first LDS store
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4* s4 = reinterpret_cast<const f4*>(src);
        const int n4 = n >> 2;
        for (int i0 = threadIdx.x; i0 < n4; i0 += 4 * 1024) {
            f4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + u * 1024 < n4) v[u] = s4[i0 + u * 1024];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + u * 1024 < n4)
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int f = 4 * (i0 + u * 1024) + k;
                        work[f + (f / ca) * a] = v[u][k];
                    }
        }
    } else {
        for (int f = threadIdx.x; f < n; f += 1024) work[f + (f / ca) * a] = src[f];
    }
    refit_stage_row(t, work, U.mu, U.sigma, a, K);
    ael_pad(work, a, K);
    __syncthreads();
    WGSTAMP(1, 3);
    const bool w = j == 0;   // slice 0 of the row writes its refit
    refit_sums(t, work, U.lo, U.hi, a, K, U.alpha, U.oma, w ? U.mu_out : nullptr, w ? U.sigma_out : nullptr,
               (w && U.fin_mu) ? U.fin_mu : nullptr, (w && U.fin_sigma) ? U.fin_sigma : nullptr,
               (w && U.fin_actions) ? U.fin_actions : nullptr, U.next_actions ? next : nullptr);
    WGSTAMP(1, 1);
    if (U.next_actions) update_draw(U, t, j, S, 0, 0u, next);
#ifdef MBRL_STAMPS
    __syncthreads();
    WGSTAMP(1, 2);
#endif
}

// The plan's first launch: workgroup (t * S + j, b) sets row t of problem b's distribution to
// (init_mu, init_sigma) and, with `actions`, draws row t of iteration 0's proposals for candidate
// slice j (fill2_kernel + sample_kernel, bit-identical: the same floats go into cem_action).
// s0_src (optional): the plan's start state, device or mapped host memory, copied once into the
// workspace (s0_dst) so that every later launch reads device memory. draw_off: the global candidate
// index of local candidate 0 (a sharded plan's rank offset; 0 otherwise). zero[2] / zero_words[2]:
// the plan's hand-off words (the column-split pairs' flags, the trajectory kernel's granules and
// status), zeroed here once per plan instead of by a memset before each launch that polls them.
struct InitZero {
    unsigned* ptr[2];
    size_t words[2];
};

__global__ void __launch_bounds__(1024) cem_init_kernel(uint64_t seed, float init_mu, float init_sigma, float lo,
                                                        float hi, int H, int a, int N, float* __restrict__ mu,
                                                        float* __restrict__ sigma, float* __restrict__ actions,
                                                        const float* __restrict__ s0_src, int s,
                                                        float* __restrict__ s0_dst, int draw_off, InitZero zero) {
    const int S = gridDim.x / H;
    const int t = blockIdx.x / S, j = blockIdx.x - (blockIdx.x / S) * S, b = blockIdx.y;
    const size_t ro = ((size_t)b * H + t) * a;
    {
        const size_t gid = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
        const size_t gsz = (size_t)gridDim.x * gridDim.y * blockDim.x;
#pragma unroll
        for (int r = 0; r < 2; ++r)
            for (size_t i = gid; zero.ptr[r] && i < zero.words[r]; i += gsz) zero.ptr[r][i] = 0u;
    }
    if (s0_src && blockIdx.x == 0 && b == 0)
        for (int d = threadIdx.x; d < s; d += blockDim.x) s0_dst[d] = s0_src[d];
    if (j == 0)
        for (int d = threadIdx.x; d < a; d += blockDim.x) { mu[ro + d] = init_mu; sigma[ro + d] = init_sigma; }
    if (!actions) return;
    const int G = (a + 3) >> 2;
    const size_t BN = (size_t)gridDim.y * N;
    const uint32_t nbase = (uint32_t)b * (uint32_t)N;
    const int NS = (N + S - 1) / S, n0 = j * NS, n1 = min(N, n0 + NS);
    for (int idx = threadIdx.x; idx < (n1 - n0) * G; idx += blockDim.x) {
        const int n = n0 + idx / G, g = idx - (idx / G) * G;
        float z[4];
        cem_normal4(seed, nbase + (uint32_t)draw_off + (uint32_t)n, (uint32_t)t, 0u, (uint32_t)g, z);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = 4 * g + j;
            if (d < a) actions[((size_t)t * BN + nbase + n) * a + d] = cem_action(init_mu, init_sigma, z[j], lo, hi);
        }
    }
}

// Batched planning: local candidate n belongs to problem n / n_env, whose distribution rows sit at
// mu + (n / n_env) * H * a (n_env = N for a single problem).
__global__ void sample_kernel(uint64_t seed, int iteration, const float* __restrict__ mu,
                              const float* __restrict__ sigma, float lo, float hi, int H, int a, int N,
                              int n_offset, float* __restrict__ out, int n_env) {
    const int G = (a + 3) >> 2;
    const size_t total = (size_t)H * N * G;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int g = (int)(i % G);
        const int n = (int)((i / G) % N);
        const int t = (int)(i / G / N);
        float z[4];
        cem_normal4(seed, (uint32_t)(n_offset + n), (uint32_t)t, (uint32_t)iteration, (uint32_t)g, z);
        const size_t mo = (size_t)(n / n_env) * H * a + (size_t)t * a;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = 4 * g + j;
            if (d < a) out[((size_t)t * N + n) * a + d] = cem_action(mu[mo + d], sigma[mo + d], z[j], lo, hi);
        }
    }
}

__global__ void fill2_kernel(float* __restrict__ x, float vx, float* __restrict__ y, float vy, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { x[i] = vx; y[i] = vy; }
}

__global__ void finalize_kernel(const float* __restrict__ mu_src, const float* __restrict__ sg_src, float lo,
                                float hi, int n, float* __restrict__ mu, float* __restrict__ sigma,
                                float* __restrict__ actions) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float m = mu_src[i];
        if (mu) mu[i] = m;
        if (sigma) sigma[i] = sg_src[i];
        actions[i] = fminf(fmaxf(m, lo), hi);
    }
}

// Sharded plans: the all-gathered costs arrive rank-major [G][E][Nl]; the selection reads [E][N] with
// candidate r * Nl + j of member e at e * N + r * Nl + j.
__global__ void shard_costs_kernel(const float* __restrict__ gathered, int G, int E, int Nl, float* __restrict__ costs) {
    const size_t total = (size_t)G * E * Nl;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / ((size_t)E * Nl), rem = i - r * E * Nl, e = rem / Nl, j = rem - e * Nl;
        costs[e * (size_t)G * Nl + r * Nl + j] = gathered[i];
    }
}

__global__ void member_mean_kernel(const float* __restrict__ src, int E, int n, float* __restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        float acc = src[i];
        for (int e = 1; e < E; ++e) acc = __fadd_rn(acc, src[(size_t)e * n + i]);
        dst[i] = E > 1 ? __fdiv_rn(acc, (float)E) : acc;
    }
}

// ------------------------------------------------------------------------------------------------
// Host helpers
// ------------------------------------------------------------------------------------------------
static int shape_geometry(const mbrl_mlp_shape* sh, Geometry* g) {
    if (!sh) return fail(MBRL_EINVAL, "shape is NULL");
    if (sh->precision != MBRL_PRECISION_F32 && sh->precision != MBRL_PRECISION_F16X3 &&
        sh->precision != MBRL_PRECISION_F16X6)
        return fail(MBRL_EINVAL, "precision %d is not an MBRL_PRECISION_* value", sh->precision);
    if (!make_geometry(sh->state_dim, sh->action_dim, sh->hidden, sh->n_hidden, sh->ensemble, sh->reward_head, g))
        return fail(MBRL_EUNSUPPORTED,
                    "unsupported MLP shape s=%d a=%d W=%d L=%d E=%d reward_head=%d (need all >= 1, W <= 1024, L <= %d)",
                    sh->state_dim, sh->action_dim, sh->hidden, sh->n_hidden, sh->ensemble, sh->reward_head, MAX_LAYERS);
    g->precision = sh->precision;
    return MBRL_OK;
}

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

__global__ void expand_rows_kernel(const float* __restrict__ src, int B, int n_rep, int s, float* __restrict__ dst) {
    const size_t total = (size_t)B * n_rep * s;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t row = i / s;
        dst[i] = src[(row / n_rep) * s + (i - row * s)];
    }
}

static int sample_impl(const mbrl_sampler* sp, int H, int a, int N, int n_offset, float* out, hipStream_t stream,
                       int n_env = 0) {
    const size_t total = (size_t)H * N * ((a + 3) / 4);
    const int blocks = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
    hipLaunchKernelGGL(sample_kernel, dim3(blocks), dim3(256), 0, stream, sp->seed, sp->iteration, sp->mu, sp->sigma,
                       sp->lo, sp->hi, H, a, N, n_offset, out, n_env > 0 ? n_env : N);
    return hip_check(hipGetLastError(), "sample launch");
}

// Column-split pair exchange area a plan workspace reserves for N candidates (0: pairs not offered:
// Wpad != 512, or more than 256 workgroups, the co-resident count of the 256-CU MI355X).
static size_t pair_area_bytes(const Geometry& g, int N) {
    const int ntiles = (N + 15) / 16;
    if (g.T != 8 || (size_t)2 * ntiles * g.E > 256) return 0;
    return pair_layout(g.Wpad, g.pw, ntiles, g.E).bytes;
}

// MBRL_OPT_ROLLOUT_PAIR = 1 on a plan whose shape or size has no pair area: an error, not a fallback.
static int pair_forced_check(const Geometry& g, int N) {
    if (g_opt[MBRL_OPT_ROLLOUT_PAIR].load(std::memory_order_relaxed) == 1 && pair_area_bytes(g, N) == 0)
        return fail(MBRL_EUNSUPPORTED, "rollout_pair forced: no pair kernel for N=%d (Wpad %d, E %d)", N, g.Wpad, g.E);
    return MBRL_OK;
}

// The hand-off words a plan's first launch zeroes (cem_init_kernel): the pair flags of a shard of Nl
// candidates (when the workspace offers pairs) and the trajectory kernel's granules with the status
// word right behind them (the workspaces lay them out so; else the trajectory launch keeps its memset).
static InitZero plan_zero(const Geometry& g, int Nl, void* pair, unsigned long long* xchg, size_t xchg_bytes,
                          unsigned* status) {
    InitZero z{};
    if (pair && pair_area_bytes(g, Nl)) {
        z.ptr[0] = static_cast<unsigned*>(pair);
        z.words[0] = pair_layout(g.Wpad, g.pw, (Nl + 15) / 16, g.E).zero_bytes / 4;
    }
    if (xchg && status && reinterpret_cast<char*>(status) == reinterpret_cast<char*>(xchg) + xchg_bytes) {
        z.ptr[1] = reinterpret_cast<unsigned*>(xchg);
        z.words[1] = (xchg_bytes + 16) / 4;
    }
    return z;
}

// The argument checks of rollout_impl that depend on the problem only (not on N or the buffers): the
// sharded plan runs them before its first collective.
static int rollout_validate(const Geometry& g, const mbrl_norm* norm, const mbrl_cost* cost) {
    if (norm) {
        if (norm->unnormalize_reward && (!norm->rew_mean || !norm->rew_std))
            return fail(MBRL_EINVAL, "reward unnormalisation requested without rew_mean/rew_std");
        if ((norm->normalize_state || norm->unnormalize_state) && (!norm->obs_mean || !norm->obs_std))
            return fail(MBRL_EINVAL, "state normalisation requested without obs_mean/obs_std");
        if (norm->normalize_action && (!norm->act_mean || !norm->act_std))
            return fail(MBRL_EINVAL, "action normalisation requested without act_mean/act_std");
    }
    if (cost && cost->kind == MBRL_COST_MODEL_REWARD) {
        if (!g.reward) return fail(MBRL_EINVAL, "MODEL_REWARD cost needs a reward_head model");
    } else if (cost) {
        if (cost->kind != MBRL_COST_GOAL_STATE) return fail(MBRL_EUNSUPPORTED, "cost kind %d", cost->kind);
        if (cost->has_state_cost && (!cost->weights || !cost->goal))
            return fail(MBRL_EINVAL, "state cost without weights/goal");
    }
    if (16 * g.a > 768) return fail(MBRL_EUNSUPPORTED, "action_dim %d too large (max 48)", g.a);
    return MBRL_OK;
}

// pair_area: a pair_area_bytes(g, N) block of the caller's workspace, or NULL (no column-split pairs).
// pair_epoch: NULL (the pair flags are zeroed by a memset before a pair launch), or the plan's counter
// of pair launches, whose flags its first launch zeroed (cem_init_kernel): each pair launch takes the
// next epoch (RolloutArgs), and a memset only when the epochs would outgrow the 32-bit flags.
static int rollout_impl(const Geometry& g, const void* packed, const mbrl_norm* norm, const mbrl_cost* cost,
                        const float* s0, int s0_per_cand, const float* actions, const mbrl_sampler* sampler,
                        int N, int H, int n_offset, float* costs, float* actions_out, float* states_out,
                        hipStream_t stream, void* pair_area = nullptr, unsigned* pair_epoch = nullptr,
                        const unsigned** pair_status_out = nullptr) {
    if (!packed || !s0 || !costs) return fail(MBRL_EINVAL, "packed, s0 and costs must be non-NULL");
    if (N < 1 || H < 1) return fail(MBRL_EINVAL, "N=%d H=%d must be >= 1", N, H);
    if (!actions && !sampler) return fail(MBRL_EINVAL, "need either actions or a sampler");
    if (n_offset < 0) return fail(MBRL_EINVAL, "n_offset=%d < 0", n_offset);
    if (int rc = rollout_validate(g, norm, cost)) return rc;
    RolloutArgs A{};
    A.packed = static_cast<const float*>(packed);
    A.member_stride = g.member_stride;
    A.stream_floats = g.stream_floats;
    A.s = g.s; A.a = g.a; A.L = g.L; A.Wpad = g.Wpad; A.K0C = g.K0C; A.NOT = g.NOT; A.E = g.E;
    A.chunks_per_step = g.C; A.lda = g.lda; A.pw = g.pw; A.k0pad_extra = 16 * g.K0C - g.s - g.a;
    A.N = N; A.H = H; A.n_offset = n_offset;
    if (norm) {
        A.obs_mean = norm->obs_mean; A.obs_std = norm->obs_std;
        A.act_mean = norm->act_mean; A.act_std = norm->act_std;
        A.norm_s = norm->normalize_state; A.unnorm_s = norm->unnormalize_state; A.norm_a = norm->normalize_action;
        A.unnorm_r = norm->unnormalize_reward; A.rew_mean = norm->rew_mean; A.rew_std = norm->rew_std;
    }
    if (cost && cost->kind == MBRL_COST_MODEL_REWARD) {
        A.reward = 1;
    } else if (cost) {
        A.has_sc = cost->has_state_cost; A.has_ac = cost->has_action_cost;
        A.cw = cost->weights; A.goal = cost->goal;
        A.alpha_s = cost->alpha_state; A.alpha_s2 = cost->alpha_state * cost->alpha_state;
        A.alpha_a = cost->alpha_action; A.alpha_a2 = cost->alpha_action * cost->alpha_action;
    }
    A.s0 = s0; A.s0_per_cand = s0_per_cand;
    if (!actions) {
        // CEM proposal: draw into actions_out first, then roll those actions out
        if (!actions_out) return fail(MBRL_EINVAL, "a sampled rollout needs actions_out to hold the draw");
        if (!sampler->mu || !sampler->sigma) return fail(MBRL_EINVAL, "sampler mu/sigma NULL");
        int rc = sample_impl(sampler, H, g.a, N, n_offset, actions_out, stream);
        if (rc) return rc;
        actions = actions_out;
    }
    A.actions = actions;
    A.costs = costs; A.states_out = states_out;
    // Tile height: two 16-row blocks per workgroup halve the weight stream per FLOP once there are
    // enough candidates to still give every CU a workgroup.
    int R = (N >= 2 * 16 * 256 && g.T <= 8) ? 2 : 1;
    const int G = (g.a + 3) / 4;
    (void)G;
    if (16 * R * g.a > 768) R = 1;
    // waves per workgroup as launch_rollout_t picks them: 8 for R = 1 (T >= 2), else 4
    A.nw = (R == 1 && g.T >= 2) ? 8 : 4;
    if ((g.precision == MBRL_PRECISION_F16X3 || g.precision == MBRL_PRECISION_F16X6) && g.split_ok && !A.reward) {
        const int P = g.precision == MBRL_PRECISION_F16X6 ? 3 : 2;
        RolloutArgs S = A;
        S.split_off = P == 3 ? g.split3_off : g.split_off;
        S.K0S = g.K0S;
        S.CS = g.CS;
        S.sr = P * (g.Wpad > 32 * g.K0S ? g.Wpad : 32 * g.K0S) + 8;
        S.nw = 8;
        // 32 candidates per workgroup once that still gives every CU a workgroup (N >= 8192): the
        // split kernel is bound by the L2 weight stream, which R = 2 halves per candidate. At
        // N = 4096 R = 2 would idle half the CUs: 0.607 vs 0.571 ms per F16X3 rollout (cheetah, r01).
        int RS = N >= 256 * 32 ? 2 : 1;
        if (const int o = g_opt[MBRL_OPT_SPLIT_TILE].load(std::memory_order_relaxed)) RS = o == 32 ? 2 : 1;
        RolloutArgs X = A;                 // the fp32 redo pass at the same tile height
        X.redo = 1;
        X.nw = RS == 1 && g.T >= 2 ? 8 : 4;
        if (RS == 2 && (!rollout_split_supported(S, g.T, 2, P) || rollout_lds_bytes(X, 32) > 160 * 1024)) {
            RS = 1;
            X.nw = g.T >= 2 ? 8 : 4;
        }
        if (rollout_split_supported(S, g.T, RS, P)) {
            hipError_t err = launch_rollout_split(S, g.T, RS, P, stream);
            if (err != hipSuccess) return hip_check(err, "split rollout launch");
            // fp32 redo of the workgroups that met an operand outside the split range (usually none:
            // every workgroup reads its candidates' costs and exits)
            return hip_check(launch_rollout(X, g.T, RS, stream), "split redo launch");
        }
    }
    // ensembles: member-major workgroup order per XCD (mbrl_internal.h xcd_unit), opt-in. The plain
    // (tile, member) grid already keeps each XCD on one member at a time (consecutive ids of one member
    // round-robin over the XCDs), so it measured the same (humanoid 75.5 ms either way)
    A.xcd_map = (g.E > 1 && g_opt[MBRL_OPT_XCD_MAP].load(std::memory_order_relaxed) == 1) ? 1 : 0;
    // 8-candidate tiles (rollout_m8_kernel, bit-identical sums) when 16-candidate tiles would leave
    // at least half the CUs idle: the shard of a strong-scaled plan, small plans.
    // MBRL_OPT_ROLLOUT_TILE = 8 / 16 forces a choice (tests, A/B).
    // column-split pairs: each 16-candidate tile on two workgroups of half the columns (16x16x4 MFMA at
    // full clock, half the weight stream per workgroup) where 16-candidate tiles would leave at least
    // half the CUs idle; opt-in until measured (MBRL_OPT_ROLLOUT_PAIR)
    if (pair_area && !A.reward && g_opt[MBRL_OPT_ROLLOUT_TILE].load(std::memory_order_relaxed) == 0) {
        const int po = g_opt[MBRL_OPT_ROLLOUT_PAIR].load(std::memory_order_relaxed);
        const int ntiles = (N + 15) / 16;
        // auto: where the pairs fill more than half the CUs and at most all of them (one workgroup per
        // CU, all co-resident): the 2048-candidate shard of walker over 8 GPUs, 0.691 vs 0.715-0.722 ms
        // per rollout on 8-candidate tiles with L2-resident hand-offs (profiles/r04/pair_l2_ab.json);
        // at 1024 (half the chip) the 8-candidate tiles stay ahead, 0.54 vs 0.69 ms
        const size_t pw = (size_t)ntiles * g.E * 2, cus = (size_t)device_cus();
        const bool want = po == 1 || (po == 0 && kPairAuto && 2 * pw > cus && pw <= cus);
        if (want && pair_area_bytes(g, N) != 0) {
            RolloutArgs P = A;
            P.pair_flags = static_cast<unsigned*>(pair_area);
            P.pair_data = reinterpret_cast<float*>(static_cast<char*>(pair_area) +
                                                   pair_layout(g.Wpad, g.pw, ntiles, g.E).flags_bytes);
            if (rollout_pair_supported(P, g.T)) {
                const int dpa = g_opt[MBRL_OPT_DEBUG_PAIR_ABORT].load(std::memory_order_relaxed);
                P.debug_abort = dpa == 1;
                P.pair_l2 = g_opt[MBRL_OPT_PAIR_L2].load(std::memory_order_relaxed) != 2;
                const unsigned qs = pair_handoffs(H, g.L);
                if (pair_epoch && (uint64_t)(*pair_epoch + 1) * qs + 16 < (1ull << 31)) {
                    P.pair_epoch = ++*pair_epoch;   // flags zeroed by the plan's first launch
                    P.pair_prezeroed = 1;
                } else {
                    P.pair_epoch = 1;               // a memset before the launch; the plan restarts its epochs
                    P.pair_prezeroed = 0;
                    if (pair_epoch) *pair_epoch = 1;
                }
                P.pair_base = (P.pair_epoch - 1) * qs;
                const hipError_t err = launch_rollout_pair(P, g.T, stream);
                if (err == hipSuccess && dpa == 2) return MBRL_OK;   // tests: the pair launch's own results
                if (err == hipSuccess && pair_status_out && P.pair_prezeroed) {
                    // the caller checks the plan's pair status word once, after the plan (a sharded plan
                    // with peers: it redoes the whole plan without pairs if any hand-off timed out), so
                    // no gated redo launch follows each pair launch
                    *pair_status_out = P.pair_flags + (size_t)2 * ntiles * g.E * 32;
                    return MBRL_OK;
                }
                if (err == hipSuccess) {
                    // A pair's halves wait on each other, and a plain launch does not promise that both
                    // are resident (another stream may hold CUs): a wait that timed out raised the status
                    // word after the flags to the launch's epoch and left its tile's costs invalid. The
                    // launch chosen below then recomputes every candidate if it did, else its workgroups
                    // exit at once (bit-identical sums on every tile height).
                    A.gate = P.pair_flags + (size_t)2 * ntiles * g.E * 32;
                    A.gate_epoch = P.pair_epoch;
                } else if (err != hipErrorCooperativeLaunchTooLarge || po == 1) {
                    return hip_check(err, "rollout pair launch");
                }
            } else if (po == 1) {
                return fail(MBRL_EUNSUPPORTED, "rollout_pair forced: shape not supported by the pair kernel");
            }
        } else if (po == 1) {
            return fail(MBRL_EUNSUPPORTED, "rollout_pair forced: no pair area for N=%d (Wpad %d, E %d)", N, g.Wpad, g.E);
        }
    }
    if (g.m8_ok) {
        A.m8_off = g.m8_off;
        A.C8 = g.C8;
        A.m4_off = g.m4_off;
        A.C4 = g.C4;
        const int o = g_opt[MBRL_OPT_ROLLOUT_TILE].load(std::memory_order_relaxed);
        // 4-candidate tiles (rollout_m4_kernel) once 8-candidate tiles would still leave at least half
        // the CUs idle (cartpole's N = 1024, shards of <= 1024 candidates); both bit-identical
        bool use4 = false;   // opt-in: slower than 8-candidate tiles at cartpole size
        bool use8 = (size_t)((N + 15) / 16) * g.E * 2 <= (size_t)device_cus();
        if (o) { use4 = o == 4; use8 = o == 8; }
        if (use4 && g.m4_ok && rollout_m4_supported(A, g.T, g.NG4))
            return hip_check(launch_rollout_m4(A, g.T, g.NG4, stream), "rollout m4 launch");
        if ((use8 || use4) && rollout_m8_supported(A, g.T))
            return hip_check(launch_rollout_m8(A, g.T, stream), "rollout m8 launch");
    }
    // partials in the activation buffer the last hidden layer does not read (rollout.hip): layer 0
    // writes act2, hidden layer l reads act2 for odd l, so with L odd the last one reads act and act2
    // is free from the barrier after layer L-2 until the next step's layer 0
    // 32-candidate tiles on 8 waves (two per SIMD) when the 8 partials fit the aliased activation
    // buffer: walker rollout 3.91 -> 3.83 ms, frac 0.883 -> 0.901 (profiles/r02_ab_r2_8waves.txt)
    if (R == 2 && g.T >= 2 && !A.reward && g.L >= 3 && (g.L & 1) && (size_t)8 * g.pw <= (size_t)g.lda) A.nw = 8;
    auto alias_ok = [&]() {
        return !A.reward && g.L >= 3 && (g.L & 1) && (size_t)(A.nw > 4 ? A.nw : 4) * g.pw <= (size_t)g.lda;
    };
    A.part_alias = alias_ok() ? 1 : 0;
    if (rollout_lds_bytes(A, 16 * R) > 160 * 1024) {
        R = 1;
        A.nw = g.T >= 2 ? 8 : 4;
        A.part_alias = alias_ok() ? 1 : 0;
        if (rollout_lds_bytes(A, 16) > 160 * 1024)
            return fail(MBRL_EUNSUPPORTED, "LDS footprint %zu B exceeds 160 KiB", rollout_lds_bytes(A, 16));
    }
    return hip_check(launch_rollout(A, g.T, R, stream), "rollout launch");
}

// prezeroed: the plan's first launch zeroed xchg and status (cem_init_kernel), so no memset here.
static int traj_impl(const Geometry& g, const void* packed, const mbrl_norm* norm, const float* s0,
                     const float* actions, int H, float* states_out, unsigned long long* xchg, size_t xchg_bytes,
                     unsigned* status, hipStream_t stream, int prezeroed = 0) {
    TrajArgs T{};
    T.prezeroed = prezeroed;
    T.packed = static_cast<const float*>(packed);
    T.member_stride = g.member_stride;
    T.bias_off = g.stream_floats;
    T.tw_base = g.stream_floats + g.bias_floats;
    for (int l = 0; l <= g.L; ++l) T.tw_off[l] = g.tw_off[l];
    T.s = g.s; T.a = g.a; T.W = g.W; T.Wpad = g.Wpad; T.L = g.L; T.H = H;
    if (norm) {
        T.obs_mean = norm->obs_mean; T.obs_std = norm->obs_std;
        T.act_mean = norm->act_mean; T.act_std = norm->act_std;
        T.norm_s = norm->normalize_state; T.unnorm_s = norm->unnormalize_state; T.norm_a = norm->normalize_action;
    }
    T.s0 = s0; T.actions = actions; T.states_out = states_out;
    if (traj_reg_supported(T) && g_opt[MBRL_OPT_DEBUG_TRAJ_ABORT].load(std::memory_order_relaxed) == 0)
        return hip_check(launch_traj_reg(T, g.E, stream), "trajectory launch");
    if (xchg && status && traj_coop_supported(T, g.E) && xchg_bytes >= traj_coop_xchg_bytes(T, g.E)) {
        T.debug_abort = g_opt[MBRL_OPT_DEBUG_TRAJ_ABORT].load(std::memory_order_relaxed) != 0;
        const int hop = g_opt[MBRL_OPT_TRAJ_HOP].load(std::memory_order_relaxed);
        T.hop_mode = hop == 0 ? kTrajHopDefault : hop - 1;
        const hipError_t err = launch_traj_coop(T, g.E, xchg, status, stream);
        if (err != hipErrorCooperativeLaunchTooLarge) {   // too large: the grid cannot be co-resident
            int rc = hip_check(err, "trajectory launch");
            if (rc) return rc;
            // The cooperative kernel needs its P*E workgroups co-resident; if a hand-off ever timed
            // out (another process holding CUs, say) it set `status` and gave up. The single-workgroup
            // kernel then recomputes the states; otherwise its E workgroups read the status word and exit.
            // (Run inside the cooperative launch instead, the fallback's registers raised the kernel's
            // from 107 to 161 VGPRs: one workgroup per CU, and two plans' trajectories on one XCD then
            // waited on each other until the hand-off timeout.)
            T.gate = status;
        }
        T.debug_abort = 0;
    }
    return hip_check(launch_traj(T, g.E, stream), "trajectory launch");
}

static int select_impl(const float* costs, int E, int N, int K, int nan_policy, int64_t* elite_idx,
                       float* returns_out, void* ws, size_t ws_bytes, hipStream_t stream, int segments = 1) {
    if (!costs || !elite_idx || !ws) return fail(MBRL_EINVAL, "costs, elite_idx and workspace must be non-NULL");
    if (N < 1 || K < 1 || K > N || E < 1 || segments < 1)
        return fail(MBRL_EINVAL, "need 1 <= K (%d) <= N (%d), E >= 1, segments >= 1", K, N);
    const size_t need = align256((size_t)N * segments * 4);
    if (ws_bytes < need) return fail(MBRL_EWORKSPACE, "select workspace %zu < %zu", ws_bytes, need);
    const int member_stride = N * segments;
#define MBRL_SEL(KPT)                                                                                       \
    if (N <= 1024 * (KPT)) {                                                                                \
        const size_t lds = select_reg_lds(KPT);                                                             \
        hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(&select_reg_kernel<KPT>), (int)lds); \
        if (err != hipSuccess) return hip_check(err, "select attribute");                                   \
        hipLaunchKernelGGL(select_reg_kernel<KPT>, dim3(segments), dim3(1024), lds, stream, costs, E, N, K,  \
                           nan_policy, elite_idx, returns_out, member_stride);                              \
        return hip_check(hipGetLastError(), "select launch");                                               \
    }
    MBRL_SEL(1) MBRL_SEL(2) MBRL_SEL(4) MBRL_SEL(8) MBRL_SEL(16) MBRL_SEL(32)
#undef MBRL_SEL
    hipLaunchKernelGGL(select_kernel, dim3(segments), dim3(1024), 0, stream, costs, E, N, K, nan_policy, elite_idx,
                       returns_out, static_cast<uint32_t*>(ws), member_stride);
    return hip_check(hipGetLastError(), "select launch");
}

static int refit_impl(const mbrl_sampler* sp, int H, int a, const int64_t* elite_idx, int K, float alpha,
                      float* aelite, float* mu_out, float* sigma_out, hipStream_t stream, float* fin_mu = nullptr,
                      float* fin_sigma = nullptr, float* fin_actions = nullptr, int B = 1, int n_env = 0) {
    if (!sp || !sp->mu || !sp->sigma || !elite_idx || !mu_out || !sigma_out)
        return fail(MBRL_EINVAL, "refit: NULL argument");
    if (H < 1 || a < 1 || a > 64 || K < 1) return fail(MBRL_EINVAL, "refit: H=%d a=%d K=%d", H, a, K);
    const float oma = 1.0f - alpha;
    const size_t lds = refit_fused_lds(a, K);
    if (lds <= REFIT_LDS_MAX) {
        hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(&refit_fused_kernel), (int)REFIT_LDS_MAX);
        if (err != hipSuccess) return hip_check(err, "refit attribute");
        hipLaunchKernelGGL(refit_fused_kernel, dim3(H, B), dim3(REFIT_THREADS), lds, stream, sp->seed,
                           sp->iteration, sp->mu, sp->sigma, sp->lo, sp->hi, a, elite_idx, K, alpha, oma, mu_out,
                           sigma_out, fin_mu, fin_sigma, fin_actions, n_env);
        return hip_check(hipGetLastError(), "refit launch");
    }
    // large K x a: elite actions staged through HBM
    if (B != 1) return fail(MBRL_EUNSUPPORTED, "batched refit: K=%d x a=%d exceeds the fused kernel's LDS", K, a);
    if (!aelite) return fail(MBRL_EINVAL, "refit: NULL workspace");
    if ((size_t)((K + ELITE_CHUNK - 1) / ELITE_CHUNK) * a * sizeof(float) > 64 * 1024)
        return fail(MBRL_EUNSUPPORTED, "refit: K=%d x a=%d exceeds the refit kernel's LDS", K, a);
    const int G = (a + 3) / 4;
    hipLaunchKernelGGL(gather_elites_kernel, dim3((K * G + 255) / 256, H), dim3(256), 0, stream, sp->seed,
                       sp->iteration, sp->mu, sp->sigma, sp->lo, sp->hi, a, elite_idx, K, aelite);
    const int nch = (K + ELITE_CHUNK - 1) / ELITE_CHUNK;
    hipLaunchKernelGGL(refit_kernel, dim3(H), dim3(256), (size_t)nch * a * sizeof(float), stream, aelite, a, K,
                       alpha, oma, sp->mu, sp->sigma, mu_out, sigma_out);
    if (fin_actions)
        hipLaunchKernelGGL(finalize_kernel, dim3((H * a + 255) / 256), dim3(256), 0, stream, mu_out, sigma_out,
                           sp->lo, sp->hi, H * a, fin_mu, fin_sigma, fin_actions);
    return hip_check(hipGetLastError(), "refit launch");
}

// The fused per-iteration update (cem_update_kernel) when its selection fits in registers (N <= 32768)
// and the selection or refit working set fits LDS; KPT of that selection, 0 if not fusable.
static int update_kpt(int N, int K, int a) {
    if (a > 64 || K < 1 || K > N) return 0;
    for (int kpt = 1; kpt <= 32; kpt *= 2)
        if (N <= 1024 * kpt) return update_lds_words(kpt, a, K) * 4 + 1024 <= 160 * 1024 ? kpt : 0;   // + static LDS
    return 0;
}

// Whether the update also draws the next iteration's proposals: at most 64 Philox blocks per thread
// (the H blocks of the launch draw N x H x a values between them).
static bool update_samples(int N, int a) { return (size_t)N * ((a + 3) / 4) <= 64 * 1024; }

// Candidate slices per row for the fused draw: about 256 workgroups in all (one per CU; each runs the
// selection too), and no slice under 256 Philox blocks.
static int draw_slices(int H, int B, int N, int a) {
    const long hb = (long)H * B;
    long s = 256 / hb;
    const long cap = ((long)N * ((a + 3) / 4) + 255) / 256;
    if (s > cap) s = cap;
    return s < 1 ? 1 : (int)s;
}

// The split update (two launches, cem_select_regen_kernel + cem_refit_draw_kernel) where the elites'
// regeneration is worth sharing out: at least SPLIT_MIN_BLOCKS Philox blocks per row (walker's K =
// 1638: 3276 blocks, ~10 us of one workgroup's VALU; cheetah's 818 would save less than the launch
// boundary costs). MBRL_OPT_UPDATE_SPLIT: 0 auto, 1 never, 2 wherever scratch is given (tests, A/B).
constexpr long SPLIT_MIN_BLOCKS = 2048;

static bool update_split(const UpdateArgs& U, int B) {
    const int o = g_opt[MBRL_OPT_UPDATE_SPLIT].load(std::memory_order_relaxed);
    if (o == 1 || B != 1 || !U.ael) return false;
    return o == 2 || (long)U.K * ((U.a + 3) / 4) >= SPLIT_MIN_BLOCKS;
}

static int update_split_impl(const UpdateArgs& U, int kpt, hipStream_t stream) {
    // workgroups per row: the draw's slices, and at least ~256 workgroups in all for the regeneration
    const int Sd = U.next_actions ? draw_slices(U.H, 1, U.draw_n, U.a) : 1;
    const int S = std::max(Sd, std::max(1, 256 / U.H));
    const int a4 = (U.a + 3) & ~3;
    const size_t lds_a = ((((size_t)U.K + 3) & ~(size_t)3) + 2 * a4 + (size_t)sel_words(kpt)) * 4;
    const size_t lds_b = (2 * a4 + refit_rows_floats(U.a, U.K)) * 4;
    if (lds_b + 1024 > 160 * 1024) return fail(MBRL_EUNSUPPORTED, "split update: K=%d a=%d exceeds LDS", U.K, U.a);
#define MBRL_SPLIT_A(KPT)                                                                                       \
    if (kpt == KPT) {                                                                                           \
        hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(&cem_select_regen_kernel<KPT>), (int)lds_a); \
        if (err != hipSuccess) return hip_check(err, "split update attribute");                                 \
        hipLaunchKernelGGL(cem_select_regen_kernel<KPT>, dim3(U.H * S), dim3(1024), lds_a, stream, U);          \
    }
    MBRL_SPLIT_A(1) MBRL_SPLIT_A(2) MBRL_SPLIT_A(4) MBRL_SPLIT_A(8) MBRL_SPLIT_A(16) MBRL_SPLIT_A(32)
#undef MBRL_SPLIT_A
    if (int rc = hip_check(hipGetLastError(), "split update launch 1")) return rc;
    hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(&cem_refit_draw_kernel), (int)lds_b);
    if (err != hipSuccess) return hip_check(err, "split update attribute");
    hipLaunchKernelGGL(cem_refit_draw_kernel, dim3(U.H * S), dim3(1024), lds_b, stream, U);
    return hip_check(hipGetLastError(), "split update launch 2");
}

static int update_impl(const UpdateArgs& U, int B, hipStream_t stream) {
    const int kpt = update_kpt(U.N, U.K, U.a);
    if (!kpt) return fail(MBRL_EUNSUPPORTED, "update: N=%d K=%d a=%d not fusable", U.N, U.K, U.a);
    if (update_split(U, B)) return update_split_impl(U, kpt, stream);
    const size_t lds = update_lds_words(kpt, U.a, U.K) * 4;
    const int S = U.next_actions ? draw_slices(U.H, B, U.draw_n, U.a) : 1;
#define MBRL_UPD(KPT)                                                                                            \
    if (kpt == KPT) {                                                                                           \
        hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(&cem_update_kernel<KPT>), (int)lds);   \
        if (err != hipSuccess) return hip_check(err, "update attribute");                                       \
        hipLaunchKernelGGL(cem_update_kernel<KPT>, dim3(U.H * S, B), dim3(1024), lds, stream, U);                \
        return hip_check(hipGetLastError(), "update launch");                                                   \
    }
    MBRL_UPD(1) MBRL_UPD(2) MBRL_UPD(4) MBRL_UPD(8) MBRL_UPD(16) MBRL_UPD(32)
#undef MBRL_UPD
    return fail(MBRL_EUNSUPPORTED, "update: KPT %d", kpt);
}

}  // namespace mbrl

using namespace mbrl;

// ================================================================================================
// extern "C" ABI
// ================================================================================================
extern "C" {

int mbrl_abi_version(void) { return MBRL_ABI_VERSION; }

#if __has_include("src_digest.h")
#include "src_digest.h"
#else
#define MBRL_SRC_DIGEST "unknown"
#endif
const char* mbrl_build_info(void) { return "src=" MBRL_SRC_DIGEST " arch=gfx950"; }

const char* mbrl_last_error(void) { return g_err.c_str(); }

int mbrl_set_option(int32_t option, int32_t value) {
    if (option < 0 || option >= MBRL_OPT_COUNT) return fail(MBRL_EINVAL, "unknown option %d", option);
    bool ok = false;
    switch (option) {
        case MBRL_OPT_ROLLOUT_TILE: ok = value == 0 || value == 4 || value == 8 || value == 16; break;
        case MBRL_OPT_SPLIT_TILE: ok = value == 0 || value == 16 || value == 32; break;
        case MBRL_OPT_ADAM_ARITH: ok = value >= 0 && value <= 16; break;
        case MBRL_OPT_TRAIN_TILE: ok = value == 0 || value == 32 || value == 64; break;
        case MBRL_OPT_ROLLOUT_PAIR: ok = value >= 0 && value <= 2; break;
        case MBRL_OPT_DEBUG_PAIR_ABORT: ok = value >= 0 && value <= 2; break;
        case MBRL_OPT_TRAJ_HOP: ok = value >= 0 && value <= 3; break;
        case MBRL_OPT_GD_HOP: ok = value >= 0 && value <= 3; break;
        case MBRL_OPT_PAIR_L2: ok = value >= 0 && value <= 2; break;
        case MBRL_OPT_DEBUG_SHARD_FAIL: ok = value >= 0 && value <= 1 << 20; break;
        case MBRL_OPT_DEBUG_SHARD_FAIL_RANK: ok = value >= 0 && value <= 1 << 20; break;
        case MBRL_OPT_SHARD_EMULATE: ok = value >= 0 && value <= 2; break;
        case MBRL_OPT_UPDATE_SPLIT: ok = value >= 0 && value <= 2; break;
        default: ok = value == 0 || value == 1; break;
    }
    if (!ok) return fail(MBRL_EINVAL, "option %d: value %d not allowed", option, value);
    return g_opt[option].exchange(value);
}

int mbrl_host_alloc(size_t bytes, void** host_ptr, void** device_ptr) {
    if (!host_ptr || !device_ptr || bytes == 0) return fail(MBRL_EINVAL, "mbrl_host_alloc: bad arguments");
    *host_ptr = nullptr;
    *device_ptr = nullptr;
    void* h = nullptr;
    int rc = hip_check(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
    if (rc) return rc;
    void* d = nullptr;
    rc = hip_check(hipHostGetDevicePointer(&d, h, 0), "hipHostGetDevicePointer");
    if (rc) {
        (void)hipHostFree(h);
        return rc;
    }
    *host_ptr = h;
    *device_ptr = d;
    return MBRL_OK;
}

int mbrl_host_free(void* host_ptr) {
    return host_ptr ? hip_check(hipHostFree(host_ptr), "hipHostFree") : MBRL_OK;
}

int mbrl_event_create(mbrl_event_t* event) {
    if (!event) return fail(MBRL_EINVAL, "event_create: NULL");
    hipEvent_t e = nullptr;
    if (int rc = hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence),
                           "hipEventCreateWithFlags"))
        return rc;
    *event = reinterpret_cast<mbrl_event_t>(e);
    return MBRL_OK;
}

int mbrl_event_record(mbrl_event_t event, mbrl_stream_t stream) {
    if (!event) return fail(MBRL_EINVAL, "event_record: NULL event");
    return hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(event), reinterpret_cast<hipStream_t>(stream)),
                     "hipEventRecord");
}

int mbrl_stream_wait_event(mbrl_stream_t stream, mbrl_event_t event) {
    if (!event) return fail(MBRL_EINVAL, "stream_wait_event: NULL event");
    return hip_check(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<hipEvent_t>(event), 0),
                     "hipStreamWaitEvent");
}

int mbrl_event_synchronize(mbrl_event_t event) {
    if (!event) return fail(MBRL_EINVAL, "event_synchronize: NULL event");
    return hip_check(hipEventSynchronize(reinterpret_cast<hipEvent_t>(event)), "hipEventSynchronize");
}

int mbrl_event_destroy(mbrl_event_t event) {
    return event ? hip_check(hipEventDestroy(reinterpret_cast<hipEvent_t>(event)), "hipEventDestroy") : MBRL_OK;
}

int mbrl_get_option(int32_t option) {
    if (option < 0 || option >= MBRL_OPT_COUNT) return fail(MBRL_EINVAL, "unknown option %d", option);
    return g_opt[option].load();
}

size_t mbrl_mlp_packed_bytes(const mbrl_mlp_shape* shape) {
    Geometry g;
    if (shape_geometry(shape, &g) != MBRL_OK) return 0;
    return g.member_stride * (size_t)g.E * sizeof(float);
}

int mbrl_mlp_pack(const mbrl_mlp_shape* shape, const float* const* weights, const float* const* biases,
                  void* packed, mbrl_stream_t stream_) {
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    Geometry g;
    int rc = shape_geometry(shape, &g);
    if (rc) return rc;
    if (!weights || !biases || !packed) return fail(MBRL_EINVAL, "pack: NULL argument");
    const int nl = g.L + 1 + g.reward;   // trunk, state head, [reward head]
    for (int e = 0; e < g.E; ++e) {
        float* base = static_cast<float*>(packed) + (size_t)e * g.member_stride;
        float* bias_base = base + g.stream_floats;
        size_t chunk = 0;
        // the 2-piece (F16X3) and 3-piece (F16X6) split streams, each followed by its flag word
        _Float16* split_base[2] = {reinterpret_cast<_Float16*>(base + g.split_off),
                                   reinterpret_cast<_Float16*>(base + g.split3_off)};
        unsigned* split_bad[2] = {reinterpret_cast<unsigned*>(base + g.split_off + (size_t)g.CS * 2048 * g.T),
                                  reinterpret_cast<unsigned*>(base + g.split3_off + (size_t)g.CS * 3072 * g.T)};
        size_t split_chunk = 0;
        float* m8_base = base + g.m8_off;
        size_t m8_chunk = 0;
        float* m4_base = base + g.m4_off;
        if (g.split_ok)
            for (int q = 0; q < 2; ++q) {
                hipError_t err = hipMemsetAsync(split_bad[q], 0, 4, stream);
                if (err != hipSuccess) return hip_check(err, "pack flag reset");
            }
        for (int l = 0; l <= g.L; ++l) {
            const float* w = weights[e * nl + l];
            const float* b = biases[e * nl + l];
            if (!w || !b) return fail(MBRL_EINVAL, "pack: NULL weight/bias for member %d layer %d", e, l);
            float* dst = base + chunk * 1024 * g.T;
            float* plain = base + g.stream_floats + g.bias_floats + g.tw_off[l];
            if (l < g.L) {
                const int in_real = l == 0 ? g.s + g.a : g.W;
                const int nkc = l == 0 ? g.K0C : 4 * g.T;
                const int rot = l > 0;   // W->W layers: the half-rotated K order of the second column half
                hipLaunchKernelGGL(pack_hidden_kernel, dim3(256), dim3(256), 0, stream, w, in_real, g.W, nkc, g.T, rot, dst);
                hipLaunchKernelGGL(pack_bias_kernel, dim3(4), dim3(256), 0, stream, b, g.W, g.Wpad, bias_base + (size_t)l * g.Wpad);
                hipLaunchKernelGGL(pack_transposed_kernel, dim3(256), dim3(256), 0, stream, w, in_real, g.W, g.Wpad, plain);
                if (g.split_ok) {
                    const int nks = l == 0 ? g.K0S : 2 * g.T;
                    for (int P = 2; P <= 3; ++P)
                        hipLaunchKernelGGL(pack_split_hidden_kernel, dim3(256), dim3(256), 0, stream, w, in_real, g.W,
                                           nks, g.T, P, split_base[P - 2] + split_chunk * 2048 * (size_t)g.T * P,
                                           split_bad[P - 2]);
                    split_chunk += nks;
                }
                if (g.m8_ok) {
                    hipLaunchKernelGGL(pack_m8_hidden_kernel, dim3(256), dim3(256), 0, stream, w, in_real, g.W, nkc,
                                       g.T, (int)(g.T == 4 && g.NOT == 2), rot, m8_base + m8_chunk * 1024 * (size_t)g.T);
                    if (g.m4_ok)   // the same chunks without KP pairing (the m8 chunk index = the m4 one here)
                        hipLaunchKernelGGL(pack_m8_hidden_kernel, dim3(256), dim3(256), 0, stream, w, in_real, g.W, nkc,
                                           g.T, 0, rot, m4_base + m8_chunk * 1024 * (size_t)g.T);
                    m8_chunk += nkc;
                }
                chunk += nkc;
            } else {
                const float* wr = g.reward ? weights[e * nl + g.L + 1] : nullptr;
                const float* br = g.reward ? biases[e * nl + g.L + 1] : nullptr;
                if (g.reward && (!wr || !br)) return fail(MBRL_EINVAL, "pack: NULL reward head for member %d", e);
                hipLaunchKernelGGL(pack_out_kernel, dim3(256), dim3(256), 0, stream, w, wr, g.W, g.s, g.NOT, g.T, dst);
                if (g.split_ok)
                    for (int P = 2; P <= 3; ++P)
                        hipLaunchKernelGGL(pack_split_out_kernel, dim3(256), dim3(256), 0, stream, w, wr, g.W, g.s,
                                           g.NOS, g.T, P, split_base[P - 2] + split_chunk * 2048 * (size_t)g.T * P,
                                           split_bad[P - 2]);
                if (g.m8_ok)
                    hipLaunchKernelGGL(pack_m8_out_kernel, dim3(256), dim3(256), 0, stream, w, g.W, g.s, g.NOP8, g.NOC8 == 2, g.T,
                                       (int)(g.T == 4 && g.NOT == 2),
                                       m8_base + m8_chunk * 1024 * (size_t)g.T);
                if (g.m4_ok)
                    hipLaunchKernelGGL(pack_m4_out_kernel, dim3(256), dim3(256), 0, stream, w, g.W, g.s, g.T,
                                       m4_base + m8_chunk * 1024 * (size_t)g.T);
                float* ob = bias_base + (size_t)g.L * g.Wpad;
                hipLaunchKernelGGL(pack_bias_kernel, dim3(1), dim3(256), 0, stream, b, g.s, 16 * g.NOT, ob);
                hipLaunchKernelGGL(copy_kernel, dim3(64), dim3(256), 0, stream, w, (size_t)g.s * g.W, plain);
                if (g.reward) {   // row s of the output block: the reward head (after the zero padding)
                    hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, stream, br, (size_t)1, ob + g.s);
                    hipLaunchKernelGGL(copy_kernel, dim3(4), dim3(256), 0, stream, wr, (size_t)g.W,
                                       plain + (size_t)g.s * g.W);
                }
                chunk += g.NOT;
            }
        }
    }
    return hip_check(hipGetLastError(), "pack launch");
}

int mbrl_rollout_cost(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const mbrl_cost* cost,
                      const float* s0, int32_t s0_per_candidate, const float* actions, const mbrl_sampler* sampler,
                      int32_t N, int32_t H, int32_t n_offset, float* costs, float* actions_out, float* states_out,
                      mbrl_stream_t stream) {
    Geometry g;
    int rc = shape_geometry(shape, &g);
    if (rc) return rc;
    return rollout_impl(g, packed, norm, cost, s0, s0_per_candidate, actions, sampler, N, H, n_offset, costs,
                        actions_out, states_out, reinterpret_cast<hipStream_t>(stream));
}

size_t mbrl_select_workspace_bytes(int32_t N) { return align256((size_t)(N > 0 ? N : 1) * 4); }

int mbrl_select_elites(const float* costs, int32_t E, int32_t N, int32_t K, int32_t nan_policy, int64_t* elite_idx,
                       float* returns_out, void* workspace, size_t ws_bytes, mbrl_stream_t stream) {
    return select_impl(costs, E, N, K, nan_policy, elite_idx, returns_out, workspace, ws_bytes,
                       reinterpret_cast<hipStream_t>(stream));
}

size_t mbrl_refit_workspace_bytes(int32_t H, int32_t a, int32_t K) {
    return align256((size_t)(H > 0 ? H : 1) * (K > 0 ? K : 1) * (a > 0 ? a : 1) * sizeof(float));
}

int mbrl_cem_refit(const mbrl_sampler* sampler, int32_t H, int32_t a, const int64_t* elite_idx, int32_t K, float alpha,
                   float* mu_out, float* sigma_out, void* workspace, size_t ws_bytes, mbrl_stream_t stream) {
    if (!workspace) return fail(MBRL_EINVAL, "refit: workspace is NULL");
    if (ws_bytes < mbrl_refit_workspace_bytes(H, a, K))
        return fail(MBRL_EWORKSPACE, "refit workspace %zu < %zu", ws_bytes, mbrl_refit_workspace_bytes(H, a, K));
    return refit_impl(sampler, H, a, elite_idx, K, alpha, static_cast<float*>(workspace), mu_out, sigma_out,
                      reinterpret_cast<hipStream_t>(stream));
}

int mbrl_sample_actions(const mbrl_sampler* sampler, int32_t H, int32_t a, int32_t N, int32_t n_offset,
                        float* actions_out, mbrl_stream_t stream) {
    if (!sampler || !sampler->mu || !sampler->sigma || !actions_out) return fail(MBRL_EINVAL, "sample: NULL argument");
    if (H < 1 || a < 1 || N < 1 || n_offset < 0) return fail(MBRL_EINVAL, "sample: bad sizes");
    return sample_impl(sampler, H, a, N, n_offset, actions_out, reinterpret_cast<hipStream_t>(stream));
}

int mbrl_cem_update(const float* costs, int32_t E, int32_t N, int32_t K, const mbrl_sampler* sampler, int32_t H,
                    int32_t a, float alpha, int64_t* elite_idx, float* returns_out, float* mu_out, float* sigma_out,
                    float* next_actions, int32_t draw_offset, int32_t draw_count, mbrl_stream_t stream) {
    if (!costs || !sampler || !sampler->mu || !sampler->sigma || !mu_out || !sigma_out)
        return fail(MBRL_EINVAL, "cem_update: NULL argument");
    if (N < 1 || K < 1 || K > N || E < 1 || H < 1 || a < 1)
        return fail(MBRL_EINVAL, "cem_update: need 1 <= K (%d) <= N (%d), E, H, a >= 1", K, N);
    if (next_actions && (draw_count < 1 || draw_offset < 0 || (int64_t)draw_offset + draw_count > N))
        return fail(MBRL_EINVAL, "cem_update: draw range [%d, %d + %d) outside [0, %d)", draw_offset, draw_offset,
                    draw_count, N);
    if (!update_kpt(N, K, a))
        return fail(MBRL_EUNSUPPORTED, "cem_update: N=%d K=%d a=%d exceeds the fused kernel (select + refit + draw)",
                    N, K, a);
    UpdateArgs U{};
    U.costs = costs; U.E = E; U.N = N; U.K = K; U.member_stride = N; U.H = H; U.a = a;
    U.elite_out = elite_idx; U.returns_out = returns_out;
    U.seed = sampler->seed; U.iteration = sampler->iteration; U.mu = sampler->mu; U.sigma = sampler->sigma;
    U.lo = sampler->lo; U.hi = sampler->hi; U.alpha = alpha; U.oma = 1.0f - alpha;
    U.mu_out = mu_out; U.sigma_out = sigma_out;
    U.next_actions = next_actions; U.draw_off = next_actions ? draw_offset : 0; U.draw_n = next_actions ? draw_count : N;
    return update_impl(U, 1, reinterpret_cast<hipStream_t>(stream));
}

int mbrl_adam_step(const mbrl_adam_tensor* tensors, int32_t count, const mbrl_adam_hparams* hparams,
                   mbrl_stream_t stream) {
    if (count < 0 || (count > 0 && !tensors) || !hparams) return fail(MBRL_EINVAL, "adam_step: NULL argument");
    for (int i = 0; i < count; ++i) {
        const mbrl_adam_tensor& t = tensors[i];
        if (t.numel < 0 || (t.numel > 0 && (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq)))
            return fail(MBRL_EINVAL, "adam_step: tensor %d: NULL pointer or negative numel", i);
    }
    const int o = g_opt[MBRL_OPT_ADAM_ARITH].load(std::memory_order_relaxed);
    return hip_check(launch_adam_step(tensors, count, *hparams, o ? o - 1 : ADAM_ARITH_TORCH,
                                      reinterpret_cast<hipStream_t>(stream)), "adam_step");
}

static int train_shape(const mbrl_train_model* m, TrainShape* t) {
    if (!m) return fail(MBRL_EINVAL, "train: NULL model");
    if (m->state_dim < 1 || m->action_dim < 0 || m->hidden < 1 || m->horizon < 1 || m->n_hidden < 1 ||
        m->n_hidden + 2 > MBRL_TRAIN_MAX_LAYERS || (m->reward_head != 0 && m->reward_head != 1))
        return fail(MBRL_EINVAL, "train: bad shape (state %d, action %d, hidden %d x %d, horizon %d, reward %d)",
                    m->state_dim, m->action_dim, m->hidden, m->n_hidden, m->horizon, m->reward_head);
    t->s = m->state_dim; t->a = m->action_dim; t->W = m->hidden; t->L = m->n_hidden; t->reward = m->reward_head;
    t->H = m->horizon;
    t->tile = g_opt[MBRL_OPT_TRAIN_TILE].load(std::memory_order_relaxed);
    t->fold = g_opt[MBRL_OPT_TRAIN_NO_FOLD].load(std::memory_order_relaxed) == 0 ? 1 : 0;
    t->xcd = g_opt[MBRL_OPT_TRAIN_XCD].load(std::memory_order_relaxed) == 1 ? 1 : 0;
    t->split = g_opt[MBRL_OPT_TRAIN_SPLIT].load(std::memory_order_relaxed) == 1 ? 1 : 0;
    t->fo_split = g_opt[MBRL_OPT_TRAIN_FO].load(std::memory_order_relaxed) == 1 ? 1 : 0;
    return MBRL_OK;
}

size_t mbrl_train_workspace_bytes(const mbrl_train_model* model, int32_t batch) {
    TrainShape t;
    if (batch < 1 || train_shape(model, &t) != MBRL_OK) return 0;
    return train_ws_floats(t, batch) * sizeof(float);
}

size_t mbrl_train_status_offset(const mbrl_train_model* model, int32_t batch) {
    TrainShape t;
    if (batch < 1 || train_shape(model, &t) != MBRL_OK) return (size_t)-1;
    return train_status_offset(t, batch);
}

int mbrl_train_grads(const mbrl_train_model* model, const mbrl_train_data* data, const int64_t* batch_idx,
                     int32_t batch, float* loss_out, void* workspace, size_t ws_bytes, mbrl_stream_t stream) {
    TrainShape t;
    if (int rc = train_shape(model, &t)) return rc;
    if (!data || !batch_idx || !workspace || !data->states || !data->next_states || (t.a > 0 && !data->actions) ||
        (t.reward && !data->rewards))
        return fail(MBRL_EINVAL, "train_grads: NULL argument");
    if (batch < 1 || (int64_t)batch > data->transitions)
        return fail(MBRL_EINVAL, "train_grads: batch %d outside [1, %lld]", batch, (long long)data->transitions);
    const int layers = t.L + 1 + t.reward;
    for (int l = 0; l < layers; ++l)
        if (!model->weight[l] || !model->bias[l] || !model->weight_grad[l] || !model->bias_grad[l])
            return fail(MBRL_EINVAL, "train_grads: layer %d: NULL weight, bias or gradient", l);
    const size_t need = train_ws_floats(t, batch) * sizeof(float);
    if (ws_bytes < need) return fail(MBRL_EWORKSPACE, "train_grads: workspace %zu < %zu bytes", ws_bytes, need);
    TrainTensors w{model->weight, model->bias, model->weight_grad, model->bias_grad,
                   data->states, data->actions, data->next_states, data->rewards};
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (int rc = hip_check(hipMemsetAsync(workspace, 0, train_counter_bytes(t, batch), st), "train_grads counters"))
        return rc;
    return hip_check(launch_train_grads(t, w, batch_idx, batch, loss_out, static_cast<float*>(workspace), st),
                     "train_grads");
}

int mbrl_train_epoch(const mbrl_train_model* model, const mbrl_train_data* data, const int64_t* order, int64_t rows,
                     int32_t batch_size, const mbrl_adam_tensor* tensors, int32_t count,
                     const mbrl_adam_hparams* hparams, const float* step_sizes, const float* bc2_sqrt, float* losses,
                     void* workspace, size_t ws_bytes, mbrl_stream_t stream) {
    TrainShape t;
    if (int rc = train_shape(model, &t)) return rc;
    if (!data || !order || !workspace || !data->states || !data->next_states || (t.a > 0 && !data->actions) ||
        (t.reward && !data->rewards) || !tensors || count < 1 || !hparams || !step_sizes || !bc2_sqrt)
        return fail(MBRL_EINVAL, "train_epoch: NULL argument");
    if (batch_size < 1 || rows < 1 || rows > data->transitions)
        return fail(MBRL_EINVAL, "train_epoch: rows %lld / batch %d outside [1, %lld]", (long long)rows, batch_size,
                    (long long)data->transitions);
    const int layers = t.L + 1 + t.reward;
    for (int l = 0; l < layers; ++l)
        if (!model->weight[l] || !model->bias[l] || !model->weight_grad[l] || !model->bias_grad[l])
            return fail(MBRL_EINVAL, "train_epoch: layer %d: NULL weight, bias or gradient", l);
    for (int i = 0; i < count; ++i)
        if (tensors[i].numel < 0 || (tensors[i].numel > 0 && (!tensors[i].param || !tensors[i].grad ||
                                                              !tensors[i].exp_avg || !tensors[i].exp_avg_sq)))
            return fail(MBRL_EINVAL, "train_epoch: Adam tensor %d: NULL pointer or negative numel", i);
    const int bs = (int)std::min<int64_t>(batch_size, rows);
    const size_t need = train_ws_floats(t, bs) * sizeof(float);
    if (ws_bytes < need) return fail(MBRL_EWORKSPACE, "train_epoch: workspace %zu < %zu bytes", ws_bytes, need);
    TrainTensors w{model->weight, model->bias, model->weight_grad, model->bias_grad,
                   data->states, data->actions, data->next_states, data->rewards};
    const int arith = g_opt[MBRL_OPT_ADAM_ARITH].load(std::memory_order_relaxed);
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // the tickets and band counters start the epoch at zero whatever the workspace held
    if (int rc = hip_check(hipMemsetAsync(workspace, 0, train_counter_bytes(t, bs), st), "train_epoch counters"))
        return rc;
    std::vector<mbrl_adam_tensor> table(tensors, tensors + count);
    const int64_t batches = (rows + batch_size - 1) / batch_size;
    // the Adam step rides in the backward launches when the table is the model's layers in order
    // (weight, bias per Linear, gradients = the model's buffers); otherwise a separate launch
    bool fold = count == 2 * layers;
    for (int l = 0; fold && l < layers; ++l)
        fold = tensors[2 * l].param == model->weight[l] && tensors[2 * l].grad == model->weight_grad[l] &&
               tensors[2 * l + 1].param == model->bias[l] && tensors[2 * l + 1].grad == model->bias_grad[l];
    const int ar = arith ? arith - 1 : ADAM_ARITH_TORCH;
    // a layer's step the layer-0 fold defers: carried by the next batch's first launch, or launched
    // after the last batch
    mbrl_adam_tensor carry[2][4];
    int carry_n = 0;
    // the fused step's F gathers the next batch's rows while it runs when both batches are full-size
    // fused ones (alternating gather slots; the first batch gathers its own)
    TrainGather gather{};
    for (int64_t b = 0; b < batches; ++b) {
        const int n = (int)std::min<int64_t>(batch_size, rows - b * batch_size);
        const int n_next = b + 1 < batches ? (int)std::min<int64_t>(batch_size, rows - (b + 1) * batch_size) : 0;
        const bool hand = n_next == n && t.W > 32 && train_fused_applies(t, n);   // (F's second column tiles)
        gather.idx_next = hand ? order + (b + 1) * batch_size : nullptr;
        gather.batch_next = hand ? n_next : 0;
        for (int i = 0; i < count; ++i) {
            table[i].step_size = step_sizes[b * count + i];
            table[i].bc2_sqrt = bc2_sqrt[b * count + i];
        }
        mbrl_adam_tensor* next = carry[(b + 1) & 1];
        int next_n = 0;
        if (int rc = hip_check(launch_train_grads(t, w, order + b * batch_size, n, losses ? losses + 3 * b : nullptr,
                                                  static_cast<float*>(workspace), st, fold ? table.data() : nullptr,
                                                  hparams, ar, carry[b & 1], carry_n, next, &next_n, &gather),
                               "train_epoch grads"))
            return rc;
        gather.pre_rows = hand ? 1 : 0;
        if (hand) gather.slot ^= 1;
        carry_n = next_n;
        if (!fold)
            if (int rc = hip_check(launch_adam_step(table.data(), count, *hparams, ar, st), "train_epoch adam")) return rc;
    }
    if (carry_n > 0)
        if (int rc = hip_check(launch_adam_step(carry[batches & 1], carry_n, *hparams, ar, st), "train_epoch adam tail"))
            return rc;
    return MBRL_OK;
}

// Workspace for mbrl_trajectory: per-member states, exchange granules, status word.
struct TrajWs {
    float* states;
    unsigned long long* xchg;
    unsigned* status;
    size_t xchg_bytes, bytes;
};

static TrajWs traj_ws(const Geometry& g, int H, void* base) {
    TrajWs w{};
    char* b = static_cast<char*>(base);
    size_t o = 0;
    auto take = [&](size_t n) { void* r = b ? b + o : nullptr; o += align256(n); return r; };
    w.xchg_bytes = (size_t)g.E * 2 * g.Wpad * 8;
    w.xchg = (unsigned long long*)take(w.xchg_bytes);   // memset block first, 16-B multiple (G16)
    w.status = (unsigned*)take(16);
    w.states = (float*)take((size_t)g.E * H * g.s * 4);
    w.bytes = o;
    return w;
}

size_t mbrl_trajectory_workspace_bytes(const mbrl_mlp_shape* shape, int32_t H) {
    Geometry g;
    if (shape_geometry(shape, &g) != MBRL_OK || H < 1) return 0;
    return traj_ws(g, H, nullptr).bytes;
}

int mbrl_trajectory(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const float* s0,
                    const float* actions, int32_t H, float* states_out, float* member_states_out, void* workspace,
                    size_t ws_bytes, mbrl_stream_t stream_) {
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    Geometry g;
    int rc = shape_geometry(shape, &g);
    if (rc) return rc;
    if (H < 1) return fail(MBRL_EINVAL, "trajectory: H=%d", H);
    if (!packed || !s0 || !actions || !states_out || !workspace) return fail(MBRL_EINVAL, "trajectory: NULL argument");
    TrajWs w = traj_ws(g, H, workspace);
    if (ws_bytes < w.bytes) return fail(MBRL_EWORKSPACE, "trajectory workspace %zu < %zu", ws_bytes, w.bytes);
    float* per_member = member_states_out ? member_states_out : (g.E == 1 ? states_out : w.states);
    rc = traj_impl(g, packed, norm, s0, actions, H, per_member, w.xchg, w.xchg_bytes, w.status, stream);
    if (rc) return rc;
    if (per_member != states_out) {
        const int Hs = H * g.s;
        hipLaunchKernelGGL(member_mean_kernel, dim3((Hs + 255) / 256), dim3(256), 0, stream, per_member, g.E, Hs,
                           states_out);
    }
    return hip_check(hipGetLastError(), "trajectory launch");
}

// Workspace layout for mbrl_cem_plan.
struct PlanWs {
    float *costs, *mu[2], *sigma[2], *aelite, *states, *tmp_cost, *actions, *s0;
    void* pair;   // column-split pair exchange area (NULL-sized when pairs are not offered)
    unsigned long long* xchg;
    unsigned* status;
    size_t xchg_bytes;
    int64_t* elites;
    uint32_t* keys;
    size_t bytes;
};

static PlanWs plan_ws(const Geometry& g, const mbrl_cem_params* p, void* base) {
    PlanWs w{};
    char* b = static_cast<char*>(base);
    size_t o = 0;
    auto take = [&](size_t n) { void* r = b ? b + o : nullptr; o += align256(n); return r; };
    const size_t Ha = (size_t)p->H * g.a;
    w.costs = (float*)take((size_t)g.E * p->N * 4);
    w.actions = (float*)take((size_t)p->H * p->N * g.a * 4);
    w.mu[0] = (float*)take(Ha * 4); w.mu[1] = (float*)take(Ha * 4);
    w.sigma[0] = (float*)take(Ha * 4); w.sigma[1] = (float*)take(Ha * 4);
    w.aelite = (float*)take((size_t)p->H * p->K * g.a * 4);
    w.states = (float*)take((size_t)g.E * p->H * g.s * 4);
    w.tmp_cost = (float*)take((size_t)g.E * 4);
    w.elites = (int64_t*)take((size_t)p->K * 8);
    w.keys = (uint32_t*)take((size_t)p->N * 4);
    w.xchg_bytes = (size_t)g.E * 2 * g.Wpad * 8;
    w.xchg = (unsigned long long*)take(w.xchg_bytes);
    w.status = (unsigned*)take(16);
    w.s0 = (float*)take((size_t)g.s * 4);
    w.pair = take(pair_area_bytes(g, p->N));
    w.bytes = o;
    return w;
}

size_t mbrl_cem_workspace_bytes(const mbrl_mlp_shape* shape, const mbrl_cem_params* params) {
    Geometry g;
    if (shape_geometry(shape, &g) != MBRL_OK || !params) return 0;
    return plan_ws(g, params, nullptr).bytes;
}

int mbrl_cem_plan(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const mbrl_cost* cost,
                  const float* s0_in, const mbrl_cem_params* p, float* mu, float* sigma, float* actions_out,
                  float* states_out, float* cost_hist, float* returns_hist, int64_t* elite_hist,
                  mbrl_event_t* rollout_events, void* workspace, size_t ws_bytes, mbrl_stream_t stream_) {
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    Geometry g;
    int rc = shape_geometry(shape, &g);
    if (rc) return rc;
    if (!p) return fail(MBRL_EINVAL, "params is NULL");
    if (p->N < 1 || p->H < 1 || p->K < 1 || p->K > p->N || p->iterations < 1)
        return fail(MBRL_EINVAL, "bad CEM params N=%d H=%d K=%d I=%d", p->N, p->H, p->K, p->iterations);
    if (!actions_out || !states_out || !workspace) return fail(MBRL_EINVAL, "actions_out/states_out/workspace NULL");
    if (!s0_in) return fail(MBRL_EINVAL, "s0 is NULL");
    PlanWs w = plan_ws(g, p, workspace);
    if (ws_bytes < w.bytes) return fail(MBRL_EWORKSPACE, "workspace %zu < %zu", ws_bytes, w.bytes);
    if ((rc = pair_forced_check(g, p->N))) return rc;
    // Launches per iteration: rollout + one fused update (select, refit, next proposals) where it fits;
    // else the proposal draw, rollout, select and refit as separate launches.
    const bool fuse = update_kpt(p->N, p->K, g.a) != 0 && g_opt[MBRL_OPT_UNFUSED_UPDATE].load(std::memory_order_relaxed) == 0;
    const bool fuse_draw = fuse && update_samples(p->N, g.a);
    // one first launch: distribution rows, the s0 copy, iteration 0's proposals (where the update
    // fuses the draw), and the plan's hand-off words zeroed (no memset before the pair / trajectory
    // launches)
    const InitZero z = plan_zero(g, p->N, w.pair, w.xchg, w.xchg_bytes, w.status);
    hipLaunchKernelGGL(cem_init_kernel, dim3(p->H * (fuse_draw ? draw_slices(p->H, 1, p->N, g.a) : 1), 1), dim3(1024), 0,
                       stream, p->seed, p->init_mu, p->init_sigma, p->lo, p->hi, p->H, g.a, p->N, w.mu[0], w.sigma[0],
                       fuse_draw ? w.actions : nullptr, s0_in, g.s, w.s0, 0, z);
    unsigned pair_epoch = 0;
    const float* s0 = w.s0;   // the workspace copy (s0_in may be mapped host memory)
    int cur = 0;
    for (int it = 0; it < p->iterations; ++it) {
        mbrl_sampler sp{};
        sp.seed = p->seed; sp.iteration = it; sp.mu = w.mu[cur]; sp.sigma = w.sigma[cur]; sp.lo = p->lo; sp.hi = p->hi;
        float* costs = cost_hist ? cost_hist + (size_t)it * g.E * p->N : w.costs;
        int64_t* elites = elite_hist ? elite_hist + (size_t)it * p->K : w.elites;
        float* rets = returns_hist ? returns_hist + (size_t)it * p->N : nullptr;
        if (rollout_events && rollout_events[2 * it]) {
            rc = hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(rollout_events[2 * it]), stream), "event");
            if (rc) return rc;
        }
        rc = rollout_impl(g, packed, norm, cost, s0, 0, fuse_draw ? w.actions : nullptr, fuse_draw ? nullptr : &sp, p->N,
                          p->H, 0, costs, w.actions, nullptr, stream, pair_area_bytes(g, p->N) ? w.pair : nullptr,
                          z.ptr[0] ? &pair_epoch : nullptr);
        if (rc) return rc;
        if (rollout_events && rollout_events[2 * it + 1]) {
            rc = hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(rollout_events[2 * it + 1]), stream), "event");
            if (rc) return rc;
        }
        const bool last = it + 1 == p->iterations;   // the last refit also writes mu / sigma / clip(mu)
        if (fuse) {
            UpdateArgs U{};
            U.costs = costs; U.E = g.E; U.N = p->N; U.K = p->K; U.member_stride = p->N; U.H = p->H; U.a = g.a;
            U.elite_out = elites; U.returns_out = rets;
            U.seed = p->seed; U.iteration = it; U.mu = w.mu[cur]; U.sigma = w.sigma[cur];
            U.lo = p->lo; U.hi = p->hi; U.alpha = p->alpha; U.oma = 1.0f - p->alpha;
            U.mu_out = w.mu[cur ^ 1]; U.sigma_out = w.sigma[cur ^ 1];
            U.fin_mu = last ? mu : nullptr; U.fin_sigma = last ? sigma : nullptr; U.fin_actions = last ? actions_out : nullptr;
            U.next_actions = (fuse_draw && !last) ? w.actions : nullptr;
            U.draw_off = 0; U.draw_n = p->N;
            U.ael = w.aelite;   // (scratch of the split update)
            rc = update_impl(U, 1, stream);
        } else {
            rc = select_impl(costs, g.E, p->N, p->K, MBRL_NAN_LAST, elites, rets, w.keys, align256((size_t)p->N * 4), stream);
            if (rc) return rc;
            rc = refit_impl(&sp, p->H, g.a, elites, p->K, p->alpha, w.aelite, w.mu[cur ^ 1], w.sigma[cur ^ 1], stream,
                            last ? mu : nullptr, last ? sigma : nullptr, last ? actions_out : nullptr);
        }
        if (rc) return rc;
        cur ^= 1;
    }
    // final mean's rollout -> predicted states [E][H][s] (E == 1: straight into states_out), member mean
    float* per_member = g.E == 1 ? states_out : w.states;
    rc = traj_impl(g, packed, norm, s0, actions_out, p->H, per_member, w.xchg, w.xchg_bytes, w.status, stream,
                   z.ptr[1] != nullptr);
    if (rc) return rc;
    if (g.E > 1) {
        const int Hs = p->H * g.s;
        hipLaunchKernelGGL(member_mean_kernel, dim3((Hs + 255) / 256), dim3(256), 0, stream, w.states, g.E, Hs,
                           states_out);
    }
    return hip_check(hipGetLastError(), "plan launch");
}

// ---- multi-GPU: an RCCL communicator owned by the library, and the sharded plan as
// one call with the all-gather as a stream-ordered step.
//
// RCCL is resolved at run time, on the first mbrl_comm_* / sharded call (dlopen of librccl.so.1, the
// soname torch.distributed loads, so both share one RCCL in the process): the single-GPU library has
// no link-time dependency on RCCL and loads on a host without it.
struct Rccl {
    const char* (*get_error_string)(ncclResult_t);
    ncclResult_t (*get_unique_id)(ncclUniqueId*);
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*comm_destroy)(ncclComm_t);
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*group_start)();
    ncclResult_t (*group_end)();
    std::string error;   // why the library could not be loaded ("" when it was)
};

static const Rccl& rccl() {
    static Rccl r{};
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            r.error = e ? e : "dlopen(librccl.so.1) failed";
            return;
        }
        auto sym = [&](const char* name) {
            void* p = dlsym(h, name);
            if (!p && r.error.empty()) r.error = std::string("librccl: missing symbol ") + name;
            return p;
        };
        r.get_error_string = reinterpret_cast<decltype(r.get_error_string)>(sym("ncclGetErrorString"));
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(sym("ncclAllGather"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    });
    return r;
}

static int rccl_ready() {
    const Rccl& r = rccl();
    return r.error.empty() ? MBRL_OK : fail(MBRL_EUNSUPPORTED, "RCCL unavailable: %s", r.error.c_str());
}

static int nccl_check(ncclResult_t res, const char* what) {
    if (res == ncclSuccess) return MBRL_OK;
    return fail(MBRL_EHIP, "%s: %s", what, rccl().get_error_string(res));
}

int mbrl_comm_unique_id(void* id_out) {
    static_assert(sizeof(ncclUniqueId) == MBRL_COMM_ID_BYTES, "ncclUniqueId size");
    if (!id_out) return fail(MBRL_EINVAL, "comm_unique_id: NULL");
    if (int rc = rccl_ready()) return rc;
    ncclUniqueId id;
    if (int rc = nccl_check(rccl().get_unique_id(&id), "ncclGetUniqueId")) return rc;
    memcpy(id_out, &id, sizeof(id));
    return MBRL_OK;
}

int mbrl_comm_init(const void* id, int32_t nranks, int32_t rank, mbrl_comm_t* comm_out) {
    if (!id || !comm_out || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(MBRL_EINVAL, "comm_init: bad arguments (nranks %d, rank %d)", nranks, rank);
    if (int rc = rccl_ready()) return rc;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    if (int rc = nccl_check(rccl().comm_init_rank(&c, nranks, u, rank), "ncclCommInitRank")) return rc;
    *comm_out = reinterpret_cast<mbrl_comm_t>(c);
    return MBRL_OK;
}

int mbrl_comm_destroy(mbrl_comm_t comm) {
    if (!comm) return MBRL_OK;
    if (int rc = rccl_ready()) return rc;
    return nccl_check(rccl().comm_destroy(reinterpret_cast<ncclComm_t>(comm)), "ncclCommDestroy");
}

// MBRL_OPT_SHARD_EMULATE 2 (timing): the all-gather's rank-major buffer in one launch -- this rank's
// slot from its own costs, every other slot from the costs a mode-1 plan kept for this iteration --
// and the gathered status words (this rank's own, the others clear).
__global__ void emu_gather_kernel(const float* __restrict__ local, const float* __restrict__ kept, int G, int rank,
                                  size_t slot, const unsigned* __restrict__ own_status,
                                  const unsigned* __restrict__ own_pair, float* __restrict__ gathered,
                                  unsigned* __restrict__ peer) {
    const size_t total = (size_t)G * slot, lo = (size_t)rank * slot;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
        gathered[i] = (i >= lo && i < lo + slot) ? local[i - lo] : kept[i];
#ifdef MBRL_STAMPS
    if (threadIdx.x == 0 && g_cem_wg_stamps)   // (diagnostic) a workgroup's end, last writer wins
        g_cem_wg_stamps[8 * 2 * 1024 * 4 - 1] = __builtin_amdgcn_s_memrealtime();
#endif
    if (blockIdx.x == 0)
        for (int r = threadIdx.x; r < G; r += blockDim.x) {
            peer[r] = r == rank ? *own_status : 0u;
            peer[G + r] = (r == rank && own_pair) ? *own_pair : 0u;
        }
}

struct ShardWs {
    float *local, *gathered, *costs, *actions, *mu[2], *sigma[2], *aelite, *states, *s0;
    float* emu_actions;   // MBRL_OPT_SHARD_EMULATE 1: the other ranks' proposals, one shard at a time (taken
                          // in mode 2 as well, so both modes place emu_kept alike)
    float* emu_kept;      // MBRL_OPT_SHARD_EMULATE: [I][G][E][Nl] every iteration's gathered costs (mode 1
                          // writes them, mode 2 reads the other ranks' slots back)
    unsigned* peer;       // [2G] the ranks' status words, then their pair status words, gathered with the
                          // last iteration's costs
    void* pair;
    unsigned long long* xchg;
    unsigned* status;
    size_t xchg_bytes;
    int64_t* elites;
    uint32_t* keys;
    size_t bytes;
};

static int shard_emulation() { return g_opt[MBRL_OPT_SHARD_EMULATE].load(std::memory_order_relaxed); }

static ShardWs shard_ws(const Geometry& g, const mbrl_cem_params* p, int G, void* base) {
    ShardWs w{};
    char* b = static_cast<char*>(base);
    size_t o = 0;
    auto take = [&](size_t n) { void* r = b ? b + o : nullptr; o += align256(n); return r; };
    const int Nl = p->N / G;
    const size_t Ha = (size_t)p->H * g.a;
    w.xchg_bytes = (size_t)g.E * 2 * g.Wpad * 8;
    w.xchg = (unsigned long long*)take(w.xchg_bytes);   // the trajectory hand-off block, status right behind
    w.status = (unsigned*)take(16);
    w.local = (float*)take((size_t)g.E * Nl * 4);
    w.gathered = (float*)take((size_t)g.E * p->N * 4);
    w.costs = (float*)take((size_t)g.E * p->N * 4);
    w.actions = (float*)take((size_t)p->H * Nl * g.a * 4);
    w.mu[0] = (float*)take(Ha * 4); w.mu[1] = (float*)take(Ha * 4);
    w.sigma[0] = (float*)take(Ha * 4); w.sigma[1] = (float*)take(Ha * 4);
    w.aelite = (float*)take((size_t)p->H * p->K * g.a * 4);
    w.states = (float*)take((size_t)g.E * p->H * g.s * 4);
    w.elites = (int64_t*)take((size_t)p->K * 8);
    w.keys = (uint32_t*)take((size_t)p->N * 4);
    w.s0 = (float*)take((size_t)g.s * 4);
    w.pair = take(pair_area_bytes(g, Nl));
    w.peer = (unsigned*)take((size_t)2 * G * 4);
    const int emu = shard_emulation();
    w.emu_actions = (float*)take(emu != 0 && G > 1 ? (size_t)p->H * Nl * g.a * 4 : 0);
    w.emu_kept = (float*)take(emu != 0 && G > 1 ? (size_t)p->iterations * g.E * p->N * 4 : 0);
    w.bytes = o;
    return w;
}

size_t mbrl_cem_plan_sharded_workspace_bytes(const mbrl_mlp_shape* shape, const mbrl_cem_params* params,
                                             int32_t nranks) {
    Geometry g;
    if (shape_geometry(shape, &g) != MBRL_OK || !params || nranks < 1 || params->N % nranks) return 0;
    return shard_ws(g, params, nranks, nullptr).bytes;
}

// The body of mbrl_cem_plan_sharded. Every check that can reject the call runs before the first
// collective, and each is a function of arguments every rank passes alike (shape, params, nranks,
// the workspace size the same query gives), so the ranks agree on it; what can still fail later is a
// HIP launch, and then the rank keeps its place in every remaining all-gather (below).
static int plan_sharded_body(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm,
                             const mbrl_cost* cost, const float* s0_in, const mbrl_cem_params* p, mbrl_comm_t comm,
                             int32_t nranks, int32_t rank, float* mu, float* sigma, float* actions_out,
                             float* states_out, float* cost_hist, float* returns_hist, int64_t* elite_hist,
                             mbrl_event_t* rollout_events, void* workspace, size_t ws_bytes, hipStream_t stream,
                             bool allow_pairs = true) {
    Geometry g;
    int rc = shape_geometry(shape, &g);
    if (rc) return rc;
    // comm == NULL with MBRL_OPT_SHARD_EMULATE (tests, timing): this call fills the rank-major buffer the
    // all-gather would have delivered itself (mode 1: every other rank's shard rolled out here; mode 2:
    // the other ranks' costs a mode-1 plan kept)
    const int emu_mode = comm == nullptr ? shard_emulation() : 0;
    const bool emulate = emu_mode != 0;
    if (!p || (!comm && !emulate)) return fail(MBRL_EINVAL, "plan_sharded: NULL params or comm");
    if (p->N < 1 || p->H < 1 || p->K < 1 || p->K > p->N || p->iterations < 1)
        return fail(MBRL_EINVAL, "bad CEM params N=%d H=%d K=%d I=%d", p->N, p->H, p->K, p->iterations);
    if (nranks < 1 || rank < 0 || rank >= nranks || p->N % nranks)
        return fail(MBRL_EINVAL, "plan_sharded: N=%d over %d ranks (rank %d)", p->N, nranks, rank);
    if (!actions_out || !states_out || !workspace || !s0_in || !packed)
        return fail(MBRL_EINVAL, "plan_sharded: packed/s0/actions_out/states_out/workspace NULL");
    const ShardWs w = shard_ws(g, p, nranks, workspace);
    if (ws_bytes < w.bytes) return fail(MBRL_EWORKSPACE, "workspace %zu < %zu", ws_bytes, w.bytes);
    if (emulate && nranks > 1 && !w.emu_kept)
        return fail(MBRL_EINVAL, "plan_sharded: the workspace was sized without MBRL_OPT_SHARD_EMULATE");
    if ((rc = pair_forced_check(g, p->N / nranks))) return rc;
    if ((rc = rollout_validate(g, norm, cost))) return rc;
    if (!emulate && (rc = rccl_ready())) return rc;
    const int N = p->N, Nl = N / nranks, H = p->H, a = g.a, E = g.E;
    const int off = rank * Nl;   // this rank's global candidates [off, off + Nl)
    const size_t slot = (size_t)E * Nl;   // one rank's floats in the gathered buffer
    const bool fuse = update_kpt(N, p->K, a) != 0 && g_opt[MBRL_OPT_UNFUSED_UPDATE].load(std::memory_order_relaxed) == 0;
    const bool fuse_draw = fuse && update_samples(Nl, a);
    // injected failure (tests): iteration fail_it on rank fail_rank (the calling rank unless one is named)
    const int fail_it = g_opt[MBRL_OPT_DEBUG_SHARD_FAIL].load(std::memory_order_relaxed) - 1;
    const int fail_opt = g_opt[MBRL_OPT_DEBUG_SHARD_FAIL_RANK].load(std::memory_order_relaxed);
    const int fail_rank = fail_opt == 0 ? rank : fail_opt - 1;
    // From here on the ranks must issue the same collectives: a launch that fails on this rank does not
    // end the call. Its remaining compute launches are skipped, but it still joins every remaining
    // all-gather -- with its local costs poisoned to NaN (all bits set) and its status word set, which
    // the last iteration's all-gather hands to every peer -- and the first error is returned at the
    // end. (An abort of the communicator would not help: ncclCommAbort acts on the calling rank only,
    // and peers already inside an all-gather would wait on it.)
    int err = MBRL_OK;
    std::string err_msg;
    auto step = [&](int r) {
        if (r != MBRL_OK && err == MBRL_OK) {
            err = r;
            err_msg = g_err;
        }
        return err == MBRL_OK;
    };
    unsigned* own_status = w.status + 1;   // [0] is the trajectory kernel's; zeroed with it below
    unsigned* zero_word = w.status + 2;    // stays 0: the pair status gathered when no pair launch ran
    // With peers the plan checks its column-split pair launches once, after the plan (the pair status
    // word, gathered with the last iteration's costs): any hand-off that timed out on any rank sends
    // every rank through the whole plan again without pairs. No gated redo launch per iteration.
    void* const pair_ws = allow_pairs ? w.pair : nullptr;
    const unsigned* pair_status = nullptr;
    const unsigned** const defer = nranks > 1 ? &pair_status : nullptr;
    // one first launch: distribution rows, the workspace copy of s0, iteration 0's proposals of this
    // shard (global candidates [off, off + Nl)), the hand-off words and this rank's status zeroed
    const InitZero z = plan_zero(g, Nl, w.pair, w.xchg, w.xchg_bytes, w.status);
    if (!z.ptr[1]) step(hip_check(hipMemsetAsync(own_status, 0, 2 * sizeof(unsigned), stream), "status memset"));
    hipLaunchKernelGGL(cem_init_kernel, dim3(H * (fuse_draw ? draw_slices(H, 1, Nl, a) : 1), 1), dim3(1024), 0, stream,
                       p->seed, p->init_mu, p->init_sigma, p->lo, p->hi, H, a, Nl, w.mu[0], w.sigma[0],
                       fuse_draw ? w.actions : nullptr, s0_in, g.s, w.s0, off, z);
    step(hip_check(hipGetLastError(), "init launch"));
    if (!fuse_draw && err == MBRL_OK) {
        mbrl_sampler sp0{};
        sp0.seed = p->seed; sp0.iteration = 0; sp0.mu = w.mu[0]; sp0.sigma = w.sigma[0]; sp0.lo = p->lo; sp0.hi = p->hi;
        step(sample_impl(&sp0, H, a, Nl, off, w.actions, stream));
    }
    bool poisoned = false;   // this rank's local costs and status word carry its failure
    unsigned pair_epoch = 0;
    int cur = 0;
    for (int it = 0; it < p->iterations; ++it) {
        const bool last = it + 1 == p->iterations;
        mbrl_sampler sp{};
        sp.seed = p->seed; sp.iteration = it; sp.mu = w.mu[cur]; sp.sigma = w.sigma[cur]; sp.lo = p->lo; sp.hi = p->hi;
        if (err == MBRL_OK && rollout_events && rollout_events[2 * it])
            step(hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(rollout_events[2 * it]), stream), "event"));
        if (err == MBRL_OK)
            step(rollout_impl(g, packed, norm, cost, w.s0, 0, w.actions, nullptr, Nl, H, 0, w.local, nullptr, nullptr,
                              stream, pair_area_bytes(g, Nl) ? pair_ws : nullptr, z.ptr[0] ? &pair_epoch : nullptr,
                              defer));
        if (err == MBRL_OK && it == fail_it && fail_rank == rank)
            step(fail(MBRL_EHIP, "plan_sharded: injected launch failure at iteration %d (MBRL_OPT_DEBUG_SHARD_FAIL)", it));
        if (err == MBRL_OK && rollout_events && rollout_events[2 * it + 1])
            step(hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(rollout_events[2 * it + 1]), stream), "event"));
        if (err != MBRL_OK && !poisoned) {
            // NaN costs sort last on every rank (MBRL_NAN_LAST); the status word tells the peers. If even
            // these fail the rank still joins the collectives (and returns its first error).
            poisoned = true;
            const int m1 = hip_check(hipMemsetAsync(w.local, 0xFF, slot * 4, stream), "poison memset");
            const int m2 = hip_check(hipMemsetAsync(own_status, 0x01, sizeof(unsigned), stream), "status memset");
            if (m1 || m2) err_msg += std::string("; then ") + g_err;
        }
        // the one collective of an iteration: every rank's [E][Nl] costs, rank-major; the last one also
        // gathers the ranks' status words (grouped: one RCCL launch)
        if (!emulate) {
            const Rccl& R = rccl();
            ncclComm_t c = reinterpret_cast<ncclComm_t>(comm);
            if (last) step(nccl_check(R.group_start(), "ncclGroupStart"));
            step(nccl_check(R.all_gather(w.local, w.gathered, slot, ncclFloat, c, stream), "ncclAllGather"));
            if (last) {
                step(nccl_check(R.all_gather(own_status, w.peer, 1, ncclUint32, c, stream), "ncclAllGather status"));
                step(nccl_check(R.all_gather(pair_status ? pair_status : zero_word, w.peer + nranks, 1, ncclUint32, c,
                                             stream), "ncclAllGather pair status"));
                step(nccl_check(R.group_end(), "ncclGroupEnd"));
            }
        } else if (err == MBRL_OK && nranks == 1) {
            step(hip_check(hipMemcpyAsync(w.gathered, w.local, slot * 4, hipMemcpyDeviceToDevice, stream), "gather"));
            if (last) step(hip_check(hipMemcpyAsync(w.peer, own_status, 4, hipMemcpyDeviceToDevice, stream), "status"));
        } else if (err == MBRL_OK && emu_mode == 2) {
            float* kept = w.emu_kept + (size_t)it * nranks * slot;
            hipLaunchKernelGGL(emu_gather_kernel, dim3(256), dim3(256), 0, stream, w.local, kept, nranks, rank, slot,
                               own_status, pair_status, w.gathered, w.peer);
            step(hip_check(hipGetLastError(), "emulated gather"));
        } else if (err == MBRL_OK) {
            // rank r's slot: its proposals of this iteration (drawn at its global offset from this
            // iteration's mu / sigma, as its own previous update or initial draw made them) rolled out
            for (int r = 0; r < nranks && err == MBRL_OK; ++r) {
                float* sl = w.gathered + (size_t)r * slot;
                if (r == rank) {
                    step(hip_check(hipMemcpyAsync(sl, w.local, slot * 4, hipMemcpyDeviceToDevice, stream),
                                   "emulated gather"));
                } else if (fail_rank == r && fail_it >= 0 && it >= fail_it) {   // an emulated peer's failure
                    step(hip_check(hipMemsetAsync(sl, 0xFF, slot * 4, stream), "emulated peer poison"));
                } else if (step(sample_impl(&sp, H, a, Nl, r * Nl, w.emu_actions, stream))) {
                    step(rollout_impl(g, packed, norm, cost, w.s0, 0, w.emu_actions, nullptr, Nl, H, 0, sl, nullptr,
                                      nullptr, stream, pair_area_bytes(g, Nl) ? pair_ws : nullptr,
                                      z.ptr[0] ? &pair_epoch : nullptr));
                }
            }
            if (last && err == MBRL_OK) {
                step(hip_check(hipMemsetAsync(w.peer, 0, (size_t)2 * nranks * 4, stream), "emulated status"));
                if (fail_rank != rank && fail_rank < nranks && fail_it >= 0)
                    step(hip_check(hipMemsetAsync(w.peer + fail_rank, 0x01, 4, stream), "emulated peer status"));
                step(hip_check(hipMemcpyAsync(w.peer + rank, own_status, 4, hipMemcpyDeviceToDevice, stream),
                               "emulated status"));
                if (pair_status)
                    step(hip_check(hipMemcpyAsync(w.peer + nranks + rank, pair_status, 4, hipMemcpyDeviceToDevice,
                                                  stream), "emulated pair status"));
            }
            if (err == MBRL_OK)   // kept for mode 2
                step(hip_check(hipMemcpyAsync(w.emu_kept + (size_t)it * nranks * slot, w.gathered, nranks * slot * 4,
                                              hipMemcpyDeviceToDevice, stream), "emulated keep"));
        }
        if (err != MBRL_OK) continue;   // only the all-gathers remain for this rank
        float* costs = w.gathered;
        if (E > 1 && nranks > 1) {   // (one rank: the identity)
            hipLaunchKernelGGL(shard_costs_kernel, dim3(256), dim3(256), 0, stream, w.gathered, nranks, E, Nl, w.costs);
            costs = w.costs;
        }
        if (cost_hist)
            step(hip_check(hipMemcpyAsync(cost_hist + (size_t)it * E * N, costs, (size_t)E * N * 4,
                                          hipMemcpyDeviceToDevice, stream), "cost record"));
        int64_t* elites = elite_hist ? elite_hist + (size_t)it * p->K : w.elites;
        float* rets = returns_hist ? returns_hist + (size_t)it * N : nullptr;
        if (err != MBRL_OK) continue;
        if (fuse) {
            UpdateArgs U{};
            U.costs = costs; U.E = E; U.N = N; U.K = p->K; U.member_stride = N; U.H = H; U.a = a;
            U.elite_out = elites; U.returns_out = rets;
            U.seed = p->seed; U.iteration = it; U.mu = w.mu[cur]; U.sigma = w.sigma[cur];
            U.lo = p->lo; U.hi = p->hi; U.alpha = p->alpha; U.oma = 1.0f - p->alpha;
            U.mu_out = w.mu[cur ^ 1]; U.sigma_out = w.sigma[cur ^ 1];
            U.fin_mu = last ? mu : nullptr; U.fin_sigma = last ? sigma : nullptr; U.fin_actions = last ? actions_out : nullptr;
            U.next_actions = (fuse_draw && !last) ? w.actions : nullptr;   // this rank's shard of iteration it + 1
            U.draw_off = off; U.draw_n = Nl;
            U.ael = w.aelite;   // (scratch of the split update)
            step(update_impl(U, 1, stream));
        } else if (step(select_impl(costs, E, N, p->K, MBRL_NAN_LAST, elites, rets, w.keys, align256((size_t)N * 4),
                                    stream))) {
            step(refit_impl(&sp, H, a, elites, p->K, p->alpha, w.aelite, w.mu[cur ^ 1], w.sigma[cur ^ 1], stream,
                            last ? mu : nullptr, last ? sigma : nullptr, last ? actions_out : nullptr));
        }
        cur ^= 1;
        if (!last && !fuse_draw && err == MBRL_OK) {
            mbrl_sampler sn = sp;
            sn.iteration = it + 1; sn.mu = w.mu[cur]; sn.sigma = w.sigma[cur];
            step(sample_impl(&sn, H, a, Nl, off, w.actions, stream));
        }
    }
    if (err != MBRL_OK) return fail(err, "%s (this rank still joined every all-gather of the plan)", err_msg.c_str());
    // the final mean's states, on every rank (the same on each)
    float* per_member = E == 1 ? states_out : w.states;
    rc = traj_impl(g, packed, norm, w.s0, actions_out, H, per_member, w.xchg, w.xchg_bytes, w.status, stream,
                   z.ptr[1] != nullptr);
    if (rc) return rc;
    if (E > 1) {
        const int Hs = H * g.s;
        hipLaunchKernelGGL(member_mean_kernel, dim3((Hs + 255) / 256), dim3(256), 0, stream, w.states, E, Hs,
                           states_out);
    }
    if ((rc = hip_check(hipGetLastError(), "sharded plan launch"))) return rc;
    if (nranks == 1) return MBRL_OK;   // no peers: enqueue only, as mbrl_cem_plan
    // the peers' status and pair status words (gathered with the last iteration's costs): one copy
    // behind the plan's last launch and one stream synchronisation
    static thread_local unsigned* peer_host = nullptr;
    static thread_local int peer_cap = 0;
    if (peer_cap < 2 * nranks) {
        if (peer_host) (void)hipHostFree(peer_host);
        peer_host = nullptr;
        peer_cap = 0;
        if ((rc = hip_check(hipHostMalloc(reinterpret_cast<void**>(&peer_host), (size_t)2 * nranks * 4),
                            "hipHostMalloc")))
            return rc;
        peer_cap = 2 * nranks;
    }
    if ((rc = hip_check(hipMemcpyAsync(peer_host, w.peer, (size_t)2 * nranks * 4, hipMemcpyDeviceToHost, stream),
                        "peer status copy")))
        return rc;
    if ((rc = hip_check(hipStreamSynchronize(stream), "plan synchronise"))) return rc;
    std::string failed;
    bool pair_timeout = false;
    for (int r = 0; r < nranks; ++r) {
        if (peer_host[r] && r != rank) failed += (failed.empty() ? "" : ", ") + std::to_string(r);
        if (peer_host[nranks + r]) pair_timeout = true;
    }
    if (!failed.empty())
        return fail(MBRL_EPEER, "plan_sharded: rank(s) %s failed during this plan (each returns its own error); "
                                "this rank's outputs are void", failed.c_str());
    // a column-split hand-off timed out on some rank (its tile's costs were invalid): every rank sees
    // the same gathered words, so every rank runs the plan again, without pairs (same bits)
    if (pair_timeout && allow_pairs)
        return plan_sharded_body(shape, packed, norm, cost, s0_in, p, comm, nranks, rank, mu, sigma, actions_out,
                                 states_out, cost_hist, returns_hist, elite_hist, rollout_events, workspace, ws_bytes,
                                 stream, false);
    return MBRL_OK;
}

int mbrl_cem_plan_sharded(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm,
                          const mbrl_cost* cost, const float* s0_in, const mbrl_cem_params* p, mbrl_comm_t comm,
                          int32_t nranks, int32_t rank, float* mu, float* sigma, float* actions_out,
                          float* states_out, float* cost_hist, float* returns_hist, int64_t* elite_hist,
                          mbrl_event_t* rollout_events, void* workspace, size_t ws_bytes, mbrl_stream_t stream) {
    return plan_sharded_body(shape, packed, norm, cost, s0_in, p, comm, nranks, rank, mu, sigma, actions_out,
                             states_out, cost_hist, returns_hist, elite_hist, rollout_events, workspace, ws_bytes,
                             reinterpret_cast<hipStream_t>(stream));
}

#ifdef MBRL_STAMPS
int mbrl_diag_set_cem_stamps(void* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mbrl::g_cem_stamps), &buf, sizeof(buf));
}
int mbrl_diag_set_cem_wg_stamps(void* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mbrl::g_cem_wg_stamps), &buf, sizeof(buf));
}
#endif

// ---- batched planning: B independent CEM plans (one initial state each) in shared launches.
struct BatchWs {
    float *costs, *actions, *mu[2], *sigma[2], *s0x, *states;
    unsigned long long* xchg;
    unsigned* status;
    size_t xchg_bytes;
    int64_t* elites;
    uint32_t* keys;
    size_t bytes;
};

static BatchWs batch_ws(const Geometry& g, const mbrl_cem_params* p, int B, void* base) {
    BatchWs w{};
    char* b = static_cast<char*>(base);
    size_t o = 0;
    auto take = [&](size_t n) { void* r = b ? b + o : nullptr; o += align256(n); return r; };
    const size_t BN = (size_t)B * p->N, BHa = (size_t)B * p->H * g.a;
    w.xchg_bytes = (size_t)g.E * 2 * g.Wpad * 8;
    w.xchg = (unsigned long long*)take(w.xchg_bytes);   // memset block first, status right behind (G16)
    w.status = (unsigned*)take(16);
    w.costs = (float*)take((size_t)g.E * BN * 4);
    w.actions = (float*)take((size_t)p->H * BN * g.a * 4);
    w.mu[0] = (float*)take(BHa * 4); w.mu[1] = (float*)take(BHa * 4);
    w.sigma[0] = (float*)take(BHa * 4); w.sigma[1] = (float*)take(BHa * 4);
    w.s0x = (float*)take(BN * g.s * 4);
    w.states = (float*)take((size_t)g.E * p->H * g.s * 4);
    w.elites = (int64_t*)take((size_t)B * p->K * 8);
    w.keys = (uint32_t*)take(BN * 4);
    w.bytes = o;
    return w;
}

size_t mbrl_cem_plan_batch_workspace_bytes(const mbrl_mlp_shape* shape, const mbrl_cem_params* params, int32_t B) {
    Geometry g;
    if (shape_geometry(shape, &g) != MBRL_OK || !params || B < 1) return 0;
    return batch_ws(g, params, B, nullptr).bytes;
}

int mbrl_cem_plan_batch(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const mbrl_cost* cost,
                        const float* s0, int32_t B, const mbrl_cem_params* p, float* mu, float* sigma,
                        float* actions_out, float* states_out, void* workspace, size_t ws_bytes,
                        mbrl_stream_t stream_) {
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    Geometry g;
    int rc = shape_geometry(shape, &g);
    if (rc) return rc;
    if (!p || B < 1) return fail(MBRL_EINVAL, "params NULL or B=%d", B);
    if (p->N < 1 || p->H < 1 || p->K < 1 || p->K > p->N || p->iterations < 1)
        return fail(MBRL_EINVAL, "bad CEM params N=%d H=%d K=%d I=%d", p->N, p->H, p->K, p->iterations);
    if ((int64_t)B * p->N > INT32_MAX / 2) return fail(MBRL_EUNSUPPORTED, "B*N too large");
    if (!s0 || !actions_out || !states_out || !workspace) return fail(MBRL_EINVAL, "s0/actions_out/states_out/workspace NULL");
    BatchWs w = batch_ws(g, p, B, workspace);
    if (ws_bytes < w.bytes) return fail(MBRL_EWORKSPACE, "workspace %zu < %zu", ws_bytes, w.bytes);
    const int BN = B * p->N, BHa = B * p->H * g.a;
    // as mbrl_cem_plan: one fused update launch per iteration where it fits (grid (H, B))
    const bool fuse = update_kpt(p->N, p->K, g.a) != 0 && g_opt[MBRL_OPT_UNFUSED_UPDATE].load(std::memory_order_relaxed) == 0;
    const bool fuse_draw = fuse && update_samples(p->N, g.a);
    if (fuse_draw)
        hipLaunchKernelGGL(cem_init_kernel, dim3(p->H * draw_slices(p->H, B, p->N, g.a), B), dim3(1024), 0, stream,
                           p->seed, p->init_mu, p->init_sigma, p->lo, p->hi, p->H, g.a, p->N, w.mu[0], w.sigma[0],
                           w.actions, nullptr, 0, nullptr, 0, InitZero{});
    else
        hipLaunchKernelGGL(fill2_kernel, dim3((BHa + 255) / 256), dim3(256), 0, stream, w.mu[0], p->init_mu,
                           w.sigma[0], p->init_sigma, BHa);
    hipLaunchKernelGGL(expand_rows_kernel, dim3(256), dim3(256), 0, stream, s0, B, p->N, g.s, w.s0x);
    int cur = 0;
    for (int it = 0; it < p->iterations; ++it) {
        mbrl_sampler sp{};
        sp.seed = p->seed; sp.iteration = it; sp.mu = w.mu[cur]; sp.sigma = w.sigma[cur]; sp.lo = p->lo; sp.hi = p->hi;
        // problem b's candidate n is global candidate b*N + n (its Philox counter)
        if (!fuse_draw) {
            rc = sample_impl(&sp, p->H, g.a, BN, 0, w.actions, stream, p->N);
            if (rc) return rc;
        }
        rc = rollout_impl(g, packed, norm, cost, w.s0x, 1, w.actions, nullptr, BN, p->H, 0, w.costs, nullptr, nullptr,
                          stream);
        if (rc) return rc;
        const bool last = it + 1 == p->iterations;
        if (fuse) {
            UpdateArgs U{};
            U.costs = w.costs; U.E = g.E; U.N = p->N; U.K = p->K; U.member_stride = BN; U.H = p->H; U.a = g.a;
            U.seed = p->seed; U.iteration = it; U.mu = w.mu[cur]; U.sigma = w.sigma[cur];
            U.lo = p->lo; U.hi = p->hi; U.alpha = p->alpha; U.oma = 1.0f - p->alpha;
            U.mu_out = w.mu[cur ^ 1]; U.sigma_out = w.sigma[cur ^ 1];
            U.fin_mu = last ? mu : nullptr; U.fin_sigma = last ? sigma : nullptr; U.fin_actions = last ? actions_out : nullptr;
            U.next_actions = (fuse_draw && !last) ? w.actions : nullptr;
            U.draw_off = 0; U.draw_n = p->N;
            rc = update_impl(U, B, stream);
        } else {
            rc = select_impl(w.costs, g.E, p->N, p->K, MBRL_NAN_LAST, w.elites, nullptr, w.keys,
                             align256((size_t)BN * 4), stream, B);
            if (rc) return rc;
            rc = refit_impl(&sp, p->H, g.a, w.elites, p->K, p->alpha, nullptr, w.mu[cur ^ 1], w.sigma[cur ^ 1], stream,
                            last ? mu : nullptr, last ? sigma : nullptr, last ? actions_out : nullptr, B, p->N);
        }
        if (rc) return rc;
        cur ^= 1;
    }
    const int Hs = p->H * g.s;
    for (int b = 0; b < B; ++b) {   // each final mean's states (the cooperative trajectory kernel)
        float* per_member = g.E == 1 ? states_out + (size_t)b * Hs : w.states;
        rc = traj_impl(g, packed, norm, s0 + (size_t)b * g.s, actions_out + (size_t)b * p->H * g.a, p->H, per_member,
                       w.xchg, w.xchg_bytes, w.status, stream);
        if (rc) return rc;
        if (g.E > 1)
            hipLaunchKernelGGL(member_mean_kernel, dim3((Hs + 255) / 256), dim3(256), 0, stream, w.states, g.E, Hs,
                               states_out + (size_t)b * Hs);
    }
    return hip_check(hipGetLastError(), "batched plan launch");
}


// ---- fused gradient-descent planner (gd.hip)
// Workspace of B gradient-descent plans: the hand-off blocks of every plan first (2 Wpad granules,
// then the status word; one memset clears them all), then per plan its Adam moments and saved
// hidden vectors, plan_ws bytes apart.
struct GdWs {
    float *m, *v, *hist;
    unsigned long long* xchg;
    unsigned* status;
    size_t xchg_stride, plan_ws, bytes;
};

static GdWs gd_ws(const Geometry& g, int H, int B, void* base) {
    GdWs w{};
    char* b = static_cast<char*>(base);
    const size_t ha = (size_t)H * g.a;
    const size_t row = ((size_t)((g.s + g.a + 3) & ~3) + (size_t)g.L * g.Wpad) * (g.reward ? 2 : 1);
    // (the cooperative kernel keeps its ReLU masks in LDS; the saved layer inputs are the one-workgroup
    // kernel's)
    w.xchg_stride = (size_t)2 * g.Wpad + 2;                                  // granules, then the status word
    const size_t xbytes = align256((size_t)B * w.xchg_stride * 8);
    w.plan_ws = align256(ha * 4) * 2 + align256(H * row * 4);
    w.xchg = b ? reinterpret_cast<unsigned long long*>(b) : nullptr;
    w.status = w.xchg ? reinterpret_cast<unsigned*>(w.xchg + 2 * g.Wpad) : nullptr;
    w.m = b ? reinterpret_cast<float*>(b + xbytes) : nullptr;
    w.v = b ? reinterpret_cast<float*>(b + xbytes + align256(ha * 4)) : nullptr;
    w.hist = b ? reinterpret_cast<float*>(b + xbytes + 2 * align256(ha * 4)) : nullptr;
    w.bytes = xbytes + (size_t)B * w.plan_ws;
    return w;
}

size_t mbrl_gd_workspace_bytes(const mbrl_mlp_shape* shape, int32_t H) { return mbrl_gd_batch_workspace_bytes(shape, H, 1); }

size_t mbrl_gd_batch_workspace_bytes(const mbrl_mlp_shape* shape, int32_t H, int32_t B) {
    Geometry g;
    if (shape_geometry(shape, &g) != MBRL_OK || H < 1 || B < 1) return 0;
    return gd_ws(g, H, B, nullptr).bytes;
}

int mbrl_gd_plan(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const mbrl_cost* cost,
                 const float* s0, float* actions, int32_t H, int32_t num_iterations, float stop_condition, float lr,
                 float* states_out, int32_t* iterations_out, void* workspace, size_t ws_bytes, mbrl_stream_t stream) {
    return mbrl_gd_plan_batch(shape, packed, norm, cost, s0, actions, 1, H, num_iterations, stop_condition, lr,
                              states_out, iterations_out, workspace, ws_bytes, stream);
}

int mbrl_gd_plan_batch(const mbrl_mlp_shape* shape, const void* packed, const mbrl_norm* norm, const mbrl_cost* cost,
                       const float* s0, float* actions, int32_t B, int32_t H, int32_t num_iterations,
                       float stop_condition, float lr, float* states_out, int32_t* iterations_out, void* workspace,
                       size_t ws_bytes, mbrl_stream_t stream) {
    Geometry g;
    int rc = shape_geometry(shape, &g);
    if (rc) return rc;
    if (g.E != 1) return fail(MBRL_EUNSUPPORTED, "gd_plan: needs ensemble == 1");
    if (!cost || cost->kind != (g.reward ? MBRL_COST_MODEL_REWARD : MBRL_COST_GOAL_STATE))
        return fail(MBRL_EUNSUPPORTED, "gd_plan: needs a GOAL_STATE cost, or MODEL_REWARD with a reward-head model");
    if (!packed || !s0 || !actions || !states_out || !workspace) return fail(MBRL_EINVAL, "gd_plan: NULL argument");
    if (H < 1 || num_iterations < 0 || B < 1)
        return fail(MBRL_EINVAL, "gd_plan: H=%d iterations=%d B=%d", H, num_iterations, B);
    if (gd_lds_bytes(g.s, g.a, g.Wpad, H) > 160 * 1024) return fail(MBRL_EUNSUPPORTED, "gd_plan: H * a too large");
    if (!g.reward && cost->has_state_cost && (!cost->weights || !cost->goal))
        return fail(MBRL_EINVAL, "gd_plan: state cost without weights/goal");
    GdArgs A{};
    const GdWs w = gd_ws(g, H, B, workspace);
    if (ws_bytes < w.bytes) return fail(MBRL_EWORKSPACE, "gd workspace %zu < %zu", ws_bytes, w.bytes);
    A.packed = static_cast<const float*>(packed);
    A.bias_off = g.stream_floats;
    A.tw_base = g.stream_floats + g.bias_floats;
    for (int l = 0; l <= g.L; ++l) A.tw_off[l] = g.tw_off[l];
    A.s = g.s; A.a = g.a; A.W = g.W; A.Wpad = g.Wpad; A.L = g.L; A.H = H;
    if (norm) {
        A.obs_mean = norm->obs_mean; A.obs_std = norm->obs_std;
        A.act_mean = norm->act_mean; A.act_std = norm->act_std;
        A.norm_s = norm->normalize_state; A.unnorm_s = norm->unnormalize_state; A.norm_a = norm->normalize_action;
        if ((A.norm_s || A.unnorm_s) && (!A.obs_mean || !A.obs_std))
            return fail(MBRL_EINVAL, "state normalisation requested without obs_mean/obs_std");
        if (A.norm_a && (!A.act_mean || !A.act_std))
            return fail(MBRL_EINVAL, "action normalisation requested without act_mean/act_std");
        A.unnorm_r = g.reward ? norm->unnormalize_reward : 0;
        A.rew_std = norm->rew_std;
        if (A.unnorm_r && !A.rew_std) return fail(MBRL_EINVAL, "reward unnormalisation requested without rew_std");
    }
    A.reward = g.reward;
    if (!g.reward) {
        A.cw = cost->weights; A.goal = cost->goal;
        A.alpha_s = cost->alpha_state; A.alpha_a = cost->alpha_action;
        A.has_sc = cost->has_state_cost; A.has_ac = cost->has_action_cost;
    }
    A.hist_row = (((g.s + g.a + 3) & ~3) + g.L * g.Wpad) * (g.reward ? 2 : 1);
    A.iterations = num_iterations; A.stop = stop_condition; A.lr = lr;
    A.plan_ws = w.plan_ws;
    A.xchg_stride = w.xchg_stride;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // MBRL_OPT_GD_SINGLE (A/B and tests): the one-workgroup kernel
    const bool coop = gd_coop_supported(A) && g_opt[MBRL_OPT_GD_SINGLE].load(std::memory_order_relaxed) == 0;
    // plans run in groups whose cooperative grids fit the device together (Wpad / 16 workgroups each)
    int group = B;
    for (int i = 0; i < B; i += group) {
        const int n = std::min(group, B - i);
        A.batch = n;
        A.s0 = s0 + (size_t)i * g.s;
        A.actions = actions + (size_t)i * H * g.a;
        A.states_out = states_out + (size_t)i * (H + 1) * g.s;
        A.iterations_out = iterations_out ? iterations_out + i : nullptr;
        A.m = reinterpret_cast<float*>(reinterpret_cast<char*>(w.m) + i * w.plan_ws);
        A.v = reinterpret_cast<float*>(reinterpret_cast<char*>(w.v) + i * w.plan_ws);
        A.hist = reinterpret_cast<float*>(reinterpret_cast<char*>(w.hist) + i * w.plan_ws);
        unsigned long long* xchg = w.xchg + (size_t)i * w.xchg_stride;
        unsigned* status = reinterpret_cast<unsigned*>(xchg + 2 * g.Wpad);
        A.gate = nullptr;
        if (coop) {
            A.debug_abort = g_opt[MBRL_OPT_DEBUG_GD_ABORT].load(std::memory_order_relaxed) != 0;
            const int hop = g_opt[MBRL_OPT_GD_HOP].load(std::memory_order_relaxed);
            A.hop_mode = hop == 0 ? kTrajHopDefault : hop - 1;
            const hipError_t err = launch_gd_coop(A, xchg, status, st);
            if (err == hipErrorCooperativeLaunchTooLarge && n > 1) {   // fewer plans per group, same start
                group = std::max(1, n / 2);
                i -= group;
                continue;
            }
            if (err != hipErrorCooperativeLaunchTooLarge) {   // too large for even one plan: one workgroup each
                rc = hip_check(err, "gd_plan coop launch");
                if (rc) return rc;
                // the one-workgroup kernel redoes a plan only if its cooperative hand-offs timed out
                A.gate = status;
            }
            A.debug_abort = 0;
        }
        if ((rc = hip_check(launch_gd_plan(A, st), "gd_plan launch"))) return rc;
    }
    return MBRL_OK;
}

}  // extern "C"
