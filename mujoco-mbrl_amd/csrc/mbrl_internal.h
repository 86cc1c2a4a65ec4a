// Internal kernel-argument structs and the geometry shared by the pack kernels, the rollout kernel
// and the host launcher. Not part of the public ABI (include/mbrl_cem.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include "../../include/mbrl_cem.h"

namespace mbrl {

constexpr int MAX_LAYERS = 4;  // hidden layers

// Packed-stream geometry for one MLP shape (DESIGN.md §2 "weight stream").
struct Geometry {
    int s, a, W, L, E;
    int reward;     // 1: reward head (output rows = s + 1)
    int so;         // output rows: s + reward
    int T;          // 16-column tiles per wave per hidden layer; Wpad = 64 * T
    int Wpad;
    int K0C;        // layer-0 K chunks of 16 (even)
    int NOT;        // output tiles of 16 (even), covering so rows
    int C;          // chunks per step = K0C + (L-1)*4T + NOT
    int lda;        // LDS activation row stride (floats)
    int pw;         // LDS output-partial row stride (floats)
    size_t stream_floats;  // C * 1024 * T
    size_t bias_floats;    // L * Wpad + 16 * NOT
    // plain copies for the single-trajectory kernel (traj.hip): layer 0 and hidden layers
    // transposed W^T [in][Wpad]; the output layer row-major [so][W] (state rows, then reward)
    int Opad;
    size_t tw_off[MAX_LAYERS + 1];  // offsets inside the plain region
    size_t tw_floats;
    // F16X3 split stream (rollout_f16x3.hip): 32-deep K chunks of f16 (hi, lo) fragment pairs,
    // 8 waves x T fragments of 1 KiB per chunk. Present when split_ok (256 <= Wpad <= 512).
    int split_ok;
    int precision;         // requested MBRL_PRECISION_* (set by the ABI layer, not by make_geometry)
    int K0S;               // layer-0 chunks of 32 (K0S + NOS even)
    int NOS;               // output chunks (pairs of 16-row output tiles) = NOT / 2
    int CS;                // split chunks per step = K0S + (L-1)*2T + NOS
    size_t split_off;      // floats from the member base: the 2-piece stream (F16X3)
    size_t split_floats;   // CS * 2048 * T, then one flag word (nonzero: a weight is out of split range)
    size_t split3_off;     // the 3-piece stream (F16X6): CS * 3072 * T floats, then its flag word
    size_t split3_floats;
    // 8-candidate fp32 stream (rollout.hip rollout_m8_kernel): 16-deep chunks, T waves x 4 KiB each;
    // K0C + (L-1)*4T + NOC8 chunks per step. Present when m8_ok (Wpad 256 or 512, no reward head,
    // the ring shapes K0C, NOT in {2, 6}).
    int m8_ok;
    int NOP8;              // pairs of 32-row output tiles
    int NOC8;              // output chunks per step
    int C8;                // chunks per step
    size_t m8_off;         // floats from the member base (0: absent)
    size_t m8_floats;      // C8 * 1024 * T
    // 4-candidate fp32 stream (rollout.hip rollout_m4_kernel): layer-0 and hidden chunks in the m8
    // layout without KP pairing (wave w: row 64 w + 32 ((l >> 2) & 1) + 4 (l >> 3) + (l & 3)), then 4
    // output chunks, one per 16-feature chunk kc of the wave's own 64: float4 s = output group g,
    // element q = W[16 g + 4 (l >> 4) + (l & 3)][64 w + 16 kc + 4 q + ((l >> 2) & 3)]. Present when
    // m4_ok (m8_ok and s <= 64: NG4 <= 4 groups of 16 output rows).
    int m4_ok;
    int NG4;               // output row groups of 16
    int C4;                // chunks per step = K0C + (L-1)*4T + 4
    size_t m4_off;
    size_t m4_floats;      // C4 * 1024 * T
    size_t member_stride;  // floats per ensemble member (64-float aligned)
};

inline int round_even(int x) { return (x + 1) & ~1; }

inline bool make_geometry(int s, int a, int W, int L, int E, int reward, Geometry* g) {
    if (s < 1 || a < 1 || W < 1 || L < 1 || L > MAX_LAYERS || E < 1 || reward < 0 || reward > 1) return false;
    int T = 1;
    while (64 * T < W) T *= 2;
    if (T > 16) return false;
    g->s = s; g->a = a; g->W = W; g->L = L; g->E = E;
    g->reward = reward;
    g->so = s + reward;
    g->T = T;
    g->Wpad = 64 * T;
    g->K0C = round_even((s + a + 15) / 16);
    g->NOT = round_even((g->so + 15) / 16);
    if (g->NOT > 2 * 4 * T * 4) return false;
    g->C = g->K0C + (L - 1) * 4 * T + g->NOT;
    const int k0 = 16 * g->K0C;
    g->lda = (g->Wpad > k0 ? g->Wpad : k0) + 4;
    g->pw = 16 * g->NOT + 4;
    g->stream_floats = (size_t)g->C * 1024 * T;
    g->bias_floats = (size_t)L * g->Wpad + 16 * (size_t)g->NOT;
    g->Opad = (g->so + 3) & ~3;
    size_t o = 0;
    g->tw_off[0] = o;
    o += (size_t)(s + a) * g->Wpad;
    for (int l = 1; l < L; ++l) { g->tw_off[l] = o; o += (size_t)W * g->Wpad; }
    g->tw_off[L] = o;
    o += (size_t)g->so * W;
    g->tw_floats = o;
    size_t end = g->stream_floats + g->bias_floats + g->tw_floats;
    g->split_ok = (T == 4 || T == 8) ? 1 : 0;
    g->precision = 0;
    g->K0S = (s + a + 31) / 32;
    g->NOS = g->NOT / 2;
    if ((g->K0S + g->NOS) & 1) g->K0S += 1;   // every step then starts on the same ring phase pair
    g->CS = g->K0S + (L - 1) * 2 * T + g->NOS;
    g->split_off = (end + 63) / 64 * 64;
    g->split_floats = g->split_ok ? (size_t)g->CS * 2048 * T + 64 : 0;
    g->split3_off = g->split_off + g->split_floats;
    g->split3_floats = g->split_ok ? (size_t)g->CS * 3072 * T + 64 : 0;
    if (g->split_ok) end = g->split3_off + g->split3_floats;
    g->m8_ok = ((T == 4 || T == 8) && !reward && (g->K0C == 2 || g->K0C == 6) && (g->NOT == 2 || g->NOT == 6)) ? 1 : 0;
    g->NOP8 = (g->NOT / 2 + 1) / 2;
    g->NOC8 = g->NOT == 2 ? 2 : 4 * g->NOP8;   // one 32-row output tile: K-chunk pairs (rollout_m8_kernel)
    g->C8 = g->K0C + (L - 1) * 4 * T + g->NOC8;
    g->m8_off = g->m8_ok ? (end + 63) / 64 * 64 : 0;
    g->m8_floats = g->m8_ok ? (size_t)g->C8 * 1024 * T : 0;
    if (g->m8_ok) end = g->m8_off + g->m8_floats;
    g->NG4 = (g->so + 15) / 16;
    g->m4_ok = (g->m8_ok && g->NG4 <= 4) ? 1 : 0;
    g->C4 = g->K0C + (L - 1) * 4 * T + 4;
    g->m4_off = g->m4_ok ? (end + 63) / 64 * 64 : 0;
    g->m4_floats = g->m4_ok ? (size_t)g->C4 * 1024 * T : 0;
    if (g->m4_ok) end = g->m4_off + g->m4_floats;
    g->member_stride = (end + 63) / 64 * 64;
    return true;
}

struct RolloutArgs {
    const float* packed;
    size_t member_stride;
    size_t stream_floats;
    int s, a, L, Wpad, K0C, NOT, E, chunks_per_step, lda, pw, k0pad_extra;
    int nw;  // waves per workgroup (set by the launcher; sizes the output partials)
    int N, H, n_offset;
    const float *obs_mean, *obs_std, *act_mean, *act_std;
    int norm_s, unnorm_s, norm_a;
    int reward;                        // cost = unnormalised reward head at (s_{t+1}, a_t), 2 passes/step
    int unnorm_r;
    const float *rew_mean, *rew_std;   // [1] each (device), read once in the prologue
    const float *cw, *goal;
    float alpha_s, alpha_s2, alpha_a, alpha_a2;
    int has_sc, has_ac;
    const float* s0;
    int s0_per_cand;
    const float* actions;  // [H][N][a] (given, or drawn by the proposal kernel just before)
    float* costs;
    float* actions_out;
    float* states_out;
    // F16X3 / F16X6 (rollout_f16x3.hip) and the F32 redo pass
    size_t split_off;
    int K0S, CS, sr;       // sr: LDS activation row stride in halves
    int redo;              // F32 kernel: only workgroups whose candidates carry MBRL_REDO_MARK run
    // 8-candidate kernel (rollout_m8_kernel)
    size_t m8_off;         // 0: no 8-candidate stream in the pack
    int C8;
    // 4-candidate kernel (rollout_m4_kernel)
    size_t m4_off;         // 0: no 4-candidate stream in the pack
    int C4;
    // 16-candidate kernel, L odd >= 3, no reward head: the output partials live in the activation
    // buffer the last hidden layer does not read (act2), so 32-candidate tiles of wide states fit LDS
    int part_alias;
    // ensembles (E > 1): a 1-D grid of ntiles * E workgroups whose ids map member-major onto the 8
    // XCDs (xcd_unit), so each XCD's L2 holds the weights of one or two members instead of all E
    int xcd_map;
    // column-split pairs (rollout_kernel PAIR): two workgroups share a 16-candidate tile, each owning
    // half of every hidden layer's columns; halves cross through pair_data (sc1 stores / loads) under
    // per-workgroup flags (pair_flags: one 128-byte line per workgroup). The flags are zeroed once per
    // plan (cem_init_kernel) or, for a lone rollout, by a memset before the launch (pair_prezeroed 0);
    // within a plan every pair launch has its own epoch (1, 2, ...), so a flag that still holds an
    // earlier launch's value never reads as this launch's:
    //   hand-off q's flag value   pair_base + q + 1     (pair_base = (epoch - 1) * hand-offs per launch)
    //   roll call (word 1)        16 epoch + XCC_ID + 1
    //   status word               max(..., epoch) when one of this launch's hand-offs timed out
    float* pair_data;
    unsigned* pair_flags;
    unsigned pair_epoch, pair_base;
    int pair_prezeroed;
    int debug_abort;         // PAIR kernel: give up at once, as after a timed-out hand-off (MBRL_OPT_DEBUG_PAIR_ABORT)
    int pair_l2;             // PAIR kernel: L2-resident hand-offs when a roll call finds both halves on one XCD
    // non-PAIR fp32 kernels: NULL, or the pair launch's status word (the line after its flags); the
    // launch then recomputes its candidates only if the word reached gate_epoch (the pair launch's
    // epoch: one of its hand-offs timed out)
    const unsigned* gate;
    unsigned gate_epoch;
};

// Hand-offs one pair launch makes at most (rollout.hip: a layer hand-off per hidden layer after layer
// 0 plus the output half sums, per step): the epoch stride of the pair flags.
inline unsigned pair_handoffs(int H, int L) { return (unsigned)H * (unsigned)(L + 1) + 1u; }

// Column-split pair exchange area for ntiles * E tiles (rollout_kernel PAIR): the flags block first
// (one 128-byte line per workgroup, then a status line), then per workgroup two parities of its
// output-layer half sums as tagged 8-byte granules {value, tag} (16 x pw each), then per workgroup two
// parities of its published layer columns (16 x Wpad / 2 floats). The flags and the granules -- the
// words a reader polls -- are zeroed once per plan (zero_bytes from the start; see RolloutArgs).
struct PairLayout {
    size_t flags_bytes, gran_bytes, layer_floats, zero_bytes, bytes;
};
inline PairLayout pair_layout(int Wpad, int pw, int ntiles, int E) {
    PairLayout p;
    const size_t wgs = (size_t)2 * ntiles * E;
    p.flags_bytes = (wgs + 1) * 128;
    p.gran_bytes = wgs * 2 * 16 * (size_t)pw * 8;
    p.layer_floats = (size_t)2 * 16 * (Wpad / 2);
    p.zero_bytes = p.flags_bytes + p.gran_bytes;
    p.bytes = p.zero_bytes + wgs * p.layer_floats * sizeof(float);
    return p;
}

// Workgroup -> (tile, member). Dispatch places workgroup w on XCD w % 8 (round robin), so XCD k runs
// ids k, k + 8, k + 16, ... in that order; xcd_map hands XCD k the contiguous unit range
// [k q + min(k, r), ...) of the member-major order unit = e * ntiles + tile (q = total / 8,
// r = total % 8): a bijection, and every XCD streams at most ceil(E / 8) + 1 members' weights.
__device__ __forceinline__ void xcd_unit(int xcd_map, int ntiles, int& tile, int& e) {
    if (!xcd_map) {
        tile = blockIdx.x;
        e = blockIdx.y;
        return;
    }
    const int total = gridDim.x, q = total >> 3, r = total & 7;
    const int k = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int unit = k * q + (k < r ? k : r) + slot;
    e = unit / ntiles;
    tile = unit - e * ntiles;
}

// F16X3 operand scales (exact powers of two): activations and weights are scaled before the f16
// split so that their residual pieces stay normal; products carry X_SCALE * W_SCALE.
#define MBRL_SPLIT_X_SCALE 16.0f
#define MBRL_SPLIT_W_SCALE 256.0f

// Cost bit pattern the F16X3 kernel leaves for candidates it could not evaluate (an operand out of
// split range); the F32 redo pass recomputes exactly those workgroups. A quiet NaN payload.
constexpr uint32_t MBRL_REDO_MARK = 0x7FC0DEADu;

struct LdsMap {
    float *act, *act2, *part, *sterm, *aterm, *obs_mean, *obs_std, *act_mean, *act_std, *goal, *cw, *hbias;
    uint32_t* lflag;   // per-wave hidden-layer store counters (rollout.hip hidden_store_flag), 16 words
    size_t total_floats;
};

__host__ __device__ inline size_t lds_round4(size_t x) { return (x + 3) & ~(size_t)3; }

__host__ __device__ inline LdsMap lds_map(const RolloutArgs& A, float* base, int M) {
    LdsMap L;
    size_t o = 0;
    auto take = [&](size_t n) { float* p = base ? base + o : nullptr; o += lds_round4(n); return p; };
    L.act = take((size_t)M * A.lda);
    L.act2 = take((size_t)M * A.lda);
    L.part = A.part_alias ? L.act2 : take((size_t)(A.nw > 4 ? A.nw : 4) * M * A.pw);
    L.sterm = take((size_t)M * A.s);
    L.aterm = take((size_t)2 * M * A.a);
    L.obs_mean = take(A.s);
    L.obs_std = take(A.s);
    L.act_mean = take(A.a);
    L.act_std = take(A.a);
    L.goal = take(A.s);
    L.cw = take(A.s);
    L.hbias = take((size_t)A.L * A.Wpad + 16 * (size_t)A.NOT);
    L.lflag = reinterpret_cast<uint32_t*>(take(16));
    L.total_floats = o;
    return L;
}

// The output row value at LDS offset ro from the NP stored partials (stride ws): the canonical tree
// of rollout.hip mma_out's comment (every fp32 rollout kernel and the split kernels use it).
// NP = 8 (8-wave and 8-candidate kernels) or 4 (4-wave kernels).
template <int NP>
__device__ __forceinline__ float sum_partials(const float* part, int ws, int ro) {
    static_assert(NP == 4 || NP == 8, "partials");
    if constexpr (NP == 8)
        return ((part[ro] + part[ws + ro]) + (part[2 * ws + ro] + part[3 * ws + ro])) +
               ((part[4 * ws + ro] + part[5 * ws + ro]) + (part[6 * ws + ro] + part[7 * ws + ro]));
    else
        return (part[ro] + part[ws + ro]) + (part[2 * ws + ro] + part[3 * ws + ro]);
}

// At least 82 KiB so that one workgroup owns a CU: 256 workgroups of N = 4096 then land one per CU
// instead of doubling up on some CUs (the kernel is sized for one wave per SIMD).
inline size_t rollout_lds_bytes(const RolloutArgs& A, int M) {
    const size_t need = lds_map(A, nullptr, M).total_floats * sizeof(float);
    const size_t floor_bytes = 82 * 1024;
    return need > floor_bytes ? need : floor_bytes;
}

// Compute units of the current device (cached; cem.hip).
int device_cu_count();

// Raise `fn`'s dynamic-LDS limit to `bytes` on the current device, once per (kernel, device,
// bytes); thread-safe (cem.hip).
hipError_t ensure_dynamic_lds(const void* fn, int bytes);

// Whether `blocks` workgroups of kernel `fn` (threads each, `lds` bytes of dynamic LDS) can all be
// resident on the current device at once (occupancy query x CU count, cached; cem.hip). Kernels with
// grid-wide hand-offs check it and return hipErrorCooperativeLaunchTooLarge instead of launching.
bool grid_fits(const void* fn, int threads, size_t lds, int blocks);

hipError_t launch_rollout(const RolloutArgs& A, int T, int R, hipStream_t stream);
bool rollout_m8_supported(const RolloutArgs& A, int T);
hipError_t launch_rollout_m8(const RolloutArgs& A, int T, hipStream_t stream);
bool rollout_m4_supported(const RolloutArgs& A, int T, int NG);
hipError_t launch_rollout_m4(const RolloutArgs& A, int T, int NG, hipStream_t stream);
// Column-split pairs: 16-candidate tiles on two workgroups each (8 waves: 4 compute, 4 hand-off).
// Supported for Wpad 512, fp32, goal-state cost, compile-time chunk counts, all 2 ntiles E workgroups
// co-resident; A.pair_* point into a pair_layout() area.
bool rollout_pair_supported(const RolloutArgs& A, int T);
hipError_t launch_rollout_pair(const RolloutArgs& A, int T, hipStream_t stream);

// F16X3 rollout (8 waves, 16 R candidates per workgroup, goal-state cost). Supported for
// geometry.split_ok; the caller follows it with launch_rollout(redo = 1) at the same R.
// P = 2 (F16X3) or 3 (F16X6) operand pieces; A.split_off / A.sr must describe that stream.
bool rollout_split_supported(const RolloutArgs& A, int T, int R, int P);
size_t rollout_split_lds_bytes(const RolloutArgs& A, int R);
hipError_t launch_rollout_split(const RolloutArgs& A, int T, int R, int P, hipStream_t stream);

// Single-trajectory rollout (one candidate per ensemble member): the final CEM mean's predicted
// states. Latency-bound, so VALU dot products over plain weight copies on one workgroup per member
// instead of the 16-row MFMA tile (traj.hip).
struct TrajArgs {
    const float* packed;
    size_t member_stride, bias_off, tw_base;
    size_t tw_off[MAX_LAYERS + 1];
    int s, a, W, Wpad, L, H;
    const float *obs_mean, *obs_std, *act_mean, *act_std;
    int norm_s, unnorm_s, norm_a;
    const float* s0;
    const float* actions;  // [H][a]
    float* states_out;     // [E][H][s]
    const unsigned* gate;  // traj_kernel: when non-NULL, run only if *gate != 0 (the coop kernel gave up)
    int debug_abort;       // traj_coop_kernel: give up at once (tests of the fallback; MBRL_DEBUG_TRAJ_ABORT)
    int prezeroed;         // traj_coop_kernel: the granules and status word were zeroed by the plan's first launch
    // traj_coop_kernel hand-off placement (MBRL_OPT_TRAJ_HOP): 0 = a (P, E) grid, agent-scope (sc1)
    // granules; 1 = a 1-D grid of 8 P workgroups where member e's P share blockIdx % 8 == e (one XCD
    // under round-robin dispatch), sc1 granules; 2 = that grid, and granules written with L2-resident
    // (sc0) stores once a roll call at the start found every workgroup of the member on one XCD
    // (s_getreg XCC_ID; else sc1 as in 1)
    int hop_mode;
    int E;                 // ensemble members (hop_mode >= 1: E <= 8)
};
hipError_t launch_traj(const TrajArgs& A, int E, hipStream_t stream);

// Fused gradient-descent planner (gd.hip): one persistent workgroup runs every Adam iteration of
// planners.py:103-137 (goal-state cost, one ensemble member).
struct GdArgs {
    const float* packed;                   // member 0
    size_t bias_off, tw_base;
    size_t tw_off[MAX_LAYERS + 1];
    int s, a, W, Wpad, L, H;
    const float *obs_mean, *obs_std, *act_mean, *act_std;
    int norm_s, unnorm_s, norm_a;
    const float *cw, *goal;
    float alpha_s, alpha_a;
    int has_sc, has_ac;
    int reward;                            // cost = unnormalised reward head at (s_{t+1}, a_t): 2 passes / step
    int unnorm_r;
    const float* rew_std;                  // [1] (device) when unnorm_r
    const float* s0;                       // [s]
    float* actions;                        // [H][a], in: initial sequence, out: optimised
    float* states_out;                     // [H+1][s]: the last iteration's rollout
    float *m, *v;                          // Adam moments [H][a] (workspace)
    float* hist;                           // [H][hist_row] saved layer inputs (workspace)
    int hist_row;                          // (round4(s + a) + L * Wpad), twice with a reward head
    int iterations;
    float stop, lr;
    int* iterations_out;                   // device int or NULL
    const unsigned* gate;                  // gd_plan_kernel: when non-NULL, run only if *gate != 0
    int debug_abort;                       // gd_coop_kernel: give up at once (MBRL_DEBUG_GD_ABORT)
    int hop_mode;                          // gd_coop_kernel hand-offs, as TrajArgs.hop_mode (MBRL_OPT_GD_HOP)
    // batched plans (grid.y = batch): plan b reads s0 + b s, actions + b H a, writes states_out +
    // b (H+1) s and iterations_out + b; its m / v / hist lie plan_ws bytes after plan b-1's, its
    // hand-off block (2 Wpad granules, then the status word) xchg_stride granules after
    int batch;
    size_t plan_ws, xchg_stride;
};
size_t gd_lds_bytes(int s, int a, int Wpad, int H);
hipError_t launch_gd_plan(const GdArgs& A, hipStream_t stream);
// Cooperative variant (Wpad / 16 workgroups; hist = Wpad/16 copies of [H][L][Wpad]); `xchg` holds
// 2 Wpad 8-byte granules immediately followed by the status word (zeroed by the launcher).
bool gd_coop_supported(const GdArgs& A);
hipError_t launch_gd_coop(const GdArgs& A, unsigned long long* xchg, unsigned* status, hipStream_t stream);

// Cooperative variant: P = Wpad/16 workgroups per member each own 16 hidden units of every W -> W
// layer (slices LDS-resident); layer 0 and the output layer are computed redundantly by every
// workgroup; hidden activations are all-gathered through tagged 8-byte granules in `xchg`
// (E * 2 * Wpad granules, zeroed by the launcher before every launch). Needs the P*E workgroups co-resident (grid_fits) and
// s <= 64. `status` (one uint32, zeroed by the launcher) becomes nonzero if a bounded spin gave up.
bool traj_coop_supported(const TrajArgs& A, int E);
// Register-resident variant for narrow models (Wpad <= 256, few hidden layers): one 1024-thread
// workgroup per member with every weight in registers; no hand-off, no workspace (traj.hip).
bool traj_reg_supported(const TrajArgs& A);
hipError_t launch_traj_reg(const TrajArgs& A, int E, hipStream_t stream);
size_t traj_coop_xchg_bytes(const TrajArgs& A, int E);
hipError_t launch_traj_coop(const TrajArgs& A, int E, unsigned long long* xchg, unsigned* status,
                            hipStream_t stream);

// mbrl_adam_step (train.hip). AdamArith bits: which of torch's element-wise expressions its build
// contracts to a fused multiply-add; ADAM_ARITH_TORCH is the pattern pinned against torch.optim.Adam
// on the MI355X (tests/test_gpu_train_adam.py).
enum { ADAM_FMA_WD = 1, ADAM_FMA_LERP = 2, ADAM_FMA_ADDCMUL = 4, ADAM_FMA_ADDCDIV = 8 };
constexpr int ADAM_ARITH_TORCH = ADAM_FMA_WD | ADAM_FMA_LERP | ADAM_FMA_ADDCMUL | ADAM_FMA_ADDCDIV;
constexpr int ADAM_MAX_TENSORS = 32;   // tensors per launch (the table travels in the kernel arguments)
hipError_t launch_adam_step(const mbrl_adam_tensor* tensors, int count, const mbrl_adam_hparams& hp, int arith,
                            hipStream_t stream);

// mbrl_train_grads (train.hip): the MLP's loss gradient for one batch, n_hidden + 2 launches.
struct TrainShape {
    int s, a, W, L, reward, H;   // state / action dims, hidden width, hidden layers, reward head, horizon
    int tile;                    // backward C tile height: 0 auto, 32, 64 (MBRL_OPT_TRAIN_TILE; same bits)
    int fold;                    // 1: the layer-0 weight gradient folds into the dH_0 launch (same bits)
    int xcd;                     // 1: row-band tiles in XCD order in every launch (MBRL_OPT_TRAIN_XCD; same bits)
    int split;                   // 1: the five-launch layout where the fused step applies (MBRL_OPT_TRAIN_SPLIT; same bits)
    int fo_split;                // 1: the fused step's F and O as two launches (MBRL_OPT_TRAIN_FO; same bits)
};
struct TrainTensors {
    const float* const* weight;  // L + 1 (+ 1 reward head) nn.Linear weights [out][in]
    const float* const* bias;
    float* const* weight_grad;
    float* const* bias_grad;
    const float *states, *actions, *next_states, *rewards;   // stacked transitions [T][H][.]
};
size_t train_ws_floats(const TrainShape& t, int batch);
size_t train_status_offset(const TrainShape& t, int batch);   // bytes: the fused step's status word
size_t train_counter_bytes(const TrainShape& t, int batch);   // the tickets and band counters (offset 0)
// adam (optional): the step of every layer's weight and bias (linear1.weight, linear1.bias, ...)
// folded into the backward launches, bit-identical to a separate mbrl_adam_step after the gradient.
// With the layer-0 fold one layer's step cannot ride in this step's launches: it comes back in
// pending[0 .. *pending_n) (then required with adam) for the caller to pass as the next step's
// `prior` (taken by its first launch) or to run with launch_adam_step.
// The fused step (two hidden layers) can gather the NEXT batch's rows while it runs: `next`
// (rows idx_next[0 .. batch_next)) goes to the gather buffers of slot `slot ^ 1`, and the next call
// then passes pre_rows = 1 with that slot (mbrl_train_epoch). train_fused_applies: whether a batch of
// `batch` transitions takes the fused step.
struct TrainGather {
    const int64_t* idx_next;
    int batch_next;
    int pre_rows;
    int slot;
};
bool train_fused_applies(const TrainShape& t, int batch);
hipError_t launch_train_grads(const TrainShape& t, const TrainTensors& w, const int64_t* idx, int batch,
                              float* loss_out, float* ws, hipStream_t stream, const mbrl_adam_tensor* adam = nullptr,
                              const mbrl_adam_hparams* hp = nullptr, int arith = 0,
                              const mbrl_adam_tensor* prior = nullptr, int prior_n = 0,
                              mbrl_adam_tensor* pending = nullptr, int* pending_n = nullptr,
                              const TrainGather* gather = nullptr);

// ---- cooperative single-candidate kernels (traj.hip, gd.hip): the dot of one 16-row slice, one row
// per half-wave (32 lanes), and its reduction
typedef float coop_f32x4 __attribute__((ext_vector_type(4)));

// The same sum, complete in lane 16 of each half-wave (c == 16) only: DPP row sums (row_ror 8, 4, 2,
// 1: every lane of a 16-lane row holds its row's sum), then row_bcast:15 hands row 0's lane 15 to
// row 1 (and row 2's to row 3). DPP moves cost a few cycles where each ds_swizzle step of
// halfwave_sum waits on the LDS crossbar; a fixed order, so every workgroup gets the same bits.
__device__ __forceinline__ float halfwave_sum_hi(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x122, 0xF, 0xF, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x121, 0xF, 0xF, false));
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF,
                                                                     false));
}

// Lane c's share of a 16-row dot over K = 32 WI columns: VW-wide LDS vectors at columns
// VW c + 32 VW j + q (j < WI / VW), VW independent fmaf chains closed as a fixed tree.
template <int WI>
struct CoopDot {
    static constexpr int VW = WI >= 4 ? 4 : 2;
    static constexpr int NJ = WI / VW;
    static_assert(WI % VW == 0, "CoopDot: WI must be a multiple of the vector width (else columns are skipped)");
    static __device__ __forceinline__ int col(int c, int i) { return VW * c + 32 * VW * (i / VW) + (i % VW); }
    // w: LDS row (w[k] for column k), x: LDS vector
    static __device__ __forceinline__ float lds(const float* w, const float* x, int c) {
        float acc[VW] = {};
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int k = VW * c + 32 * VW * j;
            if constexpr (VW == 4) {
                const coop_f32x4 a = *reinterpret_cast<const coop_f32x4*>(w + k);
                const coop_f32x4 b = *reinterpret_cast<const coop_f32x4*>(x + k);
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = fmaf(a[q], b[q], acc[q]);
            } else {
#pragma unroll
                for (int q = 0; q < VW; ++q) acc[q] = fmaf(w[k + q], x[k + q], acc[q]);
            }
        }
        return close(acc);
    }
    // wr: this lane's weights in registers, wr[i] for column col(c, i)
    static __device__ __forceinline__ float reg(const float (&wr)[WI], const float* x, int c) {
        float acc[VW] = {};
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int k = VW * c + 32 * VW * j;
            if constexpr (VW == 4) {
                const coop_f32x4 b = *reinterpret_cast<const coop_f32x4*>(x + k);
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[q] = fmaf(wr[4 * j + q], b[q], acc[q]);
            } else {
#pragma unroll
                for (int q = 0; q < VW; ++q) acc[q] = fmaf(wr[VW * j + q], x[k + q], acc[q]);
            }
        }
        return close(acc);
    }
    static __device__ __forceinline__ float close(const float (&acc)[VW]) {
        if constexpr (VW == 4) return (acc[0] + acc[1]) + (acc[2] + acc[3]);
        else return acc[0] + acc[1];
    }
};

}  // namespace mbrl
