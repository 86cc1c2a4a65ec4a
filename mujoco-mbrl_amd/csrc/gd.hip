// Fused gradient-descent planner: the reference's _optimize_trajectory (planners.py:103-137) as ONE
// persistent workgroup -- every Adam iteration's rollout, loss gradient, backward pass through the
// H-step chain, Adam step and stop test on the device.
//
// One candidate is a dependent chain of batch-1 mat-vecs, so the work is latency- and
// L2-stream-bound on one CU: a forward step reads every layer's W^T once (coalesced rows, as
// traj_kernel), the backward step reads them again for W^T g (one wave per input row). The layer
// inputs of every step (normalised [s|a] and each hidden activation) are kept in the workspace for
// the backward pass (L2-resident: H * (s + a + L W) floats).
//
// Semantics per iteration (planners.py:117-135 with the GoalStateAgent closures, agents.py:219-233):
//   s_{t+1} = unnorm(MLP(norm(s_t), norm(a_t)))       for t < H      (states_out rows 1..H)
//   loss    = sum_t SmoothAbs(s_{t+1}) + CoshLoss(a_t)                (models.py:244-272)
// or, for a reward-head model behind RewardAgent's closures (agents.py:336-362; one-workgroup kernel):
//   loss    = sum_t unnorm_r(reward head of the trunk at (norm(s_{t+1}), norm(a_t)))
//   -- a second trunk pass per step, whose activations are saved and back-propagated as well.
//   grad    = d loss / d a  (reverse mode through the chain; ReLU' = [output > 0] as torch)
//   Adam(lr, betas = (0.9, 0.999), eps = 1e-8) as torch.optim.Adam: m.lerp_(g, 1 - b1),
//   v = b2 v + (1 - b2) g^2, a -= (lr / (1 - b1^k)) m / (sqrt(v) / sqrt(1 - b2^k) + eps)
//   stop once mean |a_new - a_old| < stop_condition (after the step, as the reference).
// states_out holds the LAST iteration's rollout, computed before its update, as the reference
// returns it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mbrl_internal.h"

namespace mbrl {

namespace {

constexpr int GD_THREADS = 1024;
constexpr int GD_WAVES = GD_THREADS / 64;

__device__ __forceinline__ float gd_wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// y[0..Wpad) = relu(b + W x), W^T [in][Wpad] row-major: thread (g4, ks) owns outputs 4 g4 .. 4 g4 + 3
// over a K slice; slice partials are summed in a fixed order through LDS.
__device__ void gd_dense_relu(const float* __restrict__ wt, const float* __restrict__ bias, int in, int Wpad,
                              const float* x, float* part, float* y) {
    const int G4 = Wpad / 4, KS = GD_THREADS / G4;
    const int tid = threadIdx.x, g4 = tid % G4, ks = tid / G4;
    const int per = (in + KS - 1) / KS, k0 = ks * per, k1 = min(in, k0 + per);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const float4* w4 = reinterpret_cast<const float4*>(wt) + g4;
#pragma unroll 8
    for (int k = k0; k < k1; ++k) {
        const float4 w = w4[(size_t)k * G4];
        const float xv = x[k];
        a0 += xv * w.x; a1 += xv * w.y; a2 += xv * w.z; a3 += xv * w.w;
    }
    float* pp = part + ks * Wpad + 4 * g4;
    pp[0] = a0; pp[1] = a1; pp[2] = a2; pp[3] = a3;
    __syncthreads();
    for (int n = tid; n < Wpad; n += GD_THREADS) {
        float v = bias[n];
        for (int j = 0; j < KS; ++j) v += part[j * Wpad + n];
        y[n] = fmaxf(v, 0.0f);
    }
    __syncthreads();
}

// gx[k] = sum_n W^T[k][n] gz[n] for k < in: one wave per row, lanes over n in float4 (one 1 KiB
// wave-instruction per 256 columns), four rows per pass for loads in flight
__device__ void gd_dense_back(const float* __restrict__ wt, int in, int Wpad, const float* gz, float* gx) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n4 = Wpad / 4;
    constexpr int RB = 4;
    for (int k0 = wave * RB; k0 < in; k0 += GD_WAVES * RB) {
        float v[RB];
#pragma unroll
        for (int r = 0; r < RB; ++r) v[r] = 0.f;
        for (int c = lane; c < n4; c += 64) {
            const float4 g = reinterpret_cast<const float4*>(gz)[c];
#pragma unroll
            for (int r = 0; r < RB; ++r) {
                const int k = min(k0 + r, in - 1);
                const float4 w = reinterpret_cast<const float4*>(wt + (size_t)k * Wpad)[c];
                v[r] += w.x * g.x + w.y * g.y + w.z * g.z + w.w * g.w;
            }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            const float t = gd_wave_sum(v[r]);
            if (lane == 0 && k0 + r < in) gx[k0 + r] = t;
        }
    }
    __syncthreads();
}

struct GdLds {
    float *x, *h, *part, *out, *gz, *gx, *gs, *ga, *red;
    size_t floats;
};

__host__ __device__ inline GdLds gd_lds(int s, int a, int Wpad, int H, float* base) {
    GdLds m;
    size_t o = 0;
    auto take = [&](size_t n) { float* p = base ? base + o : nullptr; o += (n + 3) & ~(size_t)3; return p; };
    const int K0 = s + a, xd = K0 > Wpad ? K0 : Wpad;
    m.x = take(xd);
    m.h = take(Wpad);
    m.part = take(4096);
    m.out = take(s);
    m.gz = take(Wpad);
    m.gx = take(xd);
    m.gs = take(s);
    m.ga = take((size_t)H * a);
    m.red = take(GD_WAVES);
    m.floats = o;
    return m;
}

__device__ float gd_block_sum(float v, float* red) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    v = gd_wave_sum(v);
    if (lane == 0) red[wave] = v;
    __syncthreads();
    float t = 0.f;
    for (int w = 0; w < GD_WAVES; ++w) t += red[w];   // fixed order, same in every thread
    __syncthreads();
    return t;
}

__global__ void __launch_bounds__(GD_THREADS) gd_plan_kernel(const GdArgs A) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // plan blockIdx.y of a batch: its own start state, actions, states, workspace block and gate
    const int pb = blockIdx.y;
    const float* s0 = A.s0 + (size_t)pb * A.s;
    float* actions = A.actions + (size_t)pb * A.H * A.a;
    float* states_out = A.states_out + (size_t)pb * (A.H + 1) * A.s;
    float* am = reinterpret_cast<float*>(reinterpret_cast<char*>(A.m) + pb * A.plan_ws);
    float* av = reinterpret_cast<float*>(reinterpret_cast<char*>(A.v) + pb * A.plan_ws);
    float* ahist = reinterpret_cast<float*>(reinterpret_cast<char*>(A.hist) + pb * A.plan_ws);
    int* iterations_out = A.iterations_out ? A.iterations_out + pb : nullptr;
    const unsigned* gate = A.gate ? A.gate + (size_t)pb * A.xchg_stride * 2 : nullptr;
    // behind the cooperative kernel: only when that one gave up (its status word set)
    if (gate != nullptr && *gate == 0u) return;
    const GdLds m = gd_lds(A.s, A.a, A.Wpad, A.H, smem);
    const int tid = threadIdx.x;
    const int s = A.s, a = A.a, Wp = A.Wpad, K0 = s + a, L = A.L, H = A.H;
    const int rowf = A.hist_row;                      // floats per step in hist: K0p + L * Wpad
    const int K0p = (K0 + 3) & ~3;
    const float* bias = A.packed + A.bias_off;
    const float* tw = A.packed + A.tw_base;
    // per-layer W^T bases (constant-index copy: a runtime index into the kernel argument would
    // move the whole argument block to scratch)
    __shared__ const float* lw[MAX_LAYERS + 1];
    if (tid == 0) {
#pragma unroll
        for (int l = 0; l <= MAX_LAYERS; ++l) lw[l] = tw + A.tw_off[l];
    }
    __syncthreads();
    const float* wout = lw[L];                         // [s][W] row-major
    const float* bout = bias + (size_t)L * Wp;
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;

    for (int i = tid; i < H * a; i += GD_THREADS) { am[i] = 0.f; av[i] = 0.f; }
    // the reference's states tensor before any iteration: s0, then zeros (returned as is when
    // num_iterations == 0)
    for (int i = tid; i < (H + 1) * s; i += GD_THREADS) states_out[i] = i < s ? s0[i] : 0.f;
    __syncthreads();
    int done = 0;
    for (int it = 0; it < A.iterations; ++it) {
        // ---------------- forward: the rollout of the current actions (states_out rows 0..H)
        for (int d = tid; d < s; d += GD_THREADS) states_out[d] = s0[d];
        __syncthreads();
        for (int t = 0; t < H; ++t) {
            float* hist = ahist + (size_t)t * rowf;
            for (int d = tid; d < K0; d += GD_THREADS) {
                float v;
                if (d < s) {
                    const float sv = states_out[(size_t)t * s + d];
                    v = A.norm_s ? (sv - A.obs_mean[d]) / A.obs_std[d] : sv;
                } else {
                    const float av = actions[t * a + d - s];
                    v = A.norm_a ? (av - A.act_mean[d - s]) / A.act_std[d - s] : av;
                }
                m.x[d] = v;
                hist[d] = v;
            }
            __syncthreads();
            gd_dense_relu(lw[0], bias, K0, Wp, m.x, m.part, m.h);
            for (int n = tid; n < Wp; n += GD_THREADS) hist[K0p + n] = m.h[n];
            for (int l = 1; l < L; ++l) {
                gd_dense_relu(lw[l], bias + (size_t)l * Wp, A.W, Wp, m.h, m.part, m.x);
                for (int n = tid; n < Wp; n += GD_THREADS) { m.h[n] = m.x[n]; hist[K0p + l * Wp + n] = m.x[n]; }
                __syncthreads();
            }
            const int wave = tid >> 6, lane = tid & 63;
            for (int n = wave; n < s; n += GD_WAVES) {
                float v = 0.f;
                for (int k = lane; k < A.W; k += 64) v += wout[(size_t)n * A.W + k] * m.h[k];
                v = gd_wave_sum(v);
                if (lane == 0) {
                    const float o = v + bout[n];
                    states_out[(size_t)(t + 1) * s + n] = A.unnorm_s ? o * A.obs_std[n] + A.obs_mean[n] : o;
                }
            }
            __threadfence_block();
            __syncthreads();
            if (A.reward) {
                // the cost call's trunk pass on (s_{t+1}, a_t): only its activations are needed (the
                // reward's derivative w.r.t. its head is the constant rew_std)
                float* hb = hist + rowf / 2;
                for (int d = tid; d < K0; d += GD_THREADS) {
                    float v;
                    if (d < s) {
                        const float sv = states_out[(size_t)(t + 1) * s + d];
                        v = A.norm_s ? (sv - A.obs_mean[d]) / A.obs_std[d] : sv;
                    } else {
                        v = hist[d];   // norm(a_t), as the state pass
                    }
                    m.x[d] = v;
                    hb[d] = v;
                }
                __syncthreads();
                gd_dense_relu(lw[0], bias, K0, Wp, m.x, m.part, m.h);
                for (int n = tid; n < Wp; n += GD_THREADS) hb[K0p + n] = m.h[n];
                for (int l = 1; l < L; ++l) {
                    gd_dense_relu(lw[l], bias + (size_t)l * Wp, A.W, Wp, m.h, m.part, m.x);
                    for (int n = tid; n < Wp; n += GD_THREADS) { m.h[n] = m.x[n]; hb[K0p + l * Wp + n] = m.x[n]; }
                    __syncthreads();
                }
            }
        }
        // ---------------- backward: d loss / d a, t = H-1 .. 0
        for (int d = tid; d < s; d += GD_THREADS) m.gs[d] = 0.f;
        __syncthreads();
        for (int t = H - 1; t >= 0; --t) {
            const float* hist = ahist + (size_t)t * rowf;
            if (A.reward) {
                // reward pass backward: d r_t / d head = rew_std (unnormalise_reward), through the
                // reward row of the output block and the pass's saved ReLU masks to its input
                // (norm(s_{t+1}), norm(a_t)); the state part joins gs, the action part waits in m.ga
                const float* hb = hist + rowf / 2;
                const float gr = A.unnorm_r ? A.rew_std[0] : 1.0f;
                const float* hl = hb + K0p + (size_t)(L - 1) * Wp;
                for (int k = tid; k < Wp; k += GD_THREADS)
                    m.gz[k] = (k < A.W && hl[k] > 0.f) ? wout[(size_t)s * A.W + k] * gr : 0.f;
                __syncthreads();
                for (int l = L - 1; l >= 1; --l) {
                    gd_dense_back(lw[l], A.W, Wp, m.gz, m.gx);
                    const float* hp = hb + K0p + (size_t)(l - 1) * Wp;
                    for (int k = tid; k < Wp; k += GD_THREADS) m.gz[k] = (k < A.W && hp[k] > 0.f) ? m.gx[k] : 0.f;
                    __syncthreads();
                }
                gd_dense_back(lw[0], K0, Wp, m.gz, m.gx);
                for (int d = tid; d < K0; d += GD_THREADS) {
                    const float g = m.gx[d];
                    if (d < s) {
                        m.gs[d] += A.norm_s ? g / A.obs_std[d] : g;
                    } else {
                        const int j = d - s;
                        m.ga[t * a + j] = A.norm_a ? g / A.act_std[j] : g;
                    }
                }
                __syncthreads();
            }
            // gs += d SmoothAbs / d s_{t+1}; g_out = gs * obs_std (s_{t+1} = out * std + mean)
            for (int d = tid; d < s; d += GD_THREADS) {
                float g = m.gs[d];
                if (A.has_sc) {
                    const float x = states_out[(size_t)(t + 1) * s + d] - A.goal[d];
                    const float wx = x * A.cw[d];
                    g += wx * A.cw[d] / sqrtf(wx * wx + A.alpha_s * A.alpha_s);
                }
                m.out[d] = A.unnorm_s ? g * A.obs_std[d] : g;
            }
            __syncthreads();
            // output layer: g_h[k] = sum_n Wout[n][k] g_out[n]; then the ReLU mask of the last hidden layer
            const float* hl = hist + K0p + (size_t)(L - 1) * Wp;
            for (int k = tid; k < Wp; k += GD_THREADS) {
                float v = 0.f;
                if (k < A.W)
                    for (int n = 0; n < s; ++n) v += wout[(size_t)n * A.W + k] * m.out[n];
                m.gz[k] = hl[k] > 0.f ? v : 0.f;
            }
            __syncthreads();
            for (int l = L - 1; l >= 1; --l) {
                gd_dense_back(lw[l], A.W, Wp, m.gz, m.gx);
                const float* hp = hist + K0p + (size_t)(l - 1) * Wp;
                for (int k = tid; k < Wp; k += GD_THREADS) m.gz[k] = (k < A.W && hp[k] > 0.f) ? m.gx[k] : 0.f;
                __syncthreads();
            }
            gd_dense_back(lw[0], K0, Wp, m.gz, m.gx);
            // split the input gradient: state part -> step t-1, action part -> grad of a_t
            for (int d = tid; d < K0; d += GD_THREADS) {
                const float g = m.gx[d];
                if (d < s) {
                    m.gs[d] = A.norm_s ? g / A.obs_std[d] : g;
                } else {
                    const int j = d - s;
                    float ga = A.norm_a ? g / A.act_std[j] : g;
                    if (A.has_ac)
                        ga += A.alpha_a * sinhf(actions[t * a + j] / A.alpha_a) / (float)a;
                    if (A.reward) ga += m.ga[t * a + j];   // the reward pass's share (above)
                    m.ga[t * a + j] = ga;
                }
            }
            __syncthreads();
        }
        // ---------------- Adam step and the stop test
        const float k = (float)(it + 1);
        const float bc1 = 1.0f - powf(b1, k), bc2 = 1.0f - powf(b2, k);
        const float step = A.lr / bc1, bc2s = sqrtf(bc2);
        float change = 0.f;
        for (int i = tid; i < H * a; i += GD_THREADS) {
            const float g = m.ga[i];
            float mm = am[i];
            mm = mm + (1.0f - b1) * (g - mm);
            const float vv = b2 * av[i] + (1.0f - b2) * g * g;
            am[i] = mm;
            av[i] = vv;
            const float old = actions[i];
            const float nw = old - step * (mm / (sqrtf(vv) / bc2s + eps));
            actions[i] = nw;
            change += fabsf(old - nw);
        }
        __threadfence_block();
        change = gd_block_sum(change, m.red);
        done = it + 1;
        if (change / (float)(H * a) < A.stop) break;
    }
    if (tid == 0 && iterations_out != nullptr) *iterations_out = done;
}

// ------------------------------------------------------------------------------------------------
// Cooperative variant (the traj_coop_kernel scheme of traj.hip, with a backward pass): P = Wpad/16
// workgroups of 512 threads. Workgroup p keeps, LDS-resident for the whole plan, rows
// [16p, 16p + 16) of every W -> W layer (forward: its 16 units) and the same rows of each layer's
// W^T (backward: its 16 input gradients). Layer 0 and the output layer, forward and backward, are
// computed redundantly by every workgroup from register-resident weights. The only cross-workgroup
// traffic is one all-gather of a hidden vector per W -> W layer and direction: 2 (L - 1) hand-offs
// per step, as R2 granules (cdna_hip_programming.md §6 G16: aligned 8-byte {epoch, value} agent-
// scope stores, gathered by one wave until every tag matches). Adam and the stop test run
// redundantly (bit-identical) in every workgroup, so no other exchange is needed. Every spin is
// bounded; on a timeout `status` is set and the single-workgroup kernel (gated on it) redoes the plan.
// ------------------------------------------------------------------------------------------------
constexpr int GC_THREADS = 512;
constexpr int GC_ROWS = 16;
typedef unsigned long long gc_u64;
typedef __attribute__((address_space(1))) gc_u64 gc_gu64;

// Diagnostic build only (-DMBRL_STAMPS): per-workgroup s_memrealtime sums (10 ns ticks) of the
// cooperative kernel's segments, written to a buffer set by mbrl_diag_set_gd_stamps()
// (tools/gd_stamps.py): forward layer 0, forward hidden (dots + hand-offs), forward output,
// backward output layer, backward hidden, backward layer 0, Adam + stop test.
#ifdef MBRL_STAMPS
constexpr int GD_NSEG = 7;
__device__ unsigned long long* g_mbrl_gd_stamps;
#define GSTAMP(k)                                                      \
    do {                                                               \
        const unsigned long long _t = __builtin_amdgcn_s_memrealtime(); \
        gseg[k] += _t - gprev;                                         \
        gprev = _t;                                                    \
    } while (0)
#else
#define GSTAMP(k) \
    do {          \
    } while (0)
#endif

struct GcLds {
    int rs;
    size_t fw, bw, x0, hA, hB, gA, gB, out, gs, red, acts, m1, m2, grad, st, flag, mk, total;
    int mk_row;   // 32-bit words of ReLU masks per (pass, step): gc_mask_words
};

// ReLU masks the backward pass needs, per (pass, step), as bits in LDS: the last hidden layer's
// whole output (the output layer's backward, one bit per unit: Wp / 32 words) and, for every other
// layer, the 16 units this workgroup owns (the hidden layers' backward: one word each).
__host__ __device__ inline int gc_mask_words(int Wp, int L) { return Wp / 32 + (L - 1); }

__host__ __device__ inline GcLds gc_lds(int s, int a, int W, int Wp, int L, int H, int K0R, int passes = 1) {
    GcLds m;
    auto al4 = [](size_t n) { return (n + 3) & ~(size_t)3; };
    m.rs = W + 32;
    size_t o = 0;
    m.fw = o;   o += (size_t)(L - 1) * GC_ROWS * m.rs;
    m.bw = o;   o += (size_t)(L - 1) * GC_ROWS * m.rs;
    m.x0 = o;   o += al4(K0R);
    m.hA = o;   o += Wp;
    m.hB = o;   o += Wp;
    m.gA = o;   o += Wp;
    m.gB = o;   o += Wp;
    m.out = o;  o += 32;
    m.gs = o;   o += 32;
    m.red = o;  o += (size_t)(GC_THREADS / 64) * K0R;
    m.acts = o; o += al4((size_t)H * a);
    m.m1 = o;   o += al4((size_t)H * a);
    m.m2 = o;   o += al4((size_t)H * a);
    m.grad = o; o += al4((size_t)H * a);
    m.st = o;   o += al4((size_t)(H + 1) * s);
    m.flag = o; o += 4;
    m.mk_row = gc_mask_words(Wp, L);
    m.mk = o;   o += al4((size_t)passes * H * m.mk_row);
    m.total = o * sizeof(float);
    return m;
}

// Publish this workgroup's 16 values (lane c == 16 of half-wave g holds value g) and gather all P
// slices into `dst`; returns false on a timeout (status set). GR = Wp / 64 granules per lane: every
// load of a sweep pass is in flight before the first compare (a runtime-bounded loop waited for
// each load in turn: GR dependent fabric round trips per pass).
// l2: every workgroup of the plan runs on this XCD (gd_roll_call), so the granules are stored with
// L2-resident (sc0) stores instead of written through (sc1); the sc1 sweep reads the shared L2.
template <int GR>
__device__ __forceinline__ bool gc_exchange(gc_gu64* xchg, int Wp, int p, unsigned& phase, float val, float* dst,
                                            int& abort_flag, unsigned* status, bool l2) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = tid >> 5, c = tid & 31;
    const unsigned epoch = phase + 1u;
    gc_gu64* buf = xchg + (size_t)(phase & 1u) * Wp;
    if (c == 16) {   // the lane holding the half-wave's sum (halfwave_sum_hi)
        const gc_u64 gr = ((gc_u64)epoch << 32) | __float_as_uint(val);
        if (l2)
            __hip_atomic_store(&buf[p * GC_ROWS + g], gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
            __hip_atomic_store(&buf[p * GC_ROWS + g], gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wave == 0) {
        const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            gc_u64 gv[GR];
#pragma unroll
            for (int q = 0; q < GR; ++q)
                gv[q] = __hip_atomic_load(&buf[lane + 64 * q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool ok = true;
#pragma unroll
            for (int q = 0; q < GR; ++q) {
                ok &= (unsigned)(gv[q] >> 32) == epoch;
                dst[lane + 64 * q] = __uint_as_float((unsigned)gv[q]);
            }
            if (__all(ok)) break;
            if (__builtin_amdgcn_s_memrealtime() - t_start > 20000000ull) {   // 200 ms
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
    ++phase;
    return abort_flag == 0;
}

// Wave-wide reduce-scatter of 32 values per lane by recursive halving: returns the sum over the
// 64 lanes of v[lane >> 1] (both lanes of a pair hold it). Each halving step adds the value a lane
// keeps to the one its partner (lane ^ m) sends: m = 32 and 16 by v_permlane32_swap /
// v_permlane16_swap (the swap hands each half-wave / row the other's value, and the two outputs
// summed are keep + partner's), m = 8, 4, 2, 1 by DPP moves (row_ror:8; row_half_mirror then the quad
// mirror for lane ^ 4; quad_perm for ^ 2, ^ 1). No LDS crossbar traffic (ds_bpermute) where the
// r03 form had 32 per lane.
// v_permlane32_swap / v_permlane16_swap as inline asm: both registers are read and written. (The
// ROCm 7.2 clang builtins return the swapped pair wrongly here: __builtin_amdgcn_permlane32_swap's two
// results were read from ONE register, v_add_f32 vX, vY, vY after the swap -- tools/ubench/rs_check.hip.)
// The s_nops cover the VALU-write -> permlane-read and permlane-write -> VALU-read hazards, which the
// compiler's hazard recognizer does not see through inline asm.
__device__ __forceinline__ void permlane32_swap(float& x, float& y) {
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void permlane16_swap(float& x, float& y) {
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
}
#define GC_DPP(v, ctrl) \
    __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, (v)), (ctrl), 0xF, 0xF, false))
__device__ __forceinline__ float wave_reduce_scatter32(const float (&v)[32], int lane) {
    float a16[16], a8[8], a4[4], a2[2];
#pragma unroll
    for (int j = 0; j < 16; ++j) {   // lane ^ 32: lanes < 32 keep v[j], lanes >= 32 keep v[j + 16]
        float x = v[j], y = v[j + 16];
        permlane32_swap(x, y);
        a16[j] = x + y;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {    // lane ^ 16: even rows keep a16[j], odd rows a16[j + 8]
        float x = a16[j], y = a16[j + 8];
        permlane16_swap(x, y);
        a8[j] = x + y;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {    // lane ^ 8 (row_ror:8)
        const bool hi = lane & 8;
        const float keep = hi ? a8[j + 4] : a8[j], send = hi ? a8[j] : a8[j + 4];
        a4[j] = keep + GC_DPP(send, 0x128);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {    // lane ^ 4: half-row mirror (7 - i), then quad mirror (i ^ 3)
        const bool hi = lane & 4;
        const float keep = hi ? a4[j + 2] : a4[j], send = hi ? a4[j] : a4[j + 2];
        a2[j] = keep + GC_DPP(GC_DPP(send, 0x141), 0x1B);
    }
    const bool hi = lane & 2;        // lane ^ 2: quad_perm [2, 3, 0, 1]
    const float keep = hi ? a2[1] : a2[0], send = hi ? a2[0] : a2[1];
    const float a1 = keep + GC_DPP(send, 0x4E);
    return a1 + GC_DPP(a1, 0xB1);    // lane ^ 1: quad_perm [1, 0, 3, 2]
}
#undef GC_DPP

// K0R >= s + a: layer-0 inputs per thread; SM: output rows per half-wave (16 SM >= s); WI = W / 32.
template <int K0R, int SM, int WI>
__global__ void __launch_bounds__(GC_THREADS) gd_coop_kernel(const GdArgs A, gc_u64* __restrict__ xchg_all,
                                                             unsigned* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    // plan pb of a batch: its own start state, actions, states, hand-off block and workspace. hop_mode
    // >= 1: plan (blockIdx.x & 7) + 8 blockIdx.y has the blocks with that blockIdx.x % 8 (one XCD under
    // round-robin dispatch; speed only), else blockIdx.y
    const bool xgrid = A.hop_mode >= 1;
    const int p = xgrid ? (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    const int pb = xgrid ? (int)((blockIdx.x & 7) + 8 * blockIdx.y) : (int)blockIdx.y;
    if (pb >= A.batch) return;
    [[maybe_unused]] const int P = xgrid ? (int)(gridDim.x >> 3) : (int)gridDim.x;
    const float* s0 = A.s0 + (size_t)pb * A.s;
    float* actions = A.actions + (size_t)pb * A.H * A.a;
    float* states_out = A.states_out + (size_t)pb * (A.H + 1) * A.s;
    int* iterations_out = A.iterations_out ? A.iterations_out + pb : nullptr;
    xchg_all += (size_t)pb * A.xchg_stride;
    status += (size_t)pb * A.xchg_stride * 2;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, g = tid >> 5, c = tid & 31;
    const int s = A.s, a = A.a, W = A.W, Wp = A.Wpad, K0 = s + a, L = A.L, H = A.H;
    const GcLds m = gc_lds(s, a, W, Wp, L, H, K0R, A.reward ? 2 : 1);
    unsigned* const mk = reinterpret_cast<unsigned*>(smem + m.mk);
    float* fw = smem + m.fw;
    float* bw = smem + m.bw;
    float* x0 = smem + m.x0;
    float* gout = smem + m.out;
    float* gs = smem + m.gs;
    float* red = smem + m.red;
    float* acts = smem + m.acts;
    float* m1 = smem + m.m1;
    float* m2 = smem + m.m2;
    float* grad = smem + m.grad;
    float* st = smem + m.st;
    int& abort_flag = *reinterpret_cast<int*>(smem + m.flag);
    const float* bias = A.packed + A.bias_off;
    const float* tw = A.packed + A.tw_base;
    gc_gu64* xchg = (gc_gu64*)xchg_all;

    if (A.debug_abort) {                       // test hook: behave as a timed-out hand-off
        if (tid == 0) atomicOr(status, 1u);
        return;
    }
    // ---- one-time staging: weight slices, register-resident layer 0 / output weights, actions
    if (tid == 0) abort_flag = 0;
    for (int k = tid; k < K0R; k += GC_THREADS) x0[k] = 0.0f;
    for (int l = 1; l < L; ++l) {
        const float* wt = tw + A.tw_off[l];                    // W^T_l [W][Wpad]
        float* f = fw + (size_t)(l - 1) * GC_ROWS * m.rs;
        float* b = bw + (size_t)(l - 1) * GC_ROWS * m.rs;
        for (int i = tid; i < GC_ROWS * W; i += GC_THREADS) {
            const int k = i >> 4, o = i & 15;
            f[o * m.rs + k] = wt[(size_t)k * Wp + p * GC_ROWS + o];   // W_l[16p + o][k]
        }
        for (int i = tid; i < GC_ROWS * W; i += GC_THREADS) {
            const int o = i / W, n = i - (i / W) * W;
            b[o * m.rs + n] = wt[(size_t)(p * GC_ROWS + o) * Wp + n];  // W_l[n][16p + o]
        }
    }
    for (int i = tid; i < H * a; i += GC_THREADS) { acts[i] = actions[i]; m1[i] = 0.f; m2[i] = 0.f; }
    for (int i = tid; i < (H + 1) * s; i += GC_THREADS) st[i] = i < s ? s0[i] : 0.f;
    for (int d = tid; d < 32; d += GC_THREADS) gout[d] = 0.f;   // entries >= s stay zero
    const bool has_unit = tid < Wp;
    const float b0 = has_unit ? bias[tid] : 0.0f;
    float w0r[K0R];                                           // W0[tid][k]
#pragma unroll
    for (int k = 0; k < K0R; ++k) w0r[k] = (has_unit && k < K0) ? tw[A.tw_off[0] + (size_t)k * Wp + tid] : 0.0f;
    const float* wo = tw + A.tw_off[L];                       // Wout [s][W]
    using Dot = CoopDot<WI>;
    float wor[SM][WI];                                        // forward: Wout[g + 16 mm][Dot::col(c, i)]
#pragma unroll
    for (int mm = 0; mm < SM; ++mm)
#pragma unroll
        for (int i = 0; i < WI; ++i) {
            const int d = g + 16 * mm, k = Dot::col(c, i);
            wor[mm][i] = (d < s && k < W) ? wo[(size_t)d * W + k] : 0.0f;
        }
    float wob[16 * SM];                                       // backward: Wout[n][tid]
#pragma unroll
    for (int n = 0; n < 16 * SM; ++n) wob[n] = (n < s && tid < W) ? wo[(size_t)n * W + tid] : 0.0f;
    // reward head (row s of the output block) and d r / d head = rew_std (unnormalise_reward)
    const float wrb = (A.reward && tid < W) ? wo[(size_t)s * W + tid] : 0.0f;
    const float grw = (A.reward && A.unnorm_r) ? A.rew_std[0] : 1.0f;
    const float* hbias = bias;                                // [L][Wpad]
    const float* obias = bias + (size_t)L * Wp;
    __syncthreads();
    // hop_mode 2: roll call (as traj_coop_kernel): XCC_IDs as granules in the parity-1 buffer, which
    // phase 1 first overwrites only after every workgroup has read them (it gathers phase 0 first)
    int& l2_flag = *(reinterpret_cast<int*>(smem + m.flag) + 1);
    if (A.hop_mode == 2) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        gc_gu64* roll = xchg + Wp;
        constexpr unsigned RTAG = 0xFFFFFFFFu;
        if (tid == 0)
            __hip_atomic_store(&roll[p], ((gc_u64)RTAG << 32) | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (wave == 0) {
            const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
            bool same = true;
            for (;;) {
                const gc_u64 gv = lane < P ? __hip_atomic_load(&roll[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : (((gc_u64)RTAG << 32) | xcc);
                if (__all((unsigned)(gv >> 32) == RTAG)) {
                    same = __all((unsigned)gv == xcc);
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t_start > 20000000ull) {   // 200 ms
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

    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;
    unsigned phase = 0;
    int done = 0;
#ifdef MBRL_STAMPS
    unsigned long long gseg[GD_NSEG] = {0, 0, 0, 0, 0, 0, 0};
    unsigned long long gprev = __builtin_amdgcn_s_memrealtime();
#endif
    float* cur = smem + m.hA;
    float* nxt = smem + m.hB;
    float* gcur = smem + m.gA;
    float* gnxt = smem + m.gB;
    // ReLU masks of layer j's output (units > 0): j = L - 1 all Wp bits (words 0 .. Wp / 32 - 1,
    // bit u % 32 of word u / 32), j < L - 1 this workgroup's units 16p .. 16p + 15 (word Wp / 32 + j,
    // bit u - 16p). Written by the forward pass from each wave's ballot; the forward's activations are
    // needed by the backward only through these signs.
    const int own_w = (GC_ROWS * p) >> 6, own_b = (GC_ROWS * p) & 63;   // the wave holding my units, bit offset
    auto put_mask = [&](unsigned* row, int j, float v) {
        const unsigned long long bal = __ballot(has_unit && v > 0.f);
        if (j == L - 1) {
            if (lane == 0 && wave < Wp / 64) {
                row[2 * wave] = (unsigned)bal;
                row[2 * wave + 1] = (unsigned)(bal >> 32);
            }
        } else if (wave == own_w && lane == 0) {
            row[Wp / 32 + j] = (unsigned)(bal >> own_b) & 0xFFFFu;
        }
    };
    // the trunk on x0 (layer 0 redundant, hidden layers through the hand-offs), masks into row;
    // leaves the last hidden vector in cur. false: a hand-off gave up.
    auto trunk = [&](unsigned* row) -> bool {
        float v0 = 0.f;
        if (has_unit) {
            float v = b0;
#pragma unroll
            for (int k = 0; k < K0R; ++k) v = fmaf(w0r[k], x0[k], v);
            v0 = fmaxf(v, 0.0f);
            cur[tid] = v0;
        }
        put_mask(row, 0, v0);
        __syncthreads();
        GSTAMP(0);
        for (int l = 1; l < L; ++l) {
            const float* f = fw + (size_t)(l - 1) * GC_ROWS * m.rs + (size_t)g * m.rs;
            float v = halfwave_sum_hi(Dot::lds(f, cur, c));
            v = fmaxf(v + hbias[(size_t)l * Wp + p * GC_ROWS + g], 0.0f);
            if (!gc_exchange<WI / 2>(xchg, Wp, p, phase, v, nxt, abort_flag, status, l2)) return false;
            float* tmp = cur; cur = nxt; nxt = tmp;
            put_mask(row, l, has_unit ? cur[tid] : 0.f);
        }
        GSTAMP(1);
        return true;
    };
    // reverse mode from gcur (d loss / d last hidden output, ReLU mask applied) through the hidden
    // layers (hand-offs) and layer 0 (redundant block reduction): use(k, d loss / d x0[k]), k < K0
    auto trunk_back = [&](const unsigned* row, auto&& use) -> bool {
        for (int l = L - 1; l >= 1; --l) {
            // my 16 input gradients of layer l: k = 16p + g, lanes over n
            const float* b = bw + (size_t)(l - 1) * GC_ROWS * m.rs + (size_t)g * m.rs;
            float v = halfwave_sum_hi(Dot::lds(b, gcur, c));
            // ReLU' of layer l - 1's output at my unit 16p + g (layer L - 1's full mask when l - 1 == L - 1
            // cannot occur here: l - 1 < L - 1)
            v = ((row[Wp / 32 + (l - 1)] >> g) & 1u) ? v : 0.f;
            if (!gc_exchange<WI / 2>(xchg, Wp, p, phase, v, gnxt, abort_flag, status, l2)) return false;
            float* tmp = gcur; gcur = gnxt; gnxt = tmp;
        }
        GSTAMP(4);
        // layer 0 backward (redundant): g_x0[k] = sum_u W0[u][k] g_z0[u], a block reduction per k
        static_assert(K0R == 32, "wave_reduce_scatter32");
        const float gu = has_unit ? gcur[tid] : 0.f;
        float vk[K0R];
#pragma unroll
        for (int k = 0; k < K0R; ++k) vk[k] = w0r[k] * gu;
        const float r = wave_reduce_scatter32(vk, lane);
        if ((lane & 1) == 0) red[wave * K0R + (lane >> 1)] = r;
        __syncthreads();
        for (int k = tid; k < K0; k += GC_THREADS) {
            float v = 0.f;
            for (int w = 0; w < GC_THREADS / 64; ++w) v += red[w * K0R + k];
            use(k, v);
        }
        __syncthreads();
        GSTAMP(5);
        return true;
    };
    for (int it = 0; it < A.iterations; ++it) {
        // ================= forward. x0 = (norm(s_t), norm(a_t)): the output lanes of step t - 1 write
        // its state part, threads d < a its action part, one barrier before layer 0
        for (int d = tid; d < K0; d += GC_THREADS) {
            if (d < s) {
                const float sv = st[d];
                x0[d] = A.norm_s ? (sv - A.obs_mean[d]) / A.obs_std[d] : sv;
            } else {
                const float av = acts[d - s];
                x0[d] = A.norm_a ? (av - A.act_mean[d - s]) / A.act_std[d - s] : av;
            }
        }
        __syncthreads();
        for (int t = 0; t < H; ++t) {
            if (!trunk(mk + (size_t)t * m.mk_row)) return;
            // output layer (redundant): half-wave g owns rows g + 16 mm; the lane holding row d's sum
            // stores s_{t+1} and its normalised copy (layer 0 read x0 before the trunk's barriers)
#pragma unroll
            for (int mm = 0; mm < SM; ++mm) {
                const float v = halfwave_sum_hi(Dot::reg(wor[mm], cur, c));
                const int d = g + 16 * mm;
                if (c == 16 && d < s) {
                    const float o = v + obias[d];
                    const float sn = A.unnorm_s ? o * A.obs_std[d] + A.obs_mean[d] : o;
                    st[(t + 1) * s + d] = sn;
                    x0[d] = A.norm_s ? (sn - A.obs_mean[d]) / A.obs_std[d] : sn;
                }
            }
            if (A.reward) {
                // the cost call's trunk pass on (norm(s_{t+1}), norm(a_t)): x0's action part still
                // holds norm(a_t); only its ReLU masks are needed for the backward pass
                __syncthreads();
                if (!trunk(mk + (size_t)(H + t) * m.mk_row)) return;
            }
            if (t + 1 < H)   // x0's action part for step t + 1 (its layer 0 reads after the barrier)
                for (int j = tid; j < a; j += GC_THREADS) {
                    const float av = acts[(t + 1) * a + j];
                    x0[s + j] = A.norm_a ? (av - A.act_mean[j]) / A.act_std[j] : av;
                }
            __syncthreads();
            GSTAMP(2);
        }
        // ================= backward, t = H-1 .. 0
        // gout[d] = d loss / d (output row d) of step t from gs[d] = d (later steps) / d s_{t+1}[d]:
        // + SmoothAbs' of the state cost at s_{t+1}, through unnormalise_state
        auto gout_of = [&](int d, float gg, int t1) {
            if (A.has_sc) {
                const float x = st[t1 * s + d] - A.goal[d];
                const float wx = x * A.cw[d];
                gg += wx * A.cw[d] / sqrtf(wx * wx + A.alpha_s * A.alpha_s);
            }
            return A.unnorm_s ? gg * A.obs_std[d] : gg;
        };
        for (int d = tid; d < 32; d += GC_THREADS) gs[d] = 0.f;
        if (!A.reward)   // step H - 1's gout (no later step); later ones come from the use() below
            for (int d = tid; d < s; d += GC_THREADS) gout[d] = gout_of(d, 0.f, H);
        __syncthreads();
        for (int t = H - 1; t >= 0; --t) {
            const unsigned* ht = mk + (size_t)t * m.mk_row;
            if (A.reward) {
                // reward pass: d r_t / d head = grw through the reward row and the pass's ReLU masks;
                // the state part joins d loss / d s_{t+1}, the action part waits in grad[t]
                const unsigned* hb = mk + (size_t)(H + t) * m.mk_row;
                if (has_unit) gcur[tid] = ((hb[tid >> 5] >> (tid & 31)) & 1u) ? wrb * grw : 0.f;
                __syncthreads();
                const bool ok = trunk_back(hb, [&](int k, float v) {
                    if (k < s) gs[k] += A.norm_s ? v / A.obs_std[k] : v;
                    else grad[t * a + k - s] = A.norm_a ? v / A.act_std[k - s] : v;
                });
                if (!ok) return;
                for (int d = tid; d < s; d += GC_THREADS) gout[d] = gout_of(d, gs[d], t + 1);
                __syncthreads();
            }
            // output layer backward (redundant): thread k = tid; ReLU mask of the last hidden layer
            if (has_unit) {
                float v = 0.f;
#pragma unroll
                for (int n = 0; n < 16 * SM; ++n) v += wob[n] * gout[n];
                gcur[tid] = ((ht[tid >> 5] >> (tid & 31)) & 1u) ? v : 0.f;
            }
            __syncthreads();
            GSTAMP(3);
            const bool ok = trunk_back(ht, [&](int k, float v) {
                if (k < s) {
                    const float gk = A.norm_s ? v / A.obs_std[k] : v;
                    gs[k] = gk;
                    // without a reward pass, step t - 1's gout follows from gk alone (read after the
                    // barrier that closes trunk_back)
                    if (!A.reward && t > 0) gout[k] = gout_of(k, gk, t);
                } else {
                    const int j = k - s;
                    float ga = A.norm_a ? v / A.act_std[j] : v;
                    if (A.has_ac) ga += A.alpha_a * sinhf(acts[t * a + j] / A.alpha_a) / (float)a;
                    if (A.reward) ga += grad[t * a + j];   // the reward pass's share (above)
                    grad[t * a + j] = ga;
                }
            });
            if (!ok) return;
        }
        // ================= Adam and the stop test (redundant, bit-identical in every workgroup)
        const float kk = (float)(it + 1);
        const float bc1 = 1.0f - powf(b1, kk), bc2 = 1.0f - powf(b2, kk);
        const float stepsz = A.lr / bc1, bc2s = sqrtf(bc2);
        float change = 0.f;
        for (int i = tid; i < H * a; i += GC_THREADS) {
            const float gg = grad[i];
            float mm = m1[i];
            mm = mm + (1.0f - b1) * (gg - mm);
            const float vv = b2 * m2[i] + (1.0f - b2) * gg * gg;
            m1[i] = mm;
            m2[i] = vv;
            const float old = acts[i];
            const float nw = old - stepsz * (mm / (sqrtf(vv) / bc2s + eps));
            acts[i] = nw;
            change += fabsf(old - nw);
        }
        {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) change += __shfl_xor(change, o, 64);
            if (lane == 0) red[wave] = change;
            __syncthreads();
            change = 0.f;
            for (int w = 0; w < GC_THREADS / 64; ++w) change += red[w];
            __syncthreads();
        }
        done = it + 1;
        GSTAMP(6);
        if (change / (float)(H * a) < A.stop) break;
    }
#ifdef MBRL_STAMPS
    if (tid == 0 && g_mbrl_gd_stamps != nullptr)
        for (int k = 0; k < GD_NSEG; ++k) g_mbrl_gd_stamps[((size_t)pb * P + p) * GD_NSEG + k] = gseg[k];
#endif
    if (p == 0) {
        for (int i = tid; i < H * a; i += GC_THREADS) actions[i] = acts[i];
        for (int i = tid; i < (H + 1) * s; i += GC_THREADS) states_out[i] = st[i];
        if (tid == 0 && iterations_out != nullptr) *iterations_out = done;
    }
}

}  // namespace

bool gd_coop_supported(const GdArgs& A) {
    const int K0 = A.s + A.a;
    if (A.L < 2 || A.W != A.Wpad || A.Wpad > GC_THREADS || A.Wpad < 64 || K0 > 32 || A.s > 32) return false;
    return gc_lds(A.s, A.a, A.W, A.Wpad, A.L, A.H, 32, A.reward ? 2 : 1).total <= 160 * 1024;
}

template <int WI>
static hipError_t launch_gd_coop_w(const GdArgs& A, gc_u64* xchg, unsigned* status, hipStream_t stream) {
    const auto fn = &gd_coop_kernel<32, 2, WI>;
    hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(fn), 160 * 1024);
    if (err != hipSuccess) return err;
    const size_t lds = gc_lds(A.s, A.a, A.W, A.Wpad, A.L, A.H, 32, A.reward ? 2 : 1).total;
    const int P = A.Wpad / GC_ROWS;
    if (!grid_fits(reinterpret_cast<const void*>(fn), GC_THREADS, lds, P * A.batch))
        return hipErrorCooperativeLaunchTooLarge;
    // the per-XCD grid puts ceil(batch / 8) plans' P workgroups on each XCD: they must fit one XCD's
    // share of the device (an eighth of the capacity), else the (P, batch) grid
    GdArgs B = A;
    if (B.hop_mode >= 1 && !grid_fits(reinterpret_cast<const void*>(fn), GC_THREADS, lds, 8 * P * ((B.batch + 7) / 8)))
        B.hop_mode = 0;
    if (B.hop_mode >= 1)   // plan b on the blocks with blockIdx.x % 8 == b % 8 (grid.y: groups of 8 plans)
        hipLaunchKernelGGL(fn, dim3(8 * P, (B.batch + 7) / 8), dim3(GC_THREADS), lds, stream, B, xchg, status);
    else
        hipLaunchKernelGGL(fn, dim3(P, B.batch), dim3(GC_THREADS), lds, stream, B, xchg, status);
    return hipGetLastError();
}

hipError_t launch_gd_coop(const GdArgs& A, unsigned long long* xchg, unsigned* status, hipStream_t stream) {
    // zero the granules and the status words (each plan's block: granules, then its status word)
    hipError_t err = hipMemsetAsync(xchg, 0, (size_t)A.batch * A.xchg_stride * 8, stream);
    if (err != hipSuccess) return err;
    switch (A.Wpad) {
        case 64: return launch_gd_coop_w<2>(A, xchg, status, stream);
        case 128: return launch_gd_coop_w<4>(A, xchg, status, stream);
        case 256: return launch_gd_coop_w<8>(A, xchg, status, stream);
        case 512: return launch_gd_coop_w<16>(A, xchg, status, stream);
        default: return hipErrorInvalidValue;
    }
}

size_t gd_lds_bytes(int s, int a, int Wpad, int H) { return gd_lds(s, a, Wpad, H, nullptr).floats * sizeof(float); }

hipError_t launch_gd_plan(const GdArgs& A, hipStream_t stream) {
    const size_t lds = gd_lds_bytes(A.s, A.a, A.Wpad, A.H);
    // the kernel also has a few bytes of static LDS: raise the dynamic limit to what it needs, not 160 KiB
    hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(&gd_plan_kernel), (int)lds);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(gd_plan_kernel, dim3(1, A.batch), dim3(GD_THREADS), lds, stream, A);
    return hipGetLastError();
}

}  // namespace mbrl

#ifdef MBRL_STAMPS
extern "C" int mbrl_diag_set_gd_stamps(void* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mbrl::g_mbrl_gd_stamps), &buf, sizeof(buf));
}
#endif
