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
    const GdLds m = gd_lds(A.s, A.a, A.Wpad, A.H, smem);
    const int tid = threadIdx.x;
    const int s = A.s, a = A.a, Wp = A.Wpad, K0 = s + a, L = A.L, H = A.H;
    const int rowf = A.hist_row;                       // floats per step in hist: K0p + L * Wpad
    const int K0p = (K0 + 3) & ~3;
    const float* bias = A.packed + A.bias_off;
    const float* tw = A.packed + A.tw_base;
    const float* wout = tw + A.tw_off[L];              // [s][W] row-major
    const float* bout = bias + (size_t)L * Wp;
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-8f;

    for (int i = tid; i < H * a; i += GD_THREADS) { A.m[i] = 0.f; A.v[i] = 0.f; }
    // the reference's states tensor before any iteration: s0, then zeros (returned as is when
    // num_iterations == 0)
    for (int i = tid; i < (H + 1) * s; i += GD_THREADS) A.states_out[i] = i < s ? A.s0[i] : 0.f;
    __syncthreads();
    int done = 0;
    for (int it = 0; it < A.iterations; ++it) {
        // ---------------- forward: the rollout of the current actions (states_out rows 0..H)
        for (int d = tid; d < s; d += GD_THREADS) A.states_out[d] = A.s0[d];
        __syncthreads();
        for (int t = 0; t < H; ++t) {
            float* hist = A.hist + (size_t)t * rowf;
            for (int d = tid; d < K0; d += GD_THREADS) {
                float v;
                if (d < s) {
                    const float sv = A.states_out[(size_t)t * s + d];
                    v = A.norm_s ? (sv - A.obs_mean[d]) / A.obs_std[d] : sv;
                } else {
                    const float av = A.actions[t * a + d - s];
                    v = A.norm_a ? (av - A.act_mean[d - s]) / A.act_std[d - s] : av;
                }
                m.x[d] = v;
                hist[d] = v;
            }
            __syncthreads();
            gd_dense_relu(tw + A.tw_off[0], bias, K0, Wp, m.x, m.part, m.h);
            for (int n = tid; n < Wp; n += GD_THREADS) hist[K0p + n] = m.h[n];
            for (int l = 1; l < L; ++l) {
                gd_dense_relu(tw + A.tw_off[l], bias + (size_t)l * Wp, A.W, Wp, m.h, m.part, m.x);
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
                    A.states_out[(size_t)(t + 1) * s + n] = A.unnorm_s ? o * A.obs_std[n] + A.obs_mean[n] : o;
                }
            }
            __threadfence_block();
            __syncthreads();
        }
        // ---------------- backward: d loss / d a, t = H-1 .. 0
        for (int d = tid; d < s; d += GD_THREADS) m.gs[d] = 0.f;
        __syncthreads();
        for (int t = H - 1; t >= 0; --t) {
            const float* hist = A.hist + (size_t)t * rowf;
            // gs += d SmoothAbs / d s_{t+1}; g_out = gs * obs_std (s_{t+1} = out * std + mean)
            for (int d = tid; d < s; d += GD_THREADS) {
                float g = m.gs[d];
                if (A.has_sc) {
                    const float x = A.states_out[(size_t)(t + 1) * s + d] - A.goal[d];
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
                gd_dense_back(tw + A.tw_off[l], A.W, Wp, m.gz, m.gx);
                const float* hp = hist + K0p + (size_t)(l - 1) * Wp;
                for (int k = tid; k < Wp; k += GD_THREADS) m.gz[k] = (k < A.W && hp[k] > 0.f) ? m.gx[k] : 0.f;
                __syncthreads();
            }
            gd_dense_back(tw + A.tw_off[0], K0, Wp, m.gz, m.gx);
            // split the input gradient: state part -> step t-1, action part -> grad of a_t
            for (int d = tid; d < K0; d += GD_THREADS) {
                const float g = m.gx[d];
                if (d < s) {
                    m.gs[d] = A.norm_s ? g / A.obs_std[d] : g;
                } else {
                    const int j = d - s;
                    float ga = A.norm_a ? g / A.act_std[j] : g;
                    if (A.has_ac)
                        ga += A.alpha_a * sinhf(A.actions[t * a + j] / A.alpha_a) / (float)a;
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
            float mm = A.m[i];
            mm = mm + (1.0f - b1) * (g - mm);
            const float vv = b2 * A.v[i] + (1.0f - b2) * g * g;
            A.m[i] = mm;
            A.v[i] = vv;
            const float old = A.actions[i];
            const float nw = old - step * (mm / (sqrtf(vv) / bc2s + eps));
            A.actions[i] = nw;
            change += fabsf(old - nw);
        }
        __threadfence_block();
        change = gd_block_sum(change, m.red);
        done = it + 1;
        if (change / (float)(H * a) < A.stop) break;
    }
    if (tid == 0 && A.iterations_out != nullptr) *A.iterations_out = done;
}

}  // namespace

size_t gd_lds_bytes(int s, int a, int Wpad, int H) { return gd_lds(s, a, Wpad, H, nullptr).floats * sizeof(float); }

hipError_t launch_gd_plan(const GdArgs& A, hipStream_t stream) {
    const size_t lds = gd_lds_bytes(A.s, A.a, A.Wpad, A.H);
    hipError_t err = ensure_dynamic_lds(reinterpret_cast<const void*>(&gd_plan_kernel), 160 * 1024);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(gd_plan_kernel, dim3(1), dim3(GD_THREADS), lds, stream, A);
    return hipGetLastError();
}

}  // namespace mbrl
