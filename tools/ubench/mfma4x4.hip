// Microtest for the 8-candidate rollout tile: the operand / result lane layout of
// v_mfma_f32_4x4x1_16b_f32 with A broadcast (CBSZ = 1, ABID = 0 / 1), and whether a chain of them
// in the k order the 16x16x4 rollout kernel consumes reproduces that kernel's sums bit for bit.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma4x4 tools/ubench/mfma4x4.hip && /tmp/mfma4x4
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// layout probe: out[(mode * 64 + lane) * 4 + v] = D for A = a_in[lane], B = b_in[lane]
__global__ void probe(const float* a_in, const float* b_in, float* out) {
    const int l = threadIdx.x;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    f32x4 d0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a_in[l], b_in[l], z, 0, 0, 0);
    f32x4 d1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a_in[l], b_in[l], z, 1, 0, 0);
    f32x4 d2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a_in[l], b_in[l], z, 1, 1, 0);
    for (int v = 0; v < 4; ++v) {
        out[(0 * 64 + l) * 4 + v] = d0[v];
        out[(1 * 64 + l) * 4 + v] = d1[v];
        out[(2 * 64 + l) * 4 + v] = d2[v];
    }
}

constexpr int K = 64;
// W [32][K] row-major, X [K][16]. y16[32][16] by 16x16x4 (rollout-kernel order), y4[32][8] by 4x4x1
// (two tiles of 32 rows packed in one A register: ABID 0 = rows 0..31 from even blocks... here one
// tile: rows 4*(l>>3) + (l&3) from even blocks, the second "tile" = rows + 32 is not needed), yv by
// a VALU fmaf chain in the same k order.
__global__ void chains(const float* W, const float* X, float* y16, float* y4, float* yv) {
    const int l = threadIdx.x;
    // (a) 16x16x4: A = weights lane l: W[16t + (l&15)][16kc + 4(l>>4) + s]; B = X[same k][l&15]
    for (int t = 0; t < 2; ++t) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int kc = 0; kc < K / 16; ++kc)
            for (int s = 0; s < 4; ++s) {
                const int k = 16 * kc + 4 * (l >> 4) + s;
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(W[(16 * t + (l & 15)) * K + k], X[k * 16 + (l & 15)], acc, 0, 0, 0);
            }
        for (int v = 0; v < 4; ++v) y16[(16 * t + 4 * (l >> 4) + v) * 16 + (l & 15)] = acc[v];
    }
    // (b) 4x4x1_16b, blocks b = 2 rs + cg, A broadcast within block pairs (CBSZ 1): even-block lanes
    // carry tile 0's A (ABID 0), odd-block lanes tile 1's (ABID 1); here tile 1 = the same rows, so
    // both results must agree. k order: chunk kc, step s, then q: k = 16 kc + 4 q + s.
    {
        const int row = 4 * (l >> 3) + (l & 3);
        const int cand = l & 7;
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
        for (int kc = 0; kc < K / 16; ++kc)
            for (int s = 0; s < 4; ++s)
                for (int q = 0; q < 4; ++q) {
                    const int k = 16 * kc + 4 * q + s;
                    const float w = W[row * K + k];
                    const float x = X[k * 16 + cand];
                    a0 = __builtin_amdgcn_mfma_f32_4x4x1f32(w, x, a0, 1, 0, 0);
                    a1 = __builtin_amdgcn_mfma_f32_4x4x1f32(w, x, a1, 1, 1, 0);
                }
        for (int v = 0; v < 4; ++v) {
            y4[(4 * (l >> 3) + v) * 8 + cand] = a0[v];
            y4[32 * 8 + (4 * (l >> 3) + v) * 8 + cand] = a1[v];
        }
    }
    // (c) VALU fmaf chain, same order
    if (l < 32) {
        for (int c = 0; c < 8; ++c) {
            float y = 0.f;
            for (int kc = 0; kc < K / 16; ++kc)
                for (int s = 0; s < 4; ++s)
                    for (int q = 0; q < 4; ++q) {
                        const int k = 16 * kc + 4 * q + s;
                        y = __builtin_fmaf(W[l * K + k], X[k * 16 + c], y);
                    }
            yv[l * 8 + c] = y;
        }
    }
}

int main() {
    float ha[64], hb[64], hout[3 * 64 * 4];
    float *da, *db, *dout;
    CHECK(hipMalloc(&da, 256)); CHECK(hipMalloc(&db, 256)); CHECK(hipMalloc(&dout, sizeof(hout)));
    // A = lane + 1, B = 1: D shows which A lane feeds each (lane, v); then the reverse
    for (int pass = 0; pass < 2; ++pass) {
        for (int l = 0; l < 64; ++l) { ha[l] = pass ? 1.f : (float)(l + 1); hb[l] = pass ? (float)(l + 1) : 1.f; }
        CHECK(hipMemcpy(da, ha, 256, hipMemcpyHostToDevice)); CHECK(hipMemcpy(db, hb, 256, hipMemcpyHostToDevice));
        probe<<<1, 64>>>(da, db, dout);
        CHECK(hipMemcpy(hout, dout, sizeof(hout), hipMemcpyDeviceToHost));
        for (int mode = 0; mode < 3; ++mode) {
            printf("%s source lane of D (cbsz/abid mode %d), lanes 0..15 x v:", pass ? "B" : "A", mode);
            for (int l = 0; l < 16; ++l) {
                printf(" [");
                for (int v = 0; v < 4; ++v) printf("%d%s", (int)hout[(mode * 64 + l) * 4 + v] - 1, v < 3 ? "," : "");
                printf("]");
            }
            printf("\n");
        }
    }
    // bitwise chains
    static float hW[32 * K], hX[K * 16], h16[32 * 16], h4[2 * 32 * 8], hv[32 * 8];
    srand(7);
    for (int i = 0; i < 32 * K; ++i) hW[i] = (float)rand() / RAND_MAX * 2.f - 1.f;
    for (int i = 0; i < K * 16; ++i) hX[i] = (float)rand() / RAND_MAX * 2.f - 1.f;
    float *dW, *dX, *d16, *d4, *dv;
    CHECK(hipMalloc(&dW, sizeof(hW))); CHECK(hipMalloc(&dX, sizeof(hX)));
    CHECK(hipMalloc(&d16, sizeof(h16))); CHECK(hipMalloc(&d4, sizeof(h4))); CHECK(hipMalloc(&dv, sizeof(hv)));
    CHECK(hipMemcpy(dW, hW, sizeof(hW), hipMemcpyHostToDevice)); CHECK(hipMemcpy(dX, hX, sizeof(hX), hipMemcpyHostToDevice));
    chains<<<1, 64>>>(dW, dX, d16, d4, dv);
    CHECK(hipMemcpy(h16, d16, sizeof(h16), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(h4, d4, sizeof(h4), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hv, dv, sizeof(hv), hipMemcpyDeviceToHost));
    int diff16v = 0, diff4v = 0, diff4ab = 0;
    double maxrel = 0;
    for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 8; ++c) {
            const float v = hv[r * 8 + c], a = h16[r * 16 + c], b = h4[r * 8 + c], b1 = h4[256 + r * 8 + c];
            diff16v += memcmp(&a, &v, 4) != 0;
            diff4v += memcmp(&b, &v, 4) != 0;
            diff4ab += memcmp(&b, &b1, 4) != 0;
            maxrel = fmax(maxrel, fabs((double)b - a) / fmax(fabs((double)a), 1e-30));
        }
    printf("bitwise mismatches of 256: 16x16x4 vs fmaf chain %d, 4x4x1 vs fmaf chain %d, 4x4x1 abid0 vs abid1 %d; "
           "max rel 4x4 vs 16x16 %.3g\n", diff16v, diff4v, diff4ab, maxrel);
    return 0;
}
