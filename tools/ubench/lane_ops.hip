// Lane-permutation semantics on gfx950 (one wave): for each primitive, which source lane each lane
// reads. Prints one line per primitive: the 64 source lanes.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define DPP(v, c) __builtin_amdgcn_mov_dpp((v), (c), 0xF, 0xF, false)

__global__ void probe(int* out) {
    const int l = threadIdx.x;
    const unsigned x = (unsigned)l, y = (unsigned)(100 + l);
    auto r32 = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    auto r16 = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    out[0 * 64 + l] = (int)r32[0];
    out[1 * 64 + l] = (int)r32[1];
    out[2 * 64 + l] = (int)r16[0];
    out[3 * 64 + l] = (int)r16[1];
    out[4 * 64 + l] = DPP(l, 0x128);
    out[5 * 64 + l] = DPP(l, 0x141);
    out[6 * 64 + l] = DPP(DPP(l, 0x141), 0x1B);
    out[7 * 64 + l] = DPP(l, 0x4E);
    out[8 * 64 + l] = DPP(l, 0xB1);
}

int main() {
    int* d;
    int h[9 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[9] = {"permlane32_swap[0]", "permlane32_swap[1]", "permlane16_swap[0]", "permlane16_swap[1]",
                            "row_ror:8", "row_half_mirror", "half_mirror+quad_mirror", "quad_perm 2301",
                            "quad_perm 1032"};
    for (int k = 0; k < 9; ++k) {
        printf("%-26s", names[k]);
        for (int l = 0; l < 64; ++l) printf(" %d", h[k * 64 + l]);
        printf("\n");
    }
    (void)hipFree(d);
    return 0;
}
