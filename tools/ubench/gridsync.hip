// Microbenchmark: cost of a grid-wide barrier for a persistent kernel of one 1024-thread workgroup
// per CU -- cooperative_groups grid.sync() vs a hand-rolled agent-scope counter barrier.
// hipcc --offload-arch=gfx950 -O3 -o /tmp/gridsync tools/ubench/gridsync.hip && /tmp/gridsync
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <stdio.h>

namespace cg = cooperative_groups;

__global__ __launch_bounds__(1024) void cg_sync(int iters, unsigned* sink) {
    cg::grid_group g = cg::this_grid();
    unsigned acc = 0;
    for (int i = 0; i < iters; ++i) {
        acc += blockIdx.x ^ i;
        g.sync();
    }
    if (threadIdx.x == 0) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(1024) void own_sync(int iters, unsigned* count, unsigned* gen, unsigned* sink) {
    unsigned acc = 0;
    __shared__ unsigned my_gen;
    if (threadIdx.x == 0) my_gen = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    for (int i = 0; i < iters; ++i) {
        acc += blockIdx.x ^ i;
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned g = my_gen;
            const unsigned a = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (a == gridDim.x - 1) {
                __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                long n = 0;
                while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g && ++n < 100000000)
                    __builtin_amdgcn_s_sleep(1);
            }
            my_gen = g + 1;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) sink[blockIdx.x] = acc;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *sink, *cnt, *gen;
    hipMalloc(&sink, 4096 * 4);
    hipMalloc(&cnt, 4);
    hipMalloc(&gen, 4);
    hipMemset(cnt, 0, 4);
    hipMemset(gen, 0, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int iters : {1, 101}) {
        int it = iters;
        void* args[] = {&it, &sink};
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            hipError_t e = hipLaunchCooperativeKernel((void*)cg_sync, dim3(cus), dim3(1024), args, 0, 0);
            hipEventRecord(b);
            hipEventSynchronize(b);
            if (e != hipSuccess) { printf("coop launch failed: %s\n", hipGetErrorString(e)); return 1; }
            hipEventElapsedTime(&ms, a, b);
        }
        printf("cg grid.sync   %d WGs  iters %3d  %8.2f us\n", cus, iters, ms * 1000);
    }
    for (int iters : {1, 101}) {
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(own_sync, dim3(cus), dim3(1024), 0, 0, iters, cnt, gen, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        printf("own barrier    %d WGs  iters %3d  %8.2f us\n", cus, iters, ms * 1000);
    }
    return 0;
}
