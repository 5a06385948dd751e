// Grid-barrier latency on MI355X: persistent grid (1 WG per CU), N barriers.
// Variants: 0 = agent-scope release/acquire (compiler memory model: wbl2 + inv),
//           1 = relaxed (lower bound, no data ordering),
//           2 = variant 0 + data exchange check (each WG publishes 64 floats, all read all).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ bool grid_sync(unsigned* c, unsigned target, bool fenced) {
    __shared__ int ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        if (fenced) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int spins = 0;
        ok = 1;
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1 << 20)) { ok = 0; break; }  // bounded: never hang the device
        }
        if (fenced) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return ok;
}

__global__ void bar_kernel(unsigned* c, float* data, int n, int variant, int* err) {
    for (int i = 0; i < n; ++i) {
        if (variant == 2) {
            if (threadIdx.x < 64) data[(size_t)(i & 1) * gridDim.x * 64 + blockIdx.x * 64 + threadIdx.x] = (float)(i + blockIdx.x);
        }
        if (!grid_sync(c, (unsigned)(i + 1) * gridDim.x, variant != 1)) {
            if (threadIdx.x == 0) atomicAdd(err, 1000000);
            return;
        }
        if (variant == 2) {
            const float* d = data + (size_t)(i & 1) * gridDim.x * 64;
            for (int j = threadIdx.x; j < (int)gridDim.x * 64; j += blockDim.x)
                if (d[j] != (float)(i + j / 64)) atomicAdd(err, 1);
        }
    }
}

int main(int argc, char** argv) {
    int n = 2000;
    int grids[] = {64, 128, 256};
    unsigned* c;
    float* data;
    int* err;
    hipMalloc(&c, 4);
    hipMalloc(&data, 2 * 1024 * 64 * 4);
    hipMalloc(&err, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int v = 0; v < 3; ++v)
        for (int g : grids) {
            for (int threads : {256, 512}) {
                hipMemset(c, 0, 4);
                hipMemset(err, 0, 4);
                hipLaunchKernelGGL(bar_kernel, dim3(g), dim3(threads), 0, 0, c, data, 10, v, err);
                hipMemset(c, 0, 4);
                hipDeviceSynchronize();
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(bar_kernel, dim3(g), dim3(threads), 0, 0, c, data, n, v, err);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                unsigned cnt;
                int e;
                hipMemcpy(&cnt, c, 4, hipMemcpyDeviceToHost);
                hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
                printf("variant=%d grid=%d threads=%d : %.3f us/barrier  (count %u/%u, data errors %d)\n", v, g, threads,
                       ms * 1000.0 / n, cnt, (unsigned)n * g, e);
            }
        }
    return 0;
}
