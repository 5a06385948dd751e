// Dataflow-phase latency on MI355X for a persistent decoder: 256 WGs (1 per CU), each phase
// every WG publishes a 64-float slice of an activation vector and a per-WG flag, waits for
// all flags, then reads the whole vector (R x 1280 f32 = 40 KB at R=8) and checks it.
// mode 0: flag array, agent-scope release store / acquire fence (wbl2 + inv)
// mode 1: single atomic counter (release add), acquire fence
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NT = 512;

__device__ __forceinline__ bool wait_flags(const unsigned* flags, int n, unsigned seq) {
    // wave 0 polls; every lane checks up to 4 flags
    __shared__ int ok;
    if (threadIdx.x < 64) {
        int spins = 0;
        bool done = false;
        while (!done) {
            bool mine = true;
            for (int i = threadIdx.x; i < n; i += 64)
                mine &= __hip_atomic_load(flags + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= seq;
            done = __all(mine);
            if (!done && ++spins > (1 << 20)) break;
        }
        if (threadIdx.x == 0) ok = done;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return ok;
}

__global__ __launch_bounds__(NT) void phase_kernel(unsigned* flags, unsigned* counter, float* x, int n_phases,
                                                   int mode, int per_wg, int* err) {
    const int wg = blockIdx.x, G = gridDim.x, tid = threadIdx.x;
    const int len = G * per_wg;
    __shared__ float red[NT / 64];
    for (int p = 1; p <= n_phases; ++p) {
        float* buf = x + (size_t)(p & 1) * len;
        if (tid < per_wg) buf[wg * per_wg + tid] = (float)(p + wg);
        __syncthreads();
        bool ok;
        if (mode == 0) {
            if (tid == 0) __hip_atomic_store(flags + wg, (unsigned)p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            ok = wait_flags(flags, G, (unsigned)p);
        } else {
            __shared__ int sok;
            if (tid == 0) {
                __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                int spins = 0;
                sok = 1;
                while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(p * G))
                    if (++spins > (1 << 20)) { sok = 0; break; }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            __syncthreads();
            ok = sok;
        }
        if (!ok) {
            if (tid == 0) atomicAdd(err, 1000000);
            return;
        }
        // consume the whole vector (vectorised)
        float s = 0.f;
        const float4* b4 = (const float4*)buf;
        for (int i = tid; i < len / 4; i += NT) {
            float4 v = b4[i];
            s += v.x + v.y + v.z + v.w;
        }
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((tid & 63) == 0) red[tid >> 6] = s;
        __syncthreads();
        if (tid == 0) {
            float t = 0.f;
            for (int w = 0; w < NT / 64; ++w) t += red[w];
            // expected: sum_wg per_wg*(p+wg)
            const float e = (float)per_wg * ((float)p * G + 0.5f * G * (G - 1));
            if (fabsf(t - e) > 1e-3f * e) atomicAdd(err, 1);
        }
    }
}

int main() {
    unsigned *flags, *counter;
    float* x;
    int* err;
    (void)hipMalloc(&flags, 4096);
    (void)hipMalloc(&counter, 4);
    (void)hipMalloc(&x, 2 * 256 * 64 * 4 * 4);
    (void)hipMalloc(&err, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int n = 2000;
    for (int mode = 0; mode < 2; ++mode)
        for (int g : {80, 256})
            for (int per_wg : {40, 160}) {
                (void)hipMemset(flags, 0, 4096);
                (void)hipMemset(counter, 0, 4);
                (void)hipMemset(err, 0, 4);
                (void)hipDeviceSynchronize();
                (void)hipEventRecord(e0, 0);
                hipLaunchKernelGGL(phase_kernel, dim3(g), dim3(NT), 0, 0, flags, counter, x, n, mode, per_wg, err);
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                int e;
                (void)hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
                printf("mode=%d grid=%d vector=%d KB : %.3f us/phase  errors %d\n", mode, g, g * per_wg * 4 / 1024,
                       ms * 1000.0 / n, e);
            }
    return 0;
}
