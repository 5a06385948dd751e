// k_init.hip -- on-device synthetic weight generation (no checkpoint I/O in the
// benchmark path) and small utility kernels.
//
// The generator is the counter-based splitmix64 stream documented in DESIGN.md
// (§Synthetic weights); every value is u * 2^e with u in [-1, 1) carrying 24
// significant bits, so it is exact in f32 and bit-identical to the CPU oracle's
// generator (oracle/wo_model.c: urand / gen_tensor).  Matrices of the bf16 model
// are rounded to bf16 with round-to-nearest-even, exactly as the oracle does.
#include "common.h"
#include "kernels.h"
#include "ggml_quant.h"

namespace spt {

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float urand(uint64_t seed, uint32_t tid, uint64_t i) {
    const uint64_t x = i + ((uint64_t)tid << 32) + seed * 0xD1B54A32D192ED03ULL;
    const uint64_t z = mix64(x);
    return (float)(uint32_t)(z >> 40) * (1.0f / 8388608.0f) - 1.0f;
}
__device__ __forceinline__ float wvalue(uint64_t seed, uint32_t tid, uint64_t i, int kind, float scale) {
    float v = urand(seed, tid, i) * scale;  // exact: scale is a power of two
    if (kind == WK_LNW) v = 1.0f + v;       // one rounding, same as the oracle
    return v;
}

template <typename T>
__global__ void gen_kernel(T* dst, int64_t n, uint64_t seed, uint32_t tid, int kind, float scale) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = from_f<T>(wvalue(seed, tid, (uint64_t)i, kind, scale));
}

template <typename T>
__global__ void gen_conv_kernel(T* dst, int N, int C, int Cp, uint64_t seed, uint32_t tid, float scale) {
    const int64_t total = (int64_t)N * 3 * Cp;
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(o % Cp);
        const int64_t nj = o / Cp;
        const int j = (int)(nj % 3);
        const int64_t nn = nj / 3;
        float v = 0.0f;
        if (c < C) v = wvalue(seed, tid, (uint64_t)((nn * C + c) * 3 + j), WK_MAT, scale);
        dst[o] = from_f<T>(v);
    }
}

__global__ void fill_kernel(float* dst, int64_t n, float v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = v;
}

template <typename T>
__global__ void checksum_kernel(const T* src, int64_t n, double* out) {
    __shared__ double sa[256], sb[256];
    double a = 0, b = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double v = (double)to_f<T>(src[i]);
        a += fabs(v);
        b += v;
    }
    sa[threadIdx.x] = a;
    sb[threadIdx.x] = b;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sa[threadIdx.x] += sa[threadIdx.x + s];
            sb[threadIdx.x] += sb[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicAdd(&out[0], sa[0]);
        atomicAdd(&out[1], sb[0]);
    }
}

inline int grid_for(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace

void gen_weights(int store_dtype, void* dst, int64_t n, uint64_t seed, uint32_t tid, int kind, int scale_exp,
                 hipStream_t st) {
    const float scale = ldexpf(1.0f, scale_exp);
    if (store_dtype == DT_BF16)
        hipLaunchKernelGGL(gen_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (bf16*)dst, n, seed, tid, kind, scale);
    else if (store_dtype == DT_F16)
        hipLaunchKernelGGL(gen_kernel<f16>, dim3(grid_for(n)), dim3(256), 0, st, (f16*)dst, n, seed, tid, kind, scale);
    else
        hipLaunchKernelGGL(gen_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (float*)dst, n, seed, tid, kind, scale);
}

void gen_conv_weights(int store_dtype, void* dst, int N, int C, int Cp, uint64_t seed, uint32_t tid, int scale_exp,
                      hipStream_t st) {
    const float scale = ldexpf(1.0f, scale_exp);
    const int64_t n = (int64_t)N * 3 * Cp;
    if (store_dtype == DT_BF16)
        hipLaunchKernelGGL(gen_conv_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, (bf16*)dst, N, C, Cp, seed, tid, scale);
    else
        hipLaunchKernelGGL(gen_conv_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, (float*)dst, N, C, Cp, seed, tid, scale);
}

// read a byte range once (16 B per lane, grid-stride): evicts the Infinity Cache / L2 before a
// measured launch so it sees the cold caches it meets inside the decode loop
__global__ __launch_bounds__(256) void touch_kernel(const uint4* __restrict__ p, int64_t n16, unsigned* sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u && threadIdx.x == 0x3ff) *sink = acc;  // keeps the loads; never true
}

void cache_flush(const void* p, int64_t bytes, unsigned* sink, hipStream_t st) {
    hipLaunchKernelGGL(touch_kernel, dim3(2048), dim3(256), 0, st, (const uint4*)p, bytes >> 4, sink);
}

// developer bandwidth probe: grid-stride 16 B per lane, 4 loads in flight per lane
__global__ void stream_kernel(const uint4* __restrict__ p, int64_t n16, unsigned* sink) {
    uint32_t acc = 0;
    const int64_t s = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * s < n16; i += 4 * s) {
        const uint4 a = p[i], b = p[i + s], c = p[i + 2 * s], d = p[i + 3 * s];
        acc ^= a.x ^ b.y ^ c.z ^ d.w;
    }
    for (; i < n16; i += s) acc ^= p[i].x;
    if (acc == 0x9e3779b9u && threadIdx.x == 0x3ff) *sink = acc;
}

void stream_read(const void* p, int64_t bytes, unsigned* sink, int grid, int tpb, hipStream_t st) {
    hipLaunchKernelGGL(stream_kernel, dim3(grid), dim3(tpb), 0, st, (const uint4*)p, bytes >> 4, sink);
}

// ---------------------------------------------------------------- ggml weight dequantisation
// Model loading (ggml_file.h): the raw ggml blocks are copied to the device as they lie in the
// file and expanded here into the engine's storage type, one thread per block (per element for
// f32 / f16), by the routine the host shares (ggml_quant.h); values are f32, then rounded once
// to bf16 (RNE) for a bf16 engine.
namespace {
template <typename T>
__global__ __launch_bounds__(256) void dequant_kernel(int type, const uint8_t* __restrict__ src, int64_t n,
                                                      T* __restrict__ dst) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    if (type == GQ_F32 || type == GQ_F16) {
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
            dst[i] = from_f<T>(type == GQ_F32 ? ((const float*)src)[i] : gq_half(src + 2 * i));
        return;
    }
    int blck, bytes;
    ggml_block_geom(type, &blck, &bytes);
    for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < n / blck; b += stride) {
        T* o = dst + b * blck;
        ggml_dequant_block(type, src + b * bytes, [o](int i, float v) { o[i] = from_f<T>(v); });
    }
}
}  // namespace

void ggml_dequant(int type, const void* src, int64_t n, int out_dtype, void* dst, hipStream_t st) {
    int blck, bytes;
    ggml_block_geom(type, &blck, &bytes);
    if (!blck || n % blck) throw std::runtime_error("ggml_dequant: unsupported type or ragged tensor");
    const int g = grid_for(n / blck);
    if (out_dtype == DT_BF16)
        hipLaunchKernelGGL(dequant_kernel<bf16>, dim3(g), dim3(256), 0, st, type, (const uint8_t*)src, n, (bf16*)dst);
    else
        hipLaunchKernelGGL(dequant_kernel<float>, dim3(g), dim3(256), 0, st, type, (const uint8_t*)src, n, (float*)dst);
    SPT_LAUNCH_CHECK();
}

void fill_f32(float* dst, int64_t n, float v, hipStream_t st) {
    hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, st, dst, n, v);
}

void tensor_checksum(int dtype, const void* src, int64_t n, double* out2, hipStream_t st) {
    int g = grid_for(n);
    if (g > 1024) g = 1024;
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(checksum_kernel<bf16>, dim3(g), dim3(256), 0, st, (const bf16*)src, n, out2);
    else if (dtype == DT_F16)
        hipLaunchKernelGGL(checksum_kernel<f16>, dim3(g), dim3(256), 0, st, (const f16*)src, n, out2);
    else
        hipLaunchKernelGGL(checksum_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)src, n, out2);
}

}  // namespace spt
