// k_norm.hip -- LayerNorm (eps 1e-5) of the f32 residual stream into the GEMM
// input dtype.  Replaces ggml_norm + ggml_mul + ggml_add of whisper.cpp's
// encoder blocks (pre-attention / pre-MLP LN and ln_post).  One wave per row,
// the whole row held in registers as float4 (d <= 1280 -> 5 per lane), two-pass
// mean / variance like ggml_compute_forward_norm_f32; HBM-bound.
#include "common.h"
#include "kernels.h"

namespace spt {

namespace {

template <typename T> __device__ __forceinline__ void store4(T* p, float a, float b, float c, float d);
template <> __device__ __forceinline__ void store4<float>(float* p, float a, float b, float c, float d) {
    *(float4*)p = make_float4(a, b, c, d);
}
template <> __device__ __forceinline__ void store4<bf16>(bf16* p, float a, float b, float c, float d) {
    *(uint2*)p = make_uint2(pack_bf2(a, b), pack_bf2(c, d));
}

// Every load of a row (x, gamma, beta) is issued up front from a clamped index and masked after
// use: under a per-element `idx < n4` guard hipcc branches around each load and waits on it in
// turn (r3: 19.7 us per launch at 12000 x 1280, 0.58 of HBM peak).
template <typename T, int NV>
__global__ __launch_bounds__(256) void ln_kernel(const float* __restrict__ x, int M, int d,
                                                 const float* __restrict__ w, const float* __restrict__ bb,
                                                 T* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int n4 = d >> 2;
    const float4* xr = (const float4*)(x + (size_t)row * d);
    const float4* w4 = (const float4*)w;
    const float4* b4 = (const float4*)bb;
    float4 v[NV], g[NV], o[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int idx = min(lane + 64 * i, n4 - 1);
        v[i] = xr[idx];
        g[i] = w4[idx];
        o[i] = b4[idx];
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        if (lane + 64 * i >= n4) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    const float mean = wave_sum(s) / (float)d;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        if (lane + 64 * i < n4) {
            const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, e = v[i].w - mean;
            s2 += (a * a + b * b) + (c * c + e * e);
        }
    }
    const float rstd = 1.0f / sqrtf(wave_sum(s2) / (float)d + 1e-5f);
    T* yr = y + (size_t)row * d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int idx = lane + 64 * i;
        if (idx < n4)
            store4<T>(yr + 4 * idx, (v[i].x - mean) * rstd * g[i].x + o[i].x, (v[i].y - mean) * rstd * g[i].y + o[i].y,
                      (v[i].z - mean) * rstd * g[i].z + o[i].z, (v[i].w - mean) * rstd * g[i].w + o[i].w);
    }
}

template <> __device__ __forceinline__ void store4<f16>(f16* p, float a, float b, float c, float d) {
    typedef __attribute__((ext_vector_type(4))) _Float16 h4;
    *(h4*)p = h4{(f16)a, (f16)b, (f16)c, (f16)d};
}

// LayerNorm with the pending split-K product of a residual GEMM folded in first.  KS > 0: the
// slab count as a template constant, so every slab, residual and bias load of a row is issued
// before the first add (a runtime slab loop waited on each load in turn: r3 profile, 10.5 us per
// launch at M = 832, 2 TB/s); KS = 0 keeps the runtime loop for other split counts.
template <typename T, int NV, int KS>
__global__ __launch_bounds__(256) void ln_pend_kernel(float* __restrict__ x, int M, int d, const float* __restrict__ slab,
                                                      int ks, int64_t sst, const float* __restrict__ pbias, float alpha,
                                                      const float* __restrict__ w, const float* __restrict__ bb,
                                                      T* __restrict__ y, int write_x) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int n4 = d >> 2;
    float4* xr = (float4*)(x + (size_t)row * d);
    float4 v[NV], g[NV], o[NV];
    const float4* w4 = (const float4*)w;
    const float4* b4 = (const float4*)bb;
#pragma unroll
    for (int i = 0; i < NV; ++i) {  // issued with the row's other operands (see ln_kernel)
        const int idx = min(lane + 64 * i, n4 - 1);
        g[i] = w4[idx];
        o[i] = b4[idx];
    }
    float s = 0.f;
    if constexpr (KS > 0) {
        float4 u[NV][KS], x0[NV], pb[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int idx = min(lane + 64 * i, n4 - 1);
#pragma unroll
            for (int q = 0; q < KS; ++q) u[i][q] = *(const float4*)(slab + q * sst + (size_t)row * d + 4 * idx);
            x0[i] = xr[idx];
            pb[i] = ((const float4*)pbias)[idx];
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            float4 p = u[i][0];
#pragma unroll
            for (int q = 1; q < KS; ++q) {
                p.x += u[i][q].x; p.y += u[i][q].y; p.z += u[i][q].z; p.w += u[i][q].w;
            }
            const int idx = lane + 64 * i;
            if (idx < n4) {
                v[i] = make_float4(x0[i].x + alpha * (p.x + pb[i].x), x0[i].y + alpha * (p.y + pb[i].y),
                                   x0[i].z + alpha * (p.z + pb[i].z), x0[i].w + alpha * (p.w + pb[i].w));
                if (write_x) xr[idx] = v[i];
                s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
            } else {
                v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int idx = lane + 64 * i;
            if (idx < n4) {
                float4 p = *(const float4*)(slab + (size_t)row * d + 4 * idx);
                for (int q = 1; q < ks; ++q) {
                    const float4 u = *(const float4*)(slab + q * sst + (size_t)row * d + 4 * idx);
                    p.x += u.x; p.y += u.y; p.z += u.z; p.w += u.w;
                }
                const float4 pb = ((const float4*)pbias)[idx], x0 = xr[idx];
                v[i] = make_float4(x0.x + alpha * (p.x + pb.x), x0.y + alpha * (p.y + pb.y), x0.z + alpha * (p.z + pb.z),
                                   x0.w + alpha * (p.w + pb.w));
                if (write_x) xr[idx] = v[i];
                s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
            } else {
                v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    }
    const float mean = wave_sum(s) / (float)d;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int idx = lane + 64 * i;
        if (idx < n4) {
            const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, e = v[i].w - mean;
            s2 += (a * a + b * b) + (c * c + e * e);
        }
    }
    const float rstd = 1.0f / sqrtf(wave_sum(s2) / (float)d + 1e-5f);
    T* yr = y + (size_t)row * d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int idx = lane + 64 * i;
        if (idx < n4)
            store4<T>(yr + 4 * idx, (v[i].x - mean) * rstd * g[i].x + o[i].x, (v[i].y - mean) * rstd * g[i].y + o[i].y,
                      (v[i].z - mean) * rstd * g[i].z + o[i].z, (v[i].w - mean) * rstd * g[i].w + o[i].w);
    }
}

// ln_pend_kernel (f32 output, x not written back) followed by a second LayerNorm of its output row,
// still in registers: the Parakeet layer boundary (the block's output LayerNorm, then the next
// block's first).  Both results are bitwise those of ln_pend_kernel + ln_kernel (the second LN
// sums the f32 row it would have read back, in the same lane order).
template <typename T2, int NV, int KS>
__global__ __launch_bounds__(256) void ln_pend2_kernel(const float* __restrict__ x, int M, int d,
                                                       const float* __restrict__ slab, int64_t sst,
                                                       const float* __restrict__ pbias, float alpha,
                                                       const float* __restrict__ w, const float* __restrict__ bb,
                                                       float* __restrict__ y, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, T2* __restrict__ y2) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const int n4 = d >> 2;
    const float4* xr = (const float4*)(x + (size_t)row * d);
    float4 v[NV], g[NV], o[NV], g2[NV], o2[NV], u[NV][KS], x0[NV], pb[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int idx = min(lane + 64 * i, n4 - 1);
#pragma unroll
        for (int q = 0; q < KS; ++q) u[i][q] = *(const float4*)(slab + q * sst + (size_t)row * d + 4 * idx);
        x0[i] = xr[idx];
        pb[i] = ((const float4*)pbias)[idx];
        g[i] = ((const float4*)w)[idx];
        o[i] = ((const float4*)bb)[idx];
        g2[i] = ((const float4*)w2)[idx];
        o2[i] = ((const float4*)b2)[idx];
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        float4 p = u[i][0];
#pragma unroll
        for (int q = 1; q < KS; ++q) {
            p.x += u[i][q].x; p.y += u[i][q].y; p.z += u[i][q].z; p.w += u[i][q].w;
        }
        if (lane + 64 * i < n4) {
            v[i] = make_float4(x0[i].x + alpha * (p.x + pb[i].x), x0[i].y + alpha * (p.y + pb[i].y),
                               x0[i].z + alpha * (p.z + pb[i].z), x0[i].w + alpha * (p.w + pb[i].w));
            s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
        } else {
            v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    float mean = wave_sum(s) / (float)d;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        if (lane + 64 * i < n4) {
            const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, e = v[i].w - mean;
            s2 += (a * a + b * b) + (c * c + e * e);
        }
    }
    float rstd = 1.0f / sqrtf(wave_sum(s2) / (float)d + 1e-5f);
    float* yr = y + (size_t)row * d;
    s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int idx = lane + 64 * i;
        if (idx < n4) {
            v[i] = make_float4((v[i].x - mean) * rstd * g[i].x + o[i].x, (v[i].y - mean) * rstd * g[i].y + o[i].y,
                               (v[i].z - mean) * rstd * g[i].z + o[i].z, (v[i].w - mean) * rstd * g[i].w + o[i].w);
            *(float4*)(yr + 4 * idx) = v[i];
        } else {
            v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    }
    mean = wave_sum(s) / (float)d;
    s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        if (lane + 64 * i < n4) {
            const float a = v[i].x - mean, b = v[i].y - mean, c = v[i].z - mean, e = v[i].w - mean;
            s2 += (a * a + b * b) + (c * c + e * e);
        }
    }
    rstd = 1.0f / sqrtf(wave_sum(s2) / (float)d + 1e-5f);
    T2* y2r = y2 + (size_t)row * d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        const int idx = lane + 64 * i;
        if (idx < n4)
            store4<T2>(y2r + 4 * idx, (v[i].x - mean) * rstd * g2[i].x + o2[i].x, (v[i].y - mean) * rstd * g2[i].y + o2[i].y,
                       (v[i].z - mean) * rstd * g2[i].z + o2[i].z, (v[i].w - mean) * rstd * g2[i].w + o2[i].w);
    }
}

template <typename T2, int NV>
void ln_pend2_nv(dim3 grid, const float* x, int M, int d, const float* slab, int ks, int64_t sst, const float* pb,
                 float alpha, const float* w, const float* b, float* y, const float* w2, const float* b2, T2* y2,
                 hipStream_t st) {
    switch (ks) {
        case 1: hipLaunchKernelGGL((ln_pend2_kernel<T2, NV, 1>), grid, dim3(256), 0, st, x, M, d, slab, sst, pb, alpha, w, b, y, w2, b2, y2); break;
        case 2: hipLaunchKernelGGL((ln_pend2_kernel<T2, NV, 2>), grid, dim3(256), 0, st, x, M, d, slab, sst, pb, alpha, w, b, y, w2, b2, y2); break;
        case 4: hipLaunchKernelGGL((ln_pend2_kernel<T2, NV, 4>), grid, dim3(256), 0, st, x, M, d, slab, sst, pb, alpha, w, b, y, w2, b2, y2); break;
        case 8: hipLaunchKernelGGL((ln_pend2_kernel<T2, NV, 8>), grid, dim3(256), 0, st, x, M, d, slab, sst, pb, alpha, w, b, y, w2, b2, y2); break;
        default: throw std::runtime_error("layernorm_pend2: split count must be 1, 2, 4 or 8");
    }
}

template <typename T2>
void ln_pend2_dispatch(const float* x, int M, int d, const float* slab, int ks, int64_t sst, const float* pb, float alpha,
                       const float* w, const float* b, float* y, const float* w2, const float* b2, T2* y2, hipStream_t st) {
    dim3 grid(cdiv(M, 4));
    switch (cdiv(d, 256)) {
        case 1: ln_pend2_nv<T2, 1>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, w2, b2, y2, st); break;
        case 2: ln_pend2_nv<T2, 2>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, w2, b2, y2, st); break;
        case 3: ln_pend2_nv<T2, 3>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, w2, b2, y2, st); break;
        case 4: ln_pend2_nv<T2, 4>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, w2, b2, y2, st); break;
        default: throw std::runtime_error("layernorm_pend2: d too large");
    }
}

template <typename T, int NV>
void ln_pend_nv(dim3 grid, float* x, int M, int d, const float* slab, int ks, int64_t sst, const float* pb, float alpha,
                const float* w, const float* b, T* y, int wx, hipStream_t st) {
    switch (ks) {
        case 1: hipLaunchKernelGGL((ln_pend_kernel<T, NV, 1>), grid, dim3(256), 0, st, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx); break;
        case 2: hipLaunchKernelGGL((ln_pend_kernel<T, NV, 2>), grid, dim3(256), 0, st, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx); break;
        case 4: hipLaunchKernelGGL((ln_pend_kernel<T, NV, 4>), grid, dim3(256), 0, st, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx); break;
        case 8: hipLaunchKernelGGL((ln_pend_kernel<T, NV, 8>), grid, dim3(256), 0, st, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx); break;
        default: hipLaunchKernelGGL((ln_pend_kernel<T, NV, 0>), grid, dim3(256), 0, st, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx); break;
    }
}

template <typename T>
void ln_pend_dispatch(float* x, int M, int d, const float* slab, int ks, int64_t sst, const float* pb, float alpha,
                      const float* w, const float* b, T* y, int wx, hipStream_t st) {
    dim3 grid(cdiv(M, 4));
    switch (cdiv(d, 256)) {
        case 1: ln_pend_nv<T, 1>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx, st); break;
        case 2: ln_pend_nv<T, 2>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx, st); break;
        case 3: ln_pend_nv<T, 3>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx, st); break;
        case 4: ln_pend_nv<T, 4>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx, st); break;
        case 5: ln_pend_nv<T, 5>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx, st); break;
        case 6: ln_pend_nv<T, 6>(grid, x, M, d, slab, ks, sst, pb, alpha, w, b, y, wx, st); break;
        default: throw std::runtime_error("layernorm_pend: d too large");
    }
}

template <typename T>
void ln_dispatch(const float* x, int M, int d, const float* w, const float* b, T* y, hipStream_t st) {
    dim3 grid(cdiv(M, 4));
    const int nv = cdiv(d, 256);
    switch (nv) {
        case 1: hipLaunchKernelGGL((ln_kernel<T, 1>), grid, dim3(256), 0, st, x, M, d, w, b, y); break;
        case 2: hipLaunchKernelGGL((ln_kernel<T, 2>), grid, dim3(256), 0, st, x, M, d, w, b, y); break;
        case 3: hipLaunchKernelGGL((ln_kernel<T, 3>), grid, dim3(256), 0, st, x, M, d, w, b, y); break;
        case 4: hipLaunchKernelGGL((ln_kernel<T, 4>), grid, dim3(256), 0, st, x, M, d, w, b, y); break;
        case 5: hipLaunchKernelGGL((ln_kernel<T, 5>), grid, dim3(256), 0, st, x, M, d, w, b, y); break;
        case 6: hipLaunchKernelGGL((ln_kernel<T, 6>), grid, dim3(256), 0, st, x, M, d, w, b, y); break;
        default: throw std::runtime_error("layernorm: d too large");
    }
}

template <typename T>
__global__ void to_f32_kernel(const T* __restrict__ s, float* __restrict__ d, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = to_f<T>(s[i]);
}

}  // namespace

void layernorm(int dtype, const float* x, int M, int d, const float* w, const float* b, void* y, hipStream_t st) {
    if (d % 4) throw std::runtime_error("layernorm: d % 4");
    if (dtype == DT_BF16) ln_dispatch<bf16>(x, M, d, w, b, (bf16*)y, st);
    else if (dtype == DT_F16) ln_dispatch<f16>(x, M, d, w, b, (f16*)y, st);
    else ln_dispatch<float>(x, M, d, w, b, (float*)y, st);
}

void layernorm_pend(int dtype, float* x, int M, int d, const float* slab, int ks, int64_t slab_stride,
                    const float* pbias, float alpha, const float* w, const float* b, void* y, bool write_x,
                    hipStream_t st) {
    if (d % 4) throw std::runtime_error("layernorm_pend: d % 4");
    if (dtype == DT_BF16) ln_pend_dispatch<bf16>(x, M, d, slab, ks, slab_stride, pbias, alpha, w, b, (bf16*)y, write_x, st);
    else if (dtype == DT_F16) ln_pend_dispatch<f16>(x, M, d, slab, ks, slab_stride, pbias, alpha, w, b, (f16*)y, write_x, st);
    else ln_pend_dispatch<float>(x, M, d, slab, ks, slab_stride, pbias, alpha, w, b, (float*)y, write_x, st);
    SPT_LAUNCH_CHECK();
}

void layernorm_pend2(int dtype2, const float* x, int M, int d, const float* slab, int ks, int64_t slab_stride,
                     const float* pbias, float alpha, const float* w, const float* b, float* y, const float* w2,
                     const float* b2, void* y2, hipStream_t st) {
    if (d % 4) throw std::runtime_error("layernorm_pend2: d % 4");
    if (dtype2 == DT_BF16) ln_pend2_dispatch<bf16>(x, M, d, slab, ks, slab_stride, pbias, alpha, w, b, y, w2, b2, (bf16*)y2, st);
    else if (dtype2 == DT_F16) ln_pend2_dispatch<f16>(x, M, d, slab, ks, slab_stride, pbias, alpha, w, b, y, w2, b2, (f16*)y2, st);
    else ln_pend2_dispatch<float>(x, M, d, slab, ks, slab_stride, pbias, alpha, w, b, y, w2, b2, (float*)y2, st);
    SPT_LAUNCH_CHECK();
}

void to_f32(int dtype, const void* src, float* dst, int64_t n, hipStream_t st) {
    int64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(to_f32_kernel<bf16>, dim3((int)g), dim3(256), 0, st, (const bf16*)src, dst, n);
    else if (dtype == DT_F16)
        hipLaunchKernelGGL(to_f32_kernel<f16>, dim3((int)g), dim3(256), 0, st, (const f16*)src, dst, n);
    else
        hipLaunchKernelGGL(to_f32_kernel<float>, dim3((int)g), dim3(256), 0, st, (const float*)src, dst, n);
}

}  // namespace spt
