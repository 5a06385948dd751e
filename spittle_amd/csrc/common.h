// common.h -- shared device/host helpers for the spittle_amd HIP backend (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

namespace spt {

typedef uint16_t bf16;  // raw bf16 storage
typedef _Float16 f16;   // IEEE half (Parakeet's fp16 encoder)
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4v;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;

#define SPT_LDS __attribute__((address_space(3)))

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define HIP_CHECK(expr)                                                                    \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            throw ::spt::HipError(std::string(#expr) + " failed: " + hipGetErrorString(_e) + \
                                  " (" __FILE__ ":" + std::to_string(__LINE__) + ")");      \
    } while (0)

// surface launch-configuration errors at the launch site (works under stream capture)
#define SPT_LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

__host__ __device__ inline float bf2f(bf16 v) {
    union { uint32_t u; float f; } x;
    x.u = (uint32_t)v << 16;
    return x.f;
}
// round-to-nearest-even; on the device one v_cvt_pk_bf16_f32 (same RNE for finite inputs,
// keeps NaNs NaN), on the host the integer form
__host__ __device__ inline bf16 f2bf(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bit_cast(bf16, (__bf16)f);
#endif
    union { uint32_t u; float f; } x;
    x.f = f;
    uint32_t u = x.u;
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (bf16)(u >> 16);
}
// packed pair -> one dword
__device__ inline uint32_t pack_bf2(float a, float b) {
    return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

template <typename T> struct TypeTag;
template <> struct TypeTag<float> { static constexpr int id = 0; };
template <> struct TypeTag<bf16> { static constexpr int id = 1; };
template <> struct TypeTag<f16> { static constexpr int id = 2; };

template <typename T> __device__ inline float to_f(T v);
template <> __device__ inline float to_f<float>(float v) { return v; }
template <> __device__ inline float to_f<bf16>(bf16 v) { return bf2f(v); }
template <> __device__ inline float to_f<f16>(f16 v) { return (float)v; }
template <typename T> __device__ inline T from_f(float v);
template <> __device__ inline float from_f<float>(float v) { return v; }
template <> __device__ inline bf16 from_f<bf16>(float v) { return f2bf(v); }
template <> __device__ inline f16 from_f<f16>(float v) { return (f16)v; }  // RNE

// GELU, tanh form (ggml / whisper.cpp): 0.5 x (1 + tanh(u)), u = sqrt(2/pi) (x + 0.044715 x^3),
// evaluated as x * sigmoid(2u) = x / (1 + 2^(-2u log2 e)): one v_exp_f32 + one v_rcp_f32
// instead of tanhf (the same function; differs from libm tanhf by a few f32 ulp)
// (contraction off: every kernel that inlines it -- the decoder's fc1 GEMV, the encoder's GEMM
// epilogues -- computes the same bits, whatever the surrounding code)
__device__ inline float gelu_tanh(float x) {
#pragma clang fp contract(off)
    const float c2 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
    const float e = __builtin_amdgcn_exp2f(c2 * (x + 0.044715f * x * x * x));
    return x * __builtin_amdgcn_rcpf(1.0f + e);
}

// the decoder rows' LayerNorm arithmetic (gemv_kernel's A_LN prologue), spelled out with
// contraction off so every instance computes the same bits: the squared deviations of four elements,
// and one normalised element
__device__ inline float ln_sq4(float4 v, float mean) {
#pragma clang fp contract(off)
    const float p = v.x - mean, q = v.y - mean, u = v.z - mean, w = v.w - mean;
    return (p * p + q * q) + (u * u + w * w);
}
__device__ inline float ln_out(float v, float mean, float rstd, float g, float b) {
#pragma clang fp contract(off)
    return (v - mean) * rstd * g + b;
}

// Swish / SiLU x * sigmoid(x) (NeMo's Swish activation): one v_exp_f32 + one v_rcp_f32
__device__ inline float swish(float x) {
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ inline float sigmoidf_(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ inline float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for the calling thread's current device, once
// per (kernel, device): the attribute is per device, and replica threads drive several devices
// from one process (r2 advisor finding).  Thread-safe.  Call outside stream capture.
void ensure_lds_attr(const void* kernel, int bytes);

}  // namespace spt
