// common.h -- shared device/host helpers for the spittle_amd HIP backend (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

namespace spt {

typedef uint16_t bf16;  // raw bf16 storage
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4v;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

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
// round-to-nearest-even (inputs are finite in this pipeline)
__host__ __device__ inline bf16 f2bf(float f) {
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

template <typename T> __device__ inline float to_f(T v);
template <> __device__ inline float to_f<float>(float v) { return v; }
template <> __device__ inline float to_f<bf16>(bf16 v) { return bf2f(v); }
template <typename T> __device__ inline T from_f(float v);
template <> __device__ inline float from_f<float>(float v) { return v; }
template <> __device__ inline bf16 from_f<bf16>(float v) { return f2bf(v); }

__device__ inline float gelu_tanh(float x) {
    const float c = 0.7978845608028654f;
    return 0.5f * x * (1.0f + tanhf(c * (x + 0.044715f * x * x * x)));
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

}  // namespace spt
