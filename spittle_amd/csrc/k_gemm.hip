// k_gemm.hip -- encoder-side GEMMs C = A . W^T on CDNA4 matrix cores.
//
// Replaces the ggml mul_mat / conv_1d_ph (im2col + mul_mat) ops that
// whisper.cpp's whisper_build_graph_conv / _encoder / _cross run for
// WhisperEngine::transcribe_samples (/root/reference/src-tauri/src/managers/transcription.rs:501-503).
//
// Tile: 128 x 128 per 256-thread workgroup (4 waves in 2 x 2, 64 x 64 each),
// one 128-byte K slab per stage (64 bf16 or 32 f32), operands staged
// global -> LDS by global_load_lds_dwordx4 (one wave-instruction = 8 rows x 128 B),
// XOR-swizzled on the source address (chunk ^ (row & 7)) so the ds_read_b128
// fragment reads are spread over the bank row, double-buffered so the next
// slab's DMA overlaps the current slab's MFMAs.
//   bf16: v_mfma_f32_16x16x32_bf16, 2 k-steps per slab.
//   f32 : v_mfma_f32_16x16x4_f32 (exact f32, no xf32 on gfx950), 8 k-steps per
//         slab with the per-lane k permutation k = 8 * (lane >> 4) + step.
// Workgroup ids are remapped so each XCD gets a contiguous run of tiles (T1).
// Fused epilogues: bias, GELU(tanh), positional add, residual add, and the
// head-split store of the cross-attention K/V cache.
//
// The conv stem needs no im2col: with tap-major weights [N][3][C] the conv
// input row for output t is a contiguous 3*C slice of the (zero-padded,
// time-major) input, i.e. an A operand with a leading dimension of C (conv1,
// stride 1) or 2*C (conv2, stride 2).
#include "common.h"
#include "kernels.h"

namespace spt {

namespace {

constexpr int BM = 128, BN = 128, SLAB = 128;  // SLAB = bytes of K per row per stage

__device__ __forceinline__ void glds16(const void* g, SPT_LDS void* l) {
    __builtin_amdgcn_global_load_lds((const void*)g, l, 16, 0, 0);
}

template <typename T, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * BM * SLAB];  // [buf][A|W][128 rows][128 B]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int nnt = g.N / BN;
    // bijective XCD-aware remap of the linear tile id
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tm = wg / nnt, tn = wg - tm * nnt;
    const int m0 = tm * BM, n0 = tn * BN;
    const int bz = blockIdx.z;
    const T* A = (const T*)g.A + (size_t)bz * g.sA;
    const T* W = (const T*)g.W;

    // per-lane source pointers for the 4 A pieces and 4 W pieces this wave stages
    const char* srcA[4];
    const char* srcW[4];
    const int prow = lane >> 3, pch = lane & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rt = (wid * 4 + i) * 8 + prow;
        const int c = pch ^ (rt & 7);
        const int ra = min(m0 + rt, g.M - 1);
        srcA[i] = (const char*)(A + (size_t)ra * g.lda) + c * 16;
        srcW[i] = (const char*)(W + (size_t)(n0 + rt) * g.ldw) + c * 16;
    }
    auto lds_a = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + (buf * 2 + 0) * BM * SLAB; };
    auto lds_w = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + (buf * 2 + 1) * BM * SLAB; };
    auto stage = [&](int buf, int kt) {
        const size_t koff = (size_t)kt * SLAB;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            glds16(srcA[i] + koff, lds_a(buf) + (wid * 4 + i) * 1024);
            glds16(srcW[i] + koff, lds_w(buf) + (wid * 4 + i) * 1024);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nkt = g.K * (int)sizeof(T) / SLAB;
    const int fr = lane & 15, fq = lane >> 4;

    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) stage(cur ^ 1, kt + 1);
        const SPT_LDS char* la = lds_a(cur);
        const SPT_LDS char* lw = lds_w(cur);
        if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 af[4], wf[4];
                const int c = 4 * s + fq;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int ra = wm * 64 + 16 * i + fr;
                    af[i] = *(const SPT_LDS bf16x8*)(la + ra * SLAB + ((c ^ (ra & 7)) << 4));
                    const int rw = wn * 64 + 16 * i + fr;
                    wf[i] = *(const SPT_LDS bf16x8*)(lw + rw * SLAB + ((c ^ (rw & 7)) << 4));
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], wf[j], acc[i][j], 0, 0, 0);
            }
        } else {
            f32x4 af[4][2], wf[4][2];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ra = wm * 64 + 16 * i + fr;
                const int rw = wn * 64 + 16 * i + fr;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int c = 2 * fq + h;
                    af[i][h] = *(const SPT_LDS f32x4*)(la + ra * SLAB + ((c ^ (ra & 7)) << 4));
                    wf[i][h] = *(const SPT_LDS f32x4*)(lw + rw * SLAB + ((c ^ (rw & 7)) << 4));
                }
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s >> 2][s & 3], wf[j][s >> 2][s & 3],
                                                                          acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---------------------------------------------------------------- epilogue
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + 16 * j + fr;
        const float bv = g.bias ? g.bias[col] : 0.0f;
        int kv_l = 0, kv_kv = 0, kv_h = 0, kv_e = 0;
        if constexpr (EPI == EPI_KVSPLIT) {
            const int d = g.kv_H * 64;
            kv_l = col / (2 * d);
            const int rem = col - kv_l * 2 * d;
            kv_kv = rem / d;
            kv_h = (rem - kv_kv * d) >> 6;
            kv_e = rem & 63;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * 64 + 16 * i + 4 * fq + r;
                if (row >= g.M) continue;
                float v = acc[i][j][r] + bv;
                if constexpr (EPI == EPI_BIAS) {
                    T* C = (T*)g.C + (size_t)bz * g.sC;
                    C[(size_t)row * g.ldc + col] = from_f<T>(v);
                } else if constexpr (EPI == EPI_BIAS_GELU) {
                    T* C = (T*)g.C + (size_t)bz * g.sC;
                    C[(size_t)row * g.ldc + col] = from_f<T>(gelu_tanh(v));
                } else if constexpr (EPI == EPI_BIAS_GELU_POS) {
                    float* C = (float*)g.C + (size_t)bz * g.sC;
                    C[(size_t)row * g.ldc + col] = gelu_tanh(v) + g.pos[(size_t)row * g.N + col];
                } else if constexpr (EPI == EPI_BIAS_RESID) {
                    float* C = (float*)g.C + (size_t)bz * g.sC;
                    C[(size_t)row * g.ldc + col] += v;
                } else if constexpr (EPI == EPI_KVSPLIT) {
                    T* C = (T*)g.C;
                    const int bb = row / g.kv_T, t = row - bb * g.kv_T;
                    const size_t off =
                        ((((size_t)(kv_l * 2 + kv_kv) * g.kv_B + bb) * g.kv_H + kv_h) * g.kv_T + t) * 64 + kv_e;
                    C[off] = from_f<T>(v);
                }
            }
    }
}

template <typename T, int EPI>
void launch_t(const GemmArgs& g, int batch, hipStream_t st) {
    dim3 grid(cdiv(g.M, BM) * (g.N / BN), 1, batch);
    hipLaunchKernelGGL((gemm_nt_kernel<T, EPI>), grid, dim3(256), 0, st, g);
}

}  // namespace

void gemm_nt(int dtype, int epi, const GemmArgs& g, int batch, hipStream_t st) {
    if (g.N % BN != 0 || (g.K * (dtype == DT_BF16 ? 2 : 4)) % SLAB != 0 || g.M <= 0)
        throw std::runtime_error("gemm_nt: unsupported shape M=" + std::to_string(g.M) + " N=" +
                                 std::to_string(g.N) + " K=" + std::to_string(g.K));
#define SPT_GEMM_CASE(T, E) \
    case E: launch_t<T, E>(g, batch, st); return;
    if (dtype == DT_BF16) {
        switch (epi) {
            SPT_GEMM_CASE(bf16, EPI_BIAS)
            SPT_GEMM_CASE(bf16, EPI_BIAS_GELU)
            SPT_GEMM_CASE(bf16, EPI_BIAS_GELU_POS)
            SPT_GEMM_CASE(bf16, EPI_BIAS_RESID)
            SPT_GEMM_CASE(bf16, EPI_KVSPLIT)
        }
    } else {
        switch (epi) {
            SPT_GEMM_CASE(float, EPI_BIAS)
            SPT_GEMM_CASE(float, EPI_BIAS_GELU)
            SPT_GEMM_CASE(float, EPI_BIAS_GELU_POS)
            SPT_GEMM_CASE(float, EPI_BIAS_RESID)
            SPT_GEMM_CASE(float, EPI_KVSPLIT)
        }
    }
#undef SPT_GEMM_CASE
    throw std::runtime_error("gemm_nt: bad epilogue");
}

}  // namespace spt
