// k_pk.hip -- Parakeet-V3 (FastConformer-TDT) kernels: front end, subsampling, rel-pos
// attention, convolution module and the TDT greedy step.  Replaces the ONNX Runtime graph
// transcribe-rs' ParakeetEngine runs (/root/reference/src-tauri/src/managers/transcription.rs:
// 278-297 load, 505-513 transcribe_samples); the model is NeMo's (oracle/parakeet_oracle.h).
//
// The dense products (DFT, pointwise convolutions, linear layers, the joint's encoder
// projection) are MFMA GEMMs (k_gemm.hip); what is here is the memory-bound glue, each kernel
// one pass over its tensor.  Activations are [rows][channels] with channels contiguous, so
// every kernel's lanes walk the channel axis (coalesced); the frame axis carries the masks.
#include "common.h"
#include "kernels.h"
#include "pk_kernels.h"

#include <algorithm>
#include <cstdlib>

namespace spt {

namespace {

inline int grid_of(int64_t n, int tpb = 256) {
    int64_t g = (n + tpb - 1) / tpb;
    return (int)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

// ---------------------------------------------------------------- front end
__global__ __launch_bounds__(256) void frames_kernel(const float* __restrict__ pcm, int64_t stride,
                                                     const int* __restrict__ nsamp, int Tp,
                                                     const float* __restrict__ win, float* __restrict__ frames) {
    const int t = blockIdx.x, b = blockIdx.y;
    const int n = nsamp[b];
    const float* x = pcm + (size_t)b * stride;
    float* row = frames + ((size_t)b * Tp + t) * PK_NFFT;
    for (int i = threadIdx.x; i < PK_NFFT; i += 256) {
        const int s = t * PK_HOP + i - PK_NFFT / 2;  // centre padding: n_fft / 2 zeros each side
        float v = 0.0f;
        if (s >= 0 && s < n) v = x[s] - (s > 0 ? __fmul_rn(0.97f, x[s - 1]) : 0.0f);  // pre-emphasis
        row[i] = __fmul_rn(v, win[i]);
    }
}

// one workgroup per frame: |X_k|^2 -> mel filterbank (fbT [257][n_mels]) -> log(x + 2^-24)
__global__ __launch_bounds__(128) void melpow_kernel(const float* __restrict__ spec, const float* __restrict__ fbT,
                                                     int n_mels, float* __restrict__ mel) {
    __shared__ float pw[PK_NBIN];
    const size_t r = blockIdx.x;
    const float* s = spec + r * PK_DFT_N;
    for (int k = threadIdx.x; k < PK_NBIN; k += 128) {
        const float re = s[k], im = s[PK_NBIN + k];
        pw[k] = re * re + im * im;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n_mels; j += 128) {
        float acc = 0.0f;
        for (int k = 0; k < PK_NBIN; ++k) acc += fbT[k * n_mels + j] * pw[k];
        mel[r * n_mels + j] = logf(acc + 5.9604644775390625e-08f);
    }
}

// per (utterance, 32 mel bands): 8 frame groups x 32 bands, f64 sums; three passes
__global__ __launch_bounds__(256) void mel_norm_kernel(float* __restrict__ mel, const int* __restrict__ lens, int Tp,
                                                       int n_mels) {
    __shared__ double red[8][33];
    const int b = blockIdx.x, jl = threadIdx.x & 31, tg = threadIdx.x >> 5;
    const int j = blockIdx.y * 32 + jl;
    const int T = lens[b * 4];
    float* base = mel + (size_t)b * Tp * n_mels;
    const bool ok = j < n_mels;
    double s = 0;
    if (ok)
        for (int t = tg; t < T; t += 8) s += base[(size_t)t * n_mels + j];
    red[tg][jl] = s;
    __syncthreads();
    double mean = 0;
    for (int g = 0; g < 8; ++g) mean += red[g][jl];
    mean /= T;
    __syncthreads();
    double v = 0;
    if (ok)
        for (int t = tg; t < T; t += 8) {
            const double e = base[(size_t)t * n_mels + j] - mean;
            v += e * e;
        }
    red[tg][jl] = v;
    __syncthreads();
    double var = 0;
    for (int g = 0; g < 8; ++g) var += red[g][jl];
    const double sd = sqrt(var / (T > 1 ? T - 1 : 1)) + 1e-5;
    if (!ok) return;
    for (int t = tg; t < Tp; t += 8) {
        float* p = base + (size_t)t * n_mels + j;
        *p = t < T ? (float)((*p - mean) / sd) : 0.0f;
    }
}

// ---------------------------------------------------------------- subsampling
// one workgroup per output frame (t, b), a thread per channel (coalesced channel-last stores);
// the three input frames it reads are staged in LDS
template <typename T>
__global__ __launch_bounds__(1024) void conv0_kernel(const float* __restrict__ mel, const int* __restrict__ lens,
                                                     int Tp, int F, const float* __restrict__ w,
                                                     const float* __restrict__ bias, int C, T* __restrict__ y, int T1p,
                                                     int F1) {
    extern __shared__ float rows[];  // [3][F]
    const int t = blockIdx.x, b = blockIdx.y, c = threadIdx.x;
    const int Tb = min(lens[b * 4], Tp);
    for (int i = threadIdx.x; i < 3 * F; i += blockDim.x) {
        const int tt = 2 * t - 1 + i / F;
        rows[i] = (tt >= 0 && tt < Tb) ? mel[((size_t)b * Tp + tt) * F + i % F] : 0.0f;
    }
    __syncthreads();
    float wc[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) wc[i] = w[c * 9 + i];
    const float bc = bias[c];
    T* out = y + ((size_t)b * T1p + t) * F1 * C + c;
    for (int f = 0; f < F1; ++f) {
        float acc = bc;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int ff = 2 * f - 1 + j;
                if (ff >= 0 && ff < F) acc += wc[i * 3 + j] * rows[i * F + ff];
            }
        out[(size_t)f * C] = from_f<T>(fmaxf(acc, 0.0f));
    }
}

// depthwise 3x3 stride 2: one workgroup per output frame (t, b), a thread per channel
template <typename T>
__global__ __launch_bounds__(1024) void dwconv_kernel(const T* __restrict__ x, const int* __restrict__ lens, int stage,
                                                      int Tip, int Fi, const float* __restrict__ w,
                                                      const float* __restrict__ bias, int C, T* __restrict__ y, int Top,
                                                      int Fo) {
    const int t = blockIdx.x, b = blockIdx.y, c = threadIdx.x;
    const int Tb = min(lens[b * 4 + stage], Tip);
    float wc[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) wc[i] = w[c * 9 + i];
    const float bc = bias[c];
    const T* in = x + (size_t)b * Tip * Fi * C + c;
    T* out = y + ((size_t)b * Top + t) * Fo * C + c;
    for (int f = 0; f < Fo; ++f) {
        float acc = bc;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int tt = 2 * t - 1 + i;
            if (tt < 0 || tt >= Tb) continue;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int ff = 2 * f - 1 + j;
                if (ff >= 0 && ff < Fi) acc += wc[i * 3 + j] * to_f<T>(in[((size_t)tt * Fi + ff) * C]);
            }
        }
        out[(size_t)f * C] = from_f<T>(acc);
    }
}

template <typename T>
__global__ void relpos_kernel(int Tp, int d, T* __restrict__ pe) {
    const int64_t total = (int64_t)(2 * Tp - 1) * (d / 2);
    for (int64_t idx = blockIdx.x * 256ll + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int k = (int)(idx % (d / 2));
        const int r = (int)(idx / (d / 2));
        const double pos = (double)(Tp - 1 - r);
        const double div = exp(-(2.0 * k) * log(10000.0) / d);
        pe[(size_t)r * d + 2 * k] = from_f<T>((float)sin(pos * div));
        pe[(size_t)r * d + 2 * k + 1] = from_f<T>((float)cos(pos * div));
    }
}

// ---------------------------------------------------------------- rel-pos attention
// One wave per (query, head, utterance).  Scores for 64 keys at a time (a lane per key, its
// k row and p row read as 16-byte vectors), kept in LDS; exact softmax; P.V with lanes over
// the head dimension.  ac = (q + u) . k_j, bd = (q + v) . p_{Tp-1-i+j} (NeMo's rel_shift as an
// index), scores / sqrt(dk).
template <typename T> __device__ __forceinline__ void ld8(const T* p, float* o);
template <> __device__ __forceinline__ void ld8<float>(const float* p, float* o) {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <> __device__ __forceinline__ void ld8<f16>(const f16* p, float* o) {
    const f16x8 v = *(const f16x8*)p;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
}
template <> __device__ __forceinline__ void ld8<bf16>(const bf16* p, float* o) {
    const uint4 v = *(const uint4*)p;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[2 * i] = bf2f((bf16)(w[i] & 0xffff));
        o[2 * i + 1] = bf2f((bf16)(w[i] >> 16));
    }
}

template <typename T>
__global__ __launch_bounds__(64) void rel_attn_kernel(const T* __restrict__ qkv, const T* __restrict__ p, int ldp,
                                                      const float* __restrict__ pu, const float* __restrict__ pv,
                                                      const int* __restrict__ lens, int Tp, int H, int dk,
                                                      T* __restrict__ out) {
    extern __shared__ float sm[];  // qu[dk] | qv[dk] | scores[Tp]
    float* qu = sm;
    float* qv = sm + dk;
    float* sc = sm + 2 * dk;
    const int i = blockIdx.x, h = blockIdx.y, b = blockIdx.z, lane = threadIdx.x;
    const int d = H * dk;
    const int T3 = lens[b * 4 + 3];
    T* orow = out + ((size_t)b * Tp + i) * d + h * dk;
    if (i >= T3) {
        for (int e = lane; e < dk; e += 64) orow[e] = from_f<T>(0.0f);
        return;
    }
    const T* base = qkv + (size_t)b * Tp * 3 * d;
    for (int e = lane; e < dk; e += 64) {
        const float q = to_f<T>(base[(size_t)i * 3 * d + h * dk + e]);
        qu[e] = q + pu[h * dk + e];
        qv[e] = q + pv[h * dk + e];
    }
    __syncthreads();
    const float scale = 1.0f / sqrtf((float)dk);
    float mx = -INFINITY;
    for (int j0 = 0; j0 < T3; j0 += 64) {
        const int j = j0 + lane;
        if (j < T3) {
            const T* kr = base + (size_t)j * 3 * d + d + h * dk;
            const T* pr = p + (size_t)(Tp - 1 - i + j) * ldp + h * dk;
            float ac = 0.0f, bd = 0.0f;
            for (int e = 0; e < dk; e += 8) {
                float kv[8], pv8[8];
                ld8<T>(kr + e, kv);
                ld8<T>(pr + e, pv8);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    ac += qu[e + u] * kv[u];
                    bd += qv[e + u] * pv8[u];
                }
            }
            const float s = (ac + bd) * scale;
            sc[j] = s;
            mx = fmaxf(mx, s);
        }
    }
    mx = wave_max(mx);
    float l = 0.0f;
    for (int j = lane; j < T3; j += 64) {
        const float e = expf(sc[j] - mx);
        sc[j] = e;
        l += e;
    }
    l = wave_sum(l);
    __syncthreads();
    for (int e = lane; e < dk; e += 64) {
        float acc = 0.0f;
        const T* vc = base + 2 * d + h * dk + e;
        for (int j = 0; j < T3; ++j) acc += sc[j] * to_f<T>(vc[(size_t)j * 3 * d]);
        orow[e] = from_f<T>(acc / l);
    }
}

// MFMA variant (fp16, head dim 64 or 128): one wave per 32 queries of one (head, utterance),
// flash-style over 32-key tiles.  Per tile, with v_mfma_f32_32x32x16_f16:
//   S^T  = K . (q + u)^T                 (keys x queries; a lane owns one query column)
//   G^T  = P[r0 .. r0 + 63] . (q + v)^T  (the 63 relative positions the tile's (i, j) pairs use,
//                                         r0 = Tp - 1 + j0 - i0 - 31)
//   bd(i, j) = G^T[j - i + 31][i]        (NeMo's rel_shift: a per-lane row skew, through LDS)
//   online softmax of (S^T + bd) / sqrt(dk); O^T += V^T . P^T, V^T read from LDS with
//   ds_read_b64_tr_b16 (the accumulator layout of P^T is directly the B operand).
template <int DK>
__global__ __launch_bounds__(64) void rel_attn_mfma_kernel(const f16* __restrict__ qkv, const f16* __restrict__ p,
                                                           int ldp, const float* __restrict__ pu,
                                                           const float* __restrict__ pv, const int* __restrict__ lens,
                                                           int Tp, int H, f16* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) char smem[32 * DK * 2 + 64 * 32 * 4];  // V tile [32][DK] | G [64][32]
    SPT_LDS char* lv = (SPT_LDS char*)smem;
    SPT_LDS float* G = (SPT_LDS float*)(smem + 32 * DK * 2);
    const int lane = threadIdx.x, l32 = lane & 31, hf = lane >> 5;
    const int i0 = blockIdx.x * 32, h = blockIdx.y, b = blockIdx.z;
    const int d = H * DK, ld = 3 * d;
    const int T3 = lens[b * 4 + 3];
    f16* obase = out + (size_t)b * Tp * d + h * DK;
    if (i0 >= T3) {  // padded frames: finite zeros
        for (int e = lane; e < 32 * DK; e += 64) {
            const int i = i0 + e / DK;
            if (i < Tp) obase[(size_t)i * d + e % DK] = (f16)0.0f;
        }
        return;
    }
    const f16* base = qkv + (size_t)b * Tp * ld;
    constexpr int NS = DK / 16;
    f16x8 qu[NS], qv[NS];
    {
        const int qi = min(i0 + l32, Tp - 1);
        const f16* qp = base + (size_t)qi * ld + h * DK + 8 * hf;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const f16x8 raw = *(const f16x8*)(qp + 16 * s);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int c = h * DK + 16 * s + 8 * hf + e;
                qu[s][e] = (f16)((float)raw[e] + pu[c]);
                qv[s][e] = (f16)((float)raw[e] + pv[c]);
            }
        }
    }
    const float sl2 = 1.4426950408889634f / sqrtf((float)DK);
    float m_run = -INFINITY, l_run = 0.0f;
    f32x16 o[DK / 32];
#pragma unroll
    for (int t = 0; t < DK / 32; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] = 0.0f;
    const int ntile = cdiv(T3, 32);
    const int g4 = lane >> 4, i16 = lane & 15;
    for (int jt = 0; jt < ntile; ++jt) {
        const int j0 = jt * 32;
        // V tile (32 keys x DK) -> registers; written to LDS after the score products
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        u32x4 vreg[DK / 16];
#pragma unroll
        for (int u = 0; u < DK / 16; ++u) {
            const int c = lane + 64 * u;
            const int key = min(j0 + c / (DK / 8), Tp - 1);
            vreg[u] = *(const u32x4*)(base + (size_t)key * ld + 2 * d + h * DK + 8 * (c % (DK / 8)));
        }
        // the tile's K rows and relative-position rows, all issued before the first product: loads
        // written inside the MFMA loop were each issued just before their MFMA and waited with
        // vmcnt(0), one dependent round trip per 16-wide slice (r3)
        f16x8 kf[NS], pf0[NS], pf1[NS];
        {
            const f16* kp = base + (size_t)min(j0 + l32, Tp - 1) * ld + d + h * DK + 8 * hf;
            const int r0 = (Tp - 1) + j0 - i0 - 31;
            const int pr0 = min(max(r0 + l32, 0), 2 * Tp - 2), pr1 = min(max(r0 + 32 + l32, 0), 2 * Tp - 2);
            const f16* p0 = p + (size_t)pr0 * ldp + h * DK + 8 * hf;
            const f16* p1 = p + (size_t)pr1 * ldp + h * DK + 8 * hf;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                kf[s] = *(const f16x8*)(kp + 16 * s);
                pf0[s] = *(const f16x8*)(p0 + 16 * s);
                pf1[s] = *(const f16x8*)(p1 + 16 * s);
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the scheduler from sinking the loads to their MFMAs
        // S^T = K . QU^T, G^T = P[r0 ..] . QV^T (two 32-row halves)
        f32x16 sc, g0, g1;
#pragma unroll
        for (int r = 0; r < 16; ++r) { sc[r] = 0.0f; g0[r] = 0.0f; g1[r] = 0.0f; }
#pragma unroll
        for (int s = 0; s < NS; ++s) sc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[s], qu[s], sc, 0, 0, 0);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            g0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(pf0[s], qv[s], g0, 0, 0, 0);
            g1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(pf1[s], qv[s], g1, 0, 0, 0);
        }
        // one wave: the LDS hand-offs need only its own lgkmcnt waits.  __syncthreads() is also a
        // release fence, and hipcc drained the tile's in-flight loads (vmcnt(0)) at each one
        // (r3: 69 -> 55 us per offline layer without them)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous tile's LDS reads are done
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * hf;
            G[row * 32 + l32] = g0[r];
            G[(row + 32) * 32 + l32] = g1[r];
        }
#pragma unroll
        for (int u = 0; u < DK / 16; ++u) *(SPT_LDS u32x4*)(lv + (lane + 64 * u) * 16) = vreg[u];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        float mloc = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int jl = (r & 3) + 8 * (r >> 2) + 4 * hf;
            float v = (sc[r] + G[(jl - l32 + 31) * 32 + l32]) * sl2;
            if (j0 + jl >= T3) v = -INFINITY;
            sc[r] = v;
            mloc = fmaxf(mloc, v);
        }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        float ls = 0.0f;
        f16x8 pf[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float e = __builtin_amdgcn_exp2f(sc[r] - m_new);
            ls += e;
            pf[r >> 3][r & 7] = (f16)e;
        }
        l_run = l_run * alpha + ls;
#pragma unroll
        for (int t = 0; t < DK / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
        // O^T += V^T . P^T
#pragma unroll
        for (int dt = 0; dt < DK / 32; ++dt) {
            const int col = 32 * dt + 16 * (g4 & 1) + 4 * (i16 & 3);
#pragma unroll
            for (int sp = 0; sp < 2; ++sp) {
                const int key0 = 16 * sp + 4 * hf + (i16 >> 2);
                const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SPT_LDS bf16x4v*)(lv + key0 * DK * 2 + col * 2));
                const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SPT_LDS bf16x4v*)(lv + (key0 + 8) * DK * 2 + col * 2));
                bf16x8 va;
                va[0] = lo[0]; va[1] = lo[1]; va[2] = lo[2]; va[3] = lo[3];
                va[4] = hi[0]; va[5] = hi[1]; va[6] = hi[2]; va[7] = hi[3];
                o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, va), pf[sp], o[dt], 0, 0, 0);
            }
        }
    }
    const float inv = 1.0f / (l_run + __shfl_xor(l_run, 32, 64));
    const int i = i0 + l32;
    if (i < Tp) {
        f16* orow = obase + (size_t)i * d;
        const bool ok = i < T3;
#pragma unroll
        for (int dt = 0; dt < DK / 32; ++dt)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const int dd = 32 * dt + 8 * gg + 4 * hf;
                typedef __attribute__((ext_vector_type(4))) _Float16 h4;
                const h4 v = ok ? h4{(f16)(o[dt][4 * gg] * inv), (f16)(o[dt][4 * gg + 1] * inv), (f16)(o[dt][4 * gg + 2] * inv),
                                     (f16)(o[dt][4 * gg + 3] * inv)}
                                : h4{(f16)0.0f, (f16)0.0f, (f16)0.0f, (f16)0.0f};
                *(h4*)(orow + dd) = v;
            }
    }
}

// ---------------------------------------------------------------- convolution module
// a workgroup per 8 output frames x 1024 channels of one utterance, a thread per 4 adjacent
// channels (8- / 16-byte loads and stores instead of one element per lane): the GLU of the
// 8 + K - 1 frames it needs is computed once into registers (not once per tap), then the
// depthwise taps, BatchNorm and Swish.  Sigmoids are exp2 + rcp (common.h sigmoidf_ / swish).
constexpr int CM_TT = 8, CM_V = 4;
template <typename T> struct Vec4;
template <> struct Vec4<f16> { typedef __attribute__((ext_vector_type(4))) _Float16 type; };
template <> struct Vec4<bf16> { typedef bf16x4v type; };
template <> struct Vec4<float> { typedef f32x4 type; };
template <typename T, int K>
__global__ __launch_bounds__(256) void conv_module_kernel(const T* __restrict__ a, const int* __restrict__ lens, int Tp,
                                                          int d, const float* __restrict__ dw_w,
                                                          const float* __restrict__ dw_b, const float* __restrict__ bn_g,
                                                          const float* __restrict__ bn_b, const float* __restrict__ bn_m,
                                                          const float* __restrict__ bn_v, T* __restrict__ out) {
    typedef typename Vec4<T>::type V4;
    const int t0 = blockIdx.x * CM_TT, b = blockIdx.y;
    const int T3 = lens[b * 4 + 3];
    const T* ab = a + (size_t)b * Tp * 2 * d;
    T* ob = out + (size_t)b * Tp * d;
    const int i = (blockIdx.z * 256 + threadIdx.x) * CM_V;  // first of this thread's 4 channels
    if (i >= d) return;
    // every frame's pair is loaded unconditionally (a clamped row) and masked after: a load under a
    // per-frame condition is branched around, and hipcc then waits for each one before the next
    // (one dependent round trip per frame)
    V4 xv[CM_TT + K - 1], gv[CM_TT + K - 1];
#pragma unroll
    for (int f = 0; f < CM_TT + K - 1; ++f) {
        const int tt = min(max(t0 - K / 2 + f, 0), Tp - 1);
        xv[f] = *(const V4*)(ab + (size_t)tt * 2 * d + i);
        gv[f] = *(const V4*)(ab + (size_t)tt * 2 * d + d + i);
    }
    float g[CM_TT + K - 1][CM_V];
#pragma unroll
    for (int f = 0; f < CM_TT + K - 1; ++f) {
        const int tt = t0 - K / 2 + f;
        const bool valid = tt >= 0 && tt < T3;
#pragma unroll
        for (int c = 0; c < CM_V; ++c) {
            const float v = to_f<T>((T)xv[f][c]) * sigmoidf_(to_f<T>((T)gv[f][c]));  // GLU
            g[f][c] = valid ? v : 0.0f;
        }
    }
    float wk[CM_V][K], bs[CM_V], bt[CM_V], bias[CM_V];
#pragma unroll
    for (int c = 0; c < CM_V; ++c) {
#pragma unroll
        for (int j = 0; j < K; ++j) wk[c][j] = dw_w[(i + c) * K + j];
        bs[c] = bn_g[i + c] / sqrtf(bn_v[i + c] + 1e-5f);
        bt[c] = bn_b[i + c] - bn_m[i + c] * bs[c];
        bias[c] = dw_b[i + c];
    }
#pragma unroll
    for (int f = 0; f < CM_TT; ++f) {
        const int t = t0 + f;
        if (t >= Tp) break;
        V4 o;
#pragma unroll
        for (int c = 0; c < CM_V; ++c) {
            float acc = bias[c];
#pragma unroll
            for (int j = 0; j < K; ++j) acc += wk[c][j] * g[f + j][c];
            const float z = acc * bs[c] + bt[c];
            o[c] = from_f<T>(t < T3 ? swish(z) : 0.0f);  // Swish
        }
        *(V4*)(ob + (size_t)t * d + i) = o;
    }
}

// ---------------------------------------------------------------- weight placement
template <typename T>
__global__ void place_copy_kernel(const float* __restrict__ s, int64_t n, T* __restrict__ d) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = from_f<T>(s[i]);
}
__global__ void place_transpose_kernel(const float* __restrict__ s, int N, int K, float* __restrict__ d, int ld,
                                       int row0) {
    const int64_t total = (int64_t)N * K;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int n = (int)(i % N), k = (int)(i / N);  // n fastest: coalesced writes
        d[(size_t)(row0 + k) * ld + n] = s[(size_t)n * K + k];
    }
}
template <typename T>
__global__ void place_subperm_kernel(const float* __restrict__ s, int N, int C, int F, T* __restrict__ d) {
    const int64_t total = (int64_t)N * C * F;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int c = (int)(i % C);
        const int64_t q = i / C;
        const int f = (int)(q % F);
        const int64_t n = q / F;
        d[i] = from_f<T>(s[(n * C + c) * F + f]);  // dst [n][f * C + c] <- src [n][c * F + f]
    }
}

// ---------------------------------------------------------------- TDT greedy step
// One kernel per stage of a decode step, 512 threads = 8 K-groups.  A workgroup owns DO outputs;
// a lane loads a float4 of W^T (4 consecutive outputs of one k row; a wave-load covers
// 256 / DO k rows x DO outputs = 1 KB), the x rows of one row group (DR = 8
// utterances; the groups spread over grid.y) sit in LDS as [k][XP] (broadcast float4 reads), so
// each lane carries 4 outputs x 8 rows of accumulators.  Every
// lane's weight loads for its K-group slice are issued together (8 per batch), the k rows of a
// wave fold by xor shuffles and the 8 K-groups through LDS; the epilogue is the stage's own: the
// LSTM cell (gate-interleaved W^T: a workgroup's 16 outputs are the i, f, g, o rows of 4 units),
// the prediction projection, or the joint's per-workgroup top-2 + duration logits.
constexpr int DG = 8, DR = 8;   // K-groups, rows per pass (accumulators: 4 outputs x 8 rows per lane)
constexpr int XP = 12;          // LDS row stride of the staged x (8 rows + 4 pad: 16-byte rows, <= 2-way conflicts)

__device__ __forceinline__ float sig_(float x) { return 1.0f / (1.0f + expf(-x)); }

// workgroup barrier for LDS hand-offs only: __syncthreads() is a release/acquire fence that
// drains vmcnt, which would stall the in-flight weight loads held in registers across it
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int MODE, int DO, int NWM, int SE>
__global__ __launch_bounds__(512) void dec_kernel(PkDecArgs a) {
    constexpr int OQ = DO / 4;       // output quads per k row
    constexpr int KS = 64 / OQ;      // k rows per wave-load
    constexpr int NU = DO / 4;       // LSTM: units per workgroup
    // NWM: wave-loads per lane held in registers (host checks K / 8 / KS <= NWM);
    // SE: staged float4 per thread (host checks K / 4 * 16 <= 512 * SE)
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* xs = sm;                    // [K][XP]
    float* red = sm + (size_t)a.K * XP;  // [DG][DR][DO]
    const int tid = threadIdx.x, lane = tid & 63, kg = tid >> 6;
    const int oq = lane % OQ, kq = lane / OQ;
    const int n0 = blockIdx.x * DO;
    const int KT = a.K / DG, kb = kg * KT, NW = KT / KS;
    const int P = a.P;
    // every operand of the stage is issued before anything waits: this lane's whole slice of the
    // blocked W^T ([N / DO][K][DO]: a workgroup's slice is contiguous, a wave-load is 1 KB), then
    // per row group the staged x rows and the epilogue's operands -- one memory round trip
    float4 w[NWM];
    {
        const float* wcol = a.WT + (size_t)blockIdx.x * a.K * DO + (size_t)(kb + kq) * DO + 4 * oq;
#pragma unroll
        for (int u = 0; u < NWM; ++u)
            w[u] = u < NW ? *(const float4*)(wcol + (size_t)u * KS * DO) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // this row group's staged x rows; a workgroup walks the row groups blockIdx.y, + gridDim.y, ..
    // and issues the next group's rows as soon as the current ones sit in LDS, so they fly under
    // the current group's products and reductions
    const int K4 = a.K / 4, NE = K4 * DR, rstep = DR * gridDim.y;
    auto load_x = [&](int rg, float4* v, float4* v2) {
        const int R = min(DR, a.B - rg);
#pragma unroll
        for (int u = 0; u < SE; ++u) {
            const int idx = min(tid + 512 * u, NE - 1);
            const int k = 4 * (idx / DR), r = idx % DR, b = rg + min(r, R - 1);
            if constexpr (MODE == PKD_LSTM) {
                const float* lo = a.xin + (size_t)b * P + k;
                const float* hi = a.h_in + (size_t)b * P + (k - P);
                v[u] = *(const float4*)(k < P ? lo : hi);
            } else if constexpr (MODE == PKD_PRED) {
                v[u] = *(const float4*)(a.xin + (size_t)b * P + k);
            } else {  // joint input ReLU(enc + pred), formed at the LDS store (a prefetch must not wait)
                v[u] = *(const float4*)(a.fe + (size_t)b * P + k);  // the row's current frame
                v2[u] = *(const float4*)(a.gp + (size_t)b * P + k);
            }
        }
    };
    float4 v[SE], v2[MODE == PKD_JOINT ? SE : 1];
    if (blockIdx.y * DR < a.B) load_x(blockIdx.y * DR, v, v2);
    // consume the weight registers here: at their first use inside the loop hipcc would wait with
    // vmcnt(0), which also drains the next row group's rows issued just before the products
#pragma unroll
    for (int u = 0; u < NWM; ++u) asm volatile("" ::"v"(w[u].x), "v"(w[u].y), "v"(w[u].z), "v"(w[u].w));
    for (int rg = blockIdx.y * DR; rg < a.B; rg += rstep) {
        const int R = min(DR, a.B - rg);
        // epilogue operands
        // (the two LSTM biases are added only at their use: an add here would wait on the loads
        // in front of the LDS hand-off)
        float eb[4] = {0.f, 0.f, 0.f, 0.f}, eb1[4] = {0.f, 0.f, 0.f, 0.f}, eh = 0.f, ec = 0.f;
        int eupd = 0;
        if constexpr (MODE == PKD_LSTM) {
            if (tid < DR * NU) {
                const int jj = tid % NU, r = min(tid / NU, R - 1), j = blockIdx.x * NU + jj;
                const size_t o = (size_t)(rg + r) * P + j;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    eb[q] = a.b0[q * P + j];
                    eb1[q] = a.b1[q * P + j];
                }
                eh = a.h_in[o];
                ec = a.c_in[o];
                eupd = a.st[rg + r].upd;
            }
        } else if constexpr (MODE == PKD_PRED) {
            if (tid < DR * DO) {
                const int o = tid % DO, r = min(tid / DO, R - 1), n = min(n0 + o, a.N - 1);
                eb[0] = a.b0[n];
                eupd = a.st[rg + r].upd;
            }
        } else {
            eb[0] = a.b0[min(n0 + (lane % DO), a.N - 1)];
        }
        lds_sync();  // the previous row group's LDS reads are done
#pragma unroll
        for (int u = 0; u < SE; ++u) {
            const int idx = tid + 512 * u;
            if (idx < NE) {
                const int k = 4 * (idx / DR), r = idx % DR;
                const bool ok = r < R;
                float4 x = v[u];
                if constexpr (MODE == PKD_JOINT)
                    x = make_float4(fmaxf(x.x + v2[u].x, 0.f), fmaxf(x.y + v2[u].y, 0.f), fmaxf(x.z + v2[u].z, 0.f),
                                    fmaxf(x.w + v2[u].w, 0.f));
                xs[(k + 0) * XP + r] = ok ? x.x : 0.f;
                xs[(k + 1) * XP + r] = ok ? x.y : 0.f;
                xs[(k + 2) * XP + r] = ok ? x.z : 0.f;
                xs[(k + 3) * XP + r] = ok ? x.w : 0.f;
            }
        }
        lds_sync();
        if (rg + rstep < a.B) load_x(rg + rstep, v, v2);
        float acc[4][DR];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < DR; ++r) acc[q][r] = 0.0f;
#pragma unroll
        for (int u = 0; u < NWM; ++u) {
            if (u < NW) {
                const float4* xr = (const float4*)(xs + (kb + kq + u * KS) * XP);
#pragma unroll
                for (int r4 = 0; r4 < DR / 4; ++r4) {
                    const float4 x = xr[r4];
                    const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        acc[0][4 * r4 + e] += w[u].x * xv[e];
                        acc[1][4 * r4 + e] += w[u].y * xv[e];
                        acc[2][4 * r4 + e] += w[u].z * xv[e];
                        acc[3][4 * r4 + e] += w[u].w * xv[e];
                    }
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < DR; ++r) {
                float t = acc[q][r];
#pragma unroll
                for (int m = OQ; m < 64; m <<= 1) t += __shfl_xor(t, m, 64);
                acc[q][r] = t;
            }
        if (kq == 0) {
#pragma unroll
            for (int r = 0; r < DR; ++r)
                *(float4*)(red + ((size_t)kg * DR + r) * DO + 4 * oq) = make_float4(acc[0][r], acc[1][r], acc[2][r], acc[3][r]);
        }
        lds_sync();
        for (int e = tid; e < DR * DO; e += 512) {  // fold the K-groups into slot 0
            const int r = e / DO, o = e % DO;
            float t = 0.0f;
#pragma unroll
            for (int g = 0; g < DG; ++g) t += red[((size_t)g * DR + r) * DO + o];
            red[(size_t)r * DO + o] = t;
        }
        lds_sync();
        if constexpr (MODE == PKD_LSTM) {
            if (tid < DR * NU) {
                const int jj = tid % NU, r = tid / NU;
                if (r < R) {
                    const int j = blockIdx.x * NU + jj;
                    float g[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) g[q] = (eb[q] + eb1[q]) + red[(size_t)r * DO + q * NU + jj];
                    float h = eh, c = ec;
                    asm volatile("" : "+v"(eupd));  // keeps the flag test here, not at its load
                    if (eupd) {
                        c = sig_(g[1]) * c + sig_(g[0]) * tanhf(g[2]);
                        h = sig_(g[3]) * tanhf(c);
                    }
                    const size_t o = (size_t)(rg + r) * P + j;
                    a.h_out[o] = h;
                    a.c_out[o] = c;
                }
            }
        } else if constexpr (MODE == PKD_PRED) {
            if (tid < DR * DO) {
                const int r = tid / DO, o = tid % DO, n = n0 + o;
                asm volatile("" : "+v"(eupd));
                if (r < R && n < a.N && eupd) a.gp[(size_t)(rg + r) * P + n] = eb[0] + red[(size_t)r * DO + o];
            }
        } else {
            // joint logits of this workgroup's DO outputs: per row (one wave per row) the token
            // top-2 (first index on ties) and the duration logits
            for (int r = kg; r < R; r += DG) {
                const int b = rg + r, n = n0 + lane;
                const float val = (lane < DO && n < a.N) ? eb[0] + red[(size_t)r * DO + lane] : -INFINITY;
                if (lane < DO && n > a.V && n < a.N) a.dur[(size_t)b * a.n_dur + (n - a.V - 1)] = val;
                const float vt = n <= a.V ? val : -INFINITY;
                const float v1 = wave_max(vt);
                int i1 = (vt == v1 && lane < DO) ? n : 0x7fffffff;
#pragma unroll
                for (int m = 32; m > 0; m >>= 1) i1 = min(i1, __shfl_xor(i1, m, 64));
                const float v2 = wave_max(n == i1 ? -INFINITY : vt);
                if (lane == 0) a.part[(size_t)b * a.n_tiles + blockIdx.x] = make_float4(v1, __int_as_float(i1), v2, 0.0f);
            }
        }
    }
}

// one workgroup per utterance: merge the joint's per-workgroup top-2 partials and the duration
// logits (first maximum wins, as the oracle's strict >), the TDT bookkeeping, and the next
// step's operand rows: the emitted token's embedding (LSTM layer 0 input) and the encoder
// projection of the row's new frame
__global__ __launch_bounds__(256) void joint_fin_kernel(PkFinArgs a) {
    __shared__ float s1[256], s2[256];
    __shared__ int i1[256];
    __shared__ PkState ns;
    const int b = blockIdx.x, tid = threadIdx.x;
    PkState* sb = a.st + b;
    if (sb->done) return;  // uniform
    float b1 = -INFINITY, b2 = -INFINITY;
    int t1 = 0x7fffffff;
    for (int i = tid; i < a.n_tiles; i += 256) {
        const float4 p = a.part[(size_t)b * a.n_tiles + i];
        const int pi = __float_as_int(p.y);
        const bool take = p.x > b1 || (p.x == b1 && pi < t1);
        b2 = fmaxf(fmaxf(b2, p.z), take ? b1 : p.x);
        if (take) { b1 = p.x; t1 = pi; }
    }
    s1[tid] = b1; s2[tid] = b2; i1[tid] = t1;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (tid < o) {
            const float a1 = s1[tid], a2 = s2[tid], c1 = s1[tid + o], c2 = s2[tid + o];
            const int ai = i1[tid], ci = i1[tid + o];
            const bool take = c1 > a1 || (c1 == a1 && ci < ai);
            s1[tid] = take ? c1 : a1;
            i1[tid] = take ? ci : ai;
            s2[tid] = fmaxf(fmaxf(a2, c2), take ? a1 : c1);
        }
        __syncthreads();
    }
    if (tid == 0) {
        PkState s = *sb;
        const int V = a.V, tk = i1[0];
        int skip = 0;
        for (int k = 1; k < a.n_dur; ++k)
            if (a.dur[(size_t)b * a.n_dur + k] > a.dur[(size_t)b * a.n_dur + skip]) skip = k;
        if (tk != V) {
            if (s.n_out < a.cap) {
                const size_t o = (size_t)b * a.cap + s.n_out;
                a.out_tok[o] = tk;
                a.out_frame[o] = s.t;
                a.out_t1[o] = s1[0];
                a.out_t2[o] = s2[0];
            }
            s.n_out++;
            s.upd = 1;
            s.tok = tk;
            s.at_t++;
        } else {
            s.upd = 0;
        }
        if (skip == 0 && (tk == V || s.at_t >= a.max_symbols)) skip = 1;
        if (skip > 0) s.at_t = 0;
        s.t += skip;
        if (s.t >= a.lens[b * 4 + 3]) s.done = 1;
        *sb = s;
        ns = s;
    }
    __syncthreads();
    const int P = a.P;
    if (ns.upd)
        for (int k = tid; k < P; k += 256) a.xemb[(size_t)b * P + k] = a.emb[(size_t)ns.tok * P + k];
    const int t = min(ns.t, ns.t3p - 1);
    for (int k = tid; k < P; k += 256) a.fecur[(size_t)b * P + k] = a.fe[((size_t)b * ns.t3p + t) * P + k];
}

// rows start at t = 0 with the blank symbol pending: zero states, the blank's (zero) embedding,
// frame 0's encoder projection
__global__ void state_init_kernel(PkState* st, int B, int V, float* h, float* c, int n, float* xemb, float* fecur,
                                  const float* fe, int T3p, int P, const int* __restrict__ lens) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < B) st[i] = PkState{0, 0, 0, lens[i * 4 + 3] <= 0 ? 1 : 0, 1, V, T3p};  // no frames: nothing to decode
    if (i < n) { h[i] = 0.0f; c[i] = 0.0f; }
    if (i < B * P) {
        const int b = i / P, k = i % P;
        xemb[i] = 0.0f;
        fecur[i] = fe[((size_t)b * T3p) * P + k];
    }
}

__global__ void place_lstm_kernel(const float* __restrict__ s, int P, float* __restrict__ d, int row0) {
    const int64_t total = (int64_t)4 * P * P;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int n = (int)(i % (4 * P)), k = (int)(i / (4 * P));  // src [4P][P]: gate row n = q P + j
        const int q = n / P, j = n % P;
        // blocked [P / 4][2P][16] (kLstmDO = 16): workgroup j / 4 owns the i, f, g, o rows of 4 units
        d[((size_t)(j / 4) * 2 * P + row0 + k) * 16 + q * 4 + (j % 4)] = s[(size_t)n * P + k];
    }
}

}  // namespace

void pk_frames(const float* pcm, int64_t stride, const int* nsamp, int B, int Tp, const float* window, float* frames,
               hipStream_t st) {
    hipLaunchKernelGGL(frames_kernel, dim3(Tp, B), dim3(256), 0, st, pcm, stride, nsamp, Tp, window, frames);
    SPT_LAUNCH_CHECK();
}

void pk_melpow(const float* spec, int M, const float* fbT, int n_mels, float* mel, hipStream_t st) {
    hipLaunchKernelGGL(melpow_kernel, dim3(M), dim3(128), 0, st, spec, fbT, n_mels, mel);
    SPT_LAUNCH_CHECK();
}

void pk_mel_norm(float* mel, const int* lens, int B, int Tp, int n_mels, hipStream_t st) {
    hipLaunchKernelGGL(mel_norm_kernel, dim3(B, cdiv(n_mels, 32)), dim3(256), 0, st, mel, lens, Tp, n_mels);
    SPT_LAUNCH_CHECK();
}

void pk_conv0(int dtype, const float* mel, const int* lens, int B, int Tp, int F, const float* w, const float* bias,
              int C, void* y, int T1p, int F1, hipStream_t st) {
    if (C > 1024) throw std::runtime_error("pk_conv0: more than 1024 channels");
    dim3 grid(T1p, B);
    const size_t sm = (size_t)3 * F * 4;
    if (dtype == DT_F16)
        hipLaunchKernelGGL(conv0_kernel<f16>, grid, dim3(C), sm, st, mel, lens, Tp, F, w, bias, C, (f16*)y, T1p, F1);
    else if (dtype == DT_BF16)
        hipLaunchKernelGGL(conv0_kernel<bf16>, grid, dim3(C), sm, st, mel, lens, Tp, F, w, bias, C, (bf16*)y, T1p, F1);
    else
        hipLaunchKernelGGL(conv0_kernel<float>, grid, dim3(C), sm, st, mel, lens, Tp, F, w, bias, C, (float*)y, T1p, F1);
    SPT_LAUNCH_CHECK();
}

void pk_dwconv(int dtype, const void* x, const int* lens, int stage, int B, int Tip, int Fi, const float* w,
               const float* bias, int C, void* y, int Top, int Fo, hipStream_t st) {
    if (C > 1024) throw std::runtime_error("pk_dwconv: more than 1024 channels");
    dim3 grid(Top, B);
    if (dtype == DT_F16)
        hipLaunchKernelGGL(dwconv_kernel<f16>, grid, dim3(C), 0, st, (const f16*)x, lens, stage, Tip, Fi, w, bias, C,
                           (f16*)y, Top, Fo);
    else if (dtype == DT_BF16)
        hipLaunchKernelGGL(dwconv_kernel<bf16>, grid, dim3(C), 0, st, (const bf16*)x, lens, stage, Tip, Fi, w, bias, C,
                           (bf16*)y, Top, Fo);
    else
        hipLaunchKernelGGL(dwconv_kernel<float>, grid, dim3(C), 0, st, (const float*)x, lens, stage, Tip, Fi, w, bias, C,
                           (float*)y, Top, Fo);
    SPT_LAUNCH_CHECK();
}

void pk_relpos(int dtype, int Tp, int d, void* pe, hipStream_t st) {
    const int g = grid_of((int64_t)(2 * Tp - 1) * (d / 2));
    if (dtype == DT_F16) hipLaunchKernelGGL(relpos_kernel<f16>, dim3(g), dim3(256), 0, st, Tp, d, (f16*)pe);
    else if (dtype == DT_BF16) hipLaunchKernelGGL(relpos_kernel<bf16>, dim3(g), dim3(256), 0, st, Tp, d, (bf16*)pe);
    else hipLaunchKernelGGL(relpos_kernel<float>, dim3(g), dim3(256), 0, st, Tp, d, (float*)pe);
    SPT_LAUNCH_CHECK();
}

void pk_rel_attn(int dtype, const void* qkv, const void* p, int ldp, const float* pu, const float* pv, const int* lens,
                 int B, int Tp, int H, int dk, void* out, hipStream_t st) {
    if (dk % 8 || dk > 256) throw std::runtime_error("pk_rel_attn: head dim must be a multiple of 8, <= 256");
    const size_t smem = (size_t)(2 * dk + Tp) * 4;
    if (smem > 64 * 1024) throw std::runtime_error("pk_rel_attn: too many frames for the LDS score row");
    static const bool valu = getenv("SPT_PK_ATTN_VALU") != nullptr;  // A/B switch
    if (dtype == DT_F16 && !valu && (dk == 64 || dk == 128)) {
        dim3 g(cdiv(Tp, 32), H, B);
        if (dk == 128)
            hipLaunchKernelGGL(rel_attn_mfma_kernel<128>, g, dim3(64), 0, st, (const f16*)qkv, (const f16*)p, ldp, pu, pv,
                               lens, Tp, H, (f16*)out);
        else
            hipLaunchKernelGGL(rel_attn_mfma_kernel<64>, g, dim3(64), 0, st, (const f16*)qkv, (const f16*)p, ldp, pu, pv,
                               lens, Tp, H, (f16*)out);
        SPT_LAUNCH_CHECK();
        return;
    }
    dim3 grid(Tp, H, B);
    if (dtype == DT_F16)
        hipLaunchKernelGGL(rel_attn_kernel<f16>, grid, dim3(64), smem, st, (const f16*)qkv, (const f16*)p, ldp, pu, pv,
                           lens, Tp, H, dk, (f16*)out);
    else if (dtype == DT_BF16)
        hipLaunchKernelGGL(rel_attn_kernel<bf16>, grid, dim3(64), smem, st, (const bf16*)qkv, (const bf16*)p, ldp, pu, pv,
                           lens, Tp, H, dk, (bf16*)out);
    else
        hipLaunchKernelGGL(rel_attn_kernel<float>, grid, dim3(64), smem, st, (const float*)qkv, (const float*)p, ldp, pu,
                           pv, lens, Tp, H, dk, (float*)out);
    SPT_LAUNCH_CHECK();
}

void pk_conv_module(int dtype, const void* a, const int* lens, int B, int Tp, int d, int K, const float* dw_w,
                    const float* dw_b, const float* bn_g, const float* bn_b, const float* bn_m, const float* bn_v,
                    void* out, hipStream_t st) {
    if (K != 9) throw std::runtime_error("pk_conv_module: depthwise kernel size 9 only");
    if (d % CM_V) throw std::runtime_error("pk_conv_module: channels must be a multiple of 4");
    dim3 grid(cdiv(Tp, CM_TT), B, cdiv(d, 256 * CM_V));
    if (dtype == DT_F16)
        hipLaunchKernelGGL((conv_module_kernel<f16, 9>), grid, dim3(256), 0, st, (const f16*)a, lens, Tp, d, dw_w, dw_b,
                           bn_g, bn_b, bn_m, bn_v, (f16*)out);
    else if (dtype == DT_BF16)
        hipLaunchKernelGGL((conv_module_kernel<bf16, 9>), grid, dim3(256), 0, st, (const bf16*)a, lens, Tp, d, dw_w, dw_b,
                           bn_g, bn_b, bn_m, bn_v, (bf16*)out);
    else
        hipLaunchKernelGGL((conv_module_kernel<float, 9>), grid, dim3(256), 0, st, (const float*)a, lens, Tp, d, dw_w,
                           dw_b, bn_g, bn_b, bn_m, bn_v, (float*)out);
    SPT_LAUNCH_CHECK();
}

void pk_place(int mode, int dtype, const float* src, int N, int K, void* dst, int ld, int row0, int C, int F,
              hipStream_t st) {
    if (mode == PK_PLACE_TRANSPOSE) {
        hipLaunchKernelGGL(place_transpose_kernel, dim3(grid_of((int64_t)N * K)), dim3(256), 0, st, src, N, K,
                           (float*)dst, ld, row0);
    } else if (mode == PK_PLACE_SUBPERM) {
        const int g = grid_of((int64_t)N * C * F);
        if (dtype == DT_F16) hipLaunchKernelGGL(place_subperm_kernel<f16>, dim3(g), dim3(256), 0, st, src, N, C, F, (f16*)dst);
        else if (dtype == DT_BF16)
            hipLaunchKernelGGL(place_subperm_kernel<bf16>, dim3(g), dim3(256), 0, st, src, N, C, F, (bf16*)dst);
        else hipLaunchKernelGGL(place_subperm_kernel<float>, dim3(g), dim3(256), 0, st, src, N, C, F, (float*)dst);
    } else {
        const int64_t n = (int64_t)N * K;
        const int g = grid_of(n);
        if (dtype == DT_F16) hipLaunchKernelGGL(place_copy_kernel<f16>, dim3(g), dim3(256), 0, st, src, n, (f16*)dst);
        else if (dtype == DT_BF16) hipLaunchKernelGGL(place_copy_kernel<bf16>, dim3(g), dim3(256), 0, st, src, n, (bf16*)dst);
        else hipLaunchKernelGGL(place_copy_kernel<float>, dim3(g), dim3(256), 0, st, src, n, (float*)dst);
    }
    SPT_LAUNCH_CHECK();
}

constexpr int kDecSmemMax = 159 * 1024;  // dynamic LDS bound (the kernel's static rows table needs the rest)
// outputs per workgroup of each stage (grids <= 256 workgroups: one round at one workgroup per CU)
constexpr int kLstmDO = 16, kPredDO = 16, kJointDO = 64;
// register-held wave-loads per lane and staged float4 per thread, sized for P <= 640
constexpr int kNWL = 10, kSEL = 5, kNWP = 5, kSEP = 3, kNWJ = 20, kSEJ = 3;
constexpr int kDecRowsWg = 2 * DR;  // utterances per decode workgroup (two row groups)

void pk_prepare() {  // > 64 KiB dynamic LDS: per kernel and device, before any stream capture
    ensure_lds_attr((const void*)dec_kernel<PKD_LSTM, kLstmDO, kNWL, kSEL>, kDecSmemMax);
    ensure_lds_attr((const void*)dec_kernel<PKD_PRED, kPredDO, kNWP, kSEP>, kDecSmemMax);
    ensure_lds_attr((const void*)dec_kernel<PKD_JOINT, kJointDO, kNWJ, kSEJ>, kDecSmemMax);
}

int pk_joint_tile() { return kJointDO; }

void pk_decode_stage(int mode, const PkDecArgs& a, hipStream_t s) {
    const int DO = mode == PKD_LSTM ? kLstmDO : mode == PKD_PRED ? kPredDO : kJointDO;
    const int nwm = mode == PKD_LSTM ? kNWL : mode == PKD_PRED ? kNWP : kNWJ;
    const int sem = mode == PKD_LSTM ? kSEL : mode == PKD_PRED ? kSEP : kSEJ;
    if (a.K % (DG * 4) || a.ld % DO || a.B < 1 || a.B > 64 || (mode == PKD_LSTM && a.P % (DO / 4)) ||
        a.K / 4 * DR > 512 * sem || (a.K / DG) % (256 / DO) || a.K / DG / (256 / DO) > nwm)
        throw std::runtime_error("pk_decode_stage: bad shape");
    const size_t smem = ((size_t)a.K * XP + (size_t)DG * DR * DO) * 4;
    if (smem > (size_t)kDecSmemMax) throw std::runtime_error("pk_decode_stage: K too large for the LDS row stage");
    // row groups (DR utterances each) spread over grid.y, kDecRowsWg utterances per workgroup: one
    // workgroup row running all 8 groups of a batch of 64 in turn took 50 us per LSTM stage (10 at
    // B = 8), 16 per workgroup 39, 8 per workgroup the same (every workgroup re-reads its weight
    // slice) and 32 slower (r3 exp_r3r: the stages are bound by rounds of workgroups, about one
    // 512-thread workgroup per CU at a time, not by the passes)
    const dim3 grid(mode == PKD_LSTM ? a.P / (DO / 4) : a.ld / DO, cdiv(a.B, kDecRowsWg));
    pk_prepare();
    switch (mode) {
        case PKD_LSTM: hipLaunchKernelGGL((dec_kernel<PKD_LSTM, kLstmDO, kNWL, kSEL>), grid, dim3(512), smem, s, a); break;
        case PKD_PRED: hipLaunchKernelGGL((dec_kernel<PKD_PRED, kPredDO, kNWP, kSEP>), grid, dim3(512), smem, s, a); break;
        case PKD_JOINT: hipLaunchKernelGGL((dec_kernel<PKD_JOINT, kJointDO, kNWJ, kSEJ>), grid, dim3(512), smem, s, a); break;
        default: throw std::runtime_error("pk_decode_stage: bad mode");
    }
    SPT_LAUNCH_CHECK();
}

void pk_joint_fin(const PkFinArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(joint_fin_kernel, dim3(a.B), dim3(256), 0, s, a);
    SPT_LAUNCH_CHECK();
}

void pk_state_init(PkState* st, int B, int V, float* h, float* c, int n, float* xemb, float* fecur, const float* fe, const int* lens,
                   int T3p, int P, hipStream_t s) {
    hipLaunchKernelGGL(state_init_kernel, dim3(cdiv(std::max(std::max(B, n), B * P), 256)), dim3(256), 0, s, st, B, V, h,
                       c, n, xemb, fecur, fe, T3p, P, lens);
    SPT_LAUNCH_CHECK();
}

__global__ void place_blocked_kernel(const float* __restrict__ s, int N, int K, int DO, float* __restrict__ d) {
    const int64_t total = (int64_t)N * K;
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int n = (int)(i % N), k = (int)(i / N);
        d[((size_t)(n / DO) * K + k) * DO + n % DO] = s[(size_t)n * K + k];
    }
}

void pk_place_blocked(const float* src, int N, int K, int mode, float* dst, hipStream_t s) {
    const int DO = mode == PKD_PRED ? kPredDO : kJointDO;
    hipLaunchKernelGGL(place_blocked_kernel, dim3(grid_of((int64_t)N * K)), dim3(256), 0, s, src, N, K, DO, dst);
    SPT_LAUNCH_CHECK();
}

void pk_place_lstm(const float* src, int P, float* dst, int row0, hipStream_t s) {
    hipLaunchKernelGGL(place_lstm_kernel, dim3(grid_of((int64_t)4 * P * P)), dim3(256), 0, s, src, P, dst, row0);
    SPT_LAUNCH_CHECK();
}

}  // namespace spt
