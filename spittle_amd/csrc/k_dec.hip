// k_dec.hip -- the autoregressive decoder step (whisper.cpp whisper_build_graph_decoder
// + whisper_process_logits + greedy whisper_sample_token), entirely on the device:
// no per-step logits copy to the host, the next token is written straight into
// the next step's input, and the per-step state (position, step index) lives in
// device memory so one captured hipGraph replays every step.
//
// At batch <= 32 rows every projection is a weight stream (HBM-bound), so the
// projections are "GEMV" kernels: a workgroup owns 16 output columns, its 4 waves
// split K, each lane streams 64 contiguous bytes of one weight row per step
// straight into registers (no LDS round trip), and the rows x 16 tile is an
// MFMA (16x16x32 bf16 / 16x16x4 f32) with the activations as the A operand.
// The pre-LayerNorm is fused into the projection that consumes it (row stats
// recomputed per workgroup from the f32 residual), and bias / GELU / residual /
// KV-cache append are fused epilogues.
#include "common.h"
#include "kernels.h"

namespace spt {

namespace {

// ------------------------------------------------------------------ embed
template <typename T>
__global__ void embed_kernel(const int* __restrict__ tok, int Tq, int d, const T* __restrict__ emb,
                             const float* __restrict__ pos, const DecState* __restrict__ ds, float* __restrict__ x) {
    const int r = blockIdx.x, t = r % Tq;
    const int p = ds->pos0 + t;
    const T* e = emb + (size_t)tok[r] * d;
    const float* pp = pos + (size_t)p * d;
    for (int i = threadIdx.x; i < d; i += blockDim.x) x[(size_t)r * d + i] = to_f<T>(e[i]) + pp[i];
}

// ------------------------------------------------------------------ GEMV
template <typename T> struct GV;
template <> struct GV<bf16> {
    static constexpr int KS = 128;  // K per super-step: 4 lane groups x 32 elements
    typedef bf16x8 frag;
};
template <> struct GV<float> {
    static constexpr int KS = 64;   // 4 lane groups x 16 elements
    typedef f32x4 frag;
};

template <typename T, int MODE, bool LN, int RG>
__global__ __launch_bounds__(256) void gemv_kernel(GemvArgs a) {
    constexpr int KS = GV<T>::KS;
    constexpr int EPL = KS / 4;  // elements per lane per super-step (64 bytes)
    __shared__ float s_stat[64][2];
    __shared__ f32x4 s_red[4][RG][64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int n0 = blockIdx.x * 16;
    const int K = a.K;

    if constexpr (LN) {
        for (int r = wid; r < a.R; r += 4) {
            const float* xr = (const float*)a.A + (size_t)r * a.lda + a.a_row0;
            float s = 0.f;
            for (int k = lane * 4; k < K; k += 256) {
                const float4 v = *(const float4*)(xr + k);
                s += (v.x + v.y) + (v.z + v.w);
            }
            const float mean = wave_sum(s) / (float)K;
            float s2 = 0.f;
            for (int k = lane * 4; k < K; k += 256) {
                const float4 v = *(const float4*)(xr + k);
                const float p = v.x - mean, q = v.y - mean, u = v.z - mean, w = v.w - mean;
                s2 += (p * p + q * q) + (u * u + w * w);
            }
            const float rstd = 1.0f / sqrtf(wave_sum(s2) / (float)K + 1e-5f);
            if (lane == 0) { s_stat[r][0] = mean; s_stat[r][1] = rstd; }
        }
        __syncthreads();
    }

    const T* wrow = (const T*)a.W + (size_t)min(n0 + fr, a.N - 1) * K;
    f32x4 acc[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nss = K / KS;
    for (int ss = wid; ss < nss; ss += 4) {
        const int kb = ss * KS + fq * EPL;  // this lane's 64-byte slice of K
        typename GV<T>::frag wf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) wf[i] = *(const typename GV<T>::frag*)(wrow + kb + i * (16 / sizeof(T)));
#pragma unroll
        for (int g = 0; g < RG; ++g) {
            const int row = g * 16 + fr;
            typename GV<T>::frag af[4];
            if (row < a.R) {
                if constexpr (LN) {
                    const float* xr = (const float*)a.A + (size_t)row * a.lda + a.a_row0 + kb;
                    const float mean = s_stat[row][0], rstd = s_stat[row][1];
                    const float* gw = a.ln_w + kb;
                    const float* gb = a.ln_b + kb;
                    if constexpr (sizeof(T) == 2) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
#pragma unroll
                            for (int j = 0; j < 8; j += 4) {
                                const float4 v = *(const float4*)(xr + 8 * i + j);
                                const float4 w = *(const float4*)(gw + 8 * i + j);
                                const float4 bb = *(const float4*)(gb + 8 * i + j);
                                af[i][j + 0] = (short)f2bf((v.x - mean) * rstd * w.x + bb.x);
                                af[i][j + 1] = (short)f2bf((v.y - mean) * rstd * w.y + bb.y);
                                af[i][j + 2] = (short)f2bf((v.z - mean) * rstd * w.z + bb.z);
                                af[i][j + 3] = (short)f2bf((v.w - mean) * rstd * w.w + bb.w);
                            }
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const float4 v = *(const float4*)(xr + 4 * i);
                            const float4 w = *(const float4*)(gw + 4 * i);
                            const float4 bb = *(const float4*)(gb + 4 * i);
                            af[i][0] = (v.x - mean) * rstd * w.x + bb.x;
                            af[i][1] = (v.y - mean) * rstd * w.y + bb.y;
                            af[i][2] = (v.z - mean) * rstd * w.z + bb.z;
                            af[i][3] = (v.w - mean) * rstd * w.w + bb.w;
                        }
                    }
                } else {
                    const T* ar = (const T*)a.A + (size_t)row * a.lda + a.a_row0 + kb;
#pragma unroll
                    for (int i = 0; i < 4; ++i) af[i] = *(const typename GV<T>::frag*)(ar + i * (16 / sizeof(T)));
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) af[i] = typename GV<T>::frag{};
            }
            if constexpr (sizeof(T) == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], wf[i], acc[g], 0, 0, 0);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e], wf[i][e], acc[g], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int g = 0; g < RG; ++g) s_red[wid][g][lane] = acc[g];
    __syncthreads();
    if (wid != 0) return;
    const int n = n0 + fr;
    if (n >= a.N) return;
    const float bv = a.bias ? a.bias[n] : 0.0f;
#pragma unroll
    for (int g = 0; g < RG; ++g) {
        const f32x4 v = s_red[0][g][lane] + s_red[1][g][lane] + s_red[2][g][lane] + s_red[3][g][lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g * 16 + 4 * fq + r;
            if (row >= a.R) continue;
            const float y = v[r] + bv;
            if constexpr (MODE == GV_BIAS) {
                ((T*)a.C)[(size_t)row * a.ldc + n] = from_f<T>(y);
            } else if constexpr (MODE == GV_BIAS_GELU) {
                ((T*)a.C)[(size_t)row * a.ldc + n] = from_f<T>(gelu_tanh(y));
            } else if constexpr (MODE == GV_BIAS_RESID) {
                ((float*)a.C)[(size_t)row * a.ldc + n] += y;
            } else if constexpr (MODE == GV_LOGITS) {
                ((float*)a.C)[(size_t)row * a.ldc + n] = v[r];
            } else if constexpr (MODE == GV_QKV_CACHE) {
                const int d = a.cache_H * 64;
                if (n < d) {
                    ((T*)a.C)[(size_t)row * a.ldc + n] = from_f<T>(y);
                } else {
                    const int part = n / d - 1;  // 0 = K, 1 = V
                    const int rem = n - (part + 1) * d;
                    const int hh = rem >> 6, e = rem & 63;
                    const int bb = row / a.Tq, t = row - bb * a.Tq;
                    const int pos = a.st->pos0 + t;
                    const size_t off = ((((size_t)part * a.cache_B + bb) * a.cache_H + hh) * a.cache_ctx + pos) * 64 + e;
                    ((T*)a.cache)[off] = from_f<T>(y);
                }
            }
        }
    }
}

template <typename T, int MODE>
void gemv_launch(const GemvArgs& a, hipStream_t st) {
    dim3 grid(cdiv(a.N, 16));
    const bool ln = a.ln_w != nullptr;
    if (a.R <= 16) {
        if (ln) hipLaunchKernelGGL((gemv_kernel<T, MODE, true, 1>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((gemv_kernel<T, MODE, false, 1>), grid, dim3(256), 0, st, a);
    } else if (a.R <= 32) {
        if (ln) hipLaunchKernelGGL((gemv_kernel<T, MODE, true, 2>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((gemv_kernel<T, MODE, false, 2>), grid, dim3(256), 0, st, a);
    } else {
        if (ln) hipLaunchKernelGGL((gemv_kernel<T, MODE, true, 4>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((gemv_kernel<T, MODE, false, 4>), grid, dim3(256), 0, st, a);
    }
}

// ------------------------------------------------------------------ attention (decode)
// One workgroup per (b, h, key chunk).  Scores thread-per-key (Tq <= 4 queries),
// softmax over the chunk, then P.V with 64 dims x 4 key groups.
template <typename T>
__device__ __forceinline__ void load_row64(const T* p, float* v) {
    if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const bf16x8 x = *(const bf16x8*)(p + 8 * c);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[8 * c + j] = bf2f((bf16)x[j]);
        }
    } else {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            const float4 x = *(const float4*)(p + 4 * c);
            v[4 * c] = x.x; v[4 * c + 1] = x.y; v[4 * c + 2] = x.z; v[4 * c + 3] = x.w;
        }
    }
}

constexpr int MAXQ = 4;       // queries per (b, h) in one pass (prompt of <= 4 tokens)
constexpr int MAXKC = 512;    // keys per workgroup chunk

// Kc: keys [kc0, kc1) of the K/V arrays (row stride 64); queries q[t] (t < Tq) see keys
// < kv_lim(t).  Writes unnormalised (m, l, o) of each query.
template <typename T>
__device__ void attn_chunk(const T* __restrict__ Kc, const T* __restrict__ Vc, int kc0, int kc1, const float* sq,
                           int Tq, const int* kv_lim, float* s_p, float* s_red, float* out_m, float* out_l,
                           float* out_o /* [Tq][64] */) {
    const int tid = threadIdx.x;
    const int nk = kc1 - kc0;
    // scores
    for (int j = tid; j < nk; j += 256) {
        float kv[64];
        load_row64<T>(Kc + (size_t)(kc0 + j) * 64, kv);
        for (int t = 0; t < Tq; ++t) {
            float s = 0.f;
#pragma unroll
            for (int e = 0; e < 64; ++e) s += sq[t * 64 + e] * kv[e];
            s_p[t * MAXKC + j] = (kc0 + j < kv_lim[t]) ? s * 0.125f : -INFINITY;
        }
    }
    __syncthreads();
    for (int t = 0; t < Tq; ++t) {
        // max
        float m = -INFINITY;
        for (int j = tid; j < nk; j += 256) m = fmaxf(m, s_p[t * MAXKC + j]);
        m = wave_max(m);
        if ((tid & 63) == 0) s_red[tid >> 6] = m;
        __syncthreads();
        m = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
        __syncthreads();
        float l = 0.f;
        for (int j = tid; j < nk; j += 256) {
            const float s = s_p[t * MAXKC + j];
            const float p = (m == -INFINITY) ? 0.f : __expf(s - m);
            s_p[t * MAXKC + j] = p;
            l += p;
        }
        l = wave_sum(l);
        if ((tid & 63) == 0) s_red[tid >> 6] = l;
        __syncthreads();
        l = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
        if (tid == 0) { out_m[t] = m; out_l[t] = l; }
        __syncthreads();
    }
    // P.V : thread (e = tid & 63, g = tid >> 6) sums keys j = g, g+4, ...
    const int e = tid & 63, g = tid >> 6;
    float accv[MAXQ] = {0.f, 0.f, 0.f, 0.f};
    for (int j = g; j < nk; j += 4) {
        const float v = to_f<T>(Vc[(size_t)(kc0 + j) * 64 + e]);
        for (int t = 0; t < Tq; ++t) accv[t] += s_p[t * MAXKC + j] * v;
    }
    __shared__ float s_acc[4][MAXQ][64];
    for (int t = 0; t < Tq; ++t) s_acc[g][t][e] = accv[t];
    __syncthreads();
    if (g == 0)
        for (int t = 0; t < Tq; ++t) out_o[t * 64 + e] = (s_acc[0][t][e] + s_acc[1][t][e]) + (s_acc[2][t][e] + s_acc[3][t][e]);
    __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(256) void self_attn_kernel(const T* __restrict__ q, const T* __restrict__ cache, int B,
                                                        int H, int ctx, int Tq, const DecState* __restrict__ ds,
                                                        T* __restrict__ out) {
    __shared__ float sq[MAXQ * 64];
    __shared__ float s_p[MAXQ * MAXKC];
    __shared__ float s_red[4];
    __shared__ float s_m[MAXQ], s_l[MAXQ], s_o[MAXQ * 64];
    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int d = H * 64;
    const int pos0 = ds->pos0;
    for (int i = threadIdx.x; i < Tq * 64; i += 256) {
        const int t = i >> 6, e = i & 63;
        sq[i] = to_f<T>(q[(size_t)(b * Tq + t) * d + h * 64 + e]);
    }
    int lim[MAXQ];
    for (int t = 0; t < MAXQ; ++t) lim[t] = pos0 + t + 1;
    __syncthreads();
    const T* Kc = cache + (((size_t)0 * B + b) * H + h) * ctx * 64;
    const T* Vc = cache + (((size_t)1 * B + b) * H + h) * ctx * 64;
    attn_chunk<T>(Kc, Vc, 0, pos0 + Tq, sq, Tq, lim, s_p, s_red, s_m, s_l, s_o);
    for (int i = threadIdx.x; i < Tq * 64; i += 256) {
        const int t = i >> 6, e = i & 63;
        out[(size_t)(b * Tq + t) * d + h * 64 + e] = from_f<T>(s_o[i] / s_l[t]);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void cross_attn_kernel(const T* __restrict__ q, const T* __restrict__ kv, int B,
                                                         int H, int Tenc, int Tq, int nsplit, float* __restrict__ part) {
    __shared__ float sq[MAXQ * 64];
    __shared__ float s_p[MAXQ * MAXKC];
    __shared__ float s_red[4];
    __shared__ float s_m[MAXQ], s_l[MAXQ], s_o[MAXQ * 64];
    const int sp = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int d = H * 64;
    for (int i = threadIdx.x; i < Tq * 64; i += 256) {
        const int t = i >> 6, e = i & 63;
        sq[i] = to_f<T>(q[(size_t)(b * Tq + t) * d + h * 64 + e]);
    }
    int lim[MAXQ];
    for (int t = 0; t < MAXQ; ++t) lim[t] = Tenc;
    __syncthreads();
    const int chunk = cdiv(Tenc, nsplit);
    const int k0 = sp * chunk, k1 = min(Tenc, k0 + chunk);
    const T* Kc = kv + (((size_t)0 * B + b) * H + h) * Tenc * 64;
    const T* Vc = kv + (((size_t)1 * B + b) * H + h) * Tenc * 64;
    attn_chunk<T>(Kc, Vc, k0, k1, sq, Tq, lim, s_p, s_red, s_m, s_l, s_o);
    // part layout [b*Tq + t][h][split][66] : m, l, o[64]
    for (int i = threadIdx.x; i < Tq * 66; i += 256) {
        const int t = i / 66, c = i - t * 66;
        const float v = c == 0 ? s_m[t] : (c == 1 ? s_l[t] : s_o[t * 64 + c - 2]);
        part[(((size_t)(b * Tq + t) * H + h) * nsplit + sp) * 66 + c] = v;
    }
}

template <typename T>
__global__ void combine_kernel(const float* __restrict__ part, int H, int nsplit, T* __restrict__ out) {
    const int r = blockIdx.x, h = blockIdx.y, e = threadIdx.x;
    const float* p = part + ((size_t)r * H + h) * nsplit * 66;
    float m = -INFINITY;
    for (int s = 0; s < nsplit; ++s) m = fmaxf(m, p[s * 66]);
    float l = 0.f, o = 0.f;
    for (int s = 0; s < nsplit; ++s) {
        const float w = __expf(p[s * 66] - m);
        l += p[s * 66 + 1] * w;
        o += p[s * 66 + 2 + e] * w;
    }
    out[(size_t)r * H * 64 + h * 64 + e] = from_f<T>(o / l);
}

// ------------------------------------------------------------------ argmax + suppression
struct Top { float v1; int i1; float v2; };
__device__ __forceinline__ Top top_merge(Top a, Top b) {
    const bool aw = (a.v1 > b.v1) || (a.v1 == b.v1 && a.i1 < b.i1);
    Top r;
    if (aw) { r.v1 = a.v1; r.i1 = a.i1; r.v2 = fmaxf(a.v2, b.v1); }
    else { r.v1 = b.v1; r.i1 = b.i1; r.v2 = fmaxf(b.v2, a.v1); }
    return r;
}

__global__ __launch_bounds__(1024) void argmax_kernel(ArgmaxArgs a) {
    __shared__ Top s_top[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int step = a.ds->step;
    const float* lg = a.logits + (size_t)b * a.V;
    Top t{-INFINITY, 0x7fffffff, -INFINITY};
    for (int i = tid; i < a.V; i += 1024) {
        float v = lg[i];
        if ((a.suppress[i >> 5] >> (i & 31)) & 1u) v = -INFINITY;
        if (step == 0 && (i == a.blank0 || i == a.blank1)) v = -INFINITY;
        Top u{v, i, -INFINITY};
        t = top_merge(t, u);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        Top u;
        u.v1 = __shfl_xor(t.v1, o, 64);
        u.i1 = __shfl_xor(t.i1, o, 64);
        u.v2 = __shfl_xor(t.v2, o, 64);
        t = top_merge(t, u);
    }
    if ((tid & 63) == 0) s_top[tid >> 6] = t;
    __syncthreads();
    if (tid != 0) return;
    for (int w = 1; w < 16; ++w) t = top_merge(t, s_top[w]);
    const int oi = b * a.out_cap + step;
    if (step >= a.out_cap) return;
    if (a.done[b]) {
        a.out_tok[oi] = -1;
        a.out_top1[oi] = -INFINITY;
        a.out_top2[oi] = -INFINITY;
        a.next_tok[b] = a.eot;
        return;
    }
    a.out_tok[oi] = t.i1;
    a.out_top1[oi] = t.v1;
    a.out_top2[oi] = t.v2;
    int nxt = t.i1;
    if (a.forced && step < a.forced_len) nxt = a.forced[b * a.forced_len + step];
    a.next_tok[b] = nxt;
    if (!a.ignore_eot && t.i1 == a.eot) a.done[b] = 1;
}

__global__ void advance_kernel(DecState* ds, int Tq) {
    ds->pos0 += Tq;
    ds->step += 1;
}
__global__ void reset_kernel(DecState* ds) {
    ds->pos0 = 0;
    ds->step = 0;
}

}  // namespace

void gemv(int dtype, int mode, const GemvArgs& a, hipStream_t st) {
    if (a.R > 64 || a.R <= 0) throw std::runtime_error("gemv: rows must be in 1..64");
    if (a.K % (dtype == DT_BF16 ? 128 : 64)) throw std::runtime_error("gemv: K alignment");
#define SPT_GV(T, M) \
    case M: gemv_launch<T, M>(a, st); return;
    if (dtype == DT_BF16) {
        switch (mode) { SPT_GV(bf16, GV_BIAS) SPT_GV(bf16, GV_BIAS_GELU) SPT_GV(bf16, GV_BIAS_RESID)
                        SPT_GV(bf16, GV_QKV_CACHE) SPT_GV(bf16, GV_LOGITS) }
    } else {
        switch (mode) { SPT_GV(float, GV_BIAS) SPT_GV(float, GV_BIAS_GELU) SPT_GV(float, GV_BIAS_RESID)
                        SPT_GV(float, GV_QKV_CACHE) SPT_GV(float, GV_LOGITS) }
    }
#undef SPT_GV
    throw std::runtime_error("gemv: bad mode");
}

void dec_embed(int dtype, const int* tok, int R, int Tq, int d, const void* tok_emb, const float* pos_emb,
               const DecState* ds, float* x, hipStream_t st) {
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(embed_kernel<bf16>, dim3(R), dim3(256), 0, st, tok, Tq, d, (const bf16*)tok_emb, pos_emb, ds, x);
    else
        hipLaunchKernelGGL(embed_kernel<float>, dim3(R), dim3(256), 0, st, tok, Tq, d, (const float*)tok_emb, pos_emb, ds, x);
}

void dec_self_attn(int dtype, const void* q, const void* cache, int B, int H, int ctx, int Tq, const DecState* ds,
                   void* out, hipStream_t st) {
    if (Tq > MAXQ || ctx > MAXKC) throw std::runtime_error("dec_self_attn: shape");
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(self_attn_kernel<bf16>, dim3(B * H), dim3(256), 0, st, (const bf16*)q, (const bf16*)cache, B, H,
                           ctx, Tq, ds, (bf16*)out);
    else
        hipLaunchKernelGGL(self_attn_kernel<float>, dim3(B * H), dim3(256), 0, st, (const float*)q, (const float*)cache, B,
                           H, ctx, Tq, ds, (float*)out);
}

void dec_cross_attn(int dtype, const void* q, const void* kv, int B, int H, int T_enc, int Tq, int n_split, float* part,
                    void* out, hipStream_t st) {
    if (Tq > MAXQ || cdiv(T_enc, n_split) > MAXKC) throw std::runtime_error("dec_cross_attn: shape");
    dim3 grid(n_split, H, B);
    if (dtype == DT_BF16) {
        hipLaunchKernelGGL(cross_attn_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)q, (const bf16*)kv, B, H, T_enc,
                           Tq, n_split, part);
        hipLaunchKernelGGL(combine_kernel<bf16>, dim3(B * Tq, H), dim3(64), 0, st, part, H, n_split, (bf16*)out);
    } else {
        hipLaunchKernelGGL(cross_attn_kernel<float>, grid, dim3(256), 0, st, (const float*)q, (const float*)kv, B, H, T_enc,
                           Tq, n_split, part);
        hipLaunchKernelGGL(combine_kernel<float>, dim3(B * Tq, H), dim3(64), 0, st, part, H, n_split, (float*)out);
    }
}

void dec_argmax(const ArgmaxArgs& a, int B, hipStream_t st) {
    hipLaunchKernelGGL(argmax_kernel, dim3(B), dim3(1024), 0, st, a);
}

void dec_advance(DecState* ds, int Tq, hipStream_t st) {
    hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, st, ds, Tq);
}
void dec_reset(DecState* ds, hipStream_t st) { hipLaunchKernelGGL(reset_kernel, dim3(1), dim3(1), 0, st, ds); }

}  // namespace spt
