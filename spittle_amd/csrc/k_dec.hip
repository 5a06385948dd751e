// k_dec.hip -- the autoregressive decoder step (whisper.cpp whisper_build_graph_decoder
// + whisper_process_logits + greedy whisper_sample_token), entirely on the device:
// no per-step logits copy to the host, the next token is written straight into
// the next step's input, and the per-step state (position, step index) lives in
// device memory so one captured hipGraph replays every step.
//
// At <= 64 rows every projection is a weight stream (HBM-bound), so projections
// are "GEMV" kernels: a workgroup owns 16 x CT output columns; its 4 waves split
// the column tiles and K; each lane streams 64 contiguous bytes of one weight
// row per step straight into registers (two steps in flight, no LDS round trip)
// and the rows x 16 tile is an MFMA (16x16x32 bf16 / 16x16x4 f32) with the
// activations as the A operand.  A fused pre-LayerNorm is computed once per
// workgroup into a bank-padded LDS image that the MFMA A fragments read;
// bias / GELU / residual / KV-cache append are fused epilogues.
//
// Attention over the caches (self: <= 448 keys, cross: 1500 keys) is a
// flash-decoding kernel: one workgroup of 8 waves per (batch, head), 8 lanes per
// key so every load is a fully coalesced 16-byte-per-lane sweep of the K/V rows,
// online softmax per wave, a one-shot cross-wave merge in LDS.
#include "common.h"
#include "kernels.h"

#include <algorithm>

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

constexpr int GV_LDS_BYTES = 98304;  // LN image budget: rows x (K + pad) x sizeof(T)
__host__ __device__ inline int gv_img_bytes(int R, int K, int esz) {
    return ((R * (K + 16 / esz) * esz) + 15) & ~15;
}

struct alignas(16) TopP { float v1; int i1; float v2; int pad; };
__device__ __forceinline__ TopP top_merge(TopP a, TopP b) {
    const bool aw = (a.v1 > b.v1) || (a.v1 == b.v1 && a.i1 < b.i1);
    TopP r;
    r.pad = 0;
    if (aw) { r.v1 = a.v1; r.i1 = a.i1; r.v2 = fmaxf(a.v2, b.v1); }
    else { r.v1 = b.v1; r.i1 = b.i1; r.v2 = fmaxf(b.v2, a.v1); }
    return r;
}
__device__ __forceinline__ TopP top_shfl(TopP t, int mask) {
    TopP u;
    u.v1 = __shfl_xor(t.v1, mask, 64);
    u.i1 = __shfl_xor(t.i1, mask, 64);
    u.v2 = __shfl_xor(t.v2, mask, 64);
    u.pad = 0;
    return u;
}

// weight loads: default cache policy. Non-temporal (SPT_GV_NT=1) measured slower on MI355X
// (r1 ubench: logits 36.8 -> 58.6 us, one decoder layer 59.6 -> 76.9 us)
#ifndef SPT_GV_NT
#define SPT_GV_NT 0
#endif
template <typename F>
__device__ __forceinline__ F load_w(const F* p) {
#if SPT_GV_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

// NWV waves; CT column tiles of 16 per workgroup; KSPLIT = NWV / CT waves share a tile
// and split its K.  Each wave keeps up to MAXJ super-steps of weights in flight.
template <typename T, int MODE, bool LN, int RG, int NWV, int CT, int MAXJ>
__global__ __launch_bounds__(64 * NWV) void gemv_kernel(GemvArgs a) {
    constexpr int KS = GV<T>::KS;
    constexpr int EPL = KS / 4;          // elements per lane per super-step (64 bytes)
    constexpr int CPE = 16 / sizeof(T);  // elements per 16-byte chunk
    constexpr int KSPLIT = NWV / CT;
    typedef typename GV<T>::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int ct = wid % CT, ks = wid / CT;
    const int tile = blockIdx.x * CT + ct;
    const int n0 = tile * 16;
    const int K = a.K;
    const int lds_ld = K + CPE;  // padded row stride (elements): rows land 4 banks apart
    // K split across the grid's y dimension: this workgroup owns super-steps [ss0, ss1)
    const int kz = blockIdx.y, kzc = gridDim.y;
    const int nss_all = K / KS, per = (nss_all + kzc - 1) / kzc;
    const int ss0 = kz * per, ss1 = min(nss_all, ss0 + per);
    const T* wrow = (const T*)a.W + (size_t)min(n0 + fr, a.N - 1) * K + fq * EPL;

    frag w[MAXJ][4];
    auto load_chunk = [&](int j0) {
#pragma unroll
        for (int j = 0; j < MAXJ; ++j) {
            const int ss = ss0 + ks + (j0 + j) * KSPLIT;
            if (ss < ss1) {
#pragma unroll
                for (int i = 0; i < 4; ++i) w[j][i] = load_w((const frag*)(wrow + (size_t)ss * KS + i * CPE));
            }
        }
    };
    // LayerNorm input rows are fetched BEFORE the weight stream: loads retire in issue
    // order, so the prologue then waits only for its own row, not for the weights
    float4 x0[6];
    if constexpr (LN) {
        if (wid < a.R) {
            const float* xr = (const float*)a.A + (size_t)wid * a.lda + a.a_row0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) x0[i] = *(const float4*)(xr + k);
            }
        }
    }
    load_chunk(0);  // the first weight fetch overlaps the LayerNorm prologue

    if constexpr (LN) {
        T* img = (T*)smem;
        for (int r = wid; r < a.R; r += NWV) {
            const float* xr = (const float*)a.A + (size_t)r * a.lda + a.a_row0;
            float4 v[6];
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    v[i] = r == wid ? x0[i] : *(const float4*)(xr + k);
                    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
                }
            }
            const float mean = wave_sum(s) / (float)K;
            float s2 = 0.f;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    const float p = v[i].x - mean, q = v[i].y - mean, u = v[i].z - mean, ww = v[i].w - mean;
                    s2 += (p * p + q * q) + (u * u + ww * ww);
                }
            }
            const float rstd = 1.0f / sqrtf(wave_sum(s2) / (float)K + 1e-5f);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    const float4 g = *(const float4*)(a.ln_w + k);
                    const float4 b = *(const float4*)(a.ln_b + k);
                    T* o = img + (size_t)r * lds_ld + k;
                    o[0] = from_f<T>((v[i].x - mean) * rstd * g.x + b.x);
                    o[1] = from_f<T>((v[i].y - mean) * rstd * g.y + b.y);
                    o[2] = from_f<T>((v[i].z - mean) * rstd * g.z + b.z);
                    o[3] = from_f<T>((v[i].w - mean) * rstd * g.w + b.w);
                }
            }
        }
        __syncthreads();
    }

    f32x4 acc[RG];
#pragma unroll
    for (int g = 0; g < RG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto compute_chunk = [&](int j0) {
#pragma unroll
        for (int j = 0; j < MAXJ; ++j) {
            const int ss = ss0 + ks + (j0 + j) * KSPLIT;
            if (ss >= ss1) break;
            const int kb = ss * KS + fq * EPL;
#pragma unroll
            for (int g = 0; g < RG; ++g) {
                const int row = g * 16 + fr;
                frag af[4];
                if (row < a.R) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if constexpr (LN)
                            af[i] = *(const frag*)((const T*)smem + (size_t)row * lds_ld + kb + i * CPE);
                        else
                            af[i] = *(const frag*)((const T*)a.A + (size_t)row * a.lda + a.a_row0 + kb + i * CPE);
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) af[i] = frag{};
                }
                if constexpr (sizeof(T) == 2) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], w[j][i], acc[g], 0, 0, 0);
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e], w[j][i][e], acc[g], 0, 0, 0);
                }
            }
        }
    };
    for (int j0 = 0; ss0 + ks + j0 * KSPLIT < ss1; j0 += MAXJ) {
        if (j0 > 0) load_chunk(j0);
        compute_chunk(j0);
    }

    // cross-wave K reduction (waves sharing a column tile)
    if constexpr (KSPLIT > 1) {
        f32x4* red = (f32x4*)(smem + (LN ? gv_img_bytes(a.R, K, sizeof(T)) : 0));
        if (LN) __syncthreads();  // the LN image region is not reused, but keep waves in step
#pragma unroll
        for (int g = 0; g < RG; ++g) red[(wid * RG + g) * 64 + lane] = acc[g];
        __syncthreads();
        if (ks != 0) return;
#pragma unroll
        for (int g = 0; g < RG; ++g) {
            f32x4 v = acc[g];
#pragma unroll
            for (int s = 1; s < KSPLIT; ++s) v += red[(((s * CT) + ct) * RG + g) * 64 + lane];
            acc[g] = v;
        }
    }
    const int n = n0 + fr;
    if constexpr (MODE == GV_LOGITS) {
        // logits + this tile's suppressed top-2 per row (finished by dec_finalize)
        const int step = a.st->step;
        const bool nvalid = n < a.N;
        bool sup = !nvalid;
        if (nvalid) {
            sup = (a.suppress[n >> 5] >> (n & 31)) & 1u;
            if (step == 0 && (n == a.blank0 || n == a.blank1)) sup = true;
        }
#pragma unroll
        for (int g = 0; g < RG; ++g) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = g * 16 + 4 * fq + r;
                const float v = acc[g][r];
                if (nvalid && row < a.R) ((float*)a.C)[(size_t)row * a.ldc + n] = v;
                TopP t{sup ? -INFINITY : v, nvalid ? n : 0x7fffffff, -INFINITY, 0};
                t = top_merge(t, top_shfl(t, 1));
                t = top_merge(t, top_shfl(t, 2));
                t = top_merge(t, top_shfl(t, 4));
                t = top_merge(t, top_shfl(t, 8));
                if (fr == 0 && row < a.R && tile < a.n_tiles) ((TopP*)a.part)[(size_t)row * a.n_tiles + tile] = t;
            }
        }
        return;
    }
    if (n >= a.N) return;
    const float bv = a.bias ? a.bias[n] : 0.0f;
#pragma unroll
    for (int g = 0; g < RG; ++g) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g * 16 + 4 * fq + r;
            if (row >= a.R) continue;
            const float y = acc[g][r] + bv;
            if constexpr (MODE == GV_BIAS) {
                ((T*)a.C)[(size_t)row * a.ldc + n] = from_f<T>(y);
            } else if constexpr (MODE == GV_BIAS_GELU) {
                ((T*)a.C)[(size_t)row * a.ldc + n] = from_f<T>(gelu_tanh(y));
            } else if constexpr (MODE == GV_BIAS_RESID) {
                ((float*)a.C)[(size_t)row * a.ldc + n] += y;
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

template <typename T, int MODE, bool LN, int RG, int NWV, int CT, int MAXJ>
void gemv_attr() {
    const int red = NWV * RG * 64 * (int)sizeof(f32x4);
    HIP_CHECK(hipFuncSetAttribute((const void*)gemv_kernel<T, MODE, LN, RG, NWV, CT, MAXJ>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, GV_LDS_BYTES + red));
}

template <typename T, int MODE, bool LN, int RG, int NWV, int CT, int MAXJ>
void gemv_launch_cfg(const GemvArgs& a, hipStream_t st) {
    const int red = NWV * RG * 64 * (int)sizeof(f32x4);
    const int lds = (LN ? gv_img_bytes(a.R, a.K, sizeof(T)) : 0) + (NWV / CT > 1 ? red : 0);
    hipLaunchKernelGGL((gemv_kernel<T, MODE, LN, RG, NWV, CT, MAXJ>), dim3(cdiv(a.N, 16 * CT), a.ksplit),
                       dim3(64 * NWV), lds, st, a);
    SPT_LAUNCH_CHECK();
}

// geometry per shape (nss = super-steps of K): every wave's whole K slice in flight
// at once where registers allow, and at most one workgroup round on 256 CUs
#define SPT_GV_CONFIGS(X)   \
    X(4, 4, 4)  /* logits: 4 column tiles x 1 wave each */ \
    X(8, 1, 1)  /* nss <= 8  */ \
    X(8, 1, 2)  /* nss <= 16 */ \
    X(16, 1, 3) /* nss <= 48 */

// > 64 KiB of dynamic LDS must be enabled per kernel, outside any stream capture
template <typename T, int MODE, bool LN>
void gemv_attr_all() {
#define SPT_ATTR(NWV, CT, MAXJ)                        \
    gemv_attr<T, MODE, LN, 1, NWV, CT, MAXJ>();         \
    gemv_attr<T, MODE, LN, 2, NWV, CT, MAXJ>();         \
    gemv_attr<T, MODE, LN, 4, NWV, CT, MAXJ>();
    SPT_GV_CONFIGS(SPT_ATTR)
#undef SPT_ATTR
}
template <typename T>
void gemv_attr_modes() {
    gemv_attr_all<T, GV_BIAS, true>(); gemv_attr_all<T, GV_BIAS, false>();
    gemv_attr_all<T, GV_BIAS_GELU, true>(); gemv_attr_all<T, GV_BIAS_GELU, false>();
    gemv_attr_all<T, GV_BIAS_RESID, true>(); gemv_attr_all<T, GV_BIAS_RESID, false>();
    gemv_attr_all<T, GV_QKV_CACHE, true>(); gemv_attr_all<T, GV_QKV_CACHE, false>();
    gemv_attr_all<T, GV_LOGITS, true>(); gemv_attr_all<T, GV_LOGITS, false>();
}

template <typename T, int MODE, bool LN, int RG>
void gemv_launch_rg(const GemvArgs& a, hipStream_t st) {
    const int nss = cdiv(a.K / GV<T>::KS, a.ksplit);  // super-steps per workgroup
    if (a.N >= 16384) gemv_launch_cfg<T, MODE, LN, RG, 4, 4, 4>(a, st);
    else if (nss <= 8) gemv_launch_cfg<T, MODE, LN, RG, 8, 1, 1>(a, st);
    else if (nss <= 16) gemv_launch_cfg<T, MODE, LN, RG, 8, 1, 2>(a, st);
    else if (nss <= 48) gemv_launch_cfg<T, MODE, LN, RG, 16, 1, 3>(a, st);
    else throw std::runtime_error("gemv: K too large");
}

template <typename T, int MODE>
void gemv_launch(const GemvArgs& a, hipStream_t st) {
    const bool ln = a.ln_w != nullptr;
    if (ln && (gv_img_bytes(a.R, a.K, sizeof(T)) > GV_LDS_BYTES || a.K > 1536))
        throw std::runtime_error("gemv: LayerNorm image exceeds LDS budget");
    if (a.R <= 16) {
        if (ln) gemv_launch_rg<T, MODE, true, 1>(a, st);
        else gemv_launch_rg<T, MODE, false, 1>(a, st);
    } else if (a.R <= 32) {
        if (ln) gemv_launch_rg<T, MODE, true, 2>(a, st);
        else gemv_launch_rg<T, MODE, false, 2>(a, st);
    } else {
        if (ln) gemv_launch_rg<T, MODE, true, 4>(a, st);
        else gemv_launch_rg<T, MODE, false, 4>(a, st);
    }
}

// ------------------------------------------------------------------ attention (decode)
constexpr float kLog2Scale = 0.125f * 1.4426950408889634f;

template <typename T> struct KVChunk;  // 8 dims of one key row per lane
template <> struct KVChunk<bf16> {
    bf16x8 v;
    __device__ __forceinline__ void load(const bf16* p) { v = *(const bf16x8*)p; }
    __device__ __forceinline__ float at(int e) const { return bf2f((bf16)v[e]); }
};
template <> struct KVChunk<float> {
    f32x4 a, b;
    __device__ __forceinline__ void load(const float* p) { a = *(const f32x4*)p; b = *(const f32x4*)(p + 4); }
    __device__ __forceinline__ float at(int e) const { return e < 4 ? a[e] : b[e - 4]; }
};

// q rows: q + (b*Tq + t)*q_ld + h*64; K/V rows of (b, h): base + ((kv*B + b)*H + h)*ctx*64
// CAUSAL: self-attention over the cache (keys 0..pos0+t); else cross-attention (all keys).
// SPLIT: the keys of one (b, h) are cut into gridDim.y chunks, one workgroup each; every chunk
// publishes its (m, l, o[64]) with write-through (sc1) stores, and the chunk whose arrival
// ticket comes last merges them in chunk order (deterministic) and writes the output row.
template <typename T, int NQ, bool CAUSAL, int AWV, bool SPLIT>
__global__ __launch_bounds__(64 * AWV) void dec_attn_kernel(const T* __restrict__ q, int q_ld,
                                                            const T* __restrict__ kv, int B, int H, int ctx,
                                                            int n_keys_static, int Tq,
                                                            const DecState* __restrict__ ds, T* __restrict__ out,
                                                            float* __restrict__ xpart, unsigned* __restrict__ xcnt) {
    constexpr bool causal = CAUSAL;
    __shared__ float s_m[AWV][NQ], s_l[AWV][NQ];
    __shared__ float s_o[AWV][NQ][64];
    __shared__ int s_last;
    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int slot = lane >> 3, g = lane & 7;  // key slot within a group of 8, dim group (8 dims)
    const int pos0 = causal ? ds->pos0 : 0;
    const int n_keys = causal ? pos0 + Tq : n_keys_static;
    const T* Kb = kv + (((size_t)0 * B + b) * H + h) * (size_t)ctx * 64 + 8 * g;
    const T* Vb = kv + (((size_t)1 * B + b) * H + h) * (size_t)ctx * 64 + 8 * g;

    float qv[NQ][8], m[NQ], l[NQ], o[NQ][8];
    int lim[NQ];
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
        const int tt = t < Tq ? t : Tq - 1;
        const T* qr = q + (size_t)(b * Tq + tt) * q_ld + h * 64 + 8 * g;
#pragma unroll
        for (int e = 0; e < 8; ++e) qv[t][e] = to_f<T>(qr[e]) * kLog2Scale;
        m[t] = -INFINITY;
        l[t] = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[t][e] = 0.f;
        lim[t] = causal ? pos0 + tt + 1 : n_keys;
    }
    // NI groups of 8 keys per block; raw K/V chunks ping-pong so the next block streams in
    constexpr int NI = (sizeof(T) == 2) ? (NQ == 1 ? 8 : 4) : (NQ == 1 ? 4 : 2);
    constexpr int KB = 8 * NI;
    const int nblk_all = cdiv(n_keys, KB);
    const int S = SPLIT ? (int)gridDim.y : 1, sp = SPLIT ? (int)blockIdx.y : 0;
    const int per = cdiv(nblk_all, S);
    const int blk0 = sp * per, nblk = min(nblk_all, blk0 + per);
    KVChunk<T> kA[NI], vA[NI], kB[NI], vB[NI];
    auto load_blk = [&](KVChunk<T>(&kc)[NI], KVChunk<T>(&vc)[NI], int blk) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int key = min(blk * KB + 8 * i + slot, n_keys - 1);
            kc[i].load(Kb + (size_t)key * 64);
            vc[i].load(Vb + (size_t)key * 64);
        }
    };
    auto process = [&](const KVChunk<T>(&kc)[NI], const KVChunk<T>(&vc)[NI], int kbase) {
#pragma unroll
        for (int t = 0; t < NQ; ++t) {
            if (t >= Tq) break;
            float s[NI];
            float mb = -INFINITY;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                float v = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) v += qv[t][e] * kc[i].at(e);
                v += __shfl_xor(v, 1, 64);
                v += __shfl_xor(v, 2, 64);
                v += __shfl_xor(v, 4, 64);
                if (kbase + 8 * i + slot >= lim[t]) v = -INFINITY;
                s[i] = v;
                mb = fmaxf(mb, v);
            }
            mb = fmaxf(mb, __shfl_xor(mb, 8, 64));
            mb = fmaxf(mb, __shfl_xor(mb, 16, 64));
            mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
            if (mb == -INFINITY) continue;
            const float mn = fmaxf(m[t], mb);
            const float alpha = exp2f(m[t] - mn);
            float ls = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[t][e] *= alpha;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const float p = exp2f(s[i] - mn);
                ls += p;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[t][e] += p * vc[i].at(e);
            }
            l[t] = l[t] * alpha + ls;
            m[t] = mn;
        }
    };
    int blk = blk0 + wid;
    if (blk < nblk) load_blk(kA, vA, blk);
    while (blk < nblk) {
        int nb = blk + AWV;
        if (nb < nblk) load_blk(kB, vB, nb);
        process(kA, vA, blk * KB);
        blk = nb;
        if (blk >= nblk) break;
        nb = blk + AWV;
        if (nb < nblk) load_blk(kA, vA, nb);
        process(kB, vB, blk * KB);
        blk = nb;
    }
    // wave merge: sum l and o over the 8 key slots (m is wave-uniform)
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
        float lt = l[t];
        lt += __shfl_xor(lt, 8, 64);
        lt += __shfl_xor(lt, 16, 64);
        lt += __shfl_xor(lt, 32, 64);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float v = o[t][e];
            v += __shfl_xor(v, 8, 64);
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            o[t][e] = v;
        }
        if (lane < 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) s_o[wid][t][8 * g + e] = o[t][e];
        }
        if (lane == 0) {
            s_m[wid][t] = m[t];
            s_l[wid][t] = lt;
        }
    }
    __syncthreads();
    // workgroup merge: thread (t, e)
    float M = -INFINITY, L = 0.f, O = 0.f;
    const int t = tid >> 6, e = tid & 63;
    if (tid < 64 * Tq) {
#pragma unroll
        for (int w = 0; w < AWV; ++w) M = fmaxf(M, s_m[w][t]);
#pragma unroll
        for (int w = 0; w < AWV; ++w) {
            if (s_m[w][t] == -INFINITY) continue;
            const float f = exp2f(s_m[w][t] - M);
            L += s_l[w][t] * f;
            O += s_o[w][t][e] * f;
        }
    }
    if constexpr (SPLIT) {
        // publish this chunk: [bh][S][NQ][66] = {o[64], m, l}, write-through stores
        float* pp = xpart + (((size_t)bh * S + sp) * NQ) * 66;
        if (tid < 64 * Tq) {
            __hip_atomic_store(pp + t * 66 + e, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (e == 0) {
                __hip_atomic_store(pp + t * 66 + 64, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(pp + t * 66 + 65, L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const unsigned prev = __hip_atomic_fetch_add(xcnt + bh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = prev == (unsigned)S - 1;
            if (last) __hip_atomic_store(xcnt + bh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = last;
        }
        __syncthreads();
        if (!s_last) return;
        if (tid < 64 * Tq) {
            const float* pb = xpart + ((size_t)bh * S * NQ) * 66;
            M = -INFINITY;
            for (int c = 0; c < S; ++c)
                M = fmaxf(M, __hip_atomic_load(pb + (c * NQ + t) * 66 + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            L = 0.f;
            O = 0.f;
            for (int c = 0; c < S; ++c) {
                const float mc = __hip_atomic_load(pb + (c * NQ + t) * 66 + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (mc == -INFINITY) continue;
                const float f = exp2f(mc - M);
                L += __hip_atomic_load(pb + (c * NQ + t) * 66 + 65, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * f;
                O += __hip_atomic_load(pb + (c * NQ + t) * 66 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * f;
            }
        }
    }
    if (tid < 64 * Tq) out[(size_t)(b * Tq + t) * (H * 64) + h * 64 + e] = from_f<T>(O / L);
}

template <typename T, int NQ, bool CAUSAL, int AWV, bool SPLIT>
void dec_attn_cfg(const T* q, const T* kv, int nseq, int B_layout, int H, int ctx, int n_keys, int Tq,
                  const DecState* ds, T* out, int S, float* xpart, unsigned* xcnt, hipStream_t st) {
    hipLaunchKernelGGL((dec_attn_kernel<T, NQ, CAUSAL, AWV, SPLIT>), dim3(nseq * H, S), dim3(64 * AWV), 0, st, q,
                       H * 64, kv, B_layout, H, ctx, n_keys, Tq, ds, out, xpart, xcnt);
    SPT_LAUNCH_CHECK();
}

template <typename T>
void dec_attn_launch(const T* q, const T* kv, int nseq, int B_layout, int H, int ctx, int n_keys, int causal, int Tq,
                     const DecState* ds, T* out, const AttnSplit& sp, hipStream_t st) {
    if (causal) {
        if (Tq == 1) dec_attn_cfg<T, 1, true, 8, false>(q, kv, nseq, B_layout, H, ctx, n_keys, Tq, ds, out, 1, nullptr, nullptr, st);
        else dec_attn_cfg<T, 4, true, 8, false>(q, kv, nseq, B_layout, H, ctx, n_keys, Tq, ds, out, 1, nullptr, nullptr, st);
        return;
    }
    const int S = (sp.xpart && sp.xcnt) ? std::max(1, std::min(sp.splits, kAttnMaxSplit)) : 1;
    const int waves = sp.waves == 16 ? 16 : 8;
#define SPT_XA(NQ_, AW_)                                                                                         \
    if (S > 1) dec_attn_cfg<T, NQ_, false, AW_, true>(q, kv, nseq, B_layout, H, ctx, n_keys, Tq, ds, out, S,     \
                                                      sp.xpart, sp.xcnt, st);                                   \
    else dec_attn_cfg<T, NQ_, false, AW_, false>(q, kv, nseq, B_layout, H, ctx, n_keys, Tq, ds, out, 1, nullptr, \
                                                 nullptr, st);
    if (Tq == 1) {
        if (waves == 16) { SPT_XA(1, 16) } else { SPT_XA(1, 8) }
    } else {
        SPT_XA(4, 8)
    }
#undef SPT_XA
}

// ------------------------------------------------------------------ finalize
// Per sequence: reduce the logits tiles' top-2, record the token, choose the next
// input (argmax or forced), embed it for the next pass; the last block advances
// the step state (every block reads it before arriving).
template <typename T>
__global__ __launch_bounds__(256) void finalize_kernel(FinalizeArgs a) {
    __shared__ TopP s_top[4];
    __shared__ int s_tok;
    const int b = blockIdx.x, tid = threadIdx.x;
    const int step = a.ds->step, pos0 = a.ds->pos0;
    TopP t{-INFINITY, 0x7fffffff, -INFINITY, 0};
    const TopP* p = (const TopP*)a.part + (size_t)b * a.n_tiles;
    for (int i = tid; i < a.n_tiles; i += 256) t = top_merge(t, p[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t = top_merge(t, top_shfl(t, o));
    if ((tid & 63) == 0) s_top[tid >> 6] = t;
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; ++w) t = top_merge(t, s_top[w]);
        // non-finite logits leave no valid winner: record the sentinel, never index with it
        if (t.i1 < 0 || t.i1 >= a.n_vocab) {
            t.i1 = -2;
            t.v1 = t.v2 = __builtin_nanf("");
        }
        int nxt = a.eot;
        if (step < a.out_cap) {
            const int oi = b * a.out_cap + step;
            if (a.done[b]) {
                a.out_tok[oi] = -1;
                a.out_top1[oi] = -INFINITY;
                a.out_top2[oi] = -INFINITY;
            } else {
                a.out_tok[oi] = t.i1;
                a.out_top1[oi] = t.v1;
                a.out_top2[oi] = t.v2;
                nxt = t.i1;
                if (a.forced && step < a.forced_len) nxt = a.forced[b * a.forced_len + step];
                if (!a.ignore_eot && t.i1 == a.eot) a.done[b] = 1;
                if (nxt < 0 || nxt >= a.n_vocab) nxt = a.eot;
            }
        }
        a.next_tok[b] = nxt;
        s_tok = nxt;
    }
    __syncthreads();
    const int tok = s_tok;
    const int pn = min(pos0 + a.Tq, a.ctx - 1);
    const T* e = (const T*)a.emb + (size_t)tok * a.d;
    const float* pp = a.pos + (size_t)pn * a.d;
    for (int i = tid; i < a.d; i += 256) a.x[(size_t)b * a.d + i] = to_f<T>(e[i]) + pp[i];
    if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)gridDim.x - 1) {
            a.ds->pos0 = pos0 + a.Tq;
            a.ds->step = step + 1;
            __hip_atomic_store(a.arrive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void reset_kernel(DecState* ds, unsigned* arrive) {
    ds->pos0 = 0;
    ds->step = 0;
    *arrive = 0u;
}

}  // namespace

void gemv_prepare(int dtype) {
    if (dtype == DT_BF16) gemv_attr_modes<bf16>();
    else gemv_attr_modes<float>();
}

void gemv(int dtype, int mode, const GemvArgs& a_in, hipStream_t st) {
    if (a_in.R > 64 || a_in.R <= 0) throw std::runtime_error("gemv: rows must be in 1..64");
    const int ks = dtype == DT_BF16 ? 128 : 64;
    if (a_in.K % ks) throw std::runtime_error("gemv: K alignment");
    GemvArgs a = a_in;
    a.ksplit = 1;
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
    if (Tq < 1 || Tq > 4) throw std::runtime_error("dec_self_attn: 1..4 queries per sequence");
    if (dtype == DT_BF16)
        dec_attn_launch<bf16>((const bf16*)q, (const bf16*)cache, B, B, H, ctx, 0, 1, Tq, ds, (bf16*)out, AttnSplit{}, st);
    else
        dec_attn_launch<float>((const float*)q, (const float*)cache, B, B, H, ctx, 0, 1, Tq, ds, (float*)out, AttnSplit{},
                               st);
}

void dec_cross_attn(int dtype, const void* q, const void* kv, int B, int B_layout, int H, int T_enc, int Tq, void* out,
                    const AttnSplit& sp, hipStream_t st) {
    if (Tq < 1 || Tq > 4) throw std::runtime_error("dec_cross_attn: 1..4 queries per sequence");
    if (dtype == DT_BF16)
        dec_attn_launch<bf16>((const bf16*)q, (const bf16*)kv, B, B_layout, H, T_enc, T_enc, 0, Tq, nullptr, (bf16*)out,
                              sp, st);
    else
        dec_attn_launch<float>((const float*)q, (const float*)kv, B, B_layout, H, T_enc, T_enc, 0, Tq, nullptr,
                               (float*)out, sp, st);
}

void dec_finalize(int dtype, const FinalizeArgs& a, int B, hipStream_t st) {
    if (dtype == DT_BF16) hipLaunchKernelGGL(finalize_kernel<bf16>, dim3(B), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(finalize_kernel<float>, dim3(B), dim3(256), 0, st, a);
}

void dec_reset(DecState* ds, unsigned* arrive, hipStream_t st) {
    hipLaunchKernelGGL(reset_kernel, dim3(1), dim3(1), 0, st, ds, arrive);
}

}  // namespace spt
