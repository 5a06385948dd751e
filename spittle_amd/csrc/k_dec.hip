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

#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#ifndef SPT_STAMP
#define SPT_STAMP 0
#endif

namespace spt {

#if SPT_STAMP
// developer timeline of the decode-step cross-attention (SPT_STAMP=1 builds): per workgroup
// {entry, streaming done, exit} in s_memrealtime ticks
__device__ unsigned long long* g_xattn_stamp;
void set_xattn_stamp(void* p) { HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_xattn_stamp), &p, sizeof(p))); }
#define XA_STAMP(i)                                                                          \
    do {                                                                                     \
        if (g_xattn_stamp && threadIdx.x == 0)                                               \
            g_xattn_stamp[3 * blockIdx.x + (i)] = __builtin_amdgcn_s_memrealtime();          \
    } while (0)
#else
#define XA_STAMP(i) do {} while (0)
#endif

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
// blockIdx.y splits K across workgroups (GV_PARTIAL only: each split writes its own
// partial slab, summed in split order by the consumer's A_LN prologue).
// ASRC selects the A operand:
//   A_DIRECT  activation rows [R][lda] of type T read straight into MFMA fragments;
//   A_LN      LayerNorm of the f32 residual rows x + pend[0..np-1] (the pending partial slabs
//             of the previous GV_PARTIAL launch), staged as a bank-padded LDS image;
//             workgroup (0, 0) also writes the combined rows to x_out;
//   A_ATTN    the cross-attention output merged from its S key-chunk partials
//             [R][H][S][66] = {o[64], m, l} (rows of this workgroup's K range), staged in LDS.
// kernel-side A source codes: A_DIRECT, LN_SRC(np) = A_LN with np pending slabs (0, 1, 2, 4), or
// ATTN_SRC(s) = A_ATTN combining s cross-attention key chunks
constexpr int LN_SRC(int np) { return 16 + np; }
constexpr bool is_ln(int asrc) { return asrc >= 16 && asrc < 32; }
constexpr int ln_np(int asrc) { return asrc - 16; }
constexpr int ATTN_SRC(int s) { return 32 + s; }
constexpr bool is_attn(int asrc) { return asrc >= 32; }
constexpr int attn_s(int asrc) { return asrc - 32; }

// developer timeline (SPT_STAMP=1 builds): thread 0's view of its workgroup's start / end
#define GV_STAMP(i)                                                                                       \
    do {                                                                                                  \
        if (SPT_STAMP && a.stamp && threadIdx.x == 0)                                                     \
            a.stamp[2 * (blockIdx.x + blockIdx.y * gridDim.x) + (i)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)

template <typename T, int MODE, int ASRC, int RG, int NWV, int CT, int MAXJ, bool EXACT = false>
__global__ __launch_bounds__(64 * NWV) void gemv_kernel(GemvArgs a) {
    GV_STAMP(0);
    constexpr int KS = GV<T>::KS;
    constexpr int CPE = 16 / sizeof(T);  // elements per 16-byte chunk
    constexpr int KSPLIT = NWV / CT;
    constexpr bool IMG = ASRC != A_DIRECT;
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
    // K order inside a super-step: MFMA step i, lane group fq takes the 16-byte chunk 4 i + fq,
    // so the four lanes of a weight row read 64 contiguous bytes per load instruction (16 rows x
    // 64 B per wave-instruction instead of 64 scattered 16-byte pieces); A uses the same order
    const T* wrow = (const T*)a.W + (size_t)min(n0 + fr, a.N - 1) * K + fq * CPE;

    frag w[MAXJ][4];
    // EXACT (every wave's K slice is exactly MAXJ super-steps, checked at launch): the weight
    // loads are unconditional, so the compiler can wait for the LayerNorm rows and prefetched
    // operands (issued before them) with a counted vmcnt that leaves the weight stream in flight.
    // Otherwise a predicated load makes every such wait a vmcnt(0) (r2: the LayerNorm then ran
    // only after the weights had landed); forcing unconditional loads there instead (waves
    // re-reading a super-step) measured slower (r2 exp_r2c).
    auto load_chunk = [&](int j0) {
#pragma unroll
        for (int j = 0; j < MAXJ; ++j) {
            const int ss = ss0 + ks + (j0 + j) * KSPLIT;
            if (EXACT || ss < ss1) {
#pragma unroll
                for (int i = 0; i < 4; ++i) w[j][i] = load_w((const frag*)(wrow + (size_t)ss * KS + i * 4 * CPE));
            }
        }
    };
    // LayerNorm input rows (x and the pending slabs) are fetched BEFORE the weight stream:
    // loads retire in issue order, so the prologue then waits only for its own row.  The slab
    // count is a template constant: loads under a runtime select are serialised by hipcc.
    constexpr int NP = is_ln(ASRC) ? ln_np(ASRC) : 0;
    float4 x0[NP + 1][6];
    if constexpr (is_ln(ASRC)) {
        if (wid < a.R) {
            const size_t ro = (size_t)wid * a.lda + a.a_row0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    x0[0][i] = *(const float4*)((const float*)a.A + ro + k);
#pragma unroll
                    for (int p = 0; p < NP; ++p) x0[p + 1][i] = *(const float4*)(a.pend[p] + ro + k);
                }
            }
        }
    }
    // Every operand of the LayerNorm and of the epilogue is fetched here, up front, beside the
    // LayerNorm rows and before the weight stream: a workgroup then pays one memory round trip
    // (kernel arguments aside) instead of one per dependent stage (r2 chain timeline: the
    // epilogue's bias / residual loads and the LayerNorm's gain / shift loads were each a round
    // trip after the weights had arrived).
    const int n_ep = n0 + fr;  // the output column this lane finishes
    const bool ep_lane = ks == 0 && n_ep < a.N;
    float bias_pre = 0.f;
    if constexpr (MODE != GV_LOGITS) {
        if (ep_lane && a.bias && kz == 0) bias_pre = a.bias[n_ep];
    }
    float resid_pre[RG][4];
    // GV_PARTIAL with p_resid: split 0 adds the residual rows into its slab, so the consumer's
    // prologue sums one slab fewer (x + p0 is formed here instead of there: the same operation)
    const float* resid = MODE == GV_BIAS_RESID ? (const float*)a.C
                         : MODE == GV_PARTIAL && kz == 0 ? a.p_resid : nullptr;
    if constexpr (MODE == GV_BIAS_RESID || MODE == GV_PARTIAL) {
#pragma unroll
        for (int g = 0; g < RG; ++g)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = g * 16 + 4 * fq + r;
                resid_pre[g][r] = (resid && ep_lane && row < a.R) ? resid[(size_t)row * a.ldc + n_ep] : 0.f;
            }
    }
    int st_pre = 0;  // decoder step state: GV_QKV_CACHE appends at pos0, GV_LOGITS reads step
    if constexpr (MODE == GV_QKV_CACHE) st_pre = a.st->pos0;
    if constexpr (MODE == GV_LOGITS) st_pre = a.st->step;
    uint32_t sup_pre = 0;
    if constexpr (MODE == GV_LOGITS) {
        if (n_ep < a.N) sup_pre = a.suppress[n_ep >> 5];
    }
    float4 lnw_pre[6], lnb_pre[6];
    if constexpr (is_ln(ASRC)) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int k = lane * 4 + 256 * i;
            if (k < K) {
                lnw_pre[i] = *(const float4*)(a.ln_w + k);
                lnb_pre[i] = *(const float4*)(a.ln_b + k);
            }
        }
    }
    load_chunk(0);  // the first weight fetch overlaps the prologue

    if constexpr (is_ln(ASRC)) {
        T* img = (T*)smem;
        const bool wr_x = a.x_out && blockIdx.x == 0 && blockIdx.y == 0;
        for (int r = wid; r < a.R; r += NWV) {
            const size_t ro = (size_t)r * a.lda + a.a_row0;
            float4 v[6];
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    float4 u[NP + 1];
                    if (r == wid) {
#pragma unroll
                        for (int p = 0; p <= NP; ++p) u[p] = x0[p][i];
                    } else {
                        u[0] = *(const float4*)((const float*)a.A + ro + k);
#pragma unroll
                        for (int p = 0; p < NP; ++p) u[p + 1] = *(const float4*)(a.pend[p] + ro + k);
                    }
                    // x + p0 + p1 + ..., always in this order (deterministic)
                    v[i] = u[0];
#pragma unroll
                    for (int p = 1; p <= NP; ++p) {
                        v[i].x += u[p].x; v[i].y += u[p].y; v[i].z += u[p].z; v[i].w += u[p].w;
                    }
                    if (wr_x) *(float4*)(a.x_out + ro + k) = v[i];
                    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
                }
            }
            const float mean = wave_sum(s) / (float)K;
            float s2 = 0.f;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    s2 += ln_sq4(v[i], mean);
                }
            }
            const float rstd = 1.0f / sqrtf(wave_sum(s2) / (float)K + 1e-5f);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    const float4 g = lnw_pre[i];
                    const float4 b = lnb_pre[i];
                    T* o = img + (size_t)r * lds_ld + k;
                    o[0] = from_f<T>(ln_out(v[i].x, mean, rstd, g.x, b.x));
                    o[1] = from_f<T>(ln_out(v[i].y, mean, rstd, g.y, b.y));
                    o[2] = from_f<T>(ln_out(v[i].z, mean, rstd, g.z, b.z));
                    o[3] = from_f<T>(ln_out(v[i].w, mean, rstd, g.w, b.w));
                }
            }
        }
        __syncthreads();
    }

    if constexpr (is_attn(ASRC)) {
        // flash-decoding merge of the S chunks: heads covering this workgroup's K range;
        // thread <-> (row r, head h, element e)
        constexpr int S = attn_s(ASRC);
        SPT_LDS T* img = (SPT_LDS T*)smem;  // LDS-typed: the stores cannot alias the partials' loads
        const int H = a.a_heads;
        const int h0 = (ss0 * KS) >> 6, h1 = min(H, (ss1 * KS + 63) >> 6);
        const int nh = h1 - h0;
        const int total = a.R * nh * 64;
        // one element per thread per round: the engine takes this prologue for one row only (B = 1:
        // 1280 elements over 512 threads); several rows merge once in attn_part_merge_kernel (r4:
        // batching four elements per round here cost the one-row pass 1.5 %, 189 VGPRs)
        for (int idx = tid; idx < total; idx += 64 * NWV) {
            const int r = idx / (nh * 64), rem = idx - r * nh * 64;
            const int h = h0 + (rem >> 6), e = rem & 63;
            const float* pp = a.apart + ((size_t)r * H + h) * S * 66;
            float mc[S], lc[S], oc[S];
#pragma unroll
            for (int c = 0; c < S; ++c) {
                mc[c] = pp[c * 66 + 64];
                lc[c] = pp[c * 66 + 65];
                oc[c] = pp[c * 66 + e];
            }
            float M = mc[0];
#pragma unroll
            for (int c = 1; c < S; ++c) M = fmaxf(M, mc[c]);
            float L = 0.f, O = 0.f;
#pragma unroll
            for (int c = 0; c < S; ++c) {  // attn_merge's operations (bitwise): skip empty chunks
                if (mc[c] == -INFINITY) continue;
                const float f = exp2f(mc[c] - M);
                L = __builtin_fmaf(lc[c], f, L);
                O = __builtin_fmaf(oc[c], f, O);
            }
            img[(size_t)r * lds_ld + h * 64 + e] = from_f<T>(O / L);
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
            if (!EXACT && ss >= ss1) break;
            const int kb = ss * KS + fq * CPE;
#pragma unroll
            for (int g = 0; g < RG; ++g) {
                const int row = g * 16 + fr;
                frag af[4];
                if (row < a.R) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if constexpr (IMG)
                            af[i] = *(const frag*)((const T*)smem + (size_t)row * lds_ld + kb + i * 4 * CPE);
                        else
                            af[i] = *(const frag*)((const T*)a.A + (size_t)row * a.lda + a.a_row0 + kb + i * 4 * CPE);
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
    if constexpr (EXACT) {
        compute_chunk(0);
    } else {
        for (int j0 = 0; ss0 + ks + j0 * KSPLIT < ss1; j0 += MAXJ) {
            if (j0 > 0) load_chunk(j0);
            compute_chunk(j0);
        }
    }

    // cross-wave K reduction (waves sharing a column tile)
    if constexpr (KSPLIT > 1) {
        f32x4* red = (f32x4*)(smem + (IMG ? gv_img_bytes(a.R, K, sizeof(T)) : 0));
        if (IMG) __syncthreads();  // the image region is not reused, but keep waves in step
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
        const int step = st_pre;
        const bool nvalid = n < a.N;
        bool sup = !nvalid;
        if (nvalid) {
            sup = (sup_pre >> (n & 31)) & 1u;
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
        GV_STAMP(1);
        return;
    }
    if (n >= a.N) return;
    const float bv = bias_pre;
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
            } else if constexpr (MODE == GV_PARTIAL) {
                ((float*)a.C + (size_t)kz * a.c_split)[(size_t)row * a.ldc + n] = resid ? resid_pre[g][r] + y : y;
            } else if constexpr (MODE == GV_BIAS_RESID) {
                ((float*)a.C)[(size_t)row * a.ldc + n] = resid_pre[g][r] + y;
            } else if constexpr (MODE == GV_QKV_CACHE) {
                const int d = a.cache_H * 64;
                if (n < d) {
                    ((T*)a.C)[(size_t)row * a.ldc + n] = from_f<T>(y);
                } else {
                    const int part = n / d - 1;  // 0 = K, 1 = V
                    const int rem = n - (part + 1) * d;
                    const int hh = rem >> 6, e = rem & 63;
                    const int bb = row / a.Tq, t = row - bb * a.Tq;
                    const int pos = st_pre + t;
                    const size_t off = ((((size_t)part * a.cache_B + bb) * a.cache_H + hh) * a.cache_ctx + pos) * 64 + e;
                    ((T*)a.cache)[off] = from_f<T>(y);
                }
            }
        }
    }
    GV_STAMP(1);
}

template <typename T, int MODE, int ASRC, int RG, int NWV, int CT, int MAXJ, bool EXACT = false>
void gemv_attr() {  // per kernel and device (ensure_lds_attr)
    const int red = NWV * RG * 64 * (int)sizeof(f32x4);
    ensure_lds_attr((const void*)gemv_kernel<T, MODE, ASRC, RG, NWV, CT, MAXJ, EXACT>, GV_LDS_BYTES + red);
}

template <typename T, int MODE, int ASRC, int RG, int NWV, int CT, int MAXJ, bool EXACT = false>
void gemv_launch_cfg(const GemvArgs& a, hipStream_t st) {
    if (EXACT && cdiv(a.K / GV<T>::KS, a.ksplit) != MAXJ * (NWV / CT))
        throw std::runtime_error("gemv: exact configuration does not match the K slice");
    const int red = NWV * RG * 64 * (int)sizeof(f32x4);
    const int lds = (ASRC != A_DIRECT ? gv_img_bytes(a.R, a.K, sizeof(T)) : 0) + (NWV / CT > 1 ? red : 0);
    hipLaunchKernelGGL((gemv_kernel<T, MODE, ASRC, RG, NWV, CT, MAXJ, EXACT>), dim3(cdiv(a.N, 16 * CT), a.ksplit),
                       dim3(64 * NWV), lds, st, a);
    SPT_LAUNCH_CHECK();
}

// geometry per shape (nss = super-steps of K per workgroup): every wave's whole K slice in
// flight at once where registers allow; logits: 4 column tiles x 1 wave each (4, 4, 4)
#define SPT_GV_CONFIGS(X)   \
    X(4, 1, 2)  /* nss <= 8  */ \
    X(8, 1, 2)  /* nss <= 16 */ \
    X(16, 1, 3) /* nss <= 48 */

// the (mode, A source) pairs the decoder uses
#define SPT_GV_PAIRS(X)                 \
    X(GV_QKV_CACHE, LN_SRC(0))          \
    X(GV_QKV_CACHE, LN_SRC(1))          \
    X(GV_QKV_CACHE, LN_SRC(2))          \
    X(GV_QKV_CACHE, LN_SRC(4))          \
    X(GV_BIAS, LN_SRC(0))               \
    X(GV_BIAS, LN_SRC(2))               \
    X(GV_BIAS_GELU, LN_SRC(0))          \
    X(GV_LOGITS, LN_SRC(0))             \
    X(GV_LOGITS, LN_SRC(1))             \
    X(GV_LOGITS, LN_SRC(2))             \
    X(GV_LOGITS, LN_SRC(4))             \
    X(GV_PARTIAL, A_DIRECT)             \
    X(GV_BIAS_RESID, A_DIRECT)          \
    X(GV_BIAS_RESID, ATTN_SRC(2))       \
    X(GV_BIAS_RESID, ATTN_SRC(3))       \
    X(GV_BIAS_RESID, ATTN_SRC(4))       \
    X(GV_BIAS_RESID, ATTN_SRC(8))

// > 64 KiB of dynamic LDS must be enabled per kernel, outside any stream capture
template <typename T, int MODE, int ASRC>
void gemv_attr_all() {
#define SPT_ATTR(NWV, CT, MAXJ)                          \
    gemv_attr<T, MODE, ASRC, 1, NWV, CT, MAXJ>();         \
    gemv_attr<T, MODE, ASRC, 2, NWV, CT, MAXJ>();         \
    gemv_attr<T, MODE, ASRC, 4, NWV, CT, MAXJ>();
    if constexpr (MODE == GV_LOGITS) {
        SPT_ATTR(4, 4, 4)
        SPT_ATTR(8, 8, 4)
    } else if constexpr (ASRC == A_DIRECT || is_attn(ASRC)) {
        SPT_GV_CONFIGS(SPT_ATTR)
        gemv_attr<T, MODE, ASRC, 1, 12, 1, 1, true>();
        gemv_attr<T, MODE, ASRC, 2, 12, 1, 1, true>();
        gemv_attr<T, MODE, ASRC, 4, 12, 1, 1, true>();
    } else {
        SPT_ATTR(4, 1, 2)
        SPT_ATTR(8, 1, 2)
        SPT_ATTR(8, 2, 3)
        gemv_attr<T, MODE, ASRC, 1, 10, 1, 1, true>();
        gemv_attr<T, MODE, ASRC, 2, 10, 1, 1, true>();
        gemv_attr<T, MODE, ASRC, 4, 10, 1, 1, true>();
        gemv_attr<T, MODE, ASRC, 1, 10, 2, 2, true>();
        gemv_attr<T, MODE, ASRC, 2, 10, 2, 2, true>();
        gemv_attr<T, MODE, ASRC, 4, 10, 2, 2, true>();
        gemv_attr<T, MODE, ASRC, 1, 12, 1, 1, true>();
        gemv_attr<T, MODE, ASRC, 2, 12, 1, 1, true>();
        gemv_attr<T, MODE, ASRC, 4, 12, 1, 1, true>();
    }
#undef SPT_ATTR
}
template <typename T>
void gemv_attr_modes() {
#define SPT_PAIR(M, S) gemv_attr_all<T, M, S>();
    SPT_GV_PAIRS(SPT_PAIR)
#undef SPT_PAIR
}

template <typename T, int MODE, int ASRC, int RG>
void gemv_launch_rg(const GemvArgs& a, hipStream_t st) {
    const int nss = cdiv(a.K / GV<T>::KS, a.ksplit);  // super-steps per workgroup
    if constexpr (MODE == GV_LOGITS) {
        // one wave per 16-column tile over all of K either way (bitwise the same logits); wider
        // workgroups stage each LayerNorm image for more tiles (SPT_GV_LOGITS_CT = 4 / 8, r4)
        static const int lct = getenv("SPT_GV_LOGITS_CT") ? atoi(getenv("SPT_GV_LOGITS_CT")) : 4;
        if (lct == 8) gemv_launch_cfg<T, MODE, ASRC, RG, 8, 8, 4>(a, st);
        else gemv_launch_cfg<T, MODE, ASRC, RG, 4, 4, 4>(a, st);
    } else {
        // Wide LayerNorm-prologue GEMVs (fc1, N = 4d >= 4096): two column tiles per workgroup,
        // so half as many workgroups re-read the residual rows for their LayerNorm image (r1
        // exp23: fc1 9.4 -> 8.6 us, RTFx +1.2 %; the QKV and cross-Q projections lose with it)
        // an attention-merge prologue (A_ATTN) takes A_DIRECT's geometry: the same waves and K
        // slices, so the cross output projection of merged key partials is bitwise the projection
        // of the 8-wave kernel's output (dec_cross_attn_vw)
        if constexpr (is_ln(ASRC)) {
            // K = 10 super-steps (large-v3's d = 1280 in bf16): 10 waves, each an exact slice, so
            // the LayerNorm does not wait for the weight stream (GV_EXACT_LN=0 restores r1's shapes)
            static const bool exact_ln = !getenv("GV_EXACT_LN") || atoi(getenv("GV_EXACT_LN")) != 0;
            // SPT_GV_CT2_MIN: the smallest N given two column tiles per workgroup (experiments)
            static const int ct2_min = getenv("SPT_GV_CT2_MIN") ? atoi(getenv("SPT_GV_CT2_MIN")) : 4096;
            if (exact_ln && nss == 10) {
                if (a.N >= ct2_min) gemv_launch_cfg<T, MODE, ASRC, RG, 10, 2, 2, true>(a, st);
                else gemv_launch_cfg<T, MODE, ASRC, RG, 10, 1, 1, true>(a, st);
                return;
            }
            // K = 12 super-steps (Whisper-small's d = 768 in f32, the C2 decoder): 12 waves, one exact
            // super-step each (experiment; SPT_GV_EXACT12=0: the 8-wave shape)
            static const bool exact12 = !getenv("SPT_GV_EXACT12") || atoi(getenv("SPT_GV_EXACT12")) != 0;
            if (exact_ln && exact12 && nss == 12) {
                gemv_launch_cfg<T, MODE, ASRC, RG, 12, 1, 1, true>(a, st);
                return;
            }
            if (a.N >= 4096 && nss <= 24) {
                gemv_launch_cfg<T, MODE, ASRC, RG, 8, 2, 3>(a, st);
                return;
            }
        }
        // the directly-read / attention-merge GEMVs of 12 super-steps (C2's self-out and cross-out) on
        // the same exact 12-wave split (r6ac: pass 0.623 -> 0.618 ms; SPT_GV_EXACT12_DIRECT=0: 8 waves).
        // A_DIRECT and A_ATTN keep one geometry, so the merged-partials projection stays bitwise the
        // merge kernel's
        static const bool exact12_direct = !getenv("SPT_GV_EXACT12_DIRECT") || atoi(getenv("SPT_GV_EXACT12_DIRECT")) != 0;
        if constexpr (!is_ln(ASRC)) {
            if (exact12_direct && nss == 12) {
                gemv_launch_cfg<T, MODE, ASRC, RG, 12, 1, 1, true>(a, st);
                return;
            }
        }
        if (nss <= 8) gemv_launch_cfg<T, MODE, ASRC, RG, 4, 1, 2>(a, st);
        else if (nss <= 16) gemv_launch_cfg<T, MODE, ASRC, RG, 8, 1, 2>(a, st);
        else if constexpr (!is_ln(ASRC)) {  // 16 waves: no room for a staged A image's registers
            if (nss <= 48) gemv_launch_cfg<T, MODE, ASRC, RG, 16, 1, 3>(a, st);
            else throw std::runtime_error("gemv: K too large");
        } else throw std::runtime_error("gemv: K too large for a staged A operand");
    }
}

template <typename T, int MODE, int ASRC>
void gemv_launch(const GemvArgs& a, hipStream_t st) {
    if (a.R <= 16) gemv_launch_rg<T, MODE, ASRC, 1>(a, st);
    else if (a.R <= 32) gemv_launch_rg<T, MODE, ASRC, 2>(a, st);
    else gemv_launch_rg<T, MODE, ASRC, 4>(a, st);
}

}  // namespace
}  // namespace spt

#include "dec_attn.h"

namespace spt {
namespace {

// Self-attention over the cache (keys 0..pos0+t), one workgroup per (b, h).
// q rows: q + (b*Tq + t)*q_ld + h*64; K/V rows of (b, h): base + ((kv*B + b)*H + h)*ctx*64.
template <typename T, int NQ, int NIX = 0>
__global__ __launch_bounds__(64 * AW) void self_attn_kernel(const T* __restrict__ q, int q_ld,
                                                            const T* __restrict__ kv, int B, int H, int ctx, int Tq,
                                                            const DecState* __restrict__ ds, T* __restrict__ out) {
    __shared__ float s_m[AW][NQ], s_l[AW][NQ];
    __shared__ float s_o[AW][NQ][64];
    const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane & 7;
    AttnWave<T, NQ, NIX> aw;
    // the wave's first key block is fetched before the position is known (every cache row is
    // readable): the K/V stream no longer waits behind the DecState round trip (run_pre)
    aw.init(kv + (((size_t)0 * B + b) * H + h) * (size_t)ctx * 64 + 8 * g,
            kv + (((size_t)1 * B + b) * H + h) * (size_t)ctx * 64 + 8 * g, ctx, lane);
    aw.load_blk(aw.kc_[0], aw.vc_[0], wid);
    const int pos0 = ds->pos0;
    const int n_keys = pos0 + Tq;
    aw.n_keys = n_keys;
    float qv[NQ][8];
    int lim[NQ];
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
        const int tt = t < Tq ? t : Tq - 1;
        const T* qr = q + (size_t)(b * Tq + tt) * q_ld + h * 64 + 8 * g;
#pragma unroll
        for (int e = 0; e < 8; ++e) qv[t][e] = to_f<T>(qr[e]) * kLog2Scale;
        lim[t] = pos0 + tt + 1;
    }
    aw.template run_pre<(448 / AttnWave<T, NQ, NIX>::KB + 1 + AW - 1) / AW>(wid, cdiv(n_keys, AttnWave<T, NQ, NIX>::KB), qv, lim, Tq);
    aw.to_lds(s_m, s_l, s_o, wid, lane);
    __syncthreads();
    if (tid < 64 * Tq) {
        const int t = tid >> 6, e = tid & 63;
        float M, L, O;
        attn_merge<NQ>(s_m, s_l, s_o, t, e, M, L, O);
        out[(size_t)(b * Tq + t) * (H * 64) + h * 64 + e] = from_f<T>(O / L);
    }
}

// Cross-attention over the cached encoder K/V (all T_enc keys), one workgroup per (row run, h).
// kv: one layer in the kv_offset layout of B_layout windows, at the group's first window (no map)
// or at the layer (kvrow: the window of each run of `share` rows).  A workgroup takes queries
// [blockIdx.y * NQ, + NQ) of its run's share * Tq query rows (rows j * share .. + share - 1, Tq
// each), so the decoders of one utterance (beam / best_of) read its window's K/V once per chunk.
// (A fused LayerNorm + cross-Q projection prologue and key-chunk splits were measured slower on
// MI355X: r1 exp_fused_xattn_pending_slabs.txt.)
template <typename T, int NQ, bool SPLIT, int NW = AW, int NIX = 0, int PF = 2>
__global__ __launch_bounds__(64 * NW) void cross_attn_kernel(const T* __restrict__ q, const T* __restrict__ kv,
                                                             int B_layout, int H, int T_enc, int Tq,
                                                             T* __restrict__ out, float* __restrict__ part,
                                                             const int* __restrict__ kvrow, int share) {
    typedef AttnWave<T, NQ, NIX, NW, PF> W;
    XA_STAMP(0);
    __shared__ float s_m[NW][NQ], s_l[NW][NQ];
    __shared__ float s_o[NW][NQ][64];
    const int bh = blockIdx.x, j = bh / H, h = bh - j * H;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane & 7;
    const int nq_all = share * Tq;                          // query rows of this run
    const int c0 = SPLIT ? 0 : (int)blockIdx.y * NQ;        // first query of this workgroup
    const int nq = min(NQ, nq_all - c0);
    const int kb = kvrow ? kvrow[j * share] : j;            // the run's window
    W aw;  // kv_offset layout: 32-key blocks [T/32][B][H][2][32][64]
    const size_t kvo = ((size_t)kb * H + h) * 4096 + 8 * g;
    aw.init(kv + kvo, kv + kvo + 2048, T_enc, lane, (int64_t)B_layout * H * 4096);
    const size_t qrow0 = (size_t)j * nq_all + c0;           // = (j * share) * Tq + c0
    float qv[NQ][8];
    int lim[NQ];
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
        const int tt = t < nq ? t : nq - 1;
        const T* qr = q + (qrow0 + tt) * (H * 64) + h * 64 + 8 * g;
#pragma unroll
        for (int e = 0; e < 8; ++e) qv[t][e] = to_f<T>(qr[e]) * kLog2Scale;
        lim[t] = T_enc;
    }
    // SPLIT: this workgroup's chunk of the key blocks (gridDim.y chunks, block-aligned)
    const int nblk_all = cdiv(T_enc, W::KB);
    const int S = SPLIT ? (int)gridDim.y : 1, sp = SPLIT ? (int)blockIdx.y : 0;
    const int per = cdiv(nblk_all, S), blk0 = sp * per, nblk = min(nblk_all, blk0 + per);
    aw.template run<(1500 / W::KB + 1 + NW - 1) / NW>(blk0 + wid, nblk, qv, lim, nq);
    if (wid == 0) XA_STAMP(1);
    aw.to_lds(s_m, s_l, s_o, wid, lane);
    __syncthreads();
    XA_STAMP(2);
    for (int i = tid; i < 64 * nq; i += 64 * NW) {
        const int t = i >> 6, e = i & 63;
        float M, L, O;
        attn_merge<NQ, NW>(s_m, s_l, s_o, t, e, M, L, O);
        if constexpr (SPLIT) {  // partial {o[64], m, l} for the output projection's merge prologue
            float* pp = part + (((qrow0 + t) * H + h) * S + sp) * 66;
            pp[e] = O;
            if (e == 0) {
                pp[64] = M;
                pp[65] = L;
            }
        } else {
            out[(qrow0 + t) * (H * 64) + h * 64 + e] = from_f<T>(O / L);
        }
    }
}

// The same cross-attention with each of the 8 waves of a (row run, h) workgroup as a workgroup
// of its own (grid.y = the wave index w, grid.z = the query chunk): wave w of the 8-wave kernel
// and workgroup w here run the same AttnWave over the same key blocks (w, w + 8, ...), and each
// writes its {o[64], m, l} as partial w of [rows][H][8][66]; the cross output projection's A_ATTN
// prologue merges the 8 partials in order w = 0..7 with attn_merge's arithmetic.  A row's result
// is therefore bitwise the 8-wave kernel's, and the choice between the two is free: this one runs
// when the 8-wave grid is small (B = 1, or the decoders of one utterance sharing a window), where
// 20 workgroups would stream 7.7 MB per layer through 20 CUs.
template <typename T, int NQ, int NIX = 0, int PF = 2>
__global__ __launch_bounds__(64) void cross_attn_vw_kernel(const T* __restrict__ q, const T* __restrict__ kv,
                                                           int B_layout, int H, int T_enc, int Tq,
                                                           float* __restrict__ part, const int* __restrict__ kvrow,
                                                           int share) {
    typedef AttnWave<T, NQ, NIX, AW, PF> W;  // block stride AW = the 8-wave kernel's waves
    __shared__ float s_m[1][NQ], s_l[1][NQ];
    __shared__ float s_o[1][NQ][64];
    const int bh = blockIdx.x, j = bh / H, h = bh - j * H;
    const int vw = blockIdx.y;                              // the 8-wave kernel's wave index
    const int lane = threadIdx.x, g = lane & 7;
    const int nq_all = share * Tq;
    const int c0 = (int)blockIdx.z * NQ;
    const int nq = min(NQ, nq_all - c0);
    const int kb = kvrow ? kvrow[j * share] : j;
    W aw;
    const size_t kvo = ((size_t)kb * H + h) * 4096 + 8 * g;
    aw.init(kv + kvo, kv + kvo + 2048, T_enc, lane, (int64_t)B_layout * H * 4096);
    const size_t qrow0 = (size_t)j * nq_all + c0;
    float qv[NQ][8];
    int lim[NQ];
#pragma unroll
    for (int t = 0; t < NQ; ++t) {
        const int tt = t < nq ? t : nq - 1;
        const T* qr = q + (qrow0 + tt) * (H * 64) + h * 64 + 8 * g;
#pragma unroll
        for (int e = 0; e < 8; ++e) qv[t][e] = to_f<T>(qr[e]) * kLog2Scale;
        lim[t] = T_enc;
    }
    aw.template run<(1500 / W::KB + 1 + AW - 1) / AW>(vw, cdiv(T_enc, W::KB), qv, lim, nq);
    aw.to_lds(s_m, s_l, s_o, 0, lane);
    __syncthreads();
    for (int i = lane; i < 64 * nq; i += 64) {
        const int t = i >> 6, e = i & 63;
        float* pp = part + (((qrow0 + t) * H + h) * AW + vw) * 66;
        pp[e] = s_o[0][t][e];
        if (e == 0) {
            pp[64] = s_m[0][t];
            pp[65] = s_l[0][t];
        }
    }
}

// The 8 partials {o[64], m, l} of each (query row, head) written by cross_attn_vw_kernel, merged
// once into the bf16 / f32 attention output: attn_merge's operations in the same order, so the
// result is bitwise the 8-wave kernel's.  Used when the cross output projection has several rows:
// its A_ATTN prologue would merge every row and head in each of its 80 workgroups (15 us at a
// beam's 5 rows, profiles/r4/exp_beam_step.txt).
template <typename T>
__global__ __launch_bounds__(64) void attn_part_merge_kernel(const float* __restrict__ part, int H, T* __restrict__ out) {
#pragma clang fp contract(off)
    const int rh = blockIdx.x, e = threadIdx.x;
    const float* pp = part + (size_t)rh * AW * 66;
    float mw[AW], lw[AW], ow[AW];
#pragma unroll
    for (int w = 0; w < AW; ++w) {
        mw[w] = pp[w * 66 + 64];
        lw[w] = pp[w * 66 + 65];
        ow[w] = pp[w * 66 + e];
    }
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < AW; ++w) M = fmaxf(M, mw[w]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < AW; ++w) {
        if (mw[w] == -INFINITY) continue;
        const float f = exp2f(mw[w] - M);
        L = __builtin_fmaf(lw[w], f, L);
        O = __builtin_fmaf(ow[w], f, O);
    }
    out[(size_t)rh * 64 + e] = from_f<T>(O / L);  // row r, head h: out[r][h * 64 + e], rh = r * H + h
}

// ------------------------------------------------------------------ finalize
// Per sequence: reduce the logits tiles' top-2, record the token, choose the next
// input (argmax or forced), embed it for the next pass; the last block advances
// the step state (every block reads it before arriving).
constexpr int FIN_T = 1024;  // finalize threads per sequence: the 3.2k top-2 partials in ~3 loads each
template <typename T>
__global__ __launch_bounds__(FIN_T) void finalize_kernel(FinalizeArgs a) {
    __shared__ TopP s_top[FIN_T / 64];
    __shared__ int s_tok;
    const int b = blockIdx.x, tid = threadIdx.x;
    const int step = a.ds->step, pos0 = a.ds->pos0;
    TopP t{-INFINITY, 0x7fffffff, -INFINITY, 0};
    const TopP* p = (const TopP*)a.part + (size_t)b * a.n_tiles;
    for (int i = tid; i < a.n_tiles; i += FIN_T) t = top_merge(t, p[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t = top_merge(t, top_shfl(t, o));
    if ((tid & 63) == 0) s_top[tid >> 6] = t;
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < FIN_T / 64; ++w) t = top_merge(t, s_top[w]);
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
    for (int i = tid; i < a.d; i += FIN_T) a.x[(size_t)b * a.d + i] = to_f<T>(e[i]) + pp[i];
    if (tid == 0) {
        // relaxed: every block's reads of the step state were consumed before it arrives, and the next
        // kernel sees the last arriver's plain stores across the launch boundary (an acq_rel RMW cost
        // an L2 write-back and invalidate in every block's tail)
        const unsigned prev = __hip_atomic_fetch_add(a.arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)gridDim.x - 1) {
            a.ds->pos0 = pos0 + a.Tq;
            a.ds->step = step + 1;
            __hip_atomic_store(a.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ void advance_kernel(DecState* ds, int n) { ds->pos0 += n; }

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

int gemv_max_image_rows(int dtype, int K) {
    const int esz = dtype == DT_BF16 ? 2 : 4;
    int r = 64;
    while (r > 1 && gv_img_bytes(r, K, esz) > GV_LDS_BYTES) --r;
    return r;
}

void gemv(int dtype, int mode, int asrc, const GemvArgs& a_in, hipStream_t st) {
    if (a_in.R > 64 || a_in.R <= 0) throw std::runtime_error("gemv: rows must be in 1..64");
    const int ks = dtype == DT_BF16 ? 128 : 64;
    if (a_in.K % ks) throw std::runtime_error("gemv: K alignment");
    GemvArgs a = a_in;
    a.ksplit = std::max(1, a.ksplit);
    if (a.ksplit > 1 && mode != GV_PARTIAL) throw std::runtime_error("gemv: K split needs partial outputs");
    if (a.ksplit > a.K / ks) throw std::runtime_error("gemv: K split exceeds the super-steps");
    const int esz = dtype == DT_BF16 ? 2 : 4;
    if (asrc != A_DIRECT && gv_img_bytes(a.R, a.K, esz) > GV_LDS_BYTES)
        throw std::runtime_error("gemv: A image exceeds the LDS budget");
    if (asrc == A_LN && (a.K > 1536 || !a.ln_w || !a.ln_b))
        throw std::runtime_error("gemv: LayerNorm prologue needs K <= 1536 and LN parameters");
    if (asrc == A_LN && (a.n_pend < 0 || a.n_pend > 4 || a.n_pend == 3))
        throw std::runtime_error("gemv: pending slab count must be 0, 1, 2 or 4");
    if (a.p_resid && mode != GV_PARTIAL) throw std::runtime_error("gemv: residual rows into slab 0 need partial outputs");
    if (asrc == A_LN)
        for (int p = 0; p < 4; ++p)
            if (!a.pend[p]) throw std::runtime_error("gemv: LayerNorm prologue needs 4 pending slabs (zero slab if none)");
    if (asrc == A_ATTN && (!a.apart || a.a_splits < 2 || (a.a_splits > 4 && a.a_splits != 8) || a.a_heads * 64 != a.K))
        throw std::runtime_error("gemv: attention-merge prologue needs 2..4 or 8 chunks over all heads");
    const int code = asrc == A_LN ? LN_SRC(a.n_pend) : asrc == A_ATTN ? ATTN_SRC(a.a_splits) : asrc;
#define SPT_GV(M, S)                                                      \
    if (mode == M && code == S) {                                         \
        if (dtype == DT_BF16) gemv_launch<bf16, M, S>(a, st);             \
        else gemv_launch<float, M, S>(a, st);                             \
        return;                                                           \
    }
    SPT_GV_PAIRS(SPT_GV)
#undef SPT_GV
    throw std::runtime_error("gemv: unsupported mode / A source");
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
    const dim3 grid(B * H), blk(64 * AW);
#define SPT_SA(T, NQ) \
    hipLaunchKernelGGL((self_attn_kernel<T, NQ>), grid, blk, 0, st, (const T*)q, H * 64, (const T*)cache, B, H, ctx, Tq, ds, (T*)out)
    if (dtype == DT_BF16) {
        if (Tq == 1) SPT_SA(bf16, 1); else SPT_SA(bf16, 4);
    } else {
        if (Tq == 1) SPT_SA(float, 1); else SPT_SA(float, 4);
    }
#undef SPT_SA
    SPT_LAUNCH_CHECK();
}

// key blocks in each cross-attention wave's register ring (SPT_XATTN_PF = 2..4; no result changes)
static int xattn_pf() {
    static const int pf = getenv("SPT_XATTN_PF") ? std::max(2, std::min(4, atoi(getenv("SPT_XATTN_PF")))) : 2;
    return pf;
}

void dec_cross_attn(int dtype, const void* q, const void* kv, int B, int B_layout, int H, int T_enc, int Tq, void* out,
                    hipStream_t st, int splits, float* part, const int* kvrow, int share) {
    if (Tq < 1 || Tq > 4) throw std::runtime_error("dec_cross_attn: 1..4 queries per sequence");
    if (splits < 1 || splits > 4 || (splits > 1 && !part)) throw std::runtime_error("dec_cross_attn: 1..4 key chunks");
    if (share < 1 || share > 8 || B % share) throw std::runtime_error("dec_cross_attn: rows per window 1..8, dividing B");
    if (share > 1 && !kvrow) throw std::runtime_error("dec_cross_attn: shared windows need the window map");
    if ((int64_t)cdiv(T_enc, 32) * B_layout * H * 4096 >= (int64_t)INT32_MAX)
        throw std::runtime_error("dec_cross_attn: a layer's cross K/V exceeds 2^31 elements");
    const int nq = share * Tq;
    // queries per workgroup: 1 or 4 as without a window map; a decode step of several rows per
    // window takes 5 (bf16: beam 5 / best_of 5 in one workgroup; 8 would spill) or 4 (f32) of
    // them.  Every variant gives each lane the
    // same keys as the one-row kernel of the same Tq (NI: keys per lane), so a row's result is
    // bitwise the same whether or not its window is shared.
    const int NQ = nq == 1 ? 1 : Tq > 1 ? 4 : (dtype == DT_BF16 ? 5 : 4);
    if (splits > 1 && nq > NQ) throw std::runtime_error("dec_cross_attn: key chunks need one query chunk per window");
    const dim3 grid((B / share) * H, splits > 1 ? splits : cdiv(nq, NQ)), blk(64 * AW);
#define SPT_XA(T, NQ_, SP, NI, ...)                                                                             \
    hipLaunchKernelGGL((cross_attn_kernel<T, NQ_, SP, AW, NI __VA_ARGS__>), grid, blk, 0, st, (const T*)q,        \
                       (const T*)kv, B_layout, H, T_enc, Tq, (T*)out, part, kvrow, share)
    // NI = 4 for the step kernels of both dtypes (AttnWave's default at NQ = 1)
#define SPT_XA_T(T)                                                                       \
    if (NQ == 1) {                                                                        \
        if (splits > 1) SPT_XA(T, 1, true, 0);                                            \
        else if (xattn_pf() == 4) SPT_XA(T, 1, false, 0, , 4);                            \
        else if (xattn_pf() == 3) SPT_XA(T, 1, false, 0, , 3);                            \
        else SPT_XA(T, 1, false, 0);                                                      \
    }                                                                                     \
    else if (NQ == 4 && Tq > 1) { if (splits > 1) SPT_XA(T, 4, true, 0); else SPT_XA(T, 4, false, 0); } \
    else if (NQ == 4) { if (splits > 1) SPT_XA(T, 4, true, 4); else SPT_XA(T, 4, false, 4); } \
    else { if (splits > 1) SPT_XA(T, 5, true, 4); else SPT_XA(T, 5, false, 4); }
    if (dtype == DT_BF16) { SPT_XA_T(bf16); }
    else { SPT_XA_T(float); }
#undef SPT_XA_T
#undef SPT_XA
    SPT_LAUNCH_CHECK();
}

void dec_cross_attn_vw(int dtype, const void* q, const void* kv, int B, int B_layout, int H, int T_enc, int Tq,
                       float* part, hipStream_t st, const int* kvrow, int share, bool per_query) {
    if (Tq < 1 || Tq > 4) throw std::runtime_error("dec_cross_attn_vw: 1..4 queries per sequence");
    if (share < 1 || share > 8 || B % share) throw std::runtime_error("dec_cross_attn_vw: rows per window 1..8, dividing B");
    if (share > 1 && !kvrow) throw std::runtime_error("dec_cross_attn_vw: shared windows need the window map");
    if ((int64_t)cdiv(T_enc, 32) * B_layout * H * 4096 >= (int64_t)INT32_MAX)
        throw std::runtime_error("dec_cross_attn_vw: a layer's cross K/V exceeds 2^31 elements");
    if (!part) throw std::runtime_error("dec_cross_attn_vw: needs the partials buffer");
    const int nq = share * Tq;
    // the same query chunks and keys per lane as dec_cross_attn (bitwise the same partials); per_query
    // (one-token steps): one query per workgroup, the window's K/V re-read per query from L2 -- the
    // same 4 keys per lane as the shared kernels' NIX = 4, so still bitwise the same partials
    const int NQ = (nq == 1 || (per_query && Tq == 1)) ? 1 : Tq > 1 ? 4 : (dtype == DT_BF16 ? 5 : 4);
    const dim3 grid((B / share) * H, AW, cdiv(nq, NQ)), blk(64);
#define SPT_XV(T, NQ_, NI, PF)                                                                               \
    hipLaunchKernelGGL((cross_attn_vw_kernel<T, NQ_, NI, PF>), grid, blk, 0, st, (const T*)q, (const T*)kv,      \
                       B_layout, H, T_enc, Tq, part, kvrow, share)
#define SPT_XV_PF(T, NQ_, NI)                                    \
    if (xattn_pf() == 4) SPT_XV(T, NQ_, NI, 4);                  \
    else if (xattn_pf() == 3) SPT_XV(T, NQ_, NI, 3);             \
    else SPT_XV(T, NQ_, NI, 2);
#define SPT_XV_T(T)                                         \
    if (NQ == 1) { SPT_XV_PF(T, 1, 0) }                     \
    else if (NQ == 4 && Tq > 1) SPT_XV(T, 4, 0, 2);         \
    else if (NQ == 4) SPT_XV(T, 4, 4, 2);                   \
    else { SPT_XV_PF(T, 5, 4) }
    if (dtype == DT_BF16) { SPT_XV_T(bf16); }
    else { SPT_XV_T(float); }
#undef SPT_XV_T
#undef SPT_XV_PF
#undef SPT_XV
    SPT_LAUNCH_CHECK();
}

void dec_attn_part_merge(int dtype, const float* part, int R, int H, void* out, hipStream_t st) {
    if (R < 1 || H < 1 || !part || !out) throw std::runtime_error("dec_attn_part_merge: empty or missing buffers");
    if (dtype == DT_BF16) hipLaunchKernelGGL(attn_part_merge_kernel<bf16>, dim3(R * H), dim3(64), 0, st, part, H, (bf16*)out);
    else hipLaunchKernelGGL(attn_part_merge_kernel<float>, dim3(R * H), dim3(64), 0, st, part, H, (float*)out);
    SPT_LAUNCH_CHECK();
}

void dec_finalize(int dtype, const FinalizeArgs& a, int B, hipStream_t st) {
    if (dtype == DT_BF16) hipLaunchKernelGGL(finalize_kernel<bf16>, dim3(B), dim3(FIN_T), 0, st, a);
    else hipLaunchKernelGGL(finalize_kernel<float>, dim3(B), dim3(FIN_T), 0, st, a);
}

void dec_advance(DecState* ds, int n, hipStream_t st) {
    hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, st, ds, n);
}

void dec_reset(DecState* ds, unsigned* arrive, hipStream_t st) {
    hipLaunchKernelGGL(reset_kernel, dim3(1), dim3(1), 0, st, ds, arrive);
}

}  // namespace spt
