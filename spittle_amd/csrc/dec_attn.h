// dec_attn.h -- the decode-step attention arithmetic of the per-stage kernels (k_dec.hip; round 5's
// persistent decoder pass shared it until round 6 deleted that pass): one definition, so every
// instance computes the same bits (AttnWave's online softmax and attn_merge are spelled out: contraction off, explicit
// fmaf).
#pragma once
#include "common.h"

namespace spt {
namespace {

// ------------------------------------------------------------------ attention (decode)
constexpr int AW = 8;  // waves per attention workgroup
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

// One wave's share of flash-decoding over key blocks [blk0, nblk) of one (b, h): 8 lanes per
// key (8 dims each, fully coalesced 16-byte sweeps of the K/V rows), online softmax in exp2
// space; raw K/V chunks ping-pong so the next block streams in during the current one.
// qv is pre-scaled by log2(e)/8.  Leaves (m, l, o) per query in the calling lanes.
// keys per lane: 4 for bf16 (r1 exp10 / exp11: lower register pressure and more resident waves
// beat more keys per lane for both the cross- and the self-attention step), 2 for f32 prompts.
// PF: key blocks in the register ring (PF - 1 in flight while one is processed); the blocks are
// processed in the same order whatever PF is, so PF changes no result bit.
template <typename T, int NQ, int NI_ = 0, int NW = AW, int PF = 2>
struct AttnWave {
    static constexpr int NI = NI_ > 0 ? NI_ : (sizeof(T) == 2) ? 4 : (NQ == 1 ? 4 : 2);
    static constexpr int KB = 8 * NI;  // keys per block
    static_assert(PF >= 2 && PF <= 4, "AttnWave: 2..4 ring slots");
    KVChunk<T> kc_[PF][NI], vc_[PF][NI];
    float m[NQ], l[NQ], o[NQ][8];
    const T *Kb, *Vb;
    int n_keys, slot;
    int bstride = 2048;  // 32-key blocks this far apart (2048: key rows contiguous, [T][64])

    __device__ __forceinline__ void init(const T* K, const T* V, int nk, int lane, int64_t blk_stride = 0) {
        slot = lane >> 3;
        Kb = K;
        Vb = V;
        n_keys = nk;
        bstride = blk_stride ? (int)blk_stride : 32 * 64;  // one branch-free offset formula for both layouts
#pragma unroll
        for (int t = 0; t < NQ; ++t) {
            m[t] = -INFINITY;
            l[t] = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[t][e] = 0.f;
        }
    }
    __device__ __forceinline__ void load_blk(KVChunk<T> (&kc)[NI], KVChunk<T> (&vc)[NI], int blk) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int key = min(blk * KB + 8 * i + slot, n_keys - 1);
            // 32-bit element offsets (the launchers check that a layer's K/V spans < 2^31 elements):
            // the 64-bit multiply per key was a third of the loop's address VALU (r4)
            const uint32_t off = (uint32_t)((key >> 5) * bstride + (key & 31) * 64);  // zero-extends for free
            kc[i].load(Kb + off);
            vc[i].load(Vb + off);
        }
    }
    // The arithmetic is spelled out (contraction off, explicit fmaf): every inlined instance of this
    // step -- per query t, per key block, per kernel (8-wave, single-wave, chunked queries) -- then
    // computes the same bits.  r4: left to the compiler, the fully unrolled schedule contracted
    // some instances differently, so identical decoder rows (a beam's first steps) in different
    // query chunks differed in the last bit and whisper.cpp's exact-equality candidate dedup failed.
    __device__ __forceinline__ void process(const KVChunk<T> (&kc)[NI], const KVChunk<T> (&vc)[NI], int kbase,
                                            const float (&qv)[NQ][8], const int (&lim)[NQ], int Tq) {
#pragma clang fp contract(off)
#pragma unroll
        for (int t = 0; t < NQ; ++t) {
            if (t >= Tq) break;
            float s[NI];
            float mb = -INFINITY;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                float v = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) v = __builtin_fmaf(qv[t][e], kc[i].at(e), v);
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
                for (int e = 0; e < 8; ++e) o[t][e] = __builtin_fmaf(p, vc[i].at(e), o[t][e]);
            }
            l[t] = __builtin_fmaf(l[t], alpha, ls);
            m[t] = mn;
        }
    }
    // blocks blk0 + w, blk0 + w + NW, ... below nblk, PF - 1 of them loading ahead.  MAXB bounds the
    // blocks one wave takes (a fully unrolled, straight-line schedule with unconditional loads:
    // past the wave's last block they repeat it, L1/L2 hits, never processed).  r4: in a rolled loop
    // whose ring registers rotate, the compiler drained every load in flight (vmcnt(0)) at the
    // loop head, so no block was ever in flight while another was processed.  More blocks than
    // MAXB (never for Whisper's 1500 keys / 448 positions) take the rolled loop.
    template <int MAXB>
    __device__ __forceinline__ void run(int blk, int nblk, const float (&qv)[NQ][8], const int (&lim)[NQ], int Tq) {
        if (blk >= nblk) return;
        const int cnt = (nblk - 1 - blk) / NW + 1;  // this wave's blocks
        const int mine = blk + (cnt - 1) * NW;      // its last one
        if (MAXB <= 8 && cnt <= MAXB) {  // (longer schedules are not unrolled: the f32 prompt kernels)
#pragma unroll
            for (int d = 0; d < PF - 1 && d < MAXB; ++d) load_blk(kc_[d], vc_[d], min(blk + d * NW, mine));
#pragma unroll
            for (int i = 0; i < (MAXB <= 8 ? MAXB : 1); ++i) {
                if (i >= cnt) break;
                if (i + PF - 1 < (MAXB <= 8 ? MAXB : 1))
                    load_blk(kc_[(i + PF - 1) % PF], vc_[(i + PF - 1) % PF], min(blk + (i + PF - 1) * NW, mine));
                process(kc_[i % PF], vc_[i % PF], (blk + i * NW) * KB, qv, lim, Tq);
            }
            return;
        }
        load_blk(kc_[0], vc_[0], blk);
        while (blk < nblk) {
            load_blk(kc_[1], vc_[1], min(blk + NW, mine));
            process(kc_[0], vc_[0], blk * KB, qv, lim, Tq);
            blk += NW;
            if (blk >= nblk) break;
            load_blk(kc_[0], vc_[0], min(blk + NW, mine));
            process(kc_[1], vc_[1], blk * KB, qv, lim, Tq);
            blk += NW;
        }
    }
    // run() with the wave's first block (blk) already in ring slot 0: loaded before n_keys was known
    // (self-attention: before the decoder position arrives), clamped to the cache's rows instead of
    // n_keys - 1.  The keys past n_keys are masked in process() either way (p = 0 against finite
    // cache rows), so the result is run()'s.
    template <int MAXB>
    __device__ __forceinline__ void run_pre(int blk, int nblk, const float (&qv)[NQ][8], const int (&lim)[NQ], int Tq) {
        if (blk >= nblk) return;
        const int cnt = (nblk - 1 - blk) / NW + 1;
        const int mine = blk + (cnt - 1) * NW;
        if (MAXB <= 8 && cnt <= MAXB) {
#pragma unroll
            for (int d = 1; d < PF - 1 && d < MAXB; ++d) load_blk(kc_[d], vc_[d], min(blk + d * NW, mine));
#pragma unroll
            for (int i = 0; i < (MAXB <= 8 ? MAXB : 1); ++i) {
                if (i >= cnt) break;
                if (i + PF - 1 < (MAXB <= 8 ? MAXB : 1))
                    load_blk(kc_[(i + PF - 1) % PF], vc_[(i + PF - 1) % PF], min(blk + (i + PF - 1) * NW, mine));
                process(kc_[i % PF], vc_[i % PF], (blk + i * NW) * KB, qv, lim, Tq);
            }
            return;
        }
        while (blk < nblk) {
            load_blk(kc_[1], vc_[1], min(blk + NW, mine));
            process(kc_[0], vc_[0], blk * KB, qv, lim, Tq);
            blk += NW;
            if (blk >= nblk) break;
            load_blk(kc_[0], vc_[0], min(blk + NW, mine));
            process(kc_[1], vc_[1], blk * KB, qv, lim, Tq);
            blk += NW;
        }
    }
    // sum l and o over the 8 key slots of the wave (m is wave-uniform) into LDS
    __device__ __forceinline__ void to_lds(float (*s_m)[NQ], float (*s_l)[NQ], float (*s_o)[NQ][64], int wid,
                                           int lane) {
        const int g = lane & 7;
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
    }
};

// workgroup merge of the NW waves' (m, l, o) for query t, element e -> (M, L, O)
template <int NQ, int NW = AW>
__device__ __forceinline__ void attn_merge(const float (*s_m)[NQ], const float (*s_l)[NQ], const float (*s_o)[NQ][64],
                                           int t, int e, float& M, float& L, float& O) {
#pragma clang fp contract(off)
    M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, s_m[w][t]);
    L = 0.f;
    O = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {  // the same operations as the GEMV's A_ATTN merge (bitwise)
        if (s_m[w][t] == -INFINITY) continue;
        const float f = exp2f(s_m[w][t] - M);
        L = __builtin_fmaf(s_l[w][t], f, L);
        O = __builtin_fmaf(s_o[w][t][e], f, O);
    }
}

}  // namespace
}  // namespace spt
