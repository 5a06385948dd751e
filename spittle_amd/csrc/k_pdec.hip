// k_pdec.hip -- the decoder pass of one-token steps as ONE persistent launch (kernels.h PdArgs).
//
// The launch chain (enqueue_layers) runs 8-9 dependent kernels per decoder layer; at the app's
// batch of one every one of them is short (a few us of weight streaming) and pays a kernel boundary
// plus a cold weight round trip that nothing overlaps.  Here one workgroup
// per CU runs every stage of every layer: the stage's work is cut into units (16 output columns of
// a projection; a (row, head) of an attention; a (row, head, key chunk) of the cross-attention), the
// units are dealt round robin over the workgroups, and each unit
//   * prefetches its operands that do not depend on the previous stage (projection weights, the
//     cached self / cross K/V) into registers while the previous unit is still finishing -- the
//     weight stream runs under the hand-off latency instead of after it;
//   * waits for its inputs: data-tagged 8-byte granules {value, epoch} that the producing units
//     store write-through (sc1) and the consumer's gather waves poll with sc1 loads
//     (MI355X_MICROARCH.md "hand-offs measured with sc1 loads", row R2: the data is the flag);
//   * computes exactly what the stage's kernel computes for those columns / rows: the same LayerNorm
//     code, the same MFMA K chains of gemv_kernel's wave geometry summed in the same order,
//     AttnWave's online softmax over the same key blocks, attn_merge's merge -- so the pass is
//     bitwise the launch chain's (tests/test_gpu_persistent.py);
//   * publishes its output granules.
// Workgroups: 8 waves, one workgroup per CU (119 KB of LDS).  Waves 0-3 gather (poll granules into
// LDS, LayerNorm); waves 4-7 compute (prefetch into registers, MFMA / attention, epilogue, publish).
//
// Every workgroup must be resident for the hand-offs to complete: each workgroup counts itself in
// a census at start, and a wait that makes no progress for 20 us while the census is incomplete (a
// kernel of another context or process holds CUs) sets the error word and every workgroup leaves.
// The engine then re-runs the call on the launch chain (Engine::run_decode), so the result never
// depends on the pass being able to run.
#include "common.h"
#include "dec_attn.h"
#include "kernels.h"

#include <stdio.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

namespace spt {
namespace {

typedef unsigned long long u64;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) u64 gu64;

constexpr int PT = 512;     // threads: waves 0-3 gather, waves 4-7 compute
constexpr int PMAXR = 8;    // rows per pass
constexpr int PMAXD = 1280; // model width (LDS image budget)
constexpr int PNPRE = 24;   // 16-byte prefetch registers per compute lane
constexpr int PMAXSS = 5;   // projection super-steps (128 K each) one compute wave holds
enum { S_A = 0, S_B, S_C, S_D, S_E, S_E2, S_F, S_G, S_H };
enum { G_X = 0, G_Q, G_K, G_V, G_A, G_XC, G_QX, G_PART, G_M, G_XF, G_H, G_P0 };

// LDS carve (bytes)
constexpr int L_IMG = 0;                                   // bf16 A image [R][K + 8], K <= 4 d
constexpr int L_RED = L_IMG + PMAXR * (4 * PMAXD + 8) * 2; // chain partials [32][64] f32x4
constexpr int L_ATT = L_RED + 32 * 64 * 16;                // s_m[8], s_l[8], s_o[8][64]
constexpr int L_QKV = L_ATT + (16 + 8 * 64) * 4;           // q, k, v rows (bf16) | 8 partials [8][66] f32
constexpr int L_RES = L_QKV + 8 * 66 * 4;                  // residual columns [R][16] f32
constexpr int L_EST = L_RES + PMAXR * 16 * 4;              // cross-attention state after 3 blocks [2][9][64] + m
constexpr int L_MISC = L_EST + 2 * (9 * 64 + 4) * 4;         // [0] abort, [1] launch index
constexpr int PMAXL = 32;                                    // decoder layers (the layer table below)
constexpr int L_LAYERS = L_MISC + 64;                        // the layers' weight pointers (PdLayer [L])
constexpr int L_KVROW = L_LAYERS + PMAXL * (int)sizeof(PdLayer);  // the rows' windows (a.kvrow) [PMAXR]
constexpr int L_TOTAL = L_KVROW + 64;
static_assert(L_TOTAL > 80 * 1024 && L_TOTAL <= 160 * 1024, "one workgroup per CU");
static_assert(sizeof(PdLayer) % 8 == 0, "layer table copy in 8-byte words");
static_assert((L_RED % 16) == 0 && (L_ATT % 16) == 0 && (L_QKV % 16) == 0 && (L_RES % 16) == 0 && (L_EST % 16) == 0 &&
                  (L_MISC % 16) == 0, "align");

__device__ __forceinline__ unsigned ld_rlx(const unsigned* p) {
    return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(unsigned* p, unsigned v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one granule: ONE 8-byte write-through store {value (low word), epoch (high word)}
__device__ __forceinline__ void gran_put(u64* base, int64_t i, unsigned ep, unsigned v) {
    __hip_atomic_store((gu64*)(base + i), ((u64)ep << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// pointers read from the LDS layer table are generic to the compiler (flat loads: counted on both
// vmcnt and lgkmcnt and waited for with both at 0); the weights and LayerNorm / bias vectors are
// global memory, so say so
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gp(const void* p) {
    return (const __attribute__((address_space(1))) T*)p;
}
// float4 (a HIP struct) has no assignment from an address-space-qualified reference: load the bits
__device__ __forceinline__ float4 gp_f4(const float* p) {
    return __builtin_bit_cast(float4, *gp<u32x4>(p));
}
__device__ __forceinline__ unsigned fbits(float f) { return __builtin_bit_cast(unsigned, f); }
__device__ __forceinline__ float bitsf(unsigned u) { return __builtin_bit_cast(float, u); }

__device__ __forceinline__ unsigned ep_of(unsigned launch, int L, int l, int s) {
    return ((launch * (unsigned)L + (unsigned)l) << 4) + (unsigned)s + 1u;
}

// a bounded wait step: false = give up (the error word is set, or set here)
__device__ __forceinline__ bool spin_ok(const PdArgs& a, unsigned& it, u64& t0) {
    __builtin_amdgcn_s_sleep(1);
    ++it;
    if (it == 1u) { t0 = wall_clock64(); return true; }  // 100 MHz
    if ((it & 7u) != 0u) return true;
    const u64 now = wall_clock64();
    if (ld_rlx(a.ctl + 2) != 0u) return false;
    const u64 el = now - t0;
    if (el > 2000u && ld_rlx(a.ctl) < (unsigned)a.nwg) {  // 20 us and not every workgroup is resident
        st_rlx(a.ctl + 2, 1u);
        return false;
    }
    if (el > 20000000u) {  // 200 ms: never in a correct run
        st_rlx(a.ctl + 2, 2u);
        return false;
    }
    return true;
}

// Poll this lane's NL 16-byte pieces (two granules each; bit k of `valid` = piece k exists) until
// every existing piece carries the epoch in both halves.  Wave-uniform result.
template <int NL>
__device__ __forceinline__ bool poll(const PdArgs& a, __amdgpu_buffer_rsrc_t rs, const unsigned (&off)[NL],
                                     unsigned valid, unsigned ep, u32x4 (&v)[NL]) {
    unsigned done = ~valid;
    unsigned it = 0;
    u64 t0 = 0;
#pragma unroll
    for (int k = 0; k < NL; ++k) v[k] = u32x4{0u, 0u, 0u, 0u};
    for (;;) {
        asm volatile("" ::: "memory");  // the loads below are re-issued every pass
#pragma unroll
        for (int k = 0; k < NL; ++k)
            if (!((done >> k) & 1u)) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off[k], 0, 16);  // sc1
#pragma unroll
        for (int k = 0; k < NL; ++k)
            if (v[k].y == ep && v[k].w == ep) done |= 1u << k;
        if (__all(done == ~0u)) return true;
        if (!spin_ok(a, it, t0)) return false;
    }
}

// diagnostics: field f of this workgroup's k-th unit record (lane 0 of the calling wave), SPT_PD_STAMP
__device__ __forceinline__ void stamp(const PdArgs& a, int wg, int k, int f, u64 v, int lane) {
    if (lane == 0 && k < kPdStampMax) a.stamps[((size_t)wg * kPdStampMax + k) * kPdStampRec + f] = v;
}

// The loop barriers between gather and compute waves hand over LDS only.  __syncthreads() carries a
// release fence, before which the compiler drains every outstanding vector-memory op (vmcnt(0)):
// the compute waves' prefetch of the NEXT unit's weights / K/V, issued just before barrier B to run
// under the next edge, was waited for there instead (r6 stage stamps: 20.7 us of a 67 us layer at
// B = 1 sat in barrier B).  So: the wave's own LDS ops (lgkmcnt(0)), then a bare s_barrier.
#define PD_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Kernel-argument arrays by constant index only: a runtime index into a.go / a.n / a.pre made the
// compiler copy the whole argument block to scratch and read EVERY field of `a` from there (scratch
// loads count on vmcnt, so each one also waited behind the weight stream in flight; r6: 376 B of
// scratch per lane).  A switch keeps each access a constant-offset argument load.
__device__ __forceinline__ int64_t go_of(const PdArgs& a, int i) {
    switch (i) {
        case 0: return a.go[0]; case 1: return a.go[1]; case 2: return a.go[2]; case 3: return a.go[3];
        case 4: return a.go[4]; case 5: return a.go[5]; case 6: return a.go[6]; case 7: return a.go[7];
        case 8: return a.go[8]; case 9: return a.go[9]; case 10: return a.go[10]; default: return a.go[11];
    }
}
__device__ __forceinline__ int n_of(const PdArgs& a, int s) {
    switch (s) {
        case 0: return a.n[0]; case 1: return a.n[1]; case 2: return a.n[2]; case 3: return a.n[3]; case 4: return a.n[4];
        case 5: return a.n[5]; case 6: return a.n[6]; case 7: return a.n[7]; default: return a.n[8];
    }
}
__device__ __forceinline__ int pre_of(const PdArgs& a, int s) {
    switch (s) {
        case 0: return a.pre[0]; case 1: return a.pre[1]; case 2: return a.pre[2]; case 3: return a.pre[3]; case 4: return a.pre[4];
        case 5: return a.pre[5]; case 6: return a.pre[6]; case 7: return a.pre[7]; default: return a.pre[8];
    }
}

// ------------------------------------------------------------------ geometry helpers
struct Cur { int l, s, u; };

__device__ __forceinline__ int unit0(const PdArgs& a, int l, int s, int wg) {
    const int base = (int)(((int64_t)l * a.U + pre_of(a, s)) % a.nwg);
    return (wg - base + a.nwg) % a.nwg;
}
// this workgroup's next unit in (layer, stage, unit) order.  The cursor is wave-uniform; readfirstlane
// says so to the compiler, so the per-stage branches are scalar (as exec-masked branches their joins
// merged the prefetch registers and waited vmcnt(0) for the loads just issued: r6 stamps, 2-3 us of
// "prefetch issue" per unit)
__device__ __forceinline__ bool advance_(const PdArgs& a, int wg, Cur& c);
__device__ __forceinline__ bool advance(const PdArgs& a, int wg, Cur& c) {
    const bool r = advance_(a, wg, c);
    c.l = __builtin_amdgcn_readfirstlane(c.l);
    c.s = __builtin_amdgcn_readfirstlane(c.s);
    c.u = __builtin_amdgcn_readfirstlane(c.u);
    return __builtin_amdgcn_readfirstlane((int)r) != 0;
}
__device__ __forceinline__ bool advance_(const PdArgs& a, int wg, Cur& c) {
    c.u += a.nwg;
    while (c.u >= n_of(a, c.s)) {
        if (++c.s == kPdStages) {
            c.s = 0;
            if (++c.l == a.L) return false;
        }
        c.u = unit0(a, c.l, c.s, wg);
    }
    return true;
}

__device__ __forceinline__ bool is_gemv(int s) { return s == S_A || s == S_C || s == S_D || s == S_F || s == S_G || s == S_H; }

struct Gv {  // one projection unit: 16 output columns n0.. of W [N][K], super-steps [s0, s1)
    const bf16* W;
    int K, n0, s0, s1, ks;
};
// fc2 (S_H) units are one K-split slab of gemv_kernel's GV_PARTIAL launch each: unit u = tile u / 2,
// slab u % 2 (super-steps z * per .. of the 4d / 128)
__device__ __forceinline__ Gv gv_of(const PdArgs& a, const PdLayer& Lw, int s, int u) {
    Gv g;
    g.n0 = 16 * u;
    g.K = a.d;
    g.s0 = 0;
    g.s1 = a.d / 128;
    // constant indices into the kernel arguments (a dynamic a.ks[s] was a vector load of the argument
    // block that the prefetch's address arithmetic waited for)
    switch (s) {
        case S_A: g.W = (const bf16*)Lw.qkv_w; g.ks = a.ks[S_A]; break;
        case S_C: g.W = (const bf16*)Lw.so_w; g.ks = a.ks[S_C]; break;
        case S_D: g.W = (const bf16*)Lw.cq_w; g.ks = a.ks[S_D]; break;
        case S_F: g.W = (const bf16*)Lw.co_w; g.ks = a.ks[S_F]; break;
        case S_G: g.W = (const bf16*)Lw.fc1_w; g.ks = a.ks[S_G]; break;
        default: {  // S_H
            const int nss = 4 * (a.d / 128), per = (nss + 1) / 2, z = u & 1;
            g.ks = a.ks[S_H];
            g.W = (const bf16*)Lw.fc2_w;
            g.n0 = 16 * (u >> 1);
            g.K = 4 * a.d;
            g.s0 = z * per;
            g.s1 = min(nss, g.s0 + per);
            break;
        }
    }
    return g;
}
// the super-steps of compute wave cw, in order: chains c = cw, cw + 4, ... (< ks) of gemv_kernel's
// K geometry (chain c: super-steps s0 + c, + ks, ... below s1)
__device__ __forceinline__ void gv_plan(const Gv& g, int cw, int (&ss)[PMAXSS], int (&gc)[PMAXSS]) {
    int c = cw, s = g.s0 + cw;
    while (c < g.ks && s >= g.s1) { c += 4; s = g.s0 + c; }
#pragma unroll
    for (int k = 0; k < PMAXSS; ++k) {
        const bool on = c < g.ks;
        ss[k] = on ? s : -1;
        gc[k] = c;
        if (on) {
            s += g.ks;
            if (s >= g.s1) {
                c += 4;
                s = g.s0 + c;
                while (c < g.ks && s >= g.s1) { c += 4; s = g.s0 + c; }
            }
        }
    }
}

// ------------------------------------------------------------------ prefetch (compute waves)
// Every register is written (zero where the unit has nothing): the previous unit's values all die
// here, so the compiler never keeps two units' operands live at once.

// the cross K/V of key block blk (32 keys) for this lane's key slot: kc[i], vc[i] (i < 4)
__device__ __forceinline__ void e_block_load(const PdArgs& a, const bf16* Kb, int blk, int slot, u32x4* kc, u32x4* vc) {
    const uint32_t bstride = (uint32_t)a.B_layout * a.H * 4096;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int key = min(blk * 32 + 8 * i + slot, a.T_enc - 1);
        const uint32_t off = (uint32_t)((key >> 5) * bstride + (key & 31) * 64);
        kc[i] = *gp<u32x4>(Kb + off);
        vc[i] = *gp<u32x4>(Kb + off + 2048);
    }
}
// cross-attention unit u: e_vw virtual waves (of the 8-wave kernel) of one (row, head); compute
// wave cw takes virtual wave vw of it, key blocks 3 * half .. + 2 (half = cw & 1: the second half
// continues the first half's online-softmax state, handed over in LDS)
struct Eu { int bh, vw, vi, half; const bf16* Kb; };
__device__ __forceinline__ Eu e_unit(const PdArgs& a, const int* kvrow, int l, int u, int cw, int lane) {
    Eu e;
    const int per_bh = 8 / a.e_vw;
    e.bh = u / per_bh;
    e.vi = cw >> 1;
    e.half = cw & 1;
    e.vw = (u - e.bh * per_bh) * a.e_vw + e.vi;
    const int b = e.bh / a.H, h = e.bh - b * a.H;
    const int kb = kvrow ? kvrow[b] : b;  // the window map, copied to LDS at kernel start
    e.Kb = (const bf16*)a.ckv + a.cross_layer * l + ((size_t)kb * a.H + h) * 4096 + 8 * (lane & 7);
    return e;
}

__device__ __forceinline__ void prefetch(const PdArgs& a, const PdLayer* layers, const int* kvrow, const Cur& c, int cw,
                                         int lane, int pos0, u32x4 (&pre)[PNPRE]) {
    const u32x4 z = {0u, 0u, 0u, 0u};
    const PdLayer& Lw = layers[c.l];
    const int fr = lane & 15, fq = lane >> 4;
    const int slot = lane >> 3;
    if (is_gemv(c.s)) {
        const Gv g = gv_of(a, Lw, c.s, c.u);
        int ss[PMAXSS], gc[PMAXSS];
        gv_plan(g, cw, ss, gc);
        const __attribute__((address_space(1))) bf16* wrow = gp<bf16>(g.W) + (size_t)(g.n0 + fr) * g.K + fq * 8;
        // unconditional loads (a super-step the wave does not own reads super-step 0 and is never
        // used): a load under a condition made hipcc wait vmcnt(0) for each before the next (r6 stamps:
        // the prefetch "issue" took 2-3 us per unit, a round trip per load)
#pragma unroll
        for (int k = 0; k < PMAXSS; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                pre[4 * k + i] = *(const __attribute__((address_space(1))) u32x4*)(wrow + max(ss[k], 0) * 128 + i * 32);
#pragma unroll
        for (int k = 4 * PMAXSS; k < PNPRE; ++k) pre[k] = z;
        return;
    }
    if (c.s == S_B) {  // the first self K/V block of virtual waves cw, cw + 4 (positions < 256; a
                       // second block, positions 256..447, is loaded when the unit runs)
        const int b = c.u / a.H, h = c.u - b * a.H;
        const int nk = pos0 + 1;
        const bf16* kv = (const bf16*)a.skv + a.self_layer * c.l;
        const bf16* Kb = kv + (((size_t)0 * a.R + b) * a.H + h) * (size_t)a.ctx * 64 + 8 * (lane & 7);
        const bf16* Vb = kv + (((size_t)1 * a.R + b) * a.H + h) * (size_t)a.ctx * 64 + 8 * (lane & 7);
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const int blk = cw + 4 * v;
#pragma unroll
            for (int i = 0; i < 4; ++i) {  // unconditional (clamped key; a block past nblk is never used)
                const int key = min(blk * 32 + 8 * i + slot, nk - 1);
                pre[(v * 4 + i) * 2 + 0] = *gp<u32x4>(Kb + key * 64);
                pre[(v * 4 + i) * 2 + 1] = *gp<u32x4>(Vb + key * 64);
            }
        }
#pragma unroll
        for (int k = 16; k < PNPRE; ++k) pre[k] = z;
        return;
    }
    if (c.s == S_E && (cw >> 1) < a.e_vw) {  // cross K/V blocks 3 half .. 3 half + 2 of virtual wave vw
        const Eu e = e_unit(a, kvrow, c.l, c.u, cw, lane);
        const int nblk = cdiv(a.T_enc, 32);
#pragma unroll
        for (int t = 0; t < 3; ++t) {  // unconditional (e_block_load clamps the key; unused past nblk)
            const int blk = e.vw + 8 * (3 * e.half + t);
            u32x4 kc[4], vc[4];
            e_block_load(a, e.Kb, min(blk, nblk - 1), slot, kc, vc);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                pre[(t * 4 + i) * 2 + 0] = kc[i];
                pre[(t * 4 + i) * 2 + 1] = vc[i];
            }
        }
#pragma unroll
        for (int k = 24; k < PNPRE; ++k) pre[k] = z;
        return;
    }
#pragma unroll
    for (int k = 0; k < PNPRE; ++k) pre[k] = z;
}

// ------------------------------------------------------------------ gathers (gather waves)
// LayerNorm of x rows into the bf16 image: gemv_kernel's A_LN prologue, row r by gather wave r % 4
// (each lane: elements lane * 4 + 256 i).  src < 0: plain f32 rows at a.x (layer 0's input).
__device__ __forceinline__ bool gather_ln(const PdArgs& a, __amdgpu_buffer_rsrc_t rs, int src, unsigned ep,
                                          const float* ln_w, const float* ln_b, bf16* img, int gw, int lane) {
    constexpr int NC = PMAXD / 256;  // float4 chunks per lane (gemv_kernel loops to 6 with k < K: the same)
    const int K = a.d, ld = K + 8;
    float4 lnw_pre[NC], lnb_pre[NC];  // fetched ahead of the rows (their wait then covers these)
#pragma unroll
    for (int i = 0; i < NC; ++i) {
        const int k = lane * 4 + 256 * i;
        if (k < K) {
            lnw_pre[i] = gp_f4(ln_w + k);
            lnb_pre[i] = gp_f4(ln_b + k);
        }
    }
    for (int r = gw; r < a.R; r += 4) {
        float4 v[NC];
        if (src < 0) {
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) v[i] = *(const float4*)(a.x + (size_t)r * K + k);
            }
        } else {
            unsigned off[2 * NC];
            unsigned valid = 0;
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                const int k = lane * 4 + 256 * i;
                const unsigned o = (unsigned)((go_of(a, src) + (int64_t)r * K + k) * 8);
                off[2 * i] = o;
                off[2 * i + 1] = o + 16;
                if (k < K) valid |= 3u << (2 * i);
            }
            u32x4 p[2 * NC];
            if (!poll<2 * NC>(a, rs, off, valid, ep, p)) return false;
#pragma unroll
            for (int i = 0; i < NC; ++i) v[i] = float4{bitsf(p[2 * i].x), bitsf(p[2 * i].z), bitsf(p[2 * i + 1].x), bitsf(p[2 * i + 1].z)};
        }
        // gemv_kernel's LayerNorm, operation for operation
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const int k = lane * 4 + 256 * i;
            if (k < K) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
        }
        const float mean = wave_sum(s) / (float)K;
        float s2 = 0.f;
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const int k = lane * 4 + 256 * i;
            if (k < K) {
                s2 += ln_sq4(v[i], mean);
            }
        }
        const float rstd = 1.0f / sqrtf(wave_sum(s2) / (float)K + 1e-5f);
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const int k = lane * 4 + 256 * i;
            if (k < K) {
                const float4 g = lnw_pre[i];
                const float4 b = lnb_pre[i];
                bf16* o = img + (size_t)r * ld + k;
                o[0] = from_f<bf16>(ln_out(v[i].x, mean, rstd, g.x, b.x));
                o[1] = from_f<bf16>(ln_out(v[i].y, mean, rstd, g.y, b.y));
                o[2] = from_f<bf16>(ln_out(v[i].z, mean, rstd, g.z, b.z));
                o[3] = from_f<bf16>(ln_out(v[i].w, mean, rstd, g.w, b.w));
            }
        }
    }
    return true;
}

// bf16 rows [R][K] (granule pairs [R][K/2]) into the image [R][K + 8]; all four gather waves
__device__ __forceinline__ bool gather_img(const PdArgs& a, __amdgpu_buffer_rsrc_t rs, int src, int K, unsigned ep,
                                           bf16* img, int gt) {
    const int ld = K + 8;
    const int pieces = a.R * K / 4;  // 16 bytes = 4 bf16 each
    for (int p0 = 0; p0 < pieces; p0 += 256 * 16) {
        unsigned off[16];
        unsigned valid = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int p = p0 + k * 256 + gt;
            off[k] = (unsigned)((go_of(a, src) + 2 * (int64_t)p) * 8);
            if (p < pieces) valid |= 1u << k;
        }
        u32x4 v[16];
        if (!poll<16>(a, rs, off, valid, ep, v)) return false;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int p = p0 + k * 256 + gt;
            if (p < pieces) {
                const int e = 4 * p, r = e / K, col = e - r * K;
                *(uint2*)(img + (size_t)r * ld + col) = uint2{v[k].x, v[k].z};
            }
        }
    }
    return true;
}

// the columns n0 .. n0 + 15 of R f32 rows (granules [R][d], or plain a.x when src < 0) into res [R][16]
// (one wave: lane = (row, pair of columns))
__device__ __forceinline__ bool gather_cols(const PdArgs& a, __amdgpu_buffer_rsrc_t rs, int src, unsigned ep, int n0,
                                            float* res, int lane) {
    const int r = lane >> 3, pc = lane & 7;
    if (src < 0) {
        if (r < a.R) {
            const float2 v = *(const float2*)(a.x + (size_t)r * a.d + n0 + 2 * pc);
            res[r * 16 + 2 * pc] = v.x;
            res[r * 16 + 2 * pc + 1] = v.y;
        }
        return true;
    }
    unsigned off[1] = {(unsigned)((go_of(a, src) + (int64_t)r * a.d + n0 + 2 * pc) * 8)};
    u32x4 v[1];
    if (!poll<1>(a, rs, off, r < a.R ? 1u : 0u, ep, v)) return false;
    if (r < a.R) {
        res[r * 16 + 2 * pc] = bitsf(v[0].x);
        res[r * 16 + 2 * pc + 1] = bitsf(v[0].z);
    }
    return true;
}

// the 64 bf16 of head h of row b from nsrc pair-granule buffers [R][d/2] into dst[j][64]
__device__ __forceinline__ bool gather_head(const PdArgs& a, __amdgpu_buffer_rsrc_t rs, const int* srcs, int nsrc,
                                            int b, int h, unsigned ep, bf16* dst, int lane) {
    const int j = lane >> 4, pc = lane & 15;  // buffer, piece of 4 bf16
    unsigned off[1] = {(unsigned)((go_of(a, j < nsrc ? srcs[j] : 0) + (int64_t)b * (a.d / 2) + 32 * h + 2 * pc) * 8)};
    u32x4 v[1];
    if (!poll<1>(a, rs, off, j < nsrc ? 1u : 0u, ep, v)) return false;
    if (j < nsrc) *(uint2*)(dst + j * 64 + 4 * pc) = uint2{v[0].x, v[0].z};
    return true;
}

// the 8 cross-attention partials {o[64], m, l} of (b, h) into part[8][66]
__device__ __forceinline__ bool gather_part(const PdArgs& a, __amdgpu_buffer_rsrc_t rs, int b, int h, unsigned ep,
                                            float* part, int gt) {
    unsigned off[2];
    unsigned valid = 0;
    const int64_t base = go_of(a, G_PART) + ((int64_t)b * a.H + h) * 8 * 66;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int p = gt + 256 * k;  // 264 pieces
        off[k] = (unsigned)((base + 2 * p) * 8);
        if (p < 264) valid |= 1u << k;
    }
    u32x4 v[2];
    if (!poll<2>(a, rs, off, valid, ep, v)) return false;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int p = gt + 256 * k;
        if (p < 264) {
            part[2 * p] = bitsf(v[k].x);
            part[2 * p + 1] = bitsf(v[k].z);
        }
    }
    return true;
}

// ------------------------------------------------------------------ the kernel
struct Smem {
    volatile unsigned* misc;
    const int* kvrow;       // LDS copy of a.kvrow (null: row b -> window b)
    const PdLayer* layers;  // LDS copy of a.layers (r6 stamps: the prefetch's scalar loads of the global
                            // table stalled its issue 2-3 us per unit)
    bf16* img;
    f32x4* red;
    float (*s_m)[1];
    float (*s_l)[1];
    float (*s_o)[1][64];
    bf16* qkv_s;
    float* part_s;
    float* res_s;
    float* est;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t gran_rsrc(const PdArgs& a) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)a.gran, (short)0, (int)(a.R * (9 * a.d + 528 * a.H) * 8), 0x00020000);
}

// waves 0-3: per unit, its inputs into LDS; the barriers of compute_loop (A, [E: mid], B); then
// (wave 0) the unit's epilogue and output granules -- and the whole of a merge (E2) unit
__device__ __forceinline__ void gather_loop(const PdArgs& a, const Smem& sm, unsigned launch, int wg, int pos0) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int L = a.L;
    const __amdgpu_buffer_rsrc_t rs = gran_rsrc(a);
    Cur c{0, 0, unit0(a, 0, 0, wg) - a.nwg};
    bool has = advance(a, wg, c);
    int img_key = -1;  // (layer, stage) of the A image in LDS
    const bool stp = a.stamps != nullptr && wave == 0;
    int nk = 0;  // units this workgroup has run (stamp record index)
    while (has) {
        const PdLayer& Lw = sm.layers[c.l];
        const int key = (c.l << 4) | c.s;
        if (stp) {
            stamp(a, wg, nk, 0, (u64)c.l | ((u64)c.s << 8) | ((u64)c.u << 16), lane);
            stamp(a, wg, nk, 1, wall_clock64(), lane);
        }
        const bool need_img = img_key != key;
        bool ok = true;
        switch (c.s) {
            case S_A:
                if (need_img)
                    ok = gather_ln(a, rs, c.l == 0 ? -1 : G_X, ep_of(launch, L, c.l - 1, S_H), Lw.ln1_w, Lw.ln1_b,
                                   sm.img, wave, lane);
                break;
            case S_D:
                if (need_img) ok = gather_ln(a, rs, G_XC, ep_of(launch, L, c.l, S_C), Lw.ln2_w, Lw.ln2_b, sm.img, wave, lane);
                break;
            case S_G:
                if (need_img) ok = gather_ln(a, rs, G_XF, ep_of(launch, L, c.l, S_F), Lw.ln3_w, Lw.ln3_b, sm.img, wave, lane);
                break;
            case S_C:
                if (need_img) ok = gather_img(a, rs, G_A, a.d, ep_of(launch, L, c.l, S_B), sm.img, tid);
                if (ok && wave == 0)  // the residual: the layer's input x (layer 0: plain rows)
                    ok = gather_cols(a, rs, c.l == 0 ? -1 : G_X, ep_of(launch, L, c.l - 1, S_H), 16 * c.u, sm.res_s, lane);
                break;
            case S_F:
                if (need_img) ok = gather_img(a, rs, G_M, a.d, ep_of(launch, L, c.l, S_E2), sm.img, tid);
                if (ok && wave == 0) ok = gather_cols(a, rs, G_XC, ep_of(launch, L, c.l, S_C), 16 * c.u, sm.res_s, lane);
                break;
            case S_H:
                if (need_img) ok = gather_img(a, rs, G_H, 4 * a.d, ep_of(launch, L, c.l, S_G), sm.img, tid);
                if (ok && wave == 0 && (c.u & 1))  // slab 1 ends with x + p0 + p1: x's columns
                    ok = gather_cols(a, rs, G_XF, ep_of(launch, L, c.l, S_F), 16 * (c.u >> 1), sm.res_s, lane);
                break;
            case S_B:
                if (wave == 0) {
                    const int srcs[3] = {G_Q, G_K, G_V};
                    ok = gather_head(a, rs, srcs, 3, c.u / a.H, c.u % a.H, ep_of(launch, L, c.l, S_A), sm.qkv_s, lane);
                }
                break;
            case S_E:
                if (wave == 0) {
                    const int bh = c.u / (8 / a.e_vw);
                    const int srcs[1] = {G_QX};
                    ok = gather_head(a, rs, srcs, 1, bh / a.H, bh % a.H, ep_of(launch, L, c.l, S_D), sm.qkv_s, lane);
                }
                break;
            default:  // S_E2
                ok = gather_part(a, rs, c.u / a.H, c.u % a.H, ep_of(launch, L, c.l, S_E), sm.part_s, tid);
                break;
        }
        if (!ok) sm.misc[0] = 1u;
        if (stp) stamp(a, wg, nk, 2, wall_clock64(), lane);
        // the epilogue's operands, fetched ahead (wave 0): the bias of this unit's columns
        float bv = 0.f;
        const unsigned ep = ep_of(launch, L, c.l, c.s);
        if (wave == 0 && is_gemv(c.s)) {
            const float* bias = c.s == S_A ? Lw.qkv_b : c.s == S_C ? Lw.so_b : c.s == S_D ? Lw.cq_b
                              : c.s == S_F ? Lw.co_b : c.s == S_G ? Lw.fc1_b : Lw.fc2_b;
            const int n0 = c.s == S_H ? 16 * (c.u >> 1) : 16 * c.u;
            bv = (bias && !(c.s == S_H && (c.u & 1))) ? gp<float>(bias)[n0 + fr] : 0.f;  // fc2: slab 0 carries the bias
        }
        PD_BARRIER();  // A: inputs in LDS
        if (sm.misc[0]) break;
        if (is_gemv(c.s)) img_key = key;
        if (c.s == S_E2 && wave == 0) {  // attn_part_merge_kernel's operations (no compute waves)
#pragma clang fp contract(off)
                const int e = lane;
                float mw[8], lw[8], ow[8];
#pragma unroll
                for (int w = 0; w < 8; ++w) {
                    mw[w] = sm.part_s[w * 66 + 64];
                    lw[w] = sm.part_s[w * 66 + 65];
                    ow[w] = sm.part_s[w * 66 + e];
                }
                float M = -INFINITY;
#pragma unroll
                for (int w = 0; w < 8; ++w) M = fmaxf(M, mw[w]);
                float Ls = 0.f, O = 0.f;
#pragma unroll
                for (int w = 0; w < 8; ++w) {
                    if (mw[w] == -INFINITY) continue;
                    const float f = exp2f(mw[w] - M);
                    Ls = __builtin_fmaf(lw[w], f, Ls);
                    O = __builtin_fmaf(ow[w], f, O);
                }
                const unsigned mine = (unsigned)f2bf(O / Ls);
                const unsigned nb = __shfl_xor(mine, 1, 64);
                if (!(e & 1)) {
                    const int b = c.u / a.H, h = c.u - b * a.H;
                    gran_put(a.gran, go_of(a, G_M) + (int64_t)b * (a.d / 2) + 32 * h + e / 2, ep, mine | (nb << 16));
                }
        }
        if (c.s == S_E) PD_BARRIER();  // E mid: the first halves' softmax state in LDS
        PD_BARRIER();  // B: chain partials / attention partials in LDS
        if (stp) stamp(a, wg, nk, 5, wall_clock64(), lane);
        // ---------------- epilogue + publish (gather wave 0)
        if (wave == 0) {
            float resv[4] = {0.f, 0.f, 0.f, 0.f};
            if (c.s == S_C || c.s == S_F || (c.s == S_H && (c.u & 1))) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = 4 * fq + r;
                    resv[r] = row < a.R ? sm.res_s[row * 16 + fr] : 0.f;
                }
            }
            f32x4* red = sm.red;
            if (is_gemv(c.s)) {
                const Gv g = gv_of(a, Lw, c.s, c.u);
                f32x4 v0 = red[0 * 64 + lane];
                for (int cc = 1; cc < g.ks; ++cc) v0 += red[cc * 64 + lane];
                const int n = g.n0 + fr;
                const bool last = c.l == L - 1;
                switch (c.s) {
                    case S_A: {  // GV_QKV_CACHE: q -> granules; k, v -> the self cache and granules
                        const int part = n / a.d;  // 0 q, 1 k, 2 v
                        const int rem = n - part * a.d;
                        const int hh = rem >> 6, e = rem & 63;
                        const int gsrc = part == 0 ? G_Q : part == 1 ? G_K : G_V;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = 4 * fq + r;
                            const float y = v0[r] + bv;
                            const bf16 yb = from_f<bf16>(y);
                            if (part > 0 && row < a.R) {
                                bf16* kv = (bf16*)a.skv + a.self_layer * c.l;
                                kv[((((size_t)(part - 1) * a.R + row) * a.H + hh) * a.ctx + pos0) * 64 + e] = yb;
                            }
                            const unsigned nb = __shfl_xor((unsigned)yb, 1, 64);
                            if (!(fr & 1) && row < a.R)
                                gran_put(a.gran, go_of(a, gsrc) + (int64_t)row * (a.d / 2) + rem / 2, ep, (unsigned)yb | (nb << 16));
                        }
                        break;
                    }
                    case S_C:
                    case S_F: {  // GV_BIAS_RESID
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = 4 * fq + r;
                            if (row >= a.R) continue;
                            const float y = v0[r] + bv;
                            const float o = resv[r] + y;
                            gran_put(a.gran, go_of(a, c.s == S_C ? G_XC : G_XF) + (int64_t)row * a.d + n, ep, fbits(o));
                            if (c.s == S_F && last) a.xo[(size_t)row * a.d + n] = o;
                        }
                        break;
                    }
                    case S_D:
                    case S_G: {  // GV_BIAS / GV_BIAS_GELU -> bf16 pairs
                        const int N = c.s == S_D ? a.d : 4 * a.d;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = 4 * fq + r;
                            const float y = v0[r] + bv;
                            const bf16 yb = from_f<bf16>(c.s == S_D ? y : gelu_tanh(y));
                            const unsigned nb = __shfl_xor((unsigned)yb, 1, 64);
                            if (!(fr & 1) && row < a.R)
                                gran_put(a.gran, go_of(a, c.s == S_D ? G_QX : G_H) + (int64_t)row * (N / 2) + n / 2, ep,
                                         (unsigned)yb | (nb << 16));
                        }
                        break;
                    }
                    default: {  // S_H: GV_PARTIAL slab z (slab 0: + bias, slab 1: + 0); slab 1 then adds up
                                // the next LayerNorm's rows x + p0 + p1 in that order
                        const bool z1 = c.u & 1;
                        float p0v[4] = {0.f, 0.f, 0.f, 0.f};
                        if (z1 && !last) {  // slab 0's columns (its unit runs beside this one)
                            const int r8 = lane >> 3, pc = lane & 7;
                            unsigned off[1] = {(unsigned)((go_of(a, G_P0) + (int64_t)r8 * a.d + g.n0 + 2 * pc) * 8)};
                            u32x4 pv[1];
                            if (!poll<1>(a, rs, off, r8 < a.R ? 1u : 0u, ep_of(launch, L, c.l, S_H), pv)) {
                                sm.misc[0] = 1u;  // seen by every wave at the next barrier A
                            } else {
                                // lane (r8, pc) holds columns 2 pc, 2 pc + 1 of row r8: lane (fr, fq) needs
                                // column fr of rows 4 fq + r
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    const int src = (4 * fq + r) * 8 + (fr >> 1);
                                    const unsigned lo = __shfl(pv[0].x, src & 63, 64), hi = __shfl(pv[0].z, src & 63, 64);
                                    p0v[r] = bitsf((fr & 1) ? hi : lo);
                                }
                            }
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = 4 * fq + r;
                            if (row >= a.R) continue;
                            const float p = v0[r] + bv;  // bv = 0 for slab 1
                            if (last) {
                                a.pend[((size_t)(z1 ? a.R : 0) + row) * a.d + n] = p;
                            } else if (!z1) {
                                gran_put(a.gran, go_of(a, G_P0) + (int64_t)row * a.d + n, ep, fbits(p));
                            } else {
                                float xn = resv[r];
                                xn += p0v[r];
                                xn += p;
                                gran_put(a.gran, go_of(a, G_X) + (int64_t)row * a.d + n, ep, fbits(xn));
                            }
                        }
                        break;
                    }
                }
            } else if (c.s == S_B) {  // self-attention merge over the 8 virtual waves
                const int b = c.u / a.H, h = c.u - b * a.H;
                float M, Ls, O;
                attn_merge<1>(sm.s_m, sm.s_l, sm.s_o, 0, lane, M, Ls, O);
                const unsigned mine = (unsigned)from_f<bf16>(O / Ls);
                const unsigned nb = __shfl_xor(mine, 1, 64);
                if (!(lane & 1)) gran_put(a.gran, go_of(a, G_A) + (int64_t)b * (a.d / 2) + 32 * h + lane / 2, ep, mine | (nb << 16));
            }
        }
        if (stp) {  // the publish has landed (diagnostic builds of a pass only: waits for the stores)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stamp(a, wg, nk, 7, wall_clock64(), lane);
        }
        ++nk;
        has = advance(a, wg, c);
    }
}

// waves 4-7: per unit, barrier A, the unit's arithmetic and the next unit's prefetch, barrier B
__device__ __forceinline__ void compute_loop(const PdArgs& a, const Smem& sm, unsigned launch, int wg, int pos0) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cw = __builtin_amdgcn_readfirstlane(wave - 4);  // wave-uniform for the compiler too
    const int fr = lane & 15, fq = lane >> 4;
    const int L = a.L;
    bf16* img = sm.img;
    f32x4* red = sm.red;
    Cur c{0, 0, unit0(a, 0, 0, wg) - a.nwg};
    bool has = advance(a, wg, c);
    u32x4 pre[PNPRE];
    const bool stp = a.stamps != nullptr && cw == 0;
    int nk = 0;
    if (has) prefetch(a, sm.layers, sm.kvrow, c, cw, lane, pos0, pre);
    while (has) {
        const PdLayer& Lw = sm.layers[c.l];
        const unsigned ep = ep_of(launch, L, c.l, c.s);
        Cur nx = c;
        const bool nhas = advance(a, wg, nx);
        PD_BARRIER();  // A: inputs in LDS
        if (sm.misc[0]) break;
        if (stp) {  // after barrier A, then once this unit's prefetched operands have landed
            stamp(a, wg, nk, 3, wall_clock64(), lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stamp(a, wg, nk, 4, wall_clock64(), lane);
        }
        if (is_gemv(c.s)) {
            const Gv g = gv_of(a, Lw, c.s, c.u);
            const int ld = g.K + 8;
            int ss[PMAXSS], gc[PMAXSS];
            gv_plan(g, cw, ss, gc);
            // a chain with no super-step contributes +0 (a gemv_kernel wave with an empty K slice)
            for (int cc = cw; cc < g.ks; cc += 4) red[cc * 64 + lane] = f32x4{0.f, 0.f, 0.f, 0.f};
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            int cur = -1;
#pragma unroll
            for (int k = 0; k < PMAXSS; ++k) {
                if (ss[k] >= 0) {
                    if (gc[k] != cur) {
                        if (cur >= 0) red[cur * 64 + lane] = acc;
                        acc = f32x4{0.f, 0.f, 0.f, 0.f};
                        cur = gc[k];
                    }
                    const int kb = ss[k] * 128 + fq * 8;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        bf16x8 af;
                        if (fr < a.R) af = *(const bf16x8*)(img + (size_t)fr * ld + kb + i * 32);
                        else af = bf16x8{};
                        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8, pre[4 * k + i]), acc, 0, 0, 0);
                    }
                }
            }
            if (cur >= 0) red[cur * 64 + lane] = acc;
        } else if (c.s == S_B) {
            const int g8 = lane & 7, slot = lane >> 3;
            float qv[1][8];
            int lim[1] = {pos0 + 1};
#pragma unroll
            for (int e = 0; e < 8; ++e) qv[0][e] = to_f<bf16>(sm.qkv_s[8 * g8 + e]) * kLog2Scale;
            const int nk = pos0 + 1, nblk = cdiv(nk, 32);
            // this pass's key / value: the QKV units' granules (the cache row they also write is not
            // visible inside the launch) in place of the cached row pos0
            const bf16x8 kcur = *(const bf16x8*)(sm.qkv_s + 64 + 8 * g8);
            const bf16x8 vcur = *(const bf16x8*)(sm.qkv_s + 128 + 8 * g8);
            const int b = c.u / a.H, h = c.u - b * a.H;
            const bf16* kv = (const bf16*)a.skv + a.self_layer * c.l;
            const bf16* Kb = kv + (((size_t)0 * a.R + b) * a.H + h) * (size_t)a.ctx * 64 + 8 * g8;
            const bf16* Vb = kv + (((size_t)1 * a.R + b) * a.H + h) * (size_t)a.ctx * 64 + 8 * g8;
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const int vw = cw + 4 * v;
                AttnWave<bf16, 1> aw;
                aw.init(nullptr, nullptr, nk, lane);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int blk = vw + 8 * j;
                    if (blk < nblk) {
                        KVChunk<bf16> kc[4], vc[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int key = min(blk * 32 + 8 * i + slot, nk - 1);
                            if (j == 0) {
                                kc[i].v = __builtin_bit_cast(bf16x8, pre[(v * 4 + i) * 2]);
                                vc[i].v = __builtin_bit_cast(bf16x8, pre[(v * 4 + i) * 2 + 1]);
                            } else {
                                kc[i].load(Kb + key * 64);
                                vc[i].load(Vb + key * 64);
                            }
                            if (key == pos0) {
                                kc[i].v = kcur;
                                vc[i].v = vcur;
                            }
                        }
                        aw.process(kc, vc, blk * 32, qv, lim, 1);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
                aw.to_lds(sm.s_m, sm.s_l, sm.s_o, vw, lane);
            }
        } else if (c.s == S_E) {
            const Eu e = e_unit(a, sm.kvrow, c.l, c.u, cw, lane);
            const bool on = e.vi < a.e_vw;
            const int g8 = lane & 7;
            float qv[1][8];
            int lim[1] = {a.T_enc};
#pragma unroll
            for (int i = 0; i < 8; ++i) qv[0][i] = to_f<bf16>(sm.qkv_s[8 * g8 + i]) * kLog2Scale;
            const int nblk = cdiv(a.T_enc, 32);
            float* st = sm.est + e.vi * (9 * 64 + 4);  // {l, o[8]} per lane, then m
            AttnWave<bf16, 1> aw;
            aw.init(nullptr, nullptr, a.T_enc, lane);
            auto run3 = [&] {  // this half's three key blocks, in order
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const int blk = e.vw + 8 * (3 * e.half + t);
                    if (blk < nblk) {
                        KVChunk<bf16> kc[4], vc[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            kc[i].v = __builtin_bit_cast(bf16x8, pre[(t * 4 + i) * 2]);
                            vc[i].v = __builtin_bit_cast(bf16x8, pre[(t * 4 + i) * 2 + 1]);
                        }
                        aw.process(kc, vc, blk * 32, qv, lim, 1);
                    }
                }
            };
            if (on && e.half == 0) {
                run3();
                st[lane] = aw.l[0];
#pragma unroll
                for (int i = 0; i < 8; ++i) st[64 * (1 + i) + lane] = aw.o[0][i];
                if (lane == 0) st[9 * 64] = aw.m[0];
            }
            PD_BARRIER();  // E mid
            if (on && e.half == 1) {
                aw.l[0] = st[lane];
#pragma unroll
                for (int i = 0; i < 8; ++i) aw.o[0][i] = st[64 * (1 + i) + lane];
                aw.m[0] = st[9 * 64];
                run3();
                aw.to_lds(sm.s_m, sm.s_l, sm.s_o, e.vi, lane);
                // partial vw of (b, h): {o[64], m, l}, as cross_attn_vw_kernel writes it
                const int64_t pb = go_of(a, G_PART) + ((int64_t)e.bh * 8 + e.vw) * 66;
                gran_put(a.gran, pb + lane, ep, fbits(sm.s_o[e.vi][0][lane]));
                if (lane == 0) {
                    gran_put(a.gran, pb + 64, ep, fbits(sm.s_m[e.vi][0]));
                    gran_put(a.gran, pb + 65, ep, fbits(sm.s_l[e.vi][0]));
                }
            }
        }
        if (stp) stamp(a, wg, nk, 6, wall_clock64(), lane);
        if (nhas) prefetch(a, sm.layers, sm.kvrow, nx, cw, lane, pos0, pre);
        if (stp) stamp(a, wg, nk, 8, wall_clock64(), lane);
        PD_BARRIER();  // B: chain partials / attention partials in LDS; the image is free again
        if (stp) stamp(a, wg, nk, 9, wall_clock64(), lane);
        ++nk;
        c = nx;
        has = nhas;
    }
}

__global__ __launch_bounds__(PT, 1) void pdec_kernel(PdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    Smem sm;
    sm.misc = (volatile unsigned*)(smem + L_MISC);
    sm.layers = (const PdLayer*)(smem + L_LAYERS);
    sm.kvrow = a.kvrow ? (const int*)(smem + L_KVROW) : nullptr;
    if (a.kvrow && tid < a.R) ((int*)(smem + L_KVROW))[tid] = a.kvrow[tid];
    for (int i = tid; i < a.L * (int)(sizeof(PdLayer) / 8); i += PT)
        ((unsigned long long*)(smem + L_LAYERS))[i] = ((const unsigned long long*)a.layers)[i];
    sm.img = (bf16*)(smem + L_IMG);
    sm.red = (f32x4*)(smem + L_RED);
    sm.s_m = (float (*)[1])(smem + L_ATT);
    sm.s_l = (float (*)[1])(smem + L_ATT + 32);
    sm.s_o = (float (*)[1][64])(smem + L_ATT + 64);
    sm.qkv_s = (bf16*)(smem + L_QKV);
    sm.part_s = (float*)(smem + L_QKV);
    sm.res_s = (float*)(smem + L_RES);
    sm.est = (float*)(smem + L_EST);
    volatile unsigned* misc = sm.misc;
    if (tid == 0) {
        unsigned err = ld_rlx(a.ctl + 2);
        const unsigned li = ld_rlx(a.ctl + 3);
        if (!err && (int)li == a.force_giveup) {  // test hook: this launch gives up as a starved one would
            st_rlx(a.ctl + 2, 3u);
            err = 3u;
        }
        misc[0] = err;
        misc[1] = li;
        if (!err) __hip_atomic_fetch_add((gu32*)a.ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (misc[0]) return;
    const unsigned launch = __builtin_amdgcn_readfirstlane(misc[1]);  // uniform (see advance)
    const int pos0 = __builtin_amdgcn_readfirstlane(a.ds->pos0);
    if ((tid >> 6) < 4) gather_loop(a, sm, launch, blockIdx.x, pos0);
    else compute_loop(a, sm, launch, blockIdx.x, pos0);
    __syncthreads();
    if (tid == 0 && !misc[0]) {
        const unsigned prev = __hip_atomic_fetch_add((gu32*)(a.ctl + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)a.nwg - 1u) {  // the last workgroup: reset the census for the next launch
            st_rlx(a.ctl, 0u);
            st_rlx(a.ctl + 1, 0u);
            st_rlx(a.ctl + 3, launch + 1u);
        }
    }
}

int oldks(bool ln, int N, int nss) {  // gemv_launch_rg's wave geometry: waves that split K (KSPLIT)
    if (ln) {
        if (nss == 10) return N >= 4096 ? 5 : 10;  // the exact-slice LayerNorm configurations
        if (N >= 4096 && nss <= 24) return 4;
    }
    if (nss <= 8) return 4;
    if (nss <= 16) return 8;
    return 16;
}

int cu_count(int dev) {
    static std::mutex m;
    static std::vector<int> cache;
    std::lock_guard<std::mutex> g(m);
    if ((int)cache.size() <= dev) cache.resize(dev + 1, 0);
    if (!cache[dev]) HIP_CHECK(hipDeviceGetAttribute(&cache[dev], hipDeviceAttributeMultiprocessorCount, dev));
    return cache[dev];
}

}  // namespace

int64_t pdec_granules(int R, int d, int H) { return (int64_t)R * (9 * (int64_t)d + 528 * (int64_t)H); }

std::string pdec_unsupported(int dtype, int d, int H, int R, int ctx, int T_enc) {
    if (dtype != DT_BF16) return "bf16 models only";
    if (d % 128 || d > PMAXD || H * 64 != d) return "model width";
    if (R < 1 || R > PMAXR) return "rows per pass";
    if (ctx > 448 || T_enc > 1536 || T_enc < 1) return "context lengths";
    return std::string();
}

void pdec_prepare() { ensure_lds_attr((const void*)pdec_kernel, L_TOTAL); }

void pdec_launch(PdArgs a, hipStream_t st) {
    const std::string why = pdec_unsupported(DT_BF16, a.d, a.H, a.R, a.ctx, a.T_enc);
    if (!why.empty()) throw std::runtime_error("persistent decoder pass: unsupported " + why);
    if (a.L < 1 || a.L > PMAXL) throw std::runtime_error("persistent decoder pass: unsupported layer count");
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    a.nwg = cu_count(dev);
    a.nss = a.d / 128;
    const int R = a.R, d = a.d, H = a.H, nss = a.nss;
    a.e_vw = R * H * 8 <= a.nwg ? 1 : 2;  // virtual waves per cross-attention unit (two compute waves each)
    a.n[S_A] = 3 * d / 16; a.n[S_B] = R * H; a.n[S_C] = d / 16; a.n[S_D] = d / 16;
    a.n[S_E] = R * H * 8 / a.e_vw; a.n[S_E2] = R * H; a.n[S_F] = d / 16; a.n[S_G] = 4 * d / 16; a.n[S_H] = 2 * d / 16;
    a.ks[S_A] = oldks(true, 3 * d, nss);
    a.ks[S_C] = oldks(false, d, nss);
    a.ks[S_D] = oldks(true, d, nss);
    a.ks[S_F] = oldks(false, d, nss);
    a.ks[S_G] = oldks(true, 4 * d, nss);
    a.ks[S_H] = oldks(false, d, (4 * nss + 1) / 2);
    a.ks[S_B] = a.ks[S_E] = a.ks[S_E2] = 0;
    for (int st2 : {S_A, S_C, S_D, S_F, S_G, S_H})  // chains per wave fit the registers, chains the partials
        if (a.ks[st2] > 32 || a.ks[st2] < 4) throw std::runtime_error("persistent decoder pass: K geometry");
    int acc = 0;
    for (int s = 0; s < kPdStages; ++s) {
        a.pre[s] = acc;
        acc += a.n[s];
    }
    a.U = acc;
    const int64_t sz[12] = {(int64_t)R * d, (int64_t)R * d / 2, (int64_t)R * d / 2, (int64_t)R * d / 2, (int64_t)R * d / 2,
                            (int64_t)R * d, (int64_t)R * d / 2, (int64_t)R * H * 8 * 66, (int64_t)R * d / 2,
                            (int64_t)R * d, (int64_t)R * 2 * d, (int64_t)R * d};
    int64_t o = 0;
    for (int i = 0; i < 12; ++i) {
        a.go[i] = o;
        o += sz[i];
    }
    if (o != pdec_granules(R, d, H)) throw std::runtime_error("persistent decoder pass: granule layout");
    hipLaunchKernelGGL(pdec_kernel, dim3(a.nwg), dim3(PT), L_TOTAL, st, a);
    SPT_LAUNCH_CHECK();
}

}  // namespace spt
