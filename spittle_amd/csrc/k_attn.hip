// k_attn.hip -- encoder self-attention (non-causal, T = 1500, d_head = 64),
// flash style: the T x T score matrix never leaves registers.
//
// Replaces whisper.cpp's encoder attention (ggml mul_mat K.Q, soft_max_ext with
// scale 1/sqrt(64), mul_mat V.P -- or flash_attn_ext) in whisper_build_graph_encoder.
//
// Workgroup = 4 waves = 128 queries of one (batch, head); each wave owns 32
// queries.  K/V tiles of 64 keys are staged global -> LDS with
// global_load_lds_dwordx4 (K XOR-swizzled on the source address), double
// buffered.  Scores are computed transposed, S^T = K . Q^T, so each lane owns one
// query column: the row max / row sum of the online softmax are in-lane plus one
// cross-half shuffle, and the accumulator is directly the B operand of the next
// product O^T += V^T . P^T (CDNA4 accumulator-as-operand layout); V^T fragments
// come from ds_read_b64_tr_b16 transposed LDS reads.
//   bf16: v_mfma_f32_32x32x16_bf16, f32 accumulate, bf16 P.
//   f32 : v_mfma_f32_32x32x2_f32 (exact f32), P kept in f32 registers.
#include "common.h"
#include "kernels.h"

#include <cstdlib>

namespace spt {

namespace {

constexpr float kScaleLog2 = 0.125f * 1.4426950408889634f;  // (1/sqrt(64)) * log2(e)
constexpr float kLazy = 8.0f;  // bf16 kernel: re-base the softmax only past a 2^8 growth

__device__ __forceinline__ void glds16(const void* g, SPT_LDS void* l) {
    __builtin_amdgcn_global_load_lds((const void*)g, l, 16, 0, 0);
}

// one v_max3_f32 (the compiler does not form it from fmaxf chains here)
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float r;
    asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// ds_read_b64_tr_b16 as inline asm at base + OFF: the caller waits lgkmcnt itself before using it
template <int OFF>
__device__ __forceinline__ bf16x4v ds_tr16_asm(const SPT_LDS char* base) {
    bf16x4v v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(OFF) : "memory");
    return v;
}

__device__ __forceinline__ int key_of(int kt2, int r, int hf) { return 32 * kt2 + (r & 3) + 8 * (r >> 2) + 4 * hf; }

// -------------------------------------------------------------------- bf16
__global__ __launch_bounds__(256, 2) void attn_bf16_kernel(const bf16* __restrict__ qkv, int T, int H,
                                                           bf16* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 64 * 128];  // [buf][K|V][64 keys][128 B]
    const int d = H * 64, ld = 3 * d;
    const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int l32 = lane & 31, hf = lane >> 5;
    const bf16* base = qkv + (size_t)b * T * ld;

    const int q_abs = qt * 128 + wid * 32 + l32;
    const bf16* qp = base + (size_t)min(q_abs, T - 1) * ld + h * 64;
    bf16x8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *(const bf16x8*)(qp + 16 * s + 8 * hf);

    auto lds_k = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + (buf * 2 + 0) * 8192; };
    auto lds_v = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + (buf * 2 + 1) * 8192; };
    const int prow = lane >> 3, pch = lane & 7;
    auto stage = [&](int buf, int kt) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int p = wid * 2 + i;
            const int rt = 8 * p + prow;
            const int key = min(kt * 64 + rt, T - 1);
            const bf16* kr = base + (size_t)key * ld + d + h * 64;
            glds16(kr + 8 * (pch ^ (rt & 7)), lds_k(buf) + p * 1024);
            glds16(kr + d + 8 * pch, lds_v(buf) + p * 1024);
        }
    };

    float m_run = -INFINITY, l_run = 0.f;
    f32x16 o[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }

    const int nkt = cdiv(T, 64);
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) stage(cur ^ 1, kt + 1);
        const SPT_LDS char* lk = lds_k(cur);
        const SPT_LDS char* lv = lds_v(cur);
        f32x16 s[2];
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2) {
#pragma unroll
            for (int i = 0; i < 16; ++i) s[kt2][i] = 0.f;
            const int row = 32 * kt2 + l32;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const int c = 2 * st + hf;
                const bf16x8 a = *(const SPT_LDS bf16x8*)(lk + row * 128 + ((c ^ (row & 7)) << 4));
                s[kt2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[st], s[kt2], 0, 0, 0);
            }
        }
        if (kt * 64 + 64 > T) {
#pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (kt * 64 + key_of(kt2, r, hf) >= T) s[kt2][r] = -INFINITY;
        }
        float mloc = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) mloc = max3f(mloc, s[0][r], s[1][r]);
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        // Lazy rescaling: the reference maximum m_run moves only when some query's new scores
        // exceed it by more than 2^kLazy (then every lane re-bases, alpha <= 1); otherwise the
        // probabilities are taken against the stale maximum (p <= 2^kLazy: no overflow in f32
        // or bf16) and the accumulator rescale -- 32 multiplies and an exp per tile, a third of
        // the softmax's vector work -- is skipped.  l and o always share the same reference,
        // so the result is the same softmax up to rounding.
        float alpha = 1.0f;
        if (__any((mloc - m_run) * kScaleLog2 > kLazy)) {
            const float m_new = fmaxf(m_run, mloc);
            // v_exp_f32 directly: exp2f's denormal-range fix-up (cmp / cndmask / ldexp per
            // score) only matters for probabilities below 2^-126 of the running maximum
            alpha = __builtin_amdgcn_exp2f((m_run - m_new) * kScaleLog2);
            m_run = m_new;
#pragma unroll
            for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; }
        }
        const float mc = m_run * kScaleLog2;
        // scores in pairs: packed f32 FMA / add (v_pk_fma_f32, v_pk_add_f32) and one
        // v_cvt_pk_bf16_f32 per pair straight into the P^T fragment dwords
        const f32x2 sc2 = {kScaleLog2, kScaleLog2}, mc2 = {-mc, -mc};
        f32x2 ls2 = {0.f, 0.f};
        union { bf16x8 v; uint32_t w[4]; } pu[2][2];
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                const f32x2 sv = {s[kt2][r], s[kt2][r + 1]};
                const f32x2 t = __builtin_elementwise_fma(sv, sc2, mc2);
                const f32x2 pv = {__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
                ls2 += pv;
                pu[kt2][r >> 3].w[(r & 7) >> 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pv, bf16x2v));
            }
        const float lsum = ls2[0] + ls2[1];
        bf16x8 pf[2][2];
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp) pf[kt2][sp] = pu[kt2][sp].v;
        l_run = l_run * alpha + lsum;
        // O^T += V^T . P^T
        const int g = lane >> 4, i16 = lane & 15;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const int col = 32 * dt + 16 * (g & 1) + 4 * (i16 & 3);
#pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {
                    const int key0 = 32 * kt2 + 16 * sp + 4 * hf + (i16 >> 2);
                    const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (SPT_LDS bf16x4v*)(lv + key0 * 128 + col * 2));
                    const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (SPT_LDS bf16x4v*)(lv + (key0 + 8) * 128 + col * 2));
                    bf16x8 va;
                    va[0] = lo[0]; va[1] = lo[1]; va[2] = lo[2]; va[3] = lo[3];
                    va[4] = hi[0]; va[5] = hi[1]; va[6] = hi[2]; va[7] = hi[3];
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[kt2][sp], o[dt], 0, 0, 0);
                }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = 1.0f / l_tot;
    if (q_abs < T) {
        bf16* orow = out + ((size_t)b * T + q_abs) * d + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const int dd = 32 * dt + 8 * gg + 4 * hf;
                *(uint2*)(orow + dd) = make_uint2(pack_bf2(o[dt][4 * gg + 0] * inv, o[dt][4 * gg + 1] * inv),
                                                  pack_bf2(o[dt][4 * gg + 2] * inv, o[dt][4 * gg + 3] * inv));
            }
    }
}

// -------------------------------------------------------------------- bf16, 64 queries per wave
// Same algorithm as attn_bf16_kernel with each wave owning two 32-query column blocks: every K
// fragment (S^T = K . Q^T) and every V^T fragment (O^T += V^T . P^T) read from LDS feeds two
// MFMAs instead of one, halving the LDS fragment traffic per flop, and a workgroup (256 queries)
// stages each K/V tile for twice the queries, halving the L2 -> LDS traffic.
// K-tile chunk swizzle: a ds_read_b128 serves 16 lanes (rows r0..r0+15 of one 16-byte chunk
// column) per pass from one 256-byte bank window; rows are 128 B, so rows r and r + 8 share their
// window half, and (r & 7) gives them the same slot (2-way conflict on every K read).  SW = 1
// keys the swizzle on (r >> 1) & 7 instead: 16 distinct slots per pass.
// V tiles (read by ds_read_b64_tr_b16: a pass covers keys k0..k0+3 x four 8-byte pieces of
// two adjacent 16-byte chunk pairs) are unswizzled at SW bit 1 clear: keys k and k + 2 share
// their bank-window half and slot (2-way).  SW bit 1 XORs the chunk index with 4 on keys with
// bit 1 set: the 32 lanes of a pass then cover all 32 8-byte positions of the window.
template <int SW>
__device__ __forceinline__ int kswz(int r) { return (SW & 1) ? ((r >> 1) & 7) : (r & 7); }
template <int SW>
__device__ __forceinline__ int vswz(int r) { return (SW & 2) ? ((r & 2) << 1) : 0; }

// QL: the wave's Q fragments (2 query blocks x 4 k-steps, 32 VGPRs) live in LDS ([8][64 lanes] x 16 B
// per wave, lane-linear: conflict-free ds_read_b128) and are re-read at the start of every tile.
// Held in registers for the whole kernel they pushed it past 256 VGPRs at two waves per SIMD: 16
// spilled, and the loop reloaded K/V stage addresses and Q pieces from scratch on every tile (r5).
template <int SUM, int SW = 1, bool QL = false>  // row sums: 0 packed f32 VALU, 1 scalar f32 VALU, 2 an MFMA with a ones operand
__global__ __launch_bounds__(256, 2) void attn_bf16_q64_kernel(const bf16* __restrict__ qkv, int T, int H,
                                                               bf16* __restrict__ out, int fulldma) {
    // [buf][K|V][64 keys][128 B] (+ QL: [wave][qb * 4 + s][lane] x 16 B)
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 64 * 128 + (QL ? 4 * 8 * 64 * 16 : 0)];
    const int d = H * 64, ld = 3 * d;
    const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int l32 = lane & 31, hf = lane >> 5;
    const bf16* base = qkv + (size_t)b * T * ld;

    bf16x8 qf[2][4];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        const int q_abs = qt * 256 + wid * 64 + 32 * qb + l32;
        const bf16* qp = base + (size_t)min(q_abs, T - 1) * ld + h * 64;
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[qb][s] = *(const bf16x8*)(qp + 16 * s + 8 * hf);
        if constexpr (SUM == 4) {  // scores come out of the MFMA in log2 units: s = (q * c) . k
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int e = 0; e < 8; ++e) qf[qb][s][e] = (short)f2bf(bf2f((bf16)qf[qb][s][e]) * kScaleLog2);
        }
    }
    SPT_LDS bf16x8* qlds = (SPT_LDS bf16x8*)(smem + 2 * 2 * 64 * 128) + wid * 8 * 64;
    if constexpr (QL) {  // this wave's own region: its later reads follow these writes in LDS order
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
            for (int s = 0; s < 4; ++s) qlds[(qb * 4 + s) * 64 + lane] = qf[qb][s];
    }

    auto lds_k = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + (buf * 2 + 0) * 8192; };
    auto lds_v = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + (buf * 2 + 1) * 8192; };
    const int prow = lane >> 3, pch = lane & 7;
    auto stage = [&](int buf, int kt) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int p = wid * 2 + i;
            const int rt = 8 * p + prow;
            const int key = min(kt * 64 + rt, T - 1);
            const bf16* kr = base + (size_t)key * ld + d + h * 64;
            glds16(kr + 8 * (pch ^ kswz<SW>(rt)), lds_k(buf) + p * 1024);
            glds16(kr + d + 8 * (pch ^ vswz<SW>(rt)), lds_v(buf) + p * 1024);
        }
    };
    // SW == 3, a tile wholly inside T: a wave-uniform row address plus two per-lane byte offsets.
    // Row 8p + prow's K swizzle (r >> 1) & 7 is (prow >> 1) ^ 4 (p & 1) and its V swizzle
    // (r & 2) << 1 is prow's, and a row is a multiple of 128 B, so the offsets are fixed per lane:
    // no per-tile clamp, multiply and 64-bit add per piece (r5)
    const uint32_t lk0 = (uint32_t)(prow * ld * 2) + ((pch ^ (prow >> 1)) << 4);
    const uint32_t lv0 = (uint32_t)(prow * ld * 2) + ((pch ^ ((prow & 2) << 1)) << 4);
    auto stage_full = [&](int buf, int kt) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int p = wid * 2 + i;
            const char* row = (const char*)(base + (size_t)(kt * 64 + 8 * p) * ld + d + h * 64);
            glds16(row + (i ? (lk0 ^ 64u) : lk0), lds_k(buf) + p * 1024);
            glds16(row + 2 * d + lv0, lds_v(buf) + p * 1024);
        }
    };

    float m_run[2] = {-INFINITY, -INFINITY}, lsum[2] = {0.f, 0.f};
    f32x16 o[2][2], lacc[2];
    bf16x8 ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;  // bf16 1.0
#pragma unroll
    for (int i = 0; i < 16; ++i) { lacc[0][i] = 0.f; lacc[1][i] = 0.f; }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 16; ++i) { o[qb][0][i] = 0.f; o[qb][1][i] = 0.f; }

    f32x16 cinit[2];  // the QK^T chains' start: 0, or (SUM == 4, after the first tile) -m_run
#pragma unroll
    for (int i = 0; i < 16; ++i) { cinit[0][i] = 0.f; cinit[1][i] = 0.f; }
    // double-buffered K/V: the DMA of tile kt + 1 is issued before tile kt's products (a third
    // buffer with two tiles in flight measured slower: 149 vs 144 us on large-v3)
    const int nkt = cdiv(T, 64);
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // one K/V tile; called with a literal buffer index (the loop below is unrolled by two), so every
    // LDS address is a constant offset from one base: no per-tile address VALU beside the MFMAs (r4)
    auto tile = [&](const int kt, const int cur) __attribute__((always_inline)) {
        if (kt + 1 < nkt) {
            if (SW == 3 && fulldma && (kt + 1) * 64 + 64 <= T) stage_full(cur ^ 1, kt + 1);
            else stage(cur ^ 1, kt + 1);
        }
        const SPT_LDS char* lk = lds_k(cur);
        const SPT_LDS char* lv = lds_v(cur);
        f32x16 s[2][2];
        bf16x8 qt[QL ? 2 : 1][4];
        if constexpr (QL) {
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                for (int st = 0; st < 4; ++st) qt[qb][st] = qlds[(qb * 4 + st) * 64 + lane];
        }
        auto qfrag = [&](int qb, int st) -> const bf16x8& {
            if constexpr (QL) return qt[qb][st];
            else return qf[qb][st];
        };
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2) {
            // SUM == 4: the accumulator starts at -m (the query's running maximum, log2 units, a
            // lane constant), so the MFMA chain leaves s - m and p = exp2(s - m) needs no FMA.  The
            // chain's first MFMA reads that start from cinit (set only when m moves) as its C
            // operand: no 64 register moves per tile (r4)
            const int row = 32 * kt2 + l32;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const int c = 2 * st + hf;
                const bf16x8 a = *(const SPT_LDS bf16x8*)(lk + row * 128 + ((c ^ kswz<SW>(row)) << 4));
                s[0][kt2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qfrag(0, st), st == 0 ? cinit[0] : s[0][kt2], 0, 0, 0);
                s[1][kt2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qfrag(1, st), st == 0 ? cinit[1] : s[1][kt2], 0, 0, 0);
            }
        }
        if (kt * 64 + 64 > T) {
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        if (kt * 64 + key_of(kt2, r, hf) >= T) s[qb][kt2][r] = -INFINITY;
        }
        bf16x8 pf[2][2][2];
        if constexpr (SUM == 4) {
            // Optimistic softmax as SUM == 3, on scores already relative to the running maximum:
            // one v_exp and one scalar add per score (no packed f32 VALU beside the MFMAs); the
            // first tile, or a lane whose tile sum leaves [0, 2^12], re-bases: m += max(0, tile max)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                union { bf16x8 v; uint32_t w[4]; } pu[2][2];
                auto expo = [&](float sub) {
                    float l0 = 0.f, l1 = 0.f;
#pragma unroll
                    for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                        for (int r = 0; r < 16; r += 2) {
                            const float p0 = __builtin_amdgcn_exp2f(s[qb][kt2][r] - sub);
                            const float p1 = __builtin_amdgcn_exp2f(s[qb][kt2][r + 1] - sub);
                            l0 += p0;
                            l1 += p1;
                            const f32x2 pv = {p0, p1};
                            pu[kt2][r >> 3].w[(r & 7) >> 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pv, bf16x2v));
                        }
                    return l0 + l1;
                };
                auto expo0 = [&]() {  // the common path: s is already s - m
                    float l0 = 0.f, l1 = 0.f;
#pragma unroll
                    for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                        for (int r = 0; r < 16; r += 2) {
                            const float p0 = __builtin_amdgcn_exp2f(s[qb][kt2][r]);
                            const float p1 = __builtin_amdgcn_exp2f(s[qb][kt2][r + 1]);
                            l0 += p0;
                            l1 += p1;
                            const f32x2 pv = {p0, p1};
                            pu[kt2][r >> 3].w[(r & 7) >> 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pv, bf16x2v));
                        }
                    return l0 + l1;
                };
                float lt = kt > 0 ? expo0() : INFINITY;
                if (__any(!(lt <= 4096.0f))) {
                    float mloc = -INFINITY;  // tile maximum of s - m (kt == 0: of s, m = -inf)
#pragma unroll
                    for (int r = 0; r < 16; ++r) mloc = max3f(mloc, s[qb][0][r], s[qb][1][r]);
                    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
                    float delta, alpha;
                    if (kt == 0) {
                        delta = mloc;
                        alpha = 0.f;
                        m_run[qb] = mloc;
                    } else {
                        delta = fmaxf(mloc, 0.f);
                        alpha = __builtin_amdgcn_exp2f(-delta);
                        m_run[qb] += delta;
                    }
#pragma unroll
                    for (int i = 0; i < 16; ++i) cinit[qb][i] = -m_run[qb];
#pragma unroll
                    for (int i = 0; i < 16; ++i) { o[qb][0][i] *= alpha; o[qb][1][i] *= alpha; }
                    lsum[qb] *= alpha;
                    lt = expo(delta);
                }
                lsum[qb] += lt;
#pragma unroll
                for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                    for (int sp = 0; sp < 2; ++sp) pf[qb][kt2][sp] = pu[kt2][sp].v;
            }
        } else if constexpr (SUM == 3) {
            // Optimistic softmax: exponentiate against the running maximum first and re-base only
            // when a lane's tile row-sum leaves [0, 2^12] (or is not finite -- always on the first
            // tile, where m_run = -inf).  Probabilities stay <= 2^12 (exact range in f32 / bf16,
            // same relative precision), and the row maximum -- 16 dependent v_max3 plus a
            // cross-half exchange per query block per tile -- is computed only on that rare path.
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                union { bf16x8 v; uint32_t w[4]; } pu[2][2];
                auto expo = [&](float mcv) {
                    const f32x2 sc2 = {kScaleLog2, kScaleLog2}, mc2 = {-mcv, -mcv};
                    f32x2 ls2 = {0.f, 0.f};
#pragma unroll
                    for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                        for (int r = 0; r < 16; r += 2) {
                            const f32x2 sv = {s[qb][kt2][r], s[qb][kt2][r + 1]};
                            const f32x2 t = __builtin_elementwise_fma(sv, sc2, mc2);
                            const f32x2 pv = {__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
                            ls2 += pv;
                            pu[kt2][r >> 3].w[(r & 7) >> 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pv, bf16x2v));
                        }
                    return ls2[0] + ls2[1];
                };
                float lt = expo(m_run[qb] * kScaleLog2);
                if (__any(!(lt <= 4096.0f))) {
                    float mloc = -INFINITY;
#pragma unroll
                    for (int r = 0; r < 16; ++r) mloc = max3f(mloc, s[qb][0][r], s[qb][1][r]);
                    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
                    const float m_new = fmaxf(m_run[qb], mloc);
                    const float alpha = __builtin_amdgcn_exp2f((m_run[qb] - m_new) * kScaleLog2);
                    m_run[qb] = m_new;
#pragma unroll
                    for (int i = 0; i < 16; ++i) { o[qb][0][i] *= alpha; o[qb][1][i] *= alpha; }
                    lsum[qb] *= alpha;
                    lt = expo(m_new * kScaleLog2);
                }
                lsum[qb] += lt;
#pragma unroll
                for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                    for (int sp = 0; sp < 2; ++sp) pf[qb][kt2][sp] = pu[kt2][sp].v;
            }
        } else
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            float mloc = -INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) mloc = max3f(mloc, s[qb][0][r], s[qb][1][r]);
            mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
            if (__any((mloc - m_run[qb]) * kScaleLog2 > kLazy)) {  // lazy re-basing (attn_bf16_kernel)
                const float m_new = fmaxf(m_run[qb], mloc);
                const float alpha = __builtin_amdgcn_exp2f((m_run[qb] - m_new) * kScaleLog2);
                m_run[qb] = m_new;
#pragma unroll
                for (int i = 0; i < 16; ++i) { o[qb][0][i] *= alpha; o[qb][1][i] *= alpha; }
                if constexpr (SUM == 2) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) lacc[qb][i] *= alpha;
                } else {
                    lsum[qb] *= alpha;
                }
            }
            const float mc = m_run[qb] * kScaleLog2;
            union { bf16x8 v; uint32_t w[4]; } pu[2][2];
            if constexpr (SUM == 0) {  // packed f32 FMA / add (v_pk_fma_f32, v_pk_add_f32)
                const f32x2 sc2 = {kScaleLog2, kScaleLog2}, mc2 = {-mc, -mc};
                f32x2 ls2 = {0.f, 0.f};
#pragma unroll
                for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                    for (int r = 0; r < 16; r += 2) {
                        const f32x2 sv = {s[qb][kt2][r], s[qb][kt2][r + 1]};
                        const f32x2 t = __builtin_elementwise_fma(sv, sc2, mc2);
                        const f32x2 pv = {__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
                        ls2 += pv;
                        pu[kt2][r >> 3].w[(r & 7) >> 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pv, bf16x2v));
                    }
                lsum[qb] += ls2[0] + ls2[1];
            } else {  // scalar f32 FMA (packed f32 VALU costs extra issue cycles beside MFMAs)
                float ls = 0.f;
#pragma unroll
                for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                    for (int r = 0; r < 16; r += 2) {
                        const float p0 = __builtin_amdgcn_exp2f(fmaf(s[qb][kt2][r], kScaleLog2, -mc));
                        const float p1 = __builtin_amdgcn_exp2f(fmaf(s[qb][kt2][r + 1], kScaleLog2, -mc));
                        if constexpr (SUM == 1) ls += p0 + p1;
                        const f32x2 pv = {p0, p1};
                        pu[kt2][r >> 3].w[(r & 7) >> 1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(pv, bf16x2v));
                    }
                if constexpr (SUM == 1) lsum[qb] += ls;
            }
#pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) pf[qb][kt2][sp] = pu[kt2][sp].v;
        }
        // O^T += V^T . P^T for both query blocks from one V^T fragment
        const int g = lane >> 4, i16 = lane & 15;
        if constexpr (QL) {
            // the V^T reads as inline asm: issued through the builtin, each made the compiler wait
            // vmcnt(0) first -- for the NEXT tile's K/V DMA, issued at this tile's start into the
            // other buffer (it cannot tell the two LDS regions apart), so no tile's DMA overlapped
            // its own PV phase.  One lgkmcnt(0) per 8 reads instead (sched_barrier: the MFMAs stay
            // behind it); the data is the previous tile's DMA, retired by its end-of-tile wait.
            // the non-QL loop's addresses, split into a lane base per dt and constant offsets: key0 =
            // 32 kt2 + 16 sp + kl (+ 8 for hi), whose swizzle bit (bit 1) is kl's; chunk 4 dt + cl
            const int kl = 4 * hf + (i16 >> 2);
            const int sb = (SW & 2) ? ((kl >> 1) & 1) : 0;  // vswz = 4: chunk ^ 4 flips dt's bit
            const int cl = 2 * (g & 1) + ((i16 & 3) >> 1), c8 = 8 * (i16 & 1);
#pragma unroll
            for (int dt = 0; dt < 2; ++dt) {
                const SPT_LDS char* vb = lv + kl * 128 + ((4 * (dt ^ sb) + cl) << 4) + c8;
                bf16x4v lo[2][2], hi[2][2];
                lo[0][0] = ds_tr16_asm<0>(vb);
                hi[0][0] = ds_tr16_asm<1024>(vb);
                lo[0][1] = ds_tr16_asm<2048>(vb);
                hi[0][1] = ds_tr16_asm<3072>(vb);
                lo[1][0] = ds_tr16_asm<4096>(vb);
                hi[1][0] = ds_tr16_asm<5120>(vb);
                lo[1][1] = ds_tr16_asm<6144>(vb);
                hi[1][1] = ds_tr16_asm<7168>(vb);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                    for (int sp = 0; sp < 2; ++sp) {
                        const bf16x8 va = __builtin_shufflevector(lo[kt2][sp], hi[kt2][sp], 0, 1, 2, 3, 4, 5, 6, 7);
                        o[0][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[0][kt2][sp], o[0][dt], 0, 0, 0);
                        o[1][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[1][kt2][sp], o[1][dt], 0, 0, 0);
                    }
            }
        } else
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
            const int col = 32 * dt + 16 * (g & 1) + 4 * (i16 & 3);
#pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                for (int sp = 0; sp < 2; ++sp) {
                    const int key0 = 32 * kt2 + 16 * sp + 4 * hf + (i16 >> 2);
                    const int cb = col * 2;  // byte in the V row: chunk cb >> 4, 8-byte half cb & 8
                    const bf16x4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (SPT_LDS bf16x4v*)(lv + key0 * 128 + ((((cb >> 4) ^ vswz<SW>(key0)) << 4) | (cb & 15))));
                    const bf16x4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (SPT_LDS bf16x4v*)(lv + (key0 + 8) * 128 + ((((cb >> 4) ^ vswz<SW>(key0 + 8)) << 4) | (cb & 15))));
                    // a concatenation, not eight element inserts (which cost ~120 shift / or /
                    // and VALU per tile beside 32 MFMAs, r4)
                    const bf16x8 va = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                    o[0][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[0][kt2][sp], o[0][dt], 0, 0, 0);
                    o[1][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pf[1][kt2][sp], o[1][dt], 0, 0, 0);
                }
        }
        // row sums of the (bf16) probabilities: ones . P^T
        if constexpr (SUM == 2)
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp) {
                lacc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[0][kt2][sp], lacc[0], 0, 0, 0);
                lacc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[1][kt2][sp], lacc[1], 0, 0, 0);
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    for (int kt = 0; kt < nkt; kt += 2) {
        tile(kt, 0);
        if (kt + 1 < nkt) tile(kt + 1, 1);
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        const float inv = 1.0f / (SUM == 2 ? lacc[qb][0] : lsum[qb] + __shfl_xor(lsum[qb], 32, 64));
        const int q_abs = qt * 256 + wid * 64 + 32 * qb + l32;
        if (q_abs < T) {
            bf16* orow = out + ((size_t)b * T + q_abs) * d + h * 64;
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int gg = 0; gg < 4; ++gg) {
                    const int dd = 32 * dt + 8 * gg + 4 * hf;
                    *(uint2*)(orow + dd) = make_uint2(pack_bf2(o[qb][dt][4 * gg + 0] * inv, o[qb][dt][4 * gg + 1] * inv),
                                                      pack_bf2(o[qb][dt][4 * gg + 2] * inv, o[qb][dt][4 * gg + 3] * inv));
                }
        }
    }
}

// -------------------------------------------------------------------- f32
__global__ __launch_bounds__(256, 1) void attn_f32_kernel(const float* __restrict__ qkv, int T, int H,
                                                          float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 64 * 256];  // [buf][K|V][64 keys][256 B]
    const int d = H * 64, ld = 3 * d;
    const int qt = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int l32 = lane & 31, hf = lane >> 5;
    const float* base = qkv + (size_t)b * T * ld;

    const int q_abs = qt * 128 + wid * 32 + l32;
    const float* qp = base + (size_t)min(q_abs, T - 1) * ld + h * 64 + 32 * hf;
    float qf[32];
#pragma unroll
    for (int s = 0; s < 32; s += 4) {
        const float4 v = *(const float4*)(qp + s);
        qf[s] = v.x; qf[s + 1] = v.y; qf[s + 2] = v.z; qf[s + 3] = v.w;
    }
    auto lds_k = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + (buf * 2 + 0) * 16384; };
    auto lds_v = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + (buf * 2 + 1) * 16384; };
    const int prow = lane >> 4, pch = lane & 15;
    auto stage = [&](int buf, int kt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = wid * 4 + i;  // 16 pieces of 4 rows x 256 B
            const int rt = 4 * p + prow;
            const int key = min(kt * 64 + rt, T - 1);
            const float* kr = base + (size_t)key * ld + d + h * 64;
            glds16(kr + 4 * (pch ^ (rt & 15)), lds_k(buf) + p * 1024);
            glds16(kr + d + 4 * pch, lds_v(buf) + p * 1024);
        }
    };
    float m_run = -INFINITY, l_run = 0.f;
    f32x16 o[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) { o[0][i] = 0.f; o[1][i] = 0.f; }
    const int nkt = cdiv(T, 64);
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) stage(cur ^ 1, kt + 1);
        const SPT_LDS char* lk = lds_k(cur);
        const SPT_LDS float* lv = (const SPT_LDS float*)lds_v(cur);
        f32x16 s[2];
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2) {
#pragma unroll
            for (int i = 0; i < 16; ++i) s[kt2][i] = 0.f;
            const int row = 32 * kt2 + l32;
#pragma unroll
            for (int c8 = 0; c8 < 8; ++c8) {
                const int c = 8 * hf + c8;
                const f32x4 kv = *(const SPT_LDS f32x4*)(lk + row * 256 + ((c ^ (row & 15)) << 4));
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    s[kt2] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[e], qf[4 * c8 + e], s[kt2], 0, 0, 0);
            }
        }
        if (kt * 64 + 64 > T) {
#pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    if (kt * 64 + key_of(kt2, r, hf) >= T) s[kt2][r] = -INFINITY;
        }
        float mloc = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r) mloc = fmaxf(mloc, fmaxf(s[0][r], s[1][r]));
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = exp2f((m_run - m_new) * kScaleLog2);
        const float mc = m_new * kScaleLog2;
        float lsum = 0.f;
#pragma unroll
        for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float p = exp2f(s[kt2][r] * kScaleLog2 - mc);
                s[kt2][r] = p;
                lsum += p;
            }
        l_run = l_run * alpha + lsum;
        m_run = m_new;
#pragma unroll
        for (int i = 0; i < 16; ++i) { o[0][i] *= alpha; o[1][i] *= alpha; }
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int kt2 = 0; kt2 < 2; ++kt2)
#pragma unroll
                for (int st = 0; st < 16; ++st) {
                    const float va = lv[key_of(kt2, st, hf) * 64 + 32 * dt + l32];
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(va, s[kt2][st], o[dt], 0, 0, 0);
                }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = 1.0f / l_tot;
    if (q_abs < T) {
        float* orow = out + ((size_t)b * T + q_abs) * d + h * 64;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
                const int dd = 32 * dt + 8 * gg + 4 * hf;
                *(float4*)(orow + dd) = make_float4(o[dt][4 * gg + 0] * inv, o[dt][4 * gg + 1] * inv,
                                                    o[dt][4 * gg + 2] * inv, o[dt][4 * gg + 3] * inv);
            }
    }
}

}  // namespace

void enc_attention(int dtype, const void* qkv, int B, int T, int H, void* out, hipStream_t st) {
    static const bool q32 = getenv("SPT_ATTN_Q32") != nullptr;  // A/B switch: 32 queries per wave
    // 4: scores relative to the running max (r4: 133 -> 127 us); 3: r2-r3 optimistic softmax.  Read per
    // launch (eager runs: debug_encode; a captured encoder keeps its variant) so a test can compare them
    const char* sum_env = getenv("SPT_ATTN_SUM");
    const int sum = sum_env ? atoi(sum_env) : 4;
    const char* ql_env = getenv("SPT_ATTN_QL");  // Q fragments in LDS (default; 0: in registers, r4)
    const bool ql = !(ql_env && atoi(ql_env) == 0);
    // read per launch, as sum.  3 (K and V tiles swizzled): r5, 129.3 -> 128.5 us in two A/B pairs,
    // bitwise equal (scripts/enc_swz_bitwise.py)
    const char* swz_env = getenv("SPT_ATTN_SWZ");
    const int swz = swz_env ? atoi(swz_env) : 3;
    // DMA sources of whole tiles as a row address + fixed lane offsets (SW = 3; 0: the clamped
    // per-tile address arithmetic of r4); read per launch, as sum
    const char* fd_env = getenv("SPT_ATTN_FULLDMA");
    const int fulldma = !(fd_env && atoi(fd_env) == 0);
    // (r5's opt-in ping-pong wave groups and 32-query-per-wave kernels measured slower in situ and were
    // removed in r6: DESIGN.md 4.1g keeps their numbers)
    if (dtype == DT_BF16 && !q32) {
        dim3 g(cdiv(T, 256), H, B);
        if (sum == 1) hipLaunchKernelGGL(attn_bf16_q64_kernel<1>, g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else if (sum == 2) hipLaunchKernelGGL(attn_bf16_q64_kernel<2>, g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else if (sum == 3 && swz == 3) hipLaunchKernelGGL((attn_bf16_q64_kernel<3, 3>), g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else if (sum == 4 && ql && swz == 3)
            hipLaunchKernelGGL((attn_bf16_q64_kernel<4, 3, true>), g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else if (sum == 4 && ql) hipLaunchKernelGGL((attn_bf16_q64_kernel<4, 1, true>), g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else if (sum == 4) hipLaunchKernelGGL(attn_bf16_q64_kernel<4>, g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else if (sum == 3) hipLaunchKernelGGL(attn_bf16_q64_kernel<3>, g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else if (swz == 0) hipLaunchKernelGGL((attn_bf16_q64_kernel<0, 0>), g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else if (swz == 1) hipLaunchKernelGGL((attn_bf16_q64_kernel<0, 1>), g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        else hipLaunchKernelGGL((attn_bf16_q64_kernel<0, 3>), g, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out, fulldma);
        return;
    }
    dim3 grid(cdiv(T, 128), H, B);
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(attn_bf16_kernel, grid, dim3(256), 0, st, (const bf16*)qkv, T, H, (bf16*)out);
    else
        hipLaunchKernelGGL(attn_f32_kernel, grid, dim3(256), 0, st, (const float*)qkv, T, H, (float*)out);
}

}  // namespace spt
