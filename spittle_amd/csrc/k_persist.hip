// k_persist.hip -- one decoder pass (all layers of whisper.cpp whisper_build_graph_decoder
// for a single new token per sequence) as ONE persistent launch.
//
// Why: at B = 8 every decoder op is a small weight/KV stream, and the per-kernel
// ramp + launch floor (~2.5 us) x 8 launches per layer was ~60 % of the pass. Here one
// workgroup per CU (8 waves) walks the 8 phases of every layer; phases are separated
// by dataflow flags instead of kernel boundaries:
//   P1 LN1 + QKV (+ self K/V append)   P2 self-attention      P3 out-proj + residual
//   P4 LN2 + cross-Q                   P5 cross-attention     P6 out-proj + residual
//   P7 LN3 + fc1 + GELU                P8 fc2 + residual
// Each phase first issues its own weight (or cross K/V) loads into registers, THEN
// waits for the producers of its input, so the weight stream overlaps the previous
// phase's tail and the flag latency. A workgroup publishes flags[wg] = seq after its
// phase-outputs are written back (agent-scope release); consumers poll the producer
// range and acquire. Every wait is bounded: a timeout raises a device abort word that
// every poller also watches, so a broken pass exits instead of hanging the device.
//
// Determinism: each output element is reduced in a fixed order (waves by rank, cross-
// attention splits by index), so results are independent of timing and of which rows
// share the batch.
#include "common.h"
#include "kernels.h"

namespace spt {

namespace {

constexpr int PW = 8;               // waves per workgroup
constexpr int PT = 64 * PW;         // threads per workgroup
constexpr int MAXKS = 20;           // 32-wide K steps per wave held in registers (GEMV phases)
constexpr int SPIN_LIMIT = 1 << 21; // polls before a wait is declared hung (~1 s)
constexpr float kL2S = 0.125f * 1.4426950408889634f;  // (1/sqrt(64)) * log2(e)

// SPT_PERSIST_DEBUG builds check every global access against the engine's two arenas
// and record the first offending site instead of touching memory (abort word = 3,
// abort_flag[1] = site, [2..3] = address).
#ifdef SPT_PERSIST_DEBUG
__device__ bool pchk(const PersistArgs& a, const void* p, int site) {
    const char* c = (const char*)p;
    if ((c >= a.ws_lo && c + 16 <= a.ws_hi) || (c >= a.wt_lo && c + 16 <= a.wt_hi)) return true;
    if (atomicCAS(a.abort_flag + 1, 0u, (unsigned)site) == 0u) {
        a.abort_flag[2] = (unsigned)(uintptr_t)c;
        a.abort_flag[3] = (unsigned)((uintptr_t)c >> 32);
    }
    __hip_atomic_store(a.abort_flag, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
}
#define PGUARD(a, p, site) if (pchk(a, p, site))
#else
#define PGUARD(a, p, site)
#endif

struct Smem {
    int ok;
    f32x4 red[PW][64];                 // GEMV cross-wave reduction
    // followed by the LayerNorm image (bf16 [R][K + 8])
};
constexpr int kSmemBytes = (int)((sizeof(Smem) + 15) & ~15);

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// ---------------------------------------------------------------- phase synchronisation
// All waves drain their own stores (vmcnt), the workgroup meets, thread 0 releases.
__device__ __forceinline__ void publish(const PersistArgs& a, unsigned seq) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(a.flags + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until flags[0 .. n_prod) >= seq. Wave 0 polls; the acquire fence (L1/L2 invalidate)
// precedes the workgroup barrier, after which every wave reads fresh data.
__device__ bool wait_for(const PersistArgs& a, int n_prod, unsigned seq, Smem* sm) {
    if (n_prod <= 0) return true;
    if (wave_id() == 0) {
        const int lane = lane_id();
        bool ok = true;
        for (int spin = 0;; ++spin) {
            bool mine = true;
            for (int i = lane; i < n_prod; i += 64)
                mine &= __hip_atomic_load(a.flags + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= seq;
            if (__all(mine)) break;
            if ((spin & 31) == 31 && __hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                ok = false;
                break;
            }
            if (spin > SPIN_LIMIT) {
                if (lane == 0) __hip_atomic_store(a.abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (lane == 0) sm->ok = ok;
    }
    __syncthreads();
    return sm->ok;
}

// ---------------------------------------------------------------- GEMV phase
enum { PM_QKV = 0, PM_BIAS = 1, PM_GELU = 2, PM_RESID = 3 };

struct GemvPhase {
    const bf16* W; int N, K;          // W [N][K]
    const float* bias;                // [N]
    const float* ln_w; const float* ln_b;  // LN of a.x (f32 rows) when non-null
    const bf16* A; int lda;           // else bf16 activations [R][lda]
    void* C; int ldc;                 // output (bf16 for QKV/BIAS/GELU, f32 residual for RESID)
    bf16* cache;                      // PM_QKV: self K/V of this layer [2][B][H][ctx][64]
    int pos;                          // PM_QKV: cache position of the new token
};

// Workgroup w owns column tiles w, w + G, ...; its waves split those tiles' K range.
template <int MODE, int JMAX, bool LN>
__device__ bool gemv_phase(const PersistArgs& a, const GemvPhase& p, int n_prod, unsigned seq_wait, Smem* sm,
                           bf16* img) {
    const int G = gridDim.x, w = blockIdx.x;
    const int n_tiles = p.N >> 4;
    const int ntl = w < n_tiles ? (n_tiles - 1 - w) / G + 1 : 0;
    if (ntl == 0) return true;
    const int lane = lane_id(), wid = wave_id(), fr = lane & 15, fq = lane >> 4;
    const int ti = wid % ntl, rank = wid / ntl;
    const int nwt = (PW - 1 - ti) / ntl + 1;  // waves on tile ti
    const int n0 = (w + ti * G) * 16;
    const int nks = p.K >> 5;
    const int R = a.B;

    // 1. this wave's weight slice (independent of the phase input): in flight during the wait
    bf16x8 wv[JMAX];
    const bf16* wr = p.W + (size_t)n0 * p.K;             // uniform base
    const int wo = fr * p.K + fq * 8 + rank * 32;         // per-lane element offset
    const int wstep = nwt * 32;
#pragma unroll
    for (int j = 0; j < JMAX; ++j) {
        const int ks = rank + j * nwt;
        if (ks < nks) PGUARD(a, wr + (wo + j * wstep), 1) wv[j] = *(const bf16x8*)(wr + (wo + j * wstep));
    }
    // 2. producers of the input
    if (!wait_for(a, n_prod, seq_wait, sm)) return false;
    const int K = p.K, ild = K + 8;
    // 3. LayerNorm prologue (one row per wave) into the bf16 image
    if constexpr (LN) {
        for (int r = wid; r < R; r += PW) {
            const float* xr = a.x + (size_t)r * a.d;
            float4 v[6];
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    PGUARD(a, xr + k, 2) v[i] = *(const float4*)(xr + k);
                    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
                }
            }
            const float mean = wave_sum(s) / (float)K;
            float s2 = 0.f;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    const float q0 = v[i].x - mean, q1 = v[i].y - mean, q2 = v[i].z - mean, q3 = v[i].w - mean;
                    s2 += (q0 * q0 + q1 * q1) + (q2 * q2 + q3 * q3);
                }
            }
            const float rstd = 1.0f / sqrtf(wave_sum(s2) / (float)K + 1e-5f);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int k = lane * 4 + 256 * i;
                if (k < K) {
                    float4 g{}, b{};
                    PGUARD(a, p.ln_w + k, 3) g = *(const float4*)(p.ln_w + k);
                    PGUARD(a, p.ln_b + k, 4) b = *(const float4*)(p.ln_b + k);
                    uint2 o;
                    o.x = pack_bf2((v[i].x - mean) * rstd * g.x + b.x, (v[i].y - mean) * rstd * g.y + b.y);
                    o.y = pack_bf2((v[i].z - mean) * rstd * g.z + b.z, (v[i].w - mean) * rstd * g.w + b.w);
                    *(uint2*)(img + (size_t)r * ild + k) = o;
                }
            }
        }
    } else {
        // bf16 activations: the whole [R][K] block staged into the image, 16 B per thread
        const int cpr = K >> 3, n_chunks = R * cpr;
        for (int c0 = threadIdx.x; c0 < n_chunks; c0 += 4 * PT) {
            bf16x8 t[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = c0 + i * PT, r = c / cpr, k = (c - r * cpr) * 8;
                if (c < n_chunks) PGUARD(a, p.A + (size_t)r * p.lda + k, 5) t[i] = *(const bf16x8*)(p.A + (size_t)r * p.lda + k);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = c0 + i * PT, r = c / cpr, k = (c - r * cpr) * 8;
                if (c < n_chunks) *(bf16x8*)(img + (size_t)r * ild + k) = t[i];
            }
        }
    }
    __syncthreads();
    // 4. MFMA over the wave's K steps (rows >= R are zero A rows)
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const bool rv = fr < R;
    const bf16* ai = img + (size_t)(rv ? fr : 0) * ild + fq * 8;  // never address past the image
#pragma unroll
    for (int j = 0; j < JMAX; ++j) {
        const int ks = rank + j * nwt;
        if (ks >= nks) break;
        const bf16x8 af = rv ? *(const bf16x8*)(ai + ks * 32) : bf16x8{};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wv[j], acc, 0, 0, 0);
    }
    // 5. reduce the tile's waves in rank order
    sm->red[wid][lane] = acc;
    __syncthreads();
    if (rank != 0) return true;
    for (int r = 1; r < nwt; ++r) acc += sm->red[ti + r * ntl][lane];
    // 6. epilogue: lane holds column n0 + fr, rows 4 fq .. 4 fq + 3
    const int n = n0 + fr;
    float bv = 0.f;
    PGUARD(a, p.bias + n, 6) bv = p.bias[n];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = 4 * fq + i;
        if (row >= R) break;
        const float y = acc[i] + bv;
        if constexpr (MODE == PM_RESID) {
            float* c = (float*)p.C + (size_t)row * p.ldc + n;
            PGUARD(a, c, 7) *c = *c + y;
        } else if constexpr (MODE == PM_GELU) {
            PGUARD(a, (bf16*)p.C + (size_t)row * p.ldc + n, 8) ((bf16*)p.C)[(size_t)row * p.ldc + n] = f2bf(gelu_tanh(y));
        } else if constexpr (MODE == PM_BIAS) {
            PGUARD(a, (bf16*)p.C + (size_t)row * p.ldc + n, 9) ((bf16*)p.C)[(size_t)row * p.ldc + n] = f2bf(y);
        } else {
            const int d = a.d;
            if (n < d) {
                PGUARD(a, (bf16*)p.C + (size_t)row * p.ldc + n, 10) ((bf16*)p.C)[(size_t)row * p.ldc + n] = f2bf(y);
            } else {
                const int part = n / d - 1, rem = n - (part + 1) * d;
                const size_t off = ((((size_t)part * a.B + row) * a.H + (rem >> 6)) * a.ctx + p.pos) * 64 + (rem & 63);
                PGUARD(a, p.cache + off, 11) p.cache[off] = f2bf(y);
            }
        }
    }
    return true;
}

// ---------------------------------------------------------------- attention phase
// Units (b, h, s): keys [s*n/S, (s+1)*n/S) of sequence b, head h, one unit per wave
// (workgroup w owns units w + G*j, wave j handles j = wid, wid + PW, ...). 8 lanes per
// key (16 B each of K and V), ANI groups of 8 keys per block, two blocks in flight.
// Each unit writes its (m, l, o[64]) partial; the wave that completes the S-th split
// of a (b, h) (counter ticket) merges the splits in index order -> bf16 output.
constexpr int ANI = 4;
constexpr int AKB = 8 * ANI;

struct AttnPhase {
    const bf16* q;                    // [B][d]
    const bf16* kv;                   // K at kv + ((b*H + h)*kv_ctx)*64, V at + v_off
    int64_t v_off; int kv_ctx;        // elements between the K and V planes; rows per (b, h)
    int n_keys, S;
    unsigned* cnt;                    // per (b, h) split tickets
    bool prefetch;                    // K/V independent of the phase input (cross-attention)
};

__device__ bool attn_phase(const PersistArgs& a, const AttnPhase& p, int n_prod, unsigned seq_wait, Smem* sm) {
    const int G = gridDim.x, w = blockIdx.x;
    const int n_units = a.B * a.H * p.S;
    const int nu = w < n_units ? (n_units - 1 - w) / G + 1 : 0;
    if (nu == 0) return true;
    const int lane = lane_id(), wid = wave_id(), slot = lane >> 3, g = lane & 7;

    bf16x8 kA[ANI], vA[ANI], kB[ANI], vB[ANI];
    const bf16* Kb = nullptr;
    const bf16* Vb = nullptr;
    int nk = 0, nblk = 0;
    auto setup = [&](int j) {
        const int u = w + j * G, bh = u / p.S, s = u - bh * p.S;
        const int k0 = (int)((int64_t)s * p.n_keys / p.S), k1 = (int)((int64_t)(s + 1) * p.n_keys / p.S);
        nk = k1 - k0;
        nblk = cdiv(nk, AKB);
        Kb = p.kv + ((size_t)bh * p.kv_ctx + k0) * 64;  // uniform bases
        Vb = Kb + p.v_off;
    };
    auto load_blk = [&](bf16x8(&kc)[ANI], bf16x8(&vc)[ANI], int blk) {
#pragma unroll
        for (int i = 0; i < ANI; ++i) {
            const int key = min(blk * AKB + 8 * i + slot, nk - 1);
            PGUARD(a, Kb + (key * 64 + 8 * g), 12) kc[i] = *(const bf16x8*)(Kb + (key * 64 + 8 * g));
            PGUARD(a, Vb + (key * 64 + 8 * g), 13) vc[i] = *(const bf16x8*)(Vb + (key * 64 + 8 * g));
        }
    };
    // the first unit's first two blocks stream in during the wait when K/V are ready
    if (p.prefetch && wid < nu) {
        setup(wid);
        if (nblk > 0) load_blk(kA, vA, 0);
        if (nblk > 1) load_blk(kB, vB, 1);
    }
    if (!wait_for(a, n_prod, seq_wait, sm)) return false;

    for (int j = wid; j < nu; j += PW) {
        const bool pre = p.prefetch && j == wid;
        if (!pre) {
            setup(j);
            if (nblk > 0) load_blk(kA, vA, 0);
            if (nblk > 1) load_blk(kB, vB, 1);
        }
        const int u = w + j * G, bh = u / p.S, b = bh / a.H, h = bh - b * a.H;
        float qv[8], o[8], m = -INFINITY, l = 0.f;
        {
            bf16x8 qr{};
            PGUARD(a, p.q + (size_t)b * a.d + h * 64 + 8 * g, 14) qr = *(const bf16x8*)(p.q + (size_t)b * a.d + h * 64 + 8 * g);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                qv[e] = bf2f((bf16)qr[e]) * kL2S;
                o[e] = 0.f;
            }
        }
        auto process = [&](const bf16x8(&kc)[ANI], const bf16x8(&vc)[ANI], int kbase) {
            float sc[ANI];
            float mb = -INFINITY;
#pragma unroll
            for (int i = 0; i < ANI; ++i) {
                float v = 0.f;
#pragma unroll
                for (int e = 0; e < 8; ++e) v += qv[e] * bf2f((bf16)kc[i][e]);
                v += __shfl_xor(v, 1, 64);
                v += __shfl_xor(v, 2, 64);
                v += __shfl_xor(v, 4, 64);
                if (kbase + 8 * i + slot >= nk) v = -INFINITY;
                sc[i] = v;
                mb = fmaxf(mb, v);
            }
            mb = fmaxf(mb, __shfl_xor(mb, 8, 64));
            mb = fmaxf(mb, __shfl_xor(mb, 16, 64));
            mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
            if (mb == -INFINITY) return;
            const float mn = fmaxf(m, mb);
            const float alpha = exp2f(m - mn);
            float ls = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] *= alpha;
#pragma unroll
            for (int i = 0; i < ANI; ++i) {
                const float pr = exp2f(sc[i] - mn);
                ls += pr;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] += pr * bf2f((bf16)vc[i][e]);
            }
            l = l * alpha + ls;
            m = mn;
        };
        // A holds blocks 0, 2, 4, ...; B holds 1, 3, 5, ...
        for (int blk = 0; blk < nblk;) {
            process(kA, vA, blk * AKB);
            if (blk + 2 < nblk) load_blk(kA, vA, blk + 2);
            if (++blk >= nblk) break;
            process(kB, vB, blk * AKB);
            if (blk + 2 < nblk) load_blk(kB, vB, blk + 2);
            ++blk;
        }
        // merge the 8 key slots (m is wave-uniform)
        l += __shfl_xor(l, 8, 64);
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float v = o[e];
            v += __shfl_xor(v, 8, 64);
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            o[e] = v;
        }
        bf16* out = a.ao + (size_t)b * a.d + h * 64;
        if (p.S == 1) {
            if (lane < 8) {
                uint4 r;
                r.x = pack_bf2(o[0] / l, o[1] / l);
                r.y = pack_bf2(o[2] / l, o[3] / l);
                r.z = pack_bf2(o[4] / l, o[5] / l);
                r.w = pack_bf2(o[6] / l, o[7] / l);
                *(uint4*)(out + 8 * g) = r;
            }
            continue;
        }
        float* pp = a.xpart + (size_t)u * 66;
        if (lane < 8) {
#pragma unroll
            for (int e = 0; e < 8; ++e) PGUARD(a, pp + 2 + 8 * g + e, 15) pp[2 + 8 * g + e] = o[e];
        }
        if (lane == 0) {
            PGUARD(a, pp, 16) pp[0] = m;
            PGUARD(a, pp + 1, 16) pp[1] = l;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned ticket = 0;
        if (lane == 0) PGUARD(a, p.cnt + bh, 17) ticket = __hip_atomic_fetch_add(p.cnt + bh, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        ticket = __shfl(ticket, 0, 64);
        if ((ticket + 1) % (unsigned)p.S != 0u) continue;
        // last split of (b, h): merge all S partials in index order, lane = output dim
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const float* pb = a.xpart + (size_t)bh * p.S * 66;
#ifdef SPT_PERSIST_DEBUG
        if (!pchk(a, pb, 19) || !pchk(a, pb + (size_t)p.S * 66 - 4, 19)) continue;
#endif
        float M = -INFINITY;
        for (int q = 0; q < p.S; ++q) M = fmaxf(M, pb[q * 66]);
        float L = 0.f, O = 0.f;
        for (int q = 0; q < p.S; ++q) {
            const float mq = pb[q * 66];
            if (mq == -INFINITY) continue;
            const float f = exp2f(mq - M);
            L += pb[q * 66 + 1] * f;
            O += pb[q * 66 + 2 + lane] * f;
        }
        PGUARD(a, out + lane, 18) out[lane] = f2bf(O / L);
    }
    return true;
}

// One decoder phase; noinline so each phase is register-allocated on its own (the
// loop in the kernel keeps only a handful of scalars live across phases).
template <int PH>
__device__ __forceinline__ bool run_phase(const PersistArgs* pa, int l, unsigned s0, int pos, Smem* sm,
                                                     bf16* img) {
    const PersistArgs& a = *pa;
    const PersistLayer& L = a.layers[l];
    const int G = gridDim.x, d = a.d, H = a.H;
    if constexpr (PH == 0) {  // P1: LN1 + QKV (+ K/V append); x from the previous layer (or the launch)
        GemvPhase gp{};
        gp.W = L.qkv_w; gp.N = 3 * d; gp.K = d; gp.bias = L.qkv_b; gp.ln_w = L.ln1_w; gp.ln_b = L.ln1_b;
        gp.C = a.q; gp.ldc = d; gp.cache = a.skv + (size_t)l * a.self_layer; gp.pos = pos;
        return gemv_phase<PM_QKV, 5, true>(a, gp, l == 0 ? 0 : min(G, d / 16), s0, sm, img);
    } else if constexpr (PH == 1) {  // P2: self-attention over keys 0..pos
        AttnPhase ap{};
        ap.q = a.q; ap.kv = a.skv + (size_t)l * a.self_layer; ap.v_off = (int64_t)a.B * H * a.ctx * 64;
        ap.kv_ctx = a.ctx; ap.n_keys = pos + 1; ap.S = a.S_self; ap.cnt = a.xcnt; ap.prefetch = false;
        return attn_phase(a, ap, min(G, 3 * d / 16), s0, sm);
    } else if constexpr (PH == 2) {  // P3: self out-proj + residual
        GemvPhase gp{};
        gp.W = L.so_w; gp.N = d; gp.K = d; gp.bias = L.so_b; gp.A = a.ao; gp.lda = d; gp.C = a.x; gp.ldc = d;
        return gemv_phase<PM_RESID, 5, false>(a, gp, min(G, a.B * H * a.S_self), s0, sm, img);
    } else if constexpr (PH == 3) {  // P4: LN2 + cross-Q
        GemvPhase gp{};
        gp.W = L.cq_w; gp.N = d; gp.K = d; gp.bias = L.cq_b; gp.ln_w = L.ln2_w; gp.ln_b = L.ln2_b;
        gp.C = a.q; gp.ldc = d;
        return gemv_phase<PM_BIAS, 5, true>(a, gp, min(G, d / 16), s0, sm, img);
    } else if constexpr (PH == 4) {  // P5: cross-attention over the encoder K/V (S splits, last merges)
        AttnPhase ap{};
        ap.q = a.q; ap.kv = a.ckv + (size_t)l * a.cross_layer; ap.v_off = (int64_t)a.B_layout * H * a.T_enc * 64;
        ap.kv_ctx = a.T_enc; ap.n_keys = a.T_enc; ap.S = a.S_cross; ap.cnt = a.xcnt + a.B * H; ap.prefetch = true;
        return attn_phase(a, ap, min(G, d / 16), s0, sm);
    } else if constexpr (PH == 5) {  // P6: cross out-proj + residual
        GemvPhase gp{};
        gp.W = L.co_w; gp.N = d; gp.K = d; gp.bias = L.co_b; gp.A = a.ao; gp.lda = d; gp.C = a.x; gp.ldc = d;
        return gemv_phase<PM_RESID, 5, false>(a, gp, min(G, a.B * H * a.S_cross), s0, sm, img);
    } else if constexpr (PH == 6) {  // P7: LN3 + fc1 + GELU
        GemvPhase gp{};
        gp.W = L.fc1_w; gp.N = 4 * d; gp.K = d; gp.bias = L.fc1_b; gp.ln_w = L.ln3_w; gp.ln_b = L.ln3_b;
        gp.C = a.ff; gp.ldc = 4 * d;
        return gemv_phase<PM_GELU, 10, true>(a, gp, min(G, d / 16), s0, sm, img);
    } else {  // P8: fc2 + residual
        GemvPhase gp{};
        gp.W = L.fc2_w; gp.N = d; gp.K = 4 * d; gp.bias = L.fc2_b; gp.A = a.ff; gp.lda = 4 * d; gp.C = a.x;
        gp.ldc = d;
        return gemv_phase<PM_RESID, MAXKS, false>(a, gp, min(G, 4 * d / 16), s0, sm, img);
    }
}

// The arguments live in device memory (one pointer kernel argument) and are re-read per
// phase through the scalar cache instead of pinning ~40 SGPRs for the whole kernel.
__global__ __launch_bounds__(PT) void persist_kernel(const PersistArgs* pa) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    Smem* sm = (Smem*)smem_raw;
    bf16* img = (bf16*)(smem_raw + kSmemBytes);
    constexpr int NPH = 8;
    const int n_layers = pa->n_layers;
    const int step = pa->ds->step, pos = pa->ds->pos0;
    if (pos < 0 || pos >= pa->ctx || step < 0) {  // never index the caches with a bad state
        if (threadIdx.x == 0) __hip_atomic_store(pa->abort_flag, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const unsigned base = (unsigned)step * (unsigned)(NPH * n_layers);
    for (int l = 0; l < n_layers; ++l) {
        const unsigned s0 = base + (unsigned)(NPH * l);  // flags after phase k: s0 + k + 1
#define SPT_PHASE(K)                                                        \
        if (!run_phase<K>(pa, l, s0 + K, pos, sm, img)) return;             \
        publish(*pa, s0 + K + 1);
        SPT_PHASE(0) SPT_PHASE(1) SPT_PHASE(2) SPT_PHASE(3)
        SPT_PHASE(4) SPT_PHASE(5) SPT_PHASE(6) SPT_PHASE(7)
#undef SPT_PHASE
    }
}

__global__ void persist_reset_kernel(unsigned* flags, int n_flags, unsigned* cnt, int n_cnt, unsigned* abort_flag) {
    for (int i = threadIdx.x; i < n_flags; i += blockDim.x) flags[i] = 0u;
    for (int i = threadIdx.x; i < n_cnt; i += blockDim.x) cnt[i] = 0u;
    if (threadIdx.x < 4) abort_flag[threadIdx.x] = 0u;  // abort word + debug site / address
}

}  // namespace

int persist_lds_bytes(int R, int d) {
    // the LN image plus padding that keeps a second workgroup off the CU (one per CU)
    const int need = kSmemBytes + R * (4 * d + 8) * 2;  // largest staged block: fc2 input
    return need < 96 * 1024 ? 96 * 1024 : need;
}

const char* persist_check(const PersistArgs& a, int G) {
    if (a.B < 1 || a.B > 16) return "persistent decoder: 1..16 sequences";
    if (a.d % 64 || a.d > 1536) return "persistent decoder: d must be a multiple of 64, <= 1536";
    if (a.d != a.H * 64) return "persistent decoder: head size must be 64";
    if (a.S_cross < 1 || a.S_cross > 64) return "persistent decoder: bad cross split";
    if (G > 256) return "persistent decoder: at most 256 workgroups";
    if (persist_lds_bytes(a.B, a.d) > 160 * 1024) return "persistent decoder: activations exceed LDS";
    // K steps per wave must fit the register slice
    const int Ns[4] = {3 * a.d, a.d, 4 * a.d, a.d};
    const int Ks[4] = {a.d, a.d, a.d, 4 * a.d};
    const int Js[4] = {5, 5, 10, MAXKS};  // JMAX of the gemv_phase instances below
    for (int i = 0; i < 4; ++i) {
        const int nt = Ns[i] / 16, ntl = (nt + G - 1) / G, nwt = PW / ntl;
        if (nwt < 1 || (Ks[i] / 32 + nwt - 1) / nwt > Js[i]) return "persistent decoder: K slice exceeds registers";
    }
    if (a.S_self < 1 || a.S_self > 64) return "persistent decoder: bad self split";
    return nullptr;
}

void persist_prepare() {
    HIP_CHECK(hipFuncSetAttribute((const void*)persist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
}

void dec_persist(const PersistArgs& a, const PersistArgs* a_dev, int G, hipStream_t st) {
    hipLaunchKernelGGL(persist_kernel, dim3(G), dim3(PT), persist_lds_bytes(a.B, a.d), st, a_dev);
    SPT_LAUNCH_CHECK();
}

void persist_reset(const PersistArgs& a, int G, hipStream_t st) {
    hipLaunchKernelGGL(persist_reset_kernel, dim3(1), dim3(256), 0, st, a.flags, G, a.xcnt, 2 * a.B * a.H, a.abort_flag);
    SPT_LAUNCH_CHECK();
}

}  // namespace spt
