// k_gemm.hip -- encoder-side GEMMs C = A . W^T on CDNA4 matrix cores.
//
// Replaces the ggml mul_mat / conv_1d_ph (im2col + mul_mat) ops that
// whisper.cpp's whisper_build_graph_conv / _encoder / _cross run for
// WhisperEngine::transcribe_samples (/root/reference/src-tauri/src/managers/transcription.rs:501-503).
//
// Tile: 128 x 128 per 256-thread workgroup (4 waves in 2 x 2, 64 x 64 each),
// one 128-byte K slab per stage (64 bf16 or 32 f32), operands staged
// global -> LDS by global_load_lds_dwordx4 (one wave-instruction = 8 rows x 128 B),
// XOR-swizzled on the source address (chunk ^ swz(row)) so the ds_read_b128
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

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <set>
#include <tuple>
#include <type_traits>
#include <vector>

namespace spt {

namespace {

constexpr int BM = 128, BN = 128, SLAB = 128;  // SLAB = bytes of K per row per stage

// LDS swizzle of 128-byte rows: a 256-byte bank row holds rows 2q and 2q+1, so 16 consecutive
// rows (one ds_read_b128 lane group) hit 16 distinct 16-byte slots with chunk' = chunk ^ ((row >> 1) & 7)
// (chunk ^ (row & 7) leaves rows r and r+8 on the same slot: 2-way conflicts)
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* g, SPT_LDS void* l) {
    __builtin_amdgcn_global_load_lds((const void*)g, l, 16, 0, 0);
}

// fused epilogue of one output element (row, column): bias, GELU, positional add, residual
// add or the head-split store of the cross-attention K/V cache
struct EpiCol { int col; float bv; int l, kvi, h, el; };
template <int EPI>
__device__ __forceinline__ EpiCol epi_col(const GemmArgs& g, int col) {
    EpiCol e{col, g.bias ? g.bias[col] : 0.0f, 0, 0, 0, 0};
    if constexpr (EPI == EPI_KVSPLIT) {
        const int d = g.kv_H * 64;
        e.l = col / (2 * d);
        const int rem = col - e.l * 2 * d;
        e.kvi = rem / d;
        e.h = (rem - e.kvi * d) >> 6;
        e.el = rem & 63;
    }
    return e;
}
// the residual / positional operand of one output element (the f32 epilogues that read one)
template <int EPI>
constexpr bool epi_reads_y() { return EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU_POS; }
template <int EPI>
__device__ __forceinline__ float epi_y(const GemmArgs& g, int bz, int row, const EpiCol& e) {
    if constexpr (EPI == EPI_BIAS_RESID) return ((const float*)g.C + (size_t)bz * g.sC)[(size_t)row * g.ldc + e.col];
    else if constexpr (EPI == EPI_BIAS_GELU_POS) return g.pos[(size_t)row * g.N + e.col];
    else return 0.0f;
}
// Every epilogue load (bias columns, residual / positional operands) is issued before the first
// store and waited for here, once.  Left to the compiler, each row-guarded store waited with
// vmcnt(0) -- for its bias value along the paths that skipped the earlier guarded blocks, and so
// for every earlier store too (vmcnt counts stores in order): the stores of a tile went one
// round trip at a time.
__device__ __forceinline__ void epi_loads_landed() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)

// No contraction here: the residual / positional add is a separate rounding after the scaled
// (or GELU'd) product, as in the 256 x 256 tile's LDS-staged epilogue, so every tile writes the same
// bits (a fused alpha * v + C differed in the last bit: r3, single-window Whisper encoder).
// y: epi_y of the element (loaded before any store)
template <typename T, int EPI>
__device__ __forceinline__ void epi_store(const GemmArgs& g, int bz, int row, const EpiCol& e, float acc, float y = 0.0f) {
#pragma clang fp contract(off)
    const float v = acc + e.bv;
    if constexpr (EPI == EPI_BIAS) {
        ((T*)g.C + (size_t)bz * g.sC)[(size_t)row * g.ldc + e.col] = from_f<T>(v);
    } else if constexpr (EPI == EPI_BIAS_SWISH) {
        ((T*)g.C + (size_t)bz * g.sC)[(size_t)row * g.ldc + e.col] = from_f<T>(swish(v));
    } else if constexpr (EPI == EPI_BIAS_RELU) {
        ((T*)g.C + (size_t)bz * g.sC)[(size_t)row * g.ldc + e.col] = from_f<T>(fmaxf(v, 0.0f));
    } else if constexpr (EPI == EPI_BIAS_F32) {
        ((float*)g.C + (size_t)bz * g.sC)[(size_t)row * g.ldc + e.col] = g.alpha * v;
    } else if constexpr (EPI == EPI_PARTIAL) {
        ((float*)g.C + (size_t)blockIdx.y * g.c_split)[(size_t)row * g.ldc + e.col] = v;
    } else if constexpr (EPI == EPI_BIAS_GELU) {
        ((T*)g.C + (size_t)bz * g.sC)[(size_t)row * g.ldc + e.col] = from_f<T>(gelu_tanh(v));
    } else if constexpr (EPI == EPI_BIAS_GELU_POS) {
        ((float*)g.C + (size_t)bz * g.sC)[(size_t)row * g.ldc + e.col] = gelu_tanh(v) + y;
    } else if constexpr (EPI == EPI_BIAS_RESID) {
        ((float*)g.C + (size_t)bz * g.sC)[(size_t)row * g.ldc + e.col] = y + g.alpha * v;
    } else if constexpr (EPI == EPI_KVSPLIT) {
        const int bb = row / g.kv_T, t = row - bb * g.kv_T;
        ((T*)g.C)[kv_offset(e.l, e.kvi, bb, e.h, t, e.el, g.kv_B, g.kv_H, g.kv_T)] = from_f<T>(v);
    }
}

// ST-slot LDS ring (ST x 32 KiB, dynamic for ST > 2): ST - 1 K-slabs in flight while one is
// computed.  The 16-slab GEMMs of a Parakeet streaming pass (M = 832, K = 1024) and Whisper's
// smaller shapes give about one workgroup per CU and no other wave to cover a slab's load
// latency; with two slots every k-step waited for its own DMA round trip.
// BMT = 64 halves the tile's rows (each wave 32 x 64 of C), BNT = 64 its columns: at M = 832 a
// 128 x 128 tile gives at most one workgroup per CU, so one wave per SIMD with every LDS read and
// DMA wait of a k-step exposed.  Every C element is the same MFMA chain in every tile shape.
template <typename T, int EPI, int ST, int BMT = BM, int BNT = BN>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmArgs g) {  // (256, 1) put the accumulators in AGPRs + ~90 copies per k-step
    static_assert((BMT == 64 || BMT == 128) && (BNT == 64 || BNT == 128), "tile shape");
    static_assert(ST == 2 || (BMT == 128 && BNT == 128), "deeper rings: 128 x 128 only");
    constexpr int MI = BMT / 32;      // 16-row A fragments per wave
    constexpr int NJ = BNT / 32;      // 16-column W fragments per wave
    constexpr int PA = BMT / 32;      // A pieces (8 rows x 128 B) a wave stages per slab
    constexpr int PW = BNT / 32;      // W pieces
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [slot][A BMT rows | W BNT rows][128 B]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int nnt = g.N / BNT;
    // bijective XCD-aware remap of the linear tile id
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int nmt = (g.M + BMT - 1) / BMT;
    const int tm = g.nmajor ? wg % nmt : wg / nnt, tn = g.nmajor ? wg / nmt : wg % nnt;
    const int m0 = tm * BMT, n0 = tn * BNT;
    const int bz = blockIdx.z;
    const int Kc = g.K / g.ksplit;  // this workgroup's K range: [blockIdx.y * Kc, + Kc)
    const T* A = (const T*)g.A + (size_t)bz * g.sA + (size_t)blockIdx.y * Kc;
    const T* W = (const T*)g.W + (size_t)blockIdx.y * Kc;

    // per-lane source pointers for the PA A pieces and PW W pieces this wave stages
    const char* srcA[PA];
    const char* srcW[PW];
    const int prow = lane >> 3, pch = lane & 7;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int rt = (wid * PW + i) * 8 + prow;
        const int c = pch ^ swz(rt);
        srcW[i] = (const char*)(W + (size_t)(n0 + rt) * g.ldw) + c * 16;
    }
#pragma unroll
    for (int i = 0; i < PA; ++i) {
        const int rt = (wid * PA + i) * 8 + prow;
        const int ra = min(m0 + rt, g.M - 1);
        srcA[i] = (const char*)(A + (size_t)ra * g.lda) + (pch ^ swz(rt)) * 16;
    }
    auto lds_a = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + buf * (BMT + BNT) * SLAB; };
    auto lds_w = [&](int buf) -> SPT_LDS char* { return (SPT_LDS char*)smem + buf * (BMT + BNT) * SLAB + BMT * SLAB; };
    auto stage = [&](int buf, int kt) {
        const size_t koff = (size_t)kt * SLAB;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i < PA) glds16(srcA[i] + koff, lds_a(buf) + (wid * PA + i) * 1024);
            if (i < PW) glds16(srcW[i] + koff, lds_w(buf) + (wid * PW + i) * 1024);
        }
    };

    f32x4 acc[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nkt = Kc * (int)sizeof(T) / SLAB;
    const int fr = lane & 15, fq = lane >> 4;


    // prologue: slabs 0 .. ST - 2.  Every iteration issues exactly one slab (past the end: the last
    // slab again, into a free slot), so each wave's vmcnt counts the same instructions everywhere.
#pragma unroll
    for (int p = 0; p < ST - 1; ++p) stage(p, min(p, nkt - 1));
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt % ST;
        // slab kt landed (8 DMA instructions per slab and wave; ST - 2 younger slabs may fly on),
        // and every wave is done with slab kt - 1, whose slot the next issue overwrites
        if constexpr (ST == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if constexpr (ST == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        // a bare s_barrier: __syncthreads()'s release fence would make the compiler drain every
        // in-flight slab (vmcnt(0)) in front of it
        asm volatile("s_barrier" ::: "memory");
        stage((kt + ST - 1) % ST, min(kt + ST - 1, nkt - 1));
        const SPT_LDS char* la = lds_a(cur);
        const SPT_LDS char* lw = lds_w(cur);
        if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 af[MI], wf[NJ];
                const int c = 4 * s + fq;
#pragma unroll
                for (int i = 0; i < NJ; ++i) {
                    const int rw = wn * (BNT / 2) + 16 * i + fr;
                    wf[i] = *(const SPT_LDS bf16x8*)(lw + rw * SLAB + ((c ^ swz(rw)) << 4));
                }
#pragma unroll
                for (int i = 0; i < MI; ++i) {
                    const int ra = wm * (BMT / 2) + 16 * i + fr;
                    af[i] = *(const SPT_LDS bf16x8*)(la + ra * SLAB + ((c ^ swz(ra)) << 4));
                }
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        if constexpr (TypeTag<T>::id == 2)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[i]),
                                                                               __builtin_bit_cast(f16x8, wf[j]), acc[i][j], 0, 0, 0);
                        else
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], wf[j], acc[i][j], 0, 0, 0);
                    }
            }
        } else {
            f32x4 af[MI][2], wf[NJ][2];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int rw = wn * (BNT / 2) + 16 * i + fr;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int c = 2 * fq + h;
                    if (i < NJ) wf[i][h] = *(const SPT_LDS f32x4*)(lw + rw * SLAB + ((c ^ swz(rw)) << 4));
                    if (i < MI) {
                        const int ra = wm * (BMT / 2) + 16 * i + fr;
                        af[i][h] = *(const SPT_LDS f32x4*)(la + ra * SLAB + ((c ^ swz(ra)) << 4));
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s >> 2][s & 3], wf[j][s >> 2][s & 3],
                                                                          acc[i][j], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing repeat slabs land before exit

    // ---------------------------------------------------------------- epilogue
    EpiCol ec[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) ec[j] = epi_col<EPI>(g, n0 + wn * (BNT / 2) + 16 * j + fr);
    float y[epi_reads_y<EPI>() ? MI : 1][NJ][4];
    if constexpr (epi_reads_y<EPI>()) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    y[i][j][r] = epi_y<EPI>(g, bz, min(m0 + wm * (BMT / 2) + 16 * i + 4 * fq + r, g.M - 1), ec[j]);
    }
    epi_loads_landed();
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * (BMT / 2) + 16 * i + 4 * fq + r;
                if (row < g.M) epi_store<T, EPI>(g, bz, row, ec[j], acc[i][j][r], y[epi_reads_y<EPI>() ? i : 0][j][r]);
            }
}

// ---------------------------------------------------------------------------------------------
// 256 x 256 tile, 512 threads = 8 waves as 2 (M) x 4 (N), each wave a 128 x 64 C tile (8 x 4
// fragments of v_mfma_f32_16x16x32_bf16), BK = 64 (128 B per row), 2 LDS buffers of 64 KiB
// (A 256 rows + W 256 rows, 128 B each, 16-byte chunk c of row r stored at slot c ^ swz(r)).
// Each buffer is staged as four half-tiles by global_load_lds_dwordx4 (2 instructions per wave
// per half-tile):
//   A0 = C rows {0..63, 128..191}   A1 = {64..127, 192..255}   (the two 64-row halves of
//   W0 = C cols {0..31, 64..95, ..} W1 = {32..63, 96..127, ..}  every wave's 128 x 64 tile)
// A K-tile is computed in four phases, one C quadrant (4 x 2 fragments x K 64 = 16 MFMAs) each:
//   P1 reads A0 + W0 -> quadrant (0,0), stages A1 of K-tile kt+1 (other buffer)
//   P2 reads W1      -> quadrant (0,1), stages A0 of kt+2 (this buffer: A0 was read in P1)
//   P3 reads A1      -> quadrant (1,1), stages W0 of kt+2
//   P4 (registers)   -> quadrant (1,0), stages W1 of kt+2
// so every half-tile is restaged one phase after its last read (behind that phase's barrier)
// and read at least four phases after it was issued.  With 2 instructions per half-tile, the
// half-tile a phase reads next always has exactly 5 half-tiles issued after it: each waiting
// phase ends with a counted s_waitcnt vmcnt(10) (never 0 in the loop) before its barrier.
// Past the last K-tile the staging repeats the last K-tile into free halves (keeps the counts
// uniform); the loop drains vmcnt(0) before the epilogue.  (A persistent variant whose staging
// runs into the next tile measured no faster: the epilogue's stores, not the prologue, were the
// per-tile cost, so the epilogue is staged through LDS into 16-byte row stores instead.)
constexpr int G2_BM = 256, G2_BN = 256, G2_ROW = 128;  // G2_ROW: bytes of K per row per K-tile
constexpr int G2_BUF = 2 * 256 * G2_ROW;               // one buffer: A + W
constexpr int G2_LDS = 2 * G2_BUF;                     // 128 KiB
constexpr int G2_LDS_ALL = 8 * 128 * (128 + 16) > G2_LDS ? 8 * 128 * (128 + 16) : G2_LDS;  // + epilogue staging

// STG: the wave groups wr = 0 (waves 0-3) and wr = 1 (waves 4-7; each SIMD holds one wave of each)
// run one phase apart -- group 1 passes one extra barrier first, group 0 one extra at the end --
// so on every SIMD one wave's MFMAs overlap the other's LDS reads and DMA issue.  With the lag a
// half-tile must be restaged >= 2 phases after its last read (A0 moves from P2 to P3) and every
// wave must have waited for a half-tile by the end of the phase two before its read, so the
// waits become vmcnt(8) at the ends of P1 / P3 / P4 (4 half-tiles in flight; see the schedule
// below).  The MFMA order per accumulator is unchanged: results are bitwise those of STG = false.
// PP (with STG): every phase gets a second barrier between its fragment reads / DMA issue and its
// MFMAs, so the two groups' half-phase lag alternates them: on each SIMD one wave reads while the
// other multiplies.  The restaging and wait rules above hold unchanged (a read completes before its
// phase's MFMAs; a half-tile is restaged >= 2 phases after its last read and read >= 2 phases after
// every wave's wait for it), and the MFMA order per accumulator is the same: bitwise equal results.
template <int EPI, bool F16, bool STG = false, bool PP = false>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;
    const int fr = lane & 15, fq = lane >> 4;
    const int nnt = g.N / G2_BN;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tm = wg / nnt, tn = wg - tm * nnt;
    const int m0 = tm * G2_BM, n0 = tn * G2_BN;
    const int bz = blockIdx.z;
    const int Kc = g.K / g.ksplit;
    const bf16* A = (const bf16*)g.A + (size_t)bz * g.sA + (size_t)blockIdx.y * Kc;
    const bf16* W = (const bf16*)g.W + (size_t)blockIdx.y * Kc;
    const int nkt = Kc / 64;

    // staging sources: half-tile h of A (or W), instruction i (0, 1) of this wave -> 8 rows
    const int prow = lane >> 3, pch = lane & 7;
    const char* srcA[2][2];
    const char* srcW[2][2];
    int dstA[2][2], dstW[2][2];  // LDS byte offsets (wave-uniform row base) inside a buffer
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int gi = wid * 2 + i;                                   // row group 0..15 of the half
            const int ra = (gi >> 3) * 128 + h * 64 + (gi & 7) * 8;       // A: 2 blocks of 64 rows
            const int rw = (gi >> 2) * 64 + h * 32 + (gi & 3) * 8;        // W: 4 blocks of 32 rows
            const int rA = ra + prow, rW = rw + prow;
            srcA[h][i] = (const char*)(A + (size_t)min(m0 + rA, g.M - 1) * g.lda) + ((pch ^ swz(rA)) << 4);
            srcW[h][i] = (const char*)(W + (size_t)(n0 + rW) * g.ldw) + ((pch ^ swz(rW)) << 4);
            dstA[h][i] = ra * G2_ROW;
            dstW[h][i] = 256 * G2_ROW + rw * G2_ROW;
        }
    auto stageA = [&](int buf, int kt, int h) {
        const size_t ko = (size_t)min(kt, nkt - 1) * G2_ROW;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(srcA[h][i] + ko),
                                             (SPT_LDS void*)(smem + buf * G2_BUF + dstA[h][i]), 16, 0, 0);
    };
    auto stageW = [&](int buf, int kt, int h) {
        const size_t ko = (size_t)min(kt, nkt - 1) * G2_ROW;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(srcW[h][i] + ko),
                                             (SPT_LDS void*)(smem + buf * G2_BUF + dstW[h][i]), 16, 0, 0);
    };
    // fragment reads: A rows of quadrant half rh, W rows (C columns) of half ch, k-steps 0/1
    bf16x8 af[4][2], bw[2][2][2];
    // k-step-major read order (s = 0 pieces first): the quadrant's first 8 MFMAs (k-step 0) can
    // start once half of a phase's reads have landed (a counted lgkmcnt instead of 0)
    auto readA = [&](int buf, int rh) {
        const SPT_LDS char* la = (const SPT_LDS char*)smem + buf * G2_BUF;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wr * 128 + rh * 64 + 16 * i + fr;
                const int c = 4 * s + fq;
                af[i][s] = *(const SPT_LDS bf16x8*)(la + r * G2_ROW + ((c ^ swz(r)) << 4));
            }
    };
    auto readW = [&](int buf, int ch) {
        const SPT_LDS char* lw = (const SPT_LDS char*)smem + buf * G2_BUF + 256 * G2_ROW;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = wc * 64 + ch * 32 + 16 * j + fr;
                const int c = 4 * s + fq;
                bw[ch][j][s] = *(const SPT_LDS bf16x8*)(lw + r * G2_ROW + ((c ^ swz(r)) << 4));
            }
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto quad = [&](int rh, int ch) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    if constexpr (F16)
                        acc[rh * 4 + i][ch * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                            __builtin_bit_cast(f16x8, af[i][s]), __builtin_bit_cast(f16x8, bw[ch][j][s]),
                            acc[rh * 4 + i][ch * 2 + j], 0, 0, 0);
                    else
                        acc[rh * 4 + i][ch * 2 + j] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bw[ch][j][s], acc[rh * 4 + i][ch * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
#define G2_BARRIER() asm volatile("s_barrier" ::: "memory")
#define G2_VMWAIT() asm volatile("s_waitcnt vmcnt(10)" ::: "memory")

    // prologue: K-tile 0 whole, K-tile 1 but its A1 (issued by K-tile 0's P1)
    stageA(0, 0, 0); stageW(0, 0, 0); stageW(0, 0, 1); stageA(0, 0, 1);
    stageA(1, 1, 0); stageW(1, 1, 0); stageW(1, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    G2_BARRIER();
    if constexpr (STG) {
        if (wr == 1) G2_BARRIER();  // group 1 starts one phase behind
        for (int kt = 0; kt < nkt; ++kt) {
            const int c = kt & 1;
            // P1: A0 W0 -> (0,0); stage A1 of kt+1.  Wait: A1(kt) (read in P3).  Each phase issues
            // its DMA before its fragment reads, so the reads are the youngest LDS-counter ops and
            // the MFMAs wait for them with counted lgkmcnt, not 0
            stageA(c ^ 1, kt + 1, 1);
            readA(c, 0);
            readW(c, 0);
            if constexpr (PP) G2_BARRIER();
            quad(0, 0);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            G2_BARRIER();
            // P2: W1 -> (0,1)
            readW(c, 1);
            if constexpr (PP) G2_BARRIER();
            quad(0, 1);
            G2_BARRIER();
            // P3: A1 -> (1,1); stage A0, W0 of kt+2.  Wait: A0(kt+1), W0(kt+1) (read in P1')
            stageA(c, kt + 2, 0);
            stageW(c, kt + 2, 0);
            readA(c, 1);
            if constexpr (PP) G2_BARRIER();
            quad(1, 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            G2_BARRIER();
            // P4: (1,0) from registers; stage W1 of kt+2.  Wait: W1(kt+1) (read in P2')
            stageW(c, kt + 2, 1);
            if constexpr (PP) G2_BARRIER();
            quad(1, 0);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            G2_BARRIER();
        }
        if (wr == 0) G2_BARRIER();  // realign: both groups have passed the same barriers
    } else
    for (int kt = 0; kt < nkt; ++kt) {
        const int c = kt & 1;
        // P1
        stageA(c ^ 1, kt + 1, 1);
        readA(c, 0);
        readW(c, 0);
        quad(0, 0);
        G2_VMWAIT();
        G2_BARRIER();
        // P2
        stageA(c, kt + 2, 0);
        readW(c, 1);
        quad(0, 1);
        G2_VMWAIT();
        G2_BARRIER();
        // P3
        stageW(c, kt + 2, 0);
        readA(c, 1);
        quad(1, 1);
        G2_BARRIER();
        // P4
        stageW(c, kt + 2, 1);
        quad(1, 0);
        G2_VMWAIT();
        G2_BARRIER();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    G2_BARRIER();  // every wave's last fragment reads are done: the LDS is free for the epilogue
#undef G2_BARRIER
#undef G2_VMWAIT

    // ---------------------------------------------------------------- epilogue
    // Per wave: the 128 x 64 C tile (after bias / GELU) goes to a private LDS region in MFMA
    // layout (a lane holds 4 rows of one column), then is read back as 16-byte row chunks
    // and written with one 16-byte global store per lane per row group (a lane's own values
    // would be 2- or 4-byte stores at a row stride).  bf16 outputs: one pass of 128 rows,
    // row stride 144 B; f32 outputs: two passes of 64 rows, row stride 272 B (the 16-byte pad
    // spreads the four row groups a store instruction writes over distinct banks).
    constexpr bool F32OUT = EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU_POS || EPI == EPI_BIAS_F32 || EPI == EPI_PARTIAL;
    constexpr int ESZ = F32OUT ? 4 : 2;
    constexpr int RS = 64 * ESZ + 16;          // LDS row stride (bytes)
    constexpr int PR = F32OUT ? 64 : 128;      // rows per pass
    constexpr int CPR = 64 * ESZ / 16;         // 16-byte chunks per row (8 or 16)
    constexpr int RPI = 64 / CPR;              // rows per wave-instruction (8 or 4)
    char* wreg = smem + wid * (PR * RS);
    float bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[j] = g.bias ? g.bias[n0 + wc * 64 + 16 * j + fr] : 0.0f;
#pragma unroll
    for (int pass = 0; pass < 128 / PR; ++pass) {
        const int ch = lane % CPR, rsub = lane / CPR;
        // the residual / positional operand of the f32 epilogues, loaded for the whole pass before
        // the LDS staging and any store.  Read inside the store loop, each load waited behind the
        // previous iteration's store to a possibly aliasing address: one dependent round trip per
        // row group (r3 ubench: the residual epilogue cost 16 us per 256 x 256 tile)
        constexpr bool YIN = EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU_POS;
        float4 ypre[YIN ? PR / RPI : 1];
        if constexpr (YIN) {
#pragma unroll
            for (int it = 0; it < PR / RPI; ++it) {
                const int row = min(m0 + wr * 128 + pass * PR + it * RPI + rsub, g.M - 1);
                const int col = n0 + wc * 64 + ch * (16 / ESZ);
                if constexpr (EPI == EPI_BIAS_RESID)
                    ypre[it] = *(const float4*)((const float*)g.C + (size_t)bz * g.sC + (size_t)row * g.ldc + col);
                else
                    ypre[it] = *(const float4*)(g.pos + (size_t)row * g.N + col);
            }
        }
#pragma unroll
        for (int ii = 0; ii < PR / 16; ++ii) {
            const int i = pass * (PR / 16) + ii;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int rl = 16 * ii + 4 * fq + r, cl = 16 * j + fr;
                    float v = acc[i][j][r] + bv[j];
                    if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_POS) v = gelu_tanh(v);
                    if constexpr (EPI == EPI_BIAS_SWISH) v = swish(v);
                    if constexpr (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.0f);
                    if constexpr (EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_F32) v *= g.alpha;
                    if constexpr (F32OUT) *(float*)(wreg + rl * RS + cl * 4) = v;
                    else if constexpr (F16) *(f16*)(wreg + rl * RS + cl * 2) = (f16)v;
                    else *(bf16*)(wreg + rl * RS + cl * 2) = f2bf(v);
                }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < PR / RPI; ++it) {
            const int rl = it * RPI + rsub;
            const int row = m0 + wr * 128 + pass * PR + rl;
            const uint4 v = *(const uint4*)(wreg + rl * RS + ch * 16);
            if (row >= g.M) continue;
            const int col = n0 + wc * 64 + ch * (16 / ESZ);
            if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_SWISH || EPI == EPI_BIAS_RELU) {
                *(uint4*)((bf16*)g.C + (size_t)bz * g.sC + (size_t)row * g.ldc + col) = v;
            } else if constexpr (EPI == EPI_KVSPLIT) {
                const int d = g.kv_H * 64;
                const int l = col / (2 * d), rem = col - l * 2 * d;
                const int kvi = rem / d, hh = (rem - kvi * d) >> 6, el = rem & 63;
                const int bb = row / g.kv_T, t = row - bb * g.kv_T;
                *(uint4*)((bf16*)g.C + kv_offset(l, kvi, bb, hh, t, el, g.kv_B, g.kv_H, g.kv_T)) = v;
            } else if constexpr (EPI == EPI_PARTIAL) {
                *(uint4*)((float*)g.C + (size_t)blockIdx.y * g.c_split + (size_t)row * g.ldc + col) = v;
            } else {
                float* cp = (float*)g.C + (size_t)bz * g.sC + (size_t)row * g.ldc + col;
                float4 o = *(const float4*)&v;
                float4 y;
                if constexpr (YIN) y = ypre[it];
                else y = make_float4(0.f, 0.f, 0.f, 0.f);
                o.x += y.x; o.y += y.y; o.z += y.z; o.w += y.w;
                *(float4*)cp = o;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------------------------
// Skinny GEMM (M <= 64 rows: a short streaming window, one utterance): the weight stream is the
// whole cost, so the grid spreads W over >= 256 workgroups -- a workgroup owns 16 columns and a
// K range (split-K over grid.y for the EPI_PARTIAL residual products), its 4 waves split that
// range again.  Operands go straight from global memory into MFMA fragments
// (v_mfma_f32_16x16x32_{bf16,f16}: a lane loads 16 B of one W row and 16 B of each 16-row A
// block per k-step), four k-steps in flight; the waves' partial tiles are summed through LDS and
// the epilogue is the shared epi_store.
template <int EPI, bool F16, int MT>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(GemmArgs g) {
    __shared__ float red[4][MT * 16][17];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int n0 = blockIdx.x * 16;
    const int Kc = g.K / g.ksplit, Kw = Kc / 4;
    const int k0 = blockIdx.y * Kc + wid * Kw;
    const bf16* wp = (const bf16*)g.W + (size_t)(n0 + fr) * g.ldw + k0 + 8 * fq;
    const bf16* ap[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) ap[mt] = (const bf16*)g.A + (size_t)min(mt * 16 + fr, g.M - 1) * g.lda + k0 + 8 * fq;
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int U = 4;
    for (int k = 0; k < Kw; k += 32 * U) {
        bf16x8 wf[U], af[U][MT];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int kk = min(k + 32 * u, Kw - 32);  // past the range: re-read, not accumulated below
            wf[u] = *(const bf16x8*)(wp + kk);
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) af[u][mt] = *(const bf16x8*)(ap[mt] + kk);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (k + 32 * u >= Kw) break;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                if constexpr (F16)
                    acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[u][mt]),
                                                                      __builtin_bit_cast(f16x8, wf[u]), acc[mt], 0, 0, 0);
                else
                    acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u][mt], wf[u], acc[mt], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wid][mt * 16 + 4 * fq + r][fr] = acc[mt][r];
    __syncthreads();
    typedef typename std::conditional<F16, f16, bf16>::type T;
    // element e = threadIdx.x + 256 u: row (threadIdx.x >> 4) + 16 u, column threadIdx.x & 15
    const int c = threadIdx.x & 15;
    const EpiCol ec = epi_col<EPI>(g, n0 + c);
    float y[MT];
#pragma unroll
    for (int u = 0; u < MT; ++u)
        y[u] = epi_reads_y<EPI>() ? epi_y<EPI>(g, 0, min((int)(threadIdx.x >> 4) + 16 * u, g.M - 1), ec) : 0.0f;
    epi_loads_landed();
#pragma unroll
    for (int u = 0; u < MT; ++u) {
        const int row = (threadIdx.x >> 4) + 16 * u;
        if (row >= g.M) continue;
        const float v = red[0][row][c] + red[1][row][c] + red[2][row][c] + red[3][row][c];
        epi_store<T, EPI>(g, 0, row, ec, v, y[u]);
    }
}

template <int EPI, bool F16>
void launch_skinny(const GemmArgs& g, hipStream_t st) {
    dim3 grid(g.N / 16, g.ksplit);
    switch (cdiv(g.M, 16)) {
        case 1: hipLaunchKernelGGL((gemm_skinny_kernel<EPI, F16, 1>), grid, dim3(256), 0, st, g); break;
        case 2: hipLaunchKernelGGL((gemm_skinny_kernel<EPI, F16, 2>), grid, dim3(256), 0, st, g); break;
        case 3: hipLaunchKernelGGL((gemm_skinny_kernel<EPI, F16, 3>), grid, dim3(256), 0, st, g); break;
        case 4: hipLaunchKernelGGL((gemm_skinny_kernel<EPI, F16, 4>), grid, dim3(256), 0, st, g); break;
        default: throw std::runtime_error("gemm_skinny: M > 64");
    }
    SPT_LAUNCH_CHECK();
}

template <int EPI, bool F16>
void launch_256(const GemmArgs& g, int batch, hipStream_t st) {
    // staggered wave groups: bitwise-identical results, encoder 21.54 -> 21.28 ms (r2, two A/B pairs);
    // SPT_G2_STAGGER=0 restores the lock-step schedule
    // (both switches read per launch: eager runs such as debug_encode pick them up; a captured encoder
    // keeps what it was captured with)
    const char* stg_env = getenv("SPT_G2_STAGGER");
    const bool stg = !stg_env || atoi(stg_env) != 0;
    // > 64 KiB dynamic LDS: per kernel and device (gemm_prepare sets them before any capture)
    ensure_lds_attr((const void*)gemm256_kernel<EPI, F16, false>, G2_LDS_ALL);
    ensure_lds_attr((const void*)gemm256_kernel<EPI, F16, true>, G2_LDS_ALL);
    ensure_lds_attr((const void*)gemm256_kernel<EPI, F16, true, true>, G2_LDS_ALL);
    // ping-pong phases (a barrier between each phase's reads and its MFMAs; r5: q/k/v 125.4 -> 119.4 us,
    // 4096^3 1182 -> 1246 TF/s standalone, encoder 20.4 -> 20.2 ms, bitwise equal); SPT_G2_PP=0: off
    const char* pp_env = getenv("SPT_G2_PP");
    const bool pp = !pp_env || atoi(pp_env) != 0;
    dim3 grid(cdiv(g.M, G2_BM) * (g.N / G2_BN), g.ksplit, batch);
    if (stg && pp) hipLaunchKernelGGL((gemm256_kernel<EPI, F16, true, true>), grid, dim3(512), G2_LDS_ALL, st, g);
    else if (stg) hipLaunchKernelGGL((gemm256_kernel<EPI, F16, true>), grid, dim3(512), G2_LDS_ALL, st, g);
    else hipLaunchKernelGGL((gemm256_kernel<EPI, F16, false>), grid, dim3(512), G2_LDS_ALL, st, g);
    SPT_LAUNCH_CHECK();
}

constexpr int kNtStages = 4;  // deepest LDS ring of the 128 x 128 kernel (4 x 32 KiB; default depth: nt_stages)
// default 2 slots: at the Parakeet streaming shapes (M = 832) the 3- and 4-slot rings measured no
// faster (r3 exp_r3e / exp_r3g: the k-step is not DMA-latency bound); SPT_GEMM_NT_STAGES = 3 / 4
int nt_stages() {
    static const int s = getenv("SPT_GEMM_NT_STAGES") ? atoi(getenv("SPT_GEMM_NT_STAGES")) : 2;
    return s == 3 || s == 4 ? s : 2;
}

template <typename T, int EPI, int ST>
void launch_t_st(const GemmArgs& g0, int batch, hipStream_t st) {
    static const int nmajor = getenv("SPT_GEMM_NT_RASTER") ? atoi(getenv("SPT_GEMM_NT_RASTER")) : 0;
    GemmArgs g = g0;
    g.nmajor = nmajor;
    constexpr int lds = ST * 2 * BM * SLAB;
    if (lds > 64 * 1024) ensure_lds_attr((const void*)gemm_nt_kernel<T, EPI, ST>, lds);
    dim3 grid(cdiv(g.M, BM) * (g.N / BN), g.ksplit, batch);
    hipLaunchKernelGGL((gemm_nt_kernel<T, EPI, ST>), grid, dim3(256), lds, st, g);
}

template <typename T, int EPI, int BMT, int BNT>
void launch_small(const GemmArgs& g0, int batch, hipStream_t st) {  // 64 x 128 / 64 x 64 tile, 2-slot ring
    static const int nmajor = getenv("SPT_GEMM_NT_RASTER") ? atoi(getenv("SPT_GEMM_NT_RASTER")) : 0;
    GemmArgs g = g0;
    g.nmajor = nmajor;
    dim3 grid(cdiv(g.M, BMT) * (g.N / BNT), g.ksplit, batch);
    hipLaunchKernelGGL((gemm_nt_kernel<T, EPI, 2, BMT, BNT>), grid, dim3(256), 2 * (BMT + BNT) * SLAB, st, g);
}

template <typename T, int EPI>
void launch_t(const GemmArgs& g, int batch, int variant, hipStream_t st) {
    if (variant == 4) return launch_small<T, EPI, 64, 128>(g, batch, st);
    if (variant == 5) return launch_small<T, EPI, 64, 64>(g, batch, st);
    switch (nt_stages()) {
        case 2: launch_t_st<T, EPI, 2>(g, batch, st); break;
        case 3: launch_t_st<T, EPI, 3>(g, batch, st); break;
        default: launch_t_st<T, EPI, kNtStages>(g, batch, st); break;
    }
}

template <int EPI>
void prepare_epi() {
    ensure_lds_attr((const void*)gemm256_kernel<EPI, false, false>, G2_LDS_ALL);
    ensure_lds_attr((const void*)gemm256_kernel<EPI, false, true>, G2_LDS_ALL);
    ensure_lds_attr((const void*)gemm256_kernel<EPI, true, false>, G2_LDS_ALL);
    ensure_lds_attr((const void*)gemm256_kernel<EPI, true, true>, G2_LDS_ALL);
    ensure_lds_attr((const void*)gemm256_kernel<EPI, false, true, true>, G2_LDS_ALL);
    ensure_lds_attr((const void*)gemm256_kernel<EPI, true, true, true>, G2_LDS_ALL);
    ensure_lds_attr((const void*)gemm_nt_kernel<bf16, EPI, 3>, 3 * 2 * BM * SLAB);
    ensure_lds_attr((const void*)gemm_nt_kernel<f16, EPI, 3>, 3 * 2 * BM * SLAB);
    ensure_lds_attr((const void*)gemm_nt_kernel<float, EPI, 3>, 3 * 2 * BM * SLAB);
    ensure_lds_attr((const void*)gemm_nt_kernel<bf16, EPI, kNtStages>, kNtStages * 2 * BM * SLAB);
    ensure_lds_attr((const void*)gemm_nt_kernel<f16, EPI, kNtStages>, kNtStages * 2 * BM * SLAB);
    ensure_lds_attr((const void*)gemm_nt_kernel<float, EPI, kNtStages>, kNtStages * 2 * BM * SLAB);
}

}  // namespace

void ensure_lds_attr(const void* kernel, int bytes) {
    static std::mutex mu;
    static std::set<std::tuple<const void*, int, int>> done;
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    if (done.count({kernel, dev, bytes})) return;
    HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done.insert({kernel, dev, bytes});
}

void gemm_prepare() {
    prepare_epi<EPI_BIAS>();
    prepare_epi<EPI_BIAS_GELU>();
    prepare_epi<EPI_BIAS_GELU_POS>();
    prepare_epi<EPI_BIAS_RESID>();
    prepare_epi<EPI_KVSPLIT>();
    prepare_epi<EPI_BIAS_SWISH>();
    prepare_epi<EPI_BIAS_RELU>();
    prepare_epi<EPI_BIAS_F32>();
    prepare_epi<EPI_PARTIAL>();
}

void gemm_nt(int dtype, int epi, const GemmArgs& g, int batch, hipStream_t st) { gemm_nt_variant(dtype, epi, g, batch, 0, st); }

void gemm_nt_variant(int dtype, int epi, const GemmArgs& g, int batch, int variant, hipStream_t st) {
    const int esz = dtype == DT_F32 ? 4 : 2;
    if (g.ksplit < 1 || g.K % g.ksplit || (g.ksplit > 1 && epi != EPI_PARTIAL))
        throw std::runtime_error("gemm_nt: split-K needs EPI_PARTIAL and K % ksplit == 0");
    if (variant != 3 && (g.N % (variant == 5 ? 64 : BN) != 0 || (g.K / g.ksplit * esz) % SLAB != 0 || g.M <= 0))
        throw std::runtime_error("gemm_nt: unsupported shape M=" + std::to_string(g.M) + " N=" +
                                 std::to_string(g.N) + " K=" + std::to_string(g.K));
#define SPT_GEMM_CASES(T)                                                          \
    switch (epi) {                                                                 \
        case EPI_BIAS: launch_t<T, EPI_BIAS>(g, batch, variant, st); return;       \
        case EPI_BIAS_GELU: launch_t<T, EPI_BIAS_GELU>(g, batch, variant, st); return; \
        case EPI_BIAS_GELU_POS: launch_t<T, EPI_BIAS_GELU_POS>(g, batch, variant, st); return; \
        case EPI_BIAS_RESID: launch_t<T, EPI_BIAS_RESID>(g, batch, variant, st); return; \
        case EPI_KVSPLIT: launch_t<T, EPI_KVSPLIT>(g, batch, variant, st); return; \
        case EPI_BIAS_SWISH: launch_t<T, EPI_BIAS_SWISH>(g, batch, variant, st); return; \
        case EPI_BIAS_RELU: launch_t<T, EPI_BIAS_RELU>(g, batch, variant, st); return; \
        case EPI_BIAS_F32: launch_t<T, EPI_BIAS_F32>(g, batch, variant, st); return; \
        case EPI_PARTIAL: launch_t<T, EPI_PARTIAL>(g, batch, variant, st); return; \
    }
#define SPT_GEMM256_CASES(F)                                                       \
    switch (epi) {                                                                 \
        case EPI_BIAS: launch_256<EPI_BIAS, F>(g, batch, st); return;              \
        case EPI_BIAS_GELU: launch_256<EPI_BIAS_GELU, F>(g, batch, st); return;    \
        case EPI_BIAS_GELU_POS: launch_256<EPI_BIAS_GELU_POS, F>(g, batch, st); return; \
        case EPI_BIAS_RESID: launch_256<EPI_BIAS_RESID, F>(g, batch, st); return;  \
        case EPI_KVSPLIT: launch_256<EPI_KVSPLIT, F>(g, batch, st); return;        \
        case EPI_BIAS_SWISH: launch_256<EPI_BIAS_SWISH, F>(g, batch, st); return;  \
        case EPI_BIAS_RELU: launch_256<EPI_BIAS_RELU, F>(g, batch, st); return;    \
        case EPI_BIAS_F32: launch_256<EPI_BIAS_F32, F>(g, batch, st); return;      \
        case EPI_PARTIAL: launch_256<EPI_PARTIAL, F>(g, batch, st); return;        \
    }
#define SPT_GEMM_SKINNY_CASES(F)                                                   \
    switch (epi) {                                                                 \
        case EPI_BIAS: launch_skinny<EPI_BIAS, F>(g, st); return;                  \
        case EPI_BIAS_GELU: launch_skinny<EPI_BIAS_GELU, F>(g, st); return;        \
        case EPI_BIAS_RESID: launch_skinny<EPI_BIAS_RESID, F>(g, st); return;      \
        case EPI_BIAS_SWISH: launch_skinny<EPI_BIAS_SWISH, F>(g, st); return;      \
        case EPI_BIAS_RELU: launch_skinny<EPI_BIAS_RELU, F>(g, st); return;        \
        case EPI_BIAS_F32: launch_skinny<EPI_BIAS_F32, F>(g, st); return;          \
        case EPI_PARTIAL: launch_skinny<EPI_PARTIAL, F>(g, st); return;            \
    }
    if (variant == 3) {  // skinny (M <= 64): bf16 / f16, N % 16, K / ksplit % 128
        if (dtype == DT_F32 || g.M > 64 || g.N % 16 || (g.K / g.ksplit) % 128)
            throw std::runtime_error("gemm_nt: skinny variant needs a 16-bit dtype, M <= 64, N % 16, (K / ksplit) % 128");
        if (dtype == DT_F16) { SPT_GEMM_SKINNY_CASES(true) }
        else { SPT_GEMM_SKINNY_CASES(false) }
        throw std::runtime_error("gemm_nt: bad epilogue for the skinny variant");
    }
#undef SPT_GEMM_SKINNY_CASES
    static const bool force128 = getenv("SPT_GEMM128") != nullptr;  // A/B switch for measurements
    // f32 (Whisper-small C2: one 30 s window gives 72-288 128 x 128 tiles on 256 CUs) takes the 64-row
    // tiles, like the 16-bit types (r6, profiles/r6/exp_f32_small_tiles.txt: C2 encoder 7.11 -> 5.42 ms);
    // SPT_GEMM_F32_SMALL=0 keeps the 128 x 128 tile
    // (read per launch, like the switches of launch_256: eager runs such as debug_encode pick it up)
    const char* f32s_env = getenv("SPT_GEMM_F32_SMALL");
    const bool f32_small = !f32s_env || atoi(f32s_env) != 0;
    if (variant == 0 && !force128 && dtype == DT_F32 && f32_small) {
        const int64_t t128 = (int64_t)cdiv(g.M, BM) * (g.N / BN) * g.ksplit * batch;
        const int64_t t64 = (int64_t)cdiv(g.M, 64) * (g.N / BN) * g.ksplit * batch;
        // below four rounds of 128 x 128 tiles (r6aa: at 256, Whisper-small's fc1 kept 288 of them,
        // 1.125 rounds; SPT_GEMM_F32_T128MIN moves the threshold)
        const char* t128_env = getenv("SPT_GEMM_F32_T128MIN");
        const int t128_min = t128_env ? atoi(t128_env) : 1024;
        if (t128 < t128_min && g.N % 64 == 0) variant = (t64 >= 512 && g.N % BN == 0) ? 4 : 5;
    }
    if (variant == 0 && !force128 && dtype != DT_F32) {
        // automatic: the 256 x 256 tile from ~96 workgroups up; below that (a single Whisper
        // window, M = 1500: 30 workgroups for the N = 1280 products) the 128 x 128 tile, or while
        // 128-row tiles would not fill the CUs once the 64 x 128 tile, or the 64 x 64 one below
        // two 64 x 128 workgroups per CU (all bitwise equal; r3 exp_r3y)
        const int64_t t256 = (int64_t)cdiv(g.M, G2_BM) * (g.N / G2_BN) * g.ksplit * batch;
        const int64_t t128 = (int64_t)cdiv(g.M, BM) * (g.N / BN) * g.ksplit * batch;
        const int64_t t64 = (int64_t)cdiv(g.M, 64) * (g.N / BN) * g.ksplit * batch;
        // r6: also below half a round of 256 x 256 tiles counted over the launches that run together (the
        // encoder's window groups, g.groups): one 30 s window's fc1 (120 tiles, alone) is 4.5 % faster
        // on the 128 x 128 tile, while two groups' 120-tile out / fc2 launches side by side are not
        // (profiles/r6/exp_bf16_tile_thresholds.txt); SPT_GEMM_BF16_T256G moves that bound (0: off)
        const char* t256g_env = getenv("SPT_GEMM_BF16_T256G");
        const int t256g = t256g_env ? atoi(t256g_env) : 128;
        if (g.N % G2_BN != 0 || t256 < 96 || t256 * std::max(1, g.groups) < t256g)
            variant = t128 >= 256 ? 1 : t64 >= 512 ? 4 : 5;
    }
    const bool use256 = variant == 2 || (variant == 0 && !force128);
    const bool fits32 = (int64_t)g.M * g.lda < (1ll << 31) && (int64_t)g.N * g.ldw < (1ll << 31);
    if (dtype != DT_F32 && use256 && fits32 && g.N % G2_BN == 0 && (g.K / g.ksplit) % 64 == 0) {
        if (dtype == DT_F16) { SPT_GEMM256_CASES(true) }
        else { SPT_GEMM256_CASES(false) }
    }
    if (dtype == DT_BF16) { SPT_GEMM_CASES(bf16) }
    else if (dtype == DT_F16) { SPT_GEMM_CASES(f16) }
    else { SPT_GEMM_CASES(float) }
#undef SPT_GEMM_CASES
#undef SPT_GEMM256_CASES
    throw std::runtime_error("gemm_nt: bad epilogue");
}

}  // namespace spt
