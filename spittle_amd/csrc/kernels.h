// kernels.h -- host launchers of the spittle_amd HIP kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace spt {

enum { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2 };  // DT_F16: the Parakeet encoder only

// ------------------------------------------------------------------ GEMM (k_gemm.hip)
// Cross-attention K/V cache layout: per decoder layer [ceil(T/32)][B][H][2][32][64] -- 32-key
// blocks, the K and V of a block side by side (4096 elements per (block, b, h)).  At any moment of
// the decode step the workgroups of all (b, h) read the same few block indices, so the bytes in
// flight form one contiguous region (r2: 15.1 -> 14.6 us per layer against [2][B][H][T][64]).
__host__ __device__ inline int64_t kv_layer_elems(int B, int H, int T) { return (int64_t)((T + 31) / 32) * B * H * 4096; }
__host__ __device__ inline int64_t kv_offset(int l, int kvi, int b, int h, int t, int e, int B, int H, int T) {
    return (int64_t)l * kv_layer_elems(B, H, T) + (((int64_t)(t >> 5) * B + b) * H + h) * 4096 + kvi * 2048 +
           (t & 31) * 64 + e;
}

// EPI_BIAS_RESID: f32 C += alpha * (acc + bias); EPI_BIAS_F32: f32 C = alpha * (acc + bias);
// SWISH / RELU: activation of acc + bias in the storage dtype
// EPI_PARTIAL: split-K slab s (grid.y) of the f32 product at C + s * c_split (no bias)
enum { EPI_BIAS = 0, EPI_BIAS_GELU = 1, EPI_BIAS_GELU_POS = 2, EPI_BIAS_RESID = 3, EPI_KVSPLIT = 4,
       EPI_BIAS_SWISH = 5, EPI_BIAS_RELU = 6, EPI_BIAS_F32 = 7, EPI_PARTIAL = 8 };

struct GemmArgs {
    const void* A; int lda; int64_t sA;   // A rows (+ batch stride, elements)
    const void* W; int ldw;               // W [N][K] row-major (K contiguous)
    int M, N, K;                          // M rows per batch item
    const float* bias;                    // [N] or nullptr
    void* C; int ldc; int64_t sC;         // output rows (+ batch stride)
    const float* pos;                     // EPI_BIAS_GELU_POS: [M][N] f32
    int kv_B, kv_T, kv_H;                 // EPI_KVSPLIT: dest = the cross K/V cache (kv_offset)
    float alpha = 1.0f;                   // EPI_BIAS_RESID / EPI_BIAS_F32 scale
    int ksplit = 1; int64_t c_split = 0;  // EPI_PARTIAL: K split over grid.y, slab stride (elements)
    int nmajor = 0;                       // 128 x 128 tile: raster tiles N-major (set by the launcher)
    int groups = 1;                       // launches of this shape running concurrently (encoder window groups)
};
void gemm_nt(int dtype, int epi, const GemmArgs& g, int batch, hipStream_t st);
// variant 0: automatic (bf16 N % 256 == 0 -> 256 x 256 tile); 1: 128 x 128 tile; 2: prefer 256 x 256;
// 3: skinny (M <= 64, 16-bit dtypes: 16 columns per workgroup, the weight stream spread over the grid)
// 4: 64 x 128 tile (16-bit or f32; small M: two workgroups per CU where the 128-row tile gives one)
// 5: 64 x 64 tile (N % 64; up to four workgroups per CU)
// sets the > 64 KiB dynamic-LDS attribute of every GEMM kernel on the current device (engine
// constructors call it before any stream capture; launches check it too)
void gemm_prepare();
void gemm_nt_variant(int dtype, int epi, const GemmArgs& g, int batch, int variant, hipStream_t st);

// ------------------------------------------------------------------ weights (k_init.hip)
enum { WK_MAT = 0, WK_BIAS = 1, WK_LNW = 2, WK_LNB = 3, WK_TOK = 4, WK_DPOS = 5 };
// dst[i] = value(seed, tid, i) for i in [0, n); stored as f32 or bf16 (RNE)
void gen_weights(int store_dtype, void* dst, int64_t n, uint64_t seed, uint32_t tid, int kind,
                 int scale_exp, hipStream_t st);
// canonical conv weight [N][C][3] -> device [N][3][Cp] (zero for c >= C)
void gen_conv_weights(int store_dtype, void* dst, int N, int C, int Cp, uint64_t seed, uint32_t tid,
                      int scale_exp, hipStream_t st);
void fill_f32(float* dst, int64_t n, float v, hipStream_t st);
// read `bytes` of p once (measurement: cold caches before a probed launch)
// ggml tensor bytes on the device -> engine storage (out_dtype DT_F32 / DT_BF16); type is the
// ggml type id (ggml_quant.h GQ_*), n a multiple of the type's block
void ggml_dequant(int type, const void* src, int64_t n, int out_dtype, void* dst, hipStream_t st);
void cache_flush(const void* p, int64_t bytes, unsigned* sink, hipStream_t st);
void set_xattn_stamp(void* p);
void dec_cross_attn_ni8(const void* q, const void* kv, int B, int B_layout, int H, int T_enc, void* out, int blocked,
                        hipStream_t st);  // ubench variant  // SPT_STAMP=1 builds only (ubench)
void stream_read(const void* p, int64_t bytes, unsigned* sink, int grid, int tpb, hipStream_t st);  // ubench probe
// weight checksum helper for tests: sum of |w| and sum of w (f64) of a device tensor
void tensor_checksum(int dtype, const void* src, int64_t n, double* out2_dev, hipStream_t st);

// ------------------------------------------------------------------ mel (k_mel.hip)
struct MelTables {
    const float* hann;   // [400]
    const float* sinv;   // [400]
    const float* cosv;   // [400]
    const float* filt;   // [n_mels][201]
    const int* grp;      // [n_mels][2] first / last+1 group of 4 bins with a nonzero weight
};
constexpr int MEL_ROWS = 3002;  // padded time-major rows of a window: [zero][3000 frames][zero]
// whole utterances (device arrays, one entry each): samples pcm[pcm_off[u] .. + n[u]), their
// mel_rows(n[u]) computed log10-mel rows at mel_raw[row_off[u]] ([rows][n_mels])
struct MelUtts {
    const int64_t* pcm_off;
    const int64_t* row_off;
    const int* n;
};
// frames whisper.cpp computes for n samples: min((n + 200) / 160 + 1, (n + 480000) / 160); later
// frames of the (n + 480000) / 160 are log10(1e-10)
int mel_rows(int n);
// log10 mel of every computed frame of each of U utterances (max_rows >= every mel_rows(n[u]));
// the maximum of each utterance as an order-preserving key in mel_max[u]
void mel_frames(const float* pcm, MelUtts u, int U, int max_rows, int n_mels, MelTables t, float* mel_raw,
                unsigned* mel_max, hipStream_t st);
// encoder windows e < E: frames [win_seek[e], + 3000) of utterance win_utt[e], clamped at that
// utterance's max - 8 and normalised -> conv1 input [E][3002][Cp] (rows 0 and 3001 zero); optional
// f32 copy [E][n_mels][3000]
void mel_norm(int dtype, const float* mel_raw, const unsigned* mel_max, MelUtts u, const int* win_utt,
              const int* win_seek, int E, int n_mels, int Cp, void* mel_in, float* dbg, hipStream_t st);

// ------------------------------------------------------------------ norm (k_norm.hip)
// y[m] = LN(x[m]) * w + b ; x f32 [M][d], y f32/bf16 [M][d]
void layernorm(int dtype, const float* x, int M, int d, const float* w, const float* b, void* y,
               hipStream_t st);
// x[m] += alpha * (slab_0[m] + .. + slab_{ks-1}[m] + pbias) (the pending split-K product of a
// residual GEMM, in slab order), then y[m] = LN(x[m]) * w + b; write_x: store the summed x back
void layernorm_pend(int dtype, float* x, int M, int d, const float* slab, int ks, int64_t slab_stride,
                    const float* pbias, float alpha, const float* w, const float* b, void* y, bool write_x,
                    hipStream_t st);
// layernorm_pend with the f32 result y (x not written back) normalised once more into y2 (w2, b2;
// dtype2): the Parakeet block boundary in one launch, bitwise the two-launch result
void layernorm_pend2(int dtype2, const float* x, int M, int d, const float* slab, int ks, int64_t slab_stride,
                     const float* pbias, float alpha, const float* w, const float* b, float* y, const float* w2,
                     const float* b2, void* y2, hipStream_t st);
// convert an activation buffer to f32 (debug / tests)
void to_f32(int dtype, const void* src, float* dst, int64_t n, hipStream_t st);

// ------------------------------------------------------------------ encoder attention (k_attn.hip)
// qkv [B*T][3*d] (q | k | v, head h at h*64), out [B*T][d]; non-causal, scale 1/8
void enc_attention(int dtype, const void* qkv, int B, int T, int H, void* out, hipStream_t st);

// ------------------------------------------------------------------ decoder (k_dec.hip)
struct DecState {        // device-resident step state
    int pos0;            // position of the first token fed this pass
    int step;            // index of the token being produced
};

enum { GV_BIAS = 0, GV_BIAS_GELU = 1, GV_PARTIAL = 2, GV_QKV_CACHE = 3, GV_LOGITS = 4, GV_BIAS_RESID = 5 };
enum { A_DIRECT = 0, A_LN = 1, A_ATTN = 2 };
struct GemvArgs {
    // A rows: row i at A + (i * lda + a_row0); A_DIRECT: dtype activations; A_LN: f32 residual rows
    const void* A; int lda; int a_row0;
    const float* ln_w; const float* ln_b; // A_LN: LayerNorm of x + pend[0] + .. + pend[3]
    const float* pend[4]; int n_pend;     // A_LN: pending partial slabs (same layout as A): n_pend = 0, 1, 2 or 4
    float* x_out;                         // A_LN: combined rows written here by workgroup (0, 0) (or nullptr)
    const float* apart; int a_splits, a_heads;  // A_ATTN: cross-attention chunk partials [R][H][S][66] (S = 2..4, 8)
    int R;                                // rows (<= 64)
    const void* W; int N, K;              // W [N][K]
    const float* bias;
    void* C; int ldc;                     // output rows (GV_BIAS*, GV_LOGITS, GV_PARTIAL; GV_BIAS_RESID: f32 C += ...)
    int ksplit; int64_t c_split;          // GV_PARTIAL: K split over workgroups, slab s at C + s * c_split (f32)
    const float* p_resid;                 // GV_PARTIAL (or nullptr): f32 rows [R][ldc] added into slab 0
    // GV_QKV_CACHE: q -> C, k/v -> cache [2][B][H][ctx][64] at position pos0 + t (row = b*Tq + t)
    void* cache; int cache_B, cache_H, cache_ctx, Tq;
    const DecState* st;
    // GV_LOGITS: suppression + per-16-column-tile top-2 partials [R][n_tiles] (16 B each)
    const uint32_t* suppress; int blank0, blank1;
    void* part; int n_tiles;
    // SPT_STAMP builds only (developer timeline): s_memrealtime at each workgroup's start / end,
    // [2 * workgroup + {0, 1}]
    unsigned long long* stamp;
};
constexpr int kMaxPend = 4;
void gemv(int dtype, int mode, int asrc, const GemvArgs& a, hipStream_t st);
// one-time per-process kernel attributes (call before any stream capture)
void gemv_prepare(int dtype);
// rows a LayerNorm / attention-merge GEMV can stage for K columns (its LDS image budget): the
// decoder's rows per pass (large-v3 bf16: 38; f32 small: 31; <= 64)
int gemv_max_image_rows(int dtype, int K);

// x[b*Tq + t] = tok_emb[tok[b*Tq+t]] + pos_emb[pos0 + t]
void dec_embed(int dtype, const int* tok, int R, int Tq, int d, const void* tok_emb,
               const float* pos_emb, const DecState* ds, float* x, hipStream_t st);
// self attention over the cache: q [R][d] (row b*Tq + t at position pos0 + t), keys 0..pos0+t
void dec_self_attn(int dtype, const void* q, const void* cache, int B, int H, int ctx, int Tq,
                   const DecState* ds, void* out, hipStream_t st);
// cross attention over all T_enc cached encoder keys: q [R][d] -> out [R][d]
// kv: [2][B_layout][H][T_enc][64] (already offset to the first of the B sequences).
// splits > 1: the keys of each (b, h) in `splits` chunks (one workgroup each) that write
// partials [R][H][splits][66] = {o[64], m, l} to `part` instead (merged by an A_ATTN GEMV)
// kv: one layer of the cross K/V cache (kv_offset layout with B_layout sequences), advanced to
// the first of the B sequences (+ b0 * H * 4096)
// kvrow (device [B], optional): rows j * share .. + share - 1 all attend to window kvrow[j * share]
// (kv then points at the layer, not at the first sequence); one workgroup per (window run, head)
// reads that window's K/V once for its share * Tq queries (the decoders of one utterance)
void dec_cross_attn(int dtype, const void* q, const void* kv, int B, int B_layout, int H, int T_enc, int Tq,
                    void* out, hipStream_t st, int splits = 1, float* part = nullptr, const int* kvrow = nullptr,
                    int share = 1);
// the same attention with each of the 8 waves of a (row run, head) workgroup as a workgroup of its
// own: writes partial w of [rows][H][8][66] = {o[64], m, l} (merged by an A_ATTN GEMV with 8
// chunks); bitwise the 8-wave kernel's result once merged, for small grids (B / share * H small)
// per_query (Tq = 1): one query row per workgroup (a beam's rows on one window: 8 x share
// workgroups per head instead of 8, each re-reading the window's K/V, mostly from L2)
void dec_cross_attn_vw(int dtype, const void* q, const void* kv, int B, int B_layout, int H, int T_enc, int Tq,
                       float* part, hipStream_t st, const int* kvrow = nullptr, int share = 1, bool per_query = false);
// the 8 partials of each of R query rows x H heads merged into out [R][H * 64] (bitwise the 8-wave
// kernel's output), for a plain (A_DIRECT) cross output projection
void dec_attn_part_merge(int dtype, const float* part, int R, int H, void* out, hipStream_t st);

struct FinalizeArgs {
    const void* part; int n_tiles;        // logits top-2 partials [B][n_tiles]
    int eot; int ignore_eot; int n_vocab;
    const int* forced; int forced_len;    // [B][forced_len] teacher forcing (nullptr = off)
    int* next_tok;                        // [B]
    int* out_tok; float* out_top1; float* out_top2; int out_cap;  // [B][out_cap]
    int* done;                            // [B]
    const void* emb; const float* pos; int d, ctx, Tq;  // next-pass embedding -> x rows 0..B-1
    float* x;
    DecState* ds; unsigned* arrive;       // step state, last-arriver counter
};
// argmax reduce + record + next-token embed + step advance (replaces embed/argmax/advance)
void dec_finalize(int dtype, const FinalizeArgs& a, int B, hipStream_t st);
void dec_reset(DecState* ds, unsigned* arrive, hipStream_t st);



// whisper_full decoding parameters of one call (device memory: read by graph-captured launches)
struct TsParams {
    float temperature;    // 0: greedy
    int suppress_blank;   // [eot] and " " at the first step
    int no_ts;            // no_timestamps: every timestamp token suppressed
    int max_initial;      // first timestamp <= beg + max_initial (round(max_initial_ts / 0.02)); < 0 off
    int n_max;            // steps per window (n_text_ctx / 2 - 4): the repetition guard
    int max_tokens;       // > 0: end the segment after this many tokens
    unsigned long long seed;
};
struct TsArgs {
    const float* logits; int ldl;        // [B][ldl] raw logits of this step
    int n_vocab, eot, beg, blank;        // blank: the " " token
    const uint32_t* suppress;            // static suppression bits
    const TsParams* prm;
    const int* seek; const int* seek_end;  // [B] window start / audio end, 10 ms frames
    int* state;                          // [B][4] has_ts, seek_delta, result_len, status
    const int* forced; int forced_len;
    int* next_tok;
    int* out_tok; float* out_plog; float* out_tid; int out_cap;  // [B][out_cap]
    int* done;
    const void* emb; const float* pos; int d, ctx, Tq;
    float* x;
    DecState* ds; unsigned* arrive;
    float* stat;                         // [B][TS_CHUNKS][6] per-chunk maxima and sums (dec_ts_stats)
};
constexpr int TS_CHUNKS = 16;  // vocabulary chunks per row in dec_ts_stats
// whisper_process_logits' maxima and exp sums of each row, over TS_CHUNKS workgroups per row
// (a.stat), then whisper_process_logits + whisper_sample_token + per-decoder bookkeeping, one
// workgroup per row (k_sample.hip)
void dec_ts_stats(const TsArgs& a, int B, hipStream_t st);
void dec_finalize_ts(int dtype, const TsArgs& a, int B, hipStream_t st);
// beam search: the k best processed candidates of each decoder row (k_sample.hip)
struct BeamArgs {
    const float* logits; int ldl;
    int n_vocab, eot, beg, blank;
    const uint32_t* suppress;
    const TsParams* prm;
    const int* row;    // [B][4] last token, previous token, has_ts, seek_delta
    const int* step;   // [1] index of the token being chosen
    int k;             // 1..8
    int* cand_id; float* cand_lp;  // [B][8]
    int* tid;          // [B] most probable timestamp (0: none)
    float* stat;       // [B][TS_CHUNKS][BEAM_STAT] per-chunk statistics and candidates (nullptr: one
                       // workgroup per row sweeps the row itself, the r4 first kernel)
};
constexpr int BEAM_STAT = 6 + 4 * 8;  // maxima + sums, then 8 (v, id) over everything and 8 over timestamps
void dec_beam_topk(const BeamArgs& a, int B, hipStream_t st);
// self-K/V cache rows for the next beam step: dst row b <- src row rows[b], positions < pos0
void dec_kv_gather(int dtype, const void* src, void* dst, const int* rows, int L, int B, int H, int ctx,
                   const DecState* ds, hipStream_t st);
// pos0 += n (after a prefill pass that produces no token)
void dec_advance(DecState* ds, int n, hipStream_t st);

}  // namespace spt
