// k_sample.hip -- whisper_full's token selection for the timestamp / temperature decode
// (the no-timestamp greedy protocol keeps the top-2 partial path of k_dec.hip).
//
// One 1024-thread workgroup per sequence reads that sequence's logits row (L2-resident, just
// written by the logits GEMV) and restates whisper.cpp (~1.7.x, whisper-rs-sys 0.11.1;
// /root/reference/src-tauri/Cargo.lock:8156-8174, not vendored):
//   whisper_process_logits: logits / temperature; the static suppression mask (sot, nosp,
//     solm, task, prev, language and optionally non-speech tokens, [not], and every timestamp
//     under no_timestamps); [eot] and " " at the first step (suppress_blank); timestamps in
//     pairs (after a timestamp that follows a timestamp no timestamp may come; after a lone
//     one only a timestamp or [eot]); the first timestamp <= max_initial_ts; timestamps never
//     before the last one (has_ts: tid < seek_delta / 2 masked); log-softmax; "if the summed
//     probability of the timestamps beats every text token, sample a timestamp".
//   whisper_sample_token: greedy = first maximum; temperature > 0 = a draw from the softmax
//     (a counter-based stream per (seed, sequence, step) replaces std::mt19937 +
//     std::discrete_distribution: the distribution is the same, the draws are not); plog =
//     the chosen token's log-probability before the timestamp rule's text mask; tid = the
//     most probable timestamp (the token itself when it is one).
//   whisper_full's per-token bookkeeping of one decoder: seek_delta / result_len / has_ts on
//     timestamps (failed when time would run backwards), end of segment on [eot], max_tokens
//     or the end of the audio (failed when no timestamp was produced), no_timestamps
//     completion (result_len = i + 1, seek_delta = 3000), and the repetition guard at
//     i == n_max - 1.
// The chosen (or forced) token is embedded for the next pass and the step advanced exactly
// as dec_finalize does.
#include "common.h"
#include "kernels.h"

namespace spt {

namespace {

constexpr int TW = 1024;  // threads per sequence

__device__ __forceinline__ float u01(uint64_t seed, int b, int step) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ULL + ((uint64_t)b << 32) + (uint64_t)step + 0x632BE59BD9B4E019ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);  // [0, 1)
}

struct MaxI { float v; int i; };
__device__ __forceinline__ MaxI max_merge(MaxI a, MaxI b) {
    return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}

// The per-row vocabulary kernels below hold a thread's logits in registers: VJ per thread, strided
// n = tid + j * TW (V <= VJ * TW = 53248 covers Whisper's 51864..51866; checked at launch), every
// load issued before the first use.  r4: a loop that loaded one logit per iteration waited a full
// memory round trip per iteration (the beam candidate kernel took 214 us per step,
// profiles/r4/exp_beam_step.txt).  The suppress bitmask is staged in LDS for the same reason.
constexpr int VJ = 52;

// whisper_process_logits' masks for one decoder row at one step, folded into per-row constants
// read once (the P fields were re-loaded inside every unrolled test) and a branch-free test:
//   suppressed token; blank / EOT at step 0; a timestamp when timestamps are off, after two
//   timestamps in a row, beyond max_initial_ts at step 0, or before the last timestamp; a text
//   token other than EOT right after a single timestamp
struct MaskRule {
    int eot, beg, blank, mi_lim, sd_lim;
    bool blank0, ts_all, tx_all;
    __device__ MaskRule(const TsParams& P, int step, int eot_, int beg_, int blank_, bool last_ts, bool pen_ts,
                        int has_ts, int seek_delta)
        : eot(eot_), beg(beg_), blank(blank_) {
        blank0 = step == 0 && P.suppress_blank;
        ts_all = P.no_ts || (last_ts && pen_ts);
        tx_all = last_ts && !pen_ts;
        mi_lim = (step == 0 && P.max_initial >= 0) ? beg + P.max_initial : 0x7fffffff;
        sd_lim = has_ts ? beg + seek_delta / 2 : -0x7fffffff;
    }
    __device__ __forceinline__ bool masked_rules(int n) const {  // everything but the suppress bits
        const bool b0 = blank0 & ((n == eot) | (n == blank));
        const bool ts = (n >= beg) & (ts_all | (n > mi_lim) | (n < sd_lim));
        const bool tx = (n < eot) & tx_all;
        return b0 | ts | tx;
    }
    __device__ __forceinline__ bool masked(const uint32_t* s_sup, int n) const {
        const bool sup = (s_sup[n >> 5] >> (n & 31)) & 1u;
        return sup | masked_rules(n);
    }
};
__device__ __forceinline__ void stage_suppress(uint32_t* s_sup, const uint32_t* __restrict__ sup, int V) {
    for (int w = threadIdx.x; w < (V + 31) / 32; w += TW) s_sup[w] = sup[w];
}

// whisper_process_logits' statistics of one row, spread over TS_CHUNKS workgroups per row: each
// workgroup takes a contiguous 1/TS_CHUNKS of the vocabulary and writes the text and timestamp
// maxima (first index on ties) of its unmasked tokens and its exp sums relative to its own maxima
// (sa over everything, st over the timestamps).  finalize_ts_kernel merges them in chunk order.
// r4: one 1024-thread workgroup per row swept all 51866 logits itself -- about 7 K VALU
// instructions per wave, 4 waves per SIMD on the one CU a row had (~50 us per step; SQ counters
// in profiles/r4/exp_beam_step.txt).
constexpr int TS_T = 256;   // threads per chunk
constexpr int TS_J = 13;    // logits per thread: V <= TS_CHUNKS * TS_T * TS_J = 53248
__global__ __launch_bounds__(TS_T) void ts_stats_kernel(TsArgs a) {
    __shared__ uint32_t s_sup[TS_T * TS_J / 32 + 2];
    __shared__ MaxI s_m[2][TS_T / 64];
    __shared__ float s_s[2][TS_T / 64];
    const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int step = a.ds->step;
    const TsParams& P = *a.prm;
    const int V = a.n_vocab, beg = a.beg, eot = a.eot;
    const int CS = (V + TS_CHUNKS - 1) / TS_CHUNKS, n0 = c * CS, n1 = min(V, n0 + CS);
    float* out = a.stat + ((size_t)b * TS_CHUNKS + c) * 6;
    const bool live = step < a.out_cap && !a.done[b];
    const int w0 = n0 >> 5, nw = n1 > n0 ? ((n1 - 1) >> 5) - w0 + 1 : 0;
    for (int w = tid; w < nw; w += TS_T) s_sup[w] = a.suppress[w0 + w];
    __syncthreads();
    if (!live) {
        if (tid == 0) {
            out[0] = -INFINITY; out[1] = __int_as_float(0x7fffffff);
            out[2] = -INFINITY; out[3] = __int_as_float(0x7fffffff);
            out[4] = 0.0f; out[5] = 0.0f;
        }
        return;
    }
    const float* lg = a.logits + (size_t)b * a.ldl;
    const int oi0 = b * a.out_cap;
    const int last = step > 0 ? a.out_tok[oi0 + step - 1] : -1;
    const int pen = step > 1 ? a.out_tok[oi0 + step - 2] : -1;
    const bool last_ts = step > 0 && last >= beg;
    const bool pen_ts = step < 2 || pen >= beg;
    const int* S = a.state + 4 * b;
    const MaskRule mr(P, step, eot, beg, a.blank, last_ts, pen_ts, S[0], S[1]);
    const float temp = P.temperature;
    float lv[TS_J];
#pragma unroll
    for (int j = 0; j < TS_J; ++j) lv[j] = lg[min(n0 + tid + j * TS_T, V - 1)];
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < TS_J; ++j) {
        const int n = n0 + tid + j * TS_T;
        const int nc = min(n, V - 1);
        const bool sup = (s_sup[(nc >> 5) - w0] >> (nc & 31)) & 1u;  // the chunk's suppress words
        const bool m = sup | mr.masked_rules(nc);
        keep |= (uint32_t)((n < n1) & !m) << j;
        if (temp > 0.0f) lv[j] = lv[j] / temp;
    }
    const MaxI none{-INFINITY, 0x7fffffff};
    MaxI mt = none, ms = none;
#pragma unroll
    for (int j = 0; j < TS_J; ++j) {
        const int n = n0 + tid + j * TS_T;
        const MaxI x = ((keep >> j) & 1) ? MaxI{lv[j], n} : none;
        const bool t = n < beg;
        mt = max_merge(mt, t ? x : none);
        ms = max_merge(ms, t ? none : x);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mt = max_merge(mt, MaxI{__shfl_xor(mt.v, o, 64), __shfl_xor(mt.i, o, 64)});
        ms = max_merge(ms, MaxI{__shfl_xor(ms.v, o, 64), __shfl_xor(ms.i, o, 64)});
    }
    if (lane == 0) { s_m[0][wv] = mt; s_m[1][wv] = ms; }
    __syncthreads();
    mt = s_m[0][0];
    ms = s_m[1][0];
    for (int w = 1; w < TS_T / 64; ++w) { mt = max_merge(mt, s_m[0][w]); ms = max_merge(ms, s_m[1][w]); }
    const float M = fmaxf(mt.v, ms.v);
    float sa = 0.0f, st = 0.0f;
#pragma unroll
    for (int j = 0; j < TS_J; ++j) {
        const bool k_ = (keep >> j) & 1;
        const float ea = expf(lv[j] - M), et = expf(lv[j] - ms.v);
        sa += k_ ? ea : 0.0f;
        st += (k_ && n0 + tid + j * TS_T >= beg) ? et : 0.0f;
    }
    sa = wave_sum(sa);
    st = wave_sum(st);
    if (lane == 0) { s_s[0][wv] = sa; s_s[1][wv] = st; }
    __syncthreads();
    if (tid == 0) {
        float za = 0.0f, zt = 0.0f;
        for (int w = 0; w < TS_T / 64; ++w) { za += s_s[0][w]; zt += s_s[1][w]; }
        out[0] = mt.v; out[1] = __int_as_float(mt.i);
        out[2] = ms.v; out[3] = __int_as_float(ms.i);
        out[4] = M > -INFINITY ? za : 0.0f;
        out[5] = ms.v > -INFINITY ? zt : 0.0f;
    }
}

template <typename T>
__global__ __launch_bounds__(TW) void finalize_ts_kernel(TsArgs a) {
    __shared__ float s_scan[TW];
    __shared__ int s_pick, s_tok;
    __shared__ float s_bc[4];  // M_all, LSE_all, M_after, ts_rule
    const int b = blockIdx.x, tid = threadIdx.x;
    const int step = a.ds->step;
    const TsParams& P = *a.prm;
    const int V = a.n_vocab, beg = a.beg, eot = a.eot;
    const float* lg = a.logits + (size_t)b * a.ldl;
    int* S = a.state + 4 * b;  // has_ts, seek_delta, result_len, status (0 run, 1 done, 2 failed)
    const bool live = step < a.out_cap && !a.done[b];
    __shared__ uint32_t s_sup[VJ * TW / 32];
    if (live && P.temperature > 0.0f) stage_suppress(s_sup, a.suppress, V);  // the sampling walk's masks
    __syncthreads();
    if (live) {
        const int oi0 = b * a.out_cap;
        const int last = step > 0 ? a.out_tok[oi0 + step - 1] : -1;
        const int pen = step > 1 ? a.out_tok[oi0 + step - 2] : -1;
        const bool last_ts = step > 0 && last >= beg;
        const bool pen_ts = step < 2 || pen >= beg;
        const int has_ts = S[0], seek_delta = S[1];
        const MaskRule mr(P, step, eot, beg, a.blank, last_ts, pen_ts, has_ts, seek_delta);
        auto masked = [&](int n) -> bool { return mr.masked(s_sup, n); };
        const float temp = P.temperature;
        auto val = [&](int n) { return temp > 0.0f ? lg[n] / temp : lg[n]; };
        // the row's maxima and exp sums: dec_ts_stats' chunks merged in chunk order (every thread
        // merges the maxima the same way; thread 0 the sums)
        const MaxI none{-INFINITY, 0x7fffffff};
        const float* sp = a.stat + (size_t)b * TS_CHUNKS * 6;
        MaxI mt = none, ms = none;
        for (int c = 0; c < TS_CHUNKS; ++c) {
            mt = max_merge(mt, MaxI{sp[c * 6 + 0], __float_as_int(sp[c * 6 + 1])});
            ms = max_merge(ms, MaxI{sp[c * 6 + 2], __float_as_int(sp[c * 6 + 3])});
        }
        const float M = fmaxf(mt.v, ms.v);
        if (tid == 0) {
            float za = 0.0f, zt = 0.0f;
            for (int c = 0; c < TS_CHUNKS; ++c) {
                const float mc = fmaxf(sp[c * 6 + 0], sp[c * 6 + 2]);
                if (mc > -INFINITY) za += sp[c * 6 + 4] * expf(mc - M);
                if (sp[c * 6 + 2] > -INFINITY) zt += sp[c * 6 + 5] * expf(sp[c * 6 + 2] - ms.v);
            }
            const float lse = logf(za) + M;
            // timestamp_logprob > max_text_token_logprob (both relative to the same LSE)
            const float ts_lp = zt > 0.0f ? logf(zt) + ms.v - lse : -INFINITY;
            const float tx_lp = mt.v - lse;
            const bool rule = ms.v > -INFINITY && ts_lp > tx_lp;
            s_bc[0] = M;
            s_bc[1] = lse;
            s_bc[2] = rule ? ms.v : M;
            s_bc[3] = rule ? 1.0f : 0.0f;
            int pick;
            if (rule) pick = ms.i;
            else pick = (ms.v > mt.v) ? ms.i : mt.i;
            s_pick = M > -INFINITY ? pick : -2;
        }
        __syncthreads();
        if (P.temperature > 0.0f && s_pick >= 0) {
            // a draw from softmax over what survived the timestamp rule: contiguous chunks, a
            // block scan of their sums, then one thread walks the chunk the draw lands in
            const bool rule = s_bc[3] != 0.0f;
            const float M2 = s_bc[2];
            const int C = (V + TW - 1) / TW, n0 = tid * C, n1 = min(V, n0 + C);
            float cv[VJ];  // this thread's contiguous chunk (C <= VJ), loaded up front
#pragma unroll
            for (int i = 0; i < VJ; ++i) cv[i] = i < C ? val(min(n0 + i, V - 1)) : 0.0f;
            float z = 0.0f;
#pragma unroll
            for (int i = 0; i < VJ; ++i) {
                const int n = n0 + i;
                if (i < C && n < n1 && !masked(n) && !(rule && n < beg)) z += expf(cv[i] - M2);
            }
            s_scan[tid] = z;
            __syncthreads();
            for (int o = 1; o < TW; o <<= 1) {  // inclusive Hillis-Steele scan
                const float add = tid >= o ? s_scan[tid - o] : 0.0f;
                __syncthreads();
                s_scan[tid] += add;
                __syncthreads();
            }
            const float total = s_scan[TW - 1];
            const float u = u01(P.seed, b, step) * total;
            const float lo = tid ? s_scan[tid - 1] : 0.0f, hi = s_scan[tid];
            if (total > 0.0f && u >= lo && (u < hi || tid == TW - 1)) {
                float c = lo;
                int last_ok = -1;
#pragma unroll
                for (int i = 0; i < VJ; ++i) {
                    const int n = n0 + i;
                    if (i >= C || n >= n1) break;
                    if (masked(n) || (rule && n < beg)) continue;
                    last_ok = n;
                    c += expf(cv[i] - M2);
                    if (u < c) break;
                }
                if (last_ok >= 0) s_pick = last_ok;
            }
            __syncthreads();
        }
        if (tid == 0) {
            const int oi = oi0 + step;
            int tok = s_pick;
            if (tok < 0 || tok >= V) {  // every logit masked or non-finite: the sequence fails
                a.out_tok[oi] = -2;
                a.out_plog[oi] = __builtin_nanf("");
                a.out_tid[oi] = 0.0f;
                S[3] = 2;
                a.done[b] = 1;
            } else {
                const float plog = val(tok) - s_bc[1];
                int tid_ts = tok >= beg ? tok : (ms.v > -INFINITY ? ms.i : 0);
                a.out_tok[oi] = tok;
                a.out_plog[oi] = plog;
                a.out_tid[oi] = (float)tid_ts;  // exact: ids < 2^24
                // whisper_full: one decoder's bookkeeping for token i = step
                const int i = step;
                int hts = S[0], sd = S[1], rl = S[2], status = 0;
                const int seek = a.seek[b], seek_end = a.seek_end[b];
                if (tok > beg) {
                    const int sdn = 2 * (tok - beg);
                    if (hts && sd > sdn && rl < i) status = 2;  // time would run backwards
                    else { sd = sdn; rl = i + 1; hts = 1; }
                }
                if (status == 0 && (tok == eot || (P.max_tokens > 0 && i >= P.max_tokens) ||
                                    (hts && seek + sd + 100 >= seek_end))) {
                    if (rl == 0 && !P.no_ts) {
                        if (seek + sd + 100 >= seek_end) rl = i + 1;
                        else status = 2;
                    }
                    if (status == 0) {
                        if (P.no_ts) { rl = i + 1; sd = 3000; }
                        status = 1;
                    }
                }
                if (status == 0 && i == P.n_max - 1 && (rl == 0 || sd < 1500)) status = 2;  // repetition guard
                S[0] = hts; S[1] = sd; S[2] = rl; S[3] = status;
                if (status != 0) a.done[b] = 1;
            }
        }
    } else if (tid == 0 && step < a.out_cap) {
        const int oi = b * a.out_cap + step;
        a.out_tok[oi] = -1;
        a.out_plog[oi] = -INFINITY;
        a.out_tid[oi] = -1.0f;
    }
    __syncthreads();
    if (tid == 0) {
        int nxt = (live && step < a.out_cap) ? a.out_tok[b * a.out_cap + step] : eot;
        if (live && a.forced && step < a.forced_len) nxt = a.forced[b * a.forced_len + step];
        if (nxt < 0 || nxt >= V) nxt = eot;
        a.next_tok[b] = nxt;
        s_tok = nxt;
    }
    __syncthreads();
    const int tok = s_tok;
    const int pos0 = a.ds->pos0;
    const int pn = min(pos0 + a.Tq, a.ctx - 1);
    const T* e = (const T*)a.emb + (size_t)tok * a.d;
    const float* pp = a.pos + (size_t)pn * a.d;
    for (int i = tid; i < a.d; i += TW) a.x[(size_t)b * a.d + i] = to_f<T>(e[i]) + pp[i];
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

// Beam search (whisper_full, WHISPER_SAMPLING_BEAM_SEARCH at temperature 0): the same
// whisper_process_logits rules for each decoder row, then its k best candidates by processed
// logit (ties: lower id) with their log-probabilities (before the timestamp rule's text mask)
// and the row's most probable timestamp.  Decoder state comes from the host per step: row
// state {last token, previous token, has_ts, seek_delta}, step index.
__global__ __launch_bounds__(TW) void beam_topk_kernel(BeamArgs a) {
    __shared__ MaxI s_m[2][TW / 64];
    __shared__ float s_s[TW / 64];
    __shared__ MaxI s_k[TW / 64];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int step = a.step[0];
    const TsParams& P = *a.prm;
    const int V = a.n_vocab, beg = a.beg, eot = a.eot;
    const float* lg = a.logits + (size_t)b * a.ldl;
    const int last = a.row[4 * b + 0], pen = a.row[4 * b + 1], has_ts = a.row[4 * b + 2], seek_delta = a.row[4 * b + 3];
    const bool last_ts = step > 0 && last >= beg;
    const bool pen_ts = step < 2 || pen >= beg;
    __shared__ uint32_t s_sup[VJ * TW / 32];
    stage_suppress(s_sup, a.suppress, V);
    __syncthreads();
    const MaskRule mr(P, step, eot, beg, a.blank, last_ts, pen_ts, has_ts, seek_delta);
    auto masked = [&](int n) -> bool { return mr.masked(s_sup, n); };
    // the row's logits stay in registers (VJ per thread): the maxima, the exp sums and the k
    // candidate rounds all read them there (the r3 kernel re-read the row from memory in each of
    // its k + 2 sweeps, one round trip per element: 214 us per step at beam 5,
    // profiles/r4/exp_beam_step.txt).  Same candidates, same order, same bits.
    float lv[VJ];  // this thread's logits (strided), all loads up front
#pragma unroll
    for (int j = 0; j < VJ; ++j) lv[j] = lg[min(tid + j * TW, V - 1)];
    uint64_t keep = 0;
#pragma unroll
    for (int j = 0; j < VJ; ++j) {  // branch-free: the LDS mask reads can all be in flight
        const int n = tid + j * TW;
        keep |= (uint64_t)((n < V) & !masked(min(n, V - 1))) << j;
    }
    // branch-free over the unrolled entries (a skipped entry offers {-inf, INT_MAX}, which never
    // wins a merge; a skipped exp adds +0.0f to a positive sum): the same maxima and sums, bit for
    // bit, without an exec-mask branch per entry
    const MaxI none{-INFINITY, 0x7fffffff};
    MaxI mt = none, ms = none;
#pragma unroll
    for (int j = 0; j < VJ; ++j) {
        const int n = tid + j * TW;
        const MaxI c = ((keep >> j) & 1) ? MaxI{lv[j], n} : none;
        const bool t = n < beg;
        mt = max_merge(mt, t ? c : none);
        ms = max_merge(ms, t ? none : c);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mt = max_merge(mt, MaxI{__shfl_xor(mt.v, o, 64), __shfl_xor(mt.i, o, 64)});
        ms = max_merge(ms, MaxI{__shfl_xor(ms.v, o, 64), __shfl_xor(ms.i, o, 64)});
    }
    if (lane == 0) { s_m[0][wv] = mt; s_m[1][wv] = ms; }
    __syncthreads();
    mt = s_m[0][0];
    ms = s_m[1][0];
    for (int w = 1; w < TW / 64; ++w) { mt = max_merge(mt, s_m[0][w]); ms = max_merge(ms, s_m[1][w]); }
    const float M = fmaxf(mt.v, ms.v);
    float sa = 0.0f, st = 0.0f;
    if (M > -INFINITY) {
#pragma unroll
        for (int j = 0; j < VJ; ++j) {
            const bool k_ = (keep >> j) & 1;
            const float ea = expf(lv[j] - M), et = expf(lv[j] - ms.v);
            sa += k_ ? ea : 0.0f;
            st += (k_ && tid + j * TW >= beg) ? et : 0.0f;
        }
    }
    sa = wave_sum(sa);
    st = wave_sum(st);
    __shared__ float s_t[TW / 64];
    __shared__ MaxI s_win;
    if (lane == 0) { s_s[wv] = sa; s_t[wv] = st; }
    __syncthreads();
    float za = 0.0f, zt = 0.0f;
    for (int w = 0; w < TW / 64; ++w) { za += s_s[w]; zt += s_t[w]; }
    const float lse = logf(za) + M;
    const float ts_lp = zt > 0.0f ? logf(zt) + ms.v - lse : -INFINITY;
    const bool rule = ms.v > -INFINITY && ts_lp > mt.v - lse;
    // k rounds of a block argmax over the candidates not taken yet (the rule: timestamps only);
    // the winner's owner drops it from its mask
    if (rule) {
#pragma unroll
        for (int j = 0; j < VJ; ++j)
            if (tid + j * TW < beg) keep &= ~(1ull << j);
    }
    // the winners stay in LDS until the rounds are over: a global store by thread 0 before a
    // __syncthreads() would hold every round's barrier until the store had completed (the
    // barrier's release waits on vmcnt)
    __shared__ int s_cid[8];
    __shared__ float s_clp[8];
    const int k = a.k;
    for (int r = 0; r < k; ++r) {
        MaxI c = none;
#pragma unroll
        for (int j = 0; j < VJ; ++j) c = max_merge(c, ((keep >> j) & 1) ? MaxI{lv[j], tid + j * TW} : none);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c = max_merge(c, MaxI{__shfl_xor(c.v, o, 64), __shfl_xor(c.i, o, 64)});
        if (lane == 0) s_k[wv] = c;
        __syncthreads();
        if (tid == 0) {
            MaxI m = s_k[0];
            for (int w = 1; w < TW / 64; ++w) m = max_merge(m, s_k[w]);
            const bool ok = m.v > -INFINITY && m.i < V;
            s_win = m;
            s_cid[r] = ok ? m.i : -1;
            s_clp[r] = ok ? m.v - lse : -INFINITY;  // m.v is lg[m.i]
        }
        __syncthreads();
        const MaxI w = s_win;
        if (w.v > -INFINITY && w.i % TW == tid) keep &= ~(1ull << (w.i / TW));
    }
    if (tid < k) {
        a.cand_id[b * 8 + tid] = s_cid[tid];
        a.cand_lp[b * 8 + tid] = s_clp[tid];
    }
    if (tid == 0) a.tid[b] = ms.v > -INFINITY ? ms.i : 0;
}

// self-K/V rows of the next beam step: dst row b <- src row src[b], positions [0, n_pos)
template <typename T>
__global__ __launch_bounds__(256) void kv_gather_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                        const int* __restrict__ rows, int L, int B, int H, int ctx,
                                                        const DecState* __restrict__ ds) {
    const int n_pos = ds->pos0;
    const int64_t per = (int64_t)n_pos * 64 / (16 / sizeof(T));  // 16-byte chunks per (l, kv, b, h)
    const int64_t total = (int64_t)L * 2 * B * H * per;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int64_t c = i % per;
        int64_t r = i / per;
        const int h = (int)(r % H); r /= H;
        const int b = (int)(r % B); r /= B;  // r = l * 2 + kv
        const int64_t dst_off = ((r * B + b) * H + h) * (int64_t)ctx * 64;
        const int64_t src_off = ((r * B + rows[b]) * H + h) * (int64_t)ctx * 64;
        ((uint4*)(dst + dst_off))[c] = ((const uint4*)(src + src_off))[c];
    }
}

}  // namespace

// The beam candidates over TS_CHUNKS workgroups per row (as ts_stats_kernel): each chunk writes
// its maxima, its exp sums relative to its own maxima, and its k best tokens by (logit desc, id
// asc) twice -- over every unmasked token and over the unmasked timestamps, since which set the
// row draws from (the timestamp rule) depends on the whole row.  beam_merge_kernel merges them.
static __global__ __launch_bounds__(TS_T) void beam_chunk_kernel(BeamArgs a) {
    __shared__ uint32_t s_sup[TS_T * TS_J / 32 + 2];
    __shared__ MaxI s_m[2][TS_T / 64];
    __shared__ float s_s[2][TS_T / 64];
    __shared__ MaxI s_k[TS_T / 64];
    __shared__ MaxI s_win;
    const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int step = a.step[0];
    const TsParams& P = *a.prm;
    const int V = a.n_vocab, beg = a.beg, eot = a.eot;
    const int CS = (V + TS_CHUNKS - 1) / TS_CHUNKS, n0 = c * CS, n1 = min(V, n0 + CS);
    float* out = a.stat + ((size_t)b * TS_CHUNKS + c) * BEAM_STAT;
    const int w0 = n0 >> 5, nw = n1 > n0 ? ((n1 - 1) >> 5) - w0 + 1 : 0;
    for (int w = tid; w < nw; w += TS_T) s_sup[w] = a.suppress[w0 + w];
    __syncthreads();
    const float* lg = a.logits + (size_t)b * a.ldl;
    const int last = a.row[4 * b + 0], pen = a.row[4 * b + 1], has_ts = a.row[4 * b + 2], seek_delta = a.row[4 * b + 3];
    const bool last_ts = step > 0 && last >= beg;
    const bool pen_ts = step < 2 || pen >= beg;
    const MaskRule mr(P, step, eot, beg, a.blank, last_ts, pen_ts, has_ts, seek_delta);
    float lv[TS_J];
#pragma unroll
    for (int j = 0; j < TS_J; ++j) lv[j] = lg[min(n0 + tid + j * TS_T, V - 1)];
    uint32_t keep = 0, tsk = 0;
#pragma unroll
    for (int j = 0; j < TS_J; ++j) {
        const int n = n0 + tid + j * TS_T;
        const int nc = min(n, V - 1);
        const bool sup = (s_sup[(nc >> 5) - w0] >> (nc & 31)) & 1u;
        const bool k_ = (n < n1) & !(sup | mr.masked_rules(nc));
        keep |= (uint32_t)k_ << j;
        tsk |= (uint32_t)(k_ & (n >= beg)) << j;
    }
    const MaxI none{-INFINITY, 0x7fffffff};
    MaxI mt = none, ms = none;
#pragma unroll
    for (int j = 0; j < TS_J; ++j) {
        const int n = n0 + tid + j * TS_T;
        const MaxI x = ((keep >> j) & 1) ? MaxI{lv[j], n} : none;
        const bool t = n < beg;
        mt = max_merge(mt, t ? x : none);
        ms = max_merge(ms, t ? none : x);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mt = max_merge(mt, MaxI{__shfl_xor(mt.v, o, 64), __shfl_xor(mt.i, o, 64)});
        ms = max_merge(ms, MaxI{__shfl_xor(ms.v, o, 64), __shfl_xor(ms.i, o, 64)});
    }
    if (lane == 0) { s_m[0][wv] = mt; s_m[1][wv] = ms; }
    __syncthreads();
    mt = s_m[0][0];
    ms = s_m[1][0];
    for (int w = 1; w < TS_T / 64; ++w) { mt = max_merge(mt, s_m[0][w]); ms = max_merge(ms, s_m[1][w]); }
    const float M = fmaxf(mt.v, ms.v);
    float sa = 0.0f, st = 0.0f;
#pragma unroll
    for (int j = 0; j < TS_J; ++j) {
        const float ea = expf(lv[j] - M), et = expf(lv[j] - ms.v);
        sa += ((keep >> j) & 1) ? ea : 0.0f;
        st += ((tsk >> j) & 1) ? et : 0.0f;
    }
    sa = wave_sum(sa);
    st = wave_sum(st);
    if (lane == 0) { s_s[0][wv] = sa; s_s[1][wv] = st; }
    __syncthreads();
    if (tid == 0) {
        float za = 0.0f, zt = 0.0f;
        for (int w = 0; w < TS_T / 64; ++w) { za += s_s[0][w]; zt += s_s[1][w]; }
        out[0] = mt.v; out[1] = __int_as_float(mt.i);
        out[2] = ms.v; out[3] = __int_as_float(ms.i);
        out[4] = M > -INFINITY ? za : 0.0f;
        out[5] = ms.v > -INFINITY ? zt : 0.0f;
    }
    // the chunk's k best, over everything (list 0) and over the timestamps (list 1)
    const int k = a.k;
    for (int list = 0; list < 2; ++list) {
        uint32_t kk = list ? tsk : keep;
        for (int r = 0; r < 8; ++r) {
            MaxI x = none;
            if (r < k) {
#pragma unroll
                for (int j = 0; j < TS_J; ++j) x = max_merge(x, ((kk >> j) & 1) ? MaxI{lv[j], n0 + tid + j * TS_T} : none);
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) x = max_merge(x, MaxI{__shfl_xor(x.v, o, 64), __shfl_xor(x.i, o, 64)});
                if (lane == 0) s_k[wv] = x;
                __syncthreads();
                if (tid == 0) {
                    MaxI m = s_k[0];
                    for (int w = 1; w < TS_T / 64; ++w) m = max_merge(m, s_k[w]);
                    s_win = m;
                }
                __syncthreads();
                x = s_win;
                const int jj = (x.i - n0 - tid) / TS_T;  // the owner drops its winner
                if (x.v > -INFINITY && x.i >= n0 && (x.i - n0) % TS_T == tid) kk &= ~(1u << jj);
            }
            if (tid == 0) {
                out[6 + list * 16 + 2 * r] = x.v;
                out[6 + list * 16 + 2 * r + 1] = __int_as_float(x.i);
            }
        }
    }
}

// One wavefront per row: the chunks' maxima and sums merged in chunk order (the log-softmax
// denominator and the timestamp rule), then the row's k best from the chunks' lists of the set the
// rule allows, by (logit desc, id asc), with their log-probabilities.
static __global__ __launch_bounds__(64) void beam_merge_kernel(BeamArgs a) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const float* sp = a.stat + (size_t)b * TS_CHUNKS * BEAM_STAT;
    const MaxI none{-INFINITY, 0x7fffffff};
    MaxI mt = none, ms = none;
    for (int c = 0; c < TS_CHUNKS; ++c) {
        mt = max_merge(mt, MaxI{sp[c * BEAM_STAT + 0], __float_as_int(sp[c * BEAM_STAT + 1])});
        ms = max_merge(ms, MaxI{sp[c * BEAM_STAT + 2], __float_as_int(sp[c * BEAM_STAT + 3])});
    }
    const float M = fmaxf(mt.v, ms.v);
    float za = 0.0f, zt = 0.0f;  // every lane the same sums, in chunk order
    for (int c = 0; c < TS_CHUNKS; ++c) {
        const float* q = sp + c * BEAM_STAT;
        const float mc = fmaxf(q[0], q[2]);
        if (mc > -INFINITY) za += q[4] * expf(mc - M);
        if (q[2] > -INFINITY) zt += q[5] * expf(q[2] - ms.v);
    }
    const float lse = logf(za) + M;
    const float ts_lp = zt > 0.0f ? logf(zt) + ms.v - lse : -INFINITY;
    const bool rule = ms.v > -INFINITY && ts_lp > mt.v - lse;
    const int list = rule ? 1 : 0, k = a.k;
    // candidates: chunk c's r-th entry at slot c * 8 + r; lane l holds slots l and l + 64
    MaxI cand[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int slot = lane + 64 * h, c = slot >> 3, r = slot & 7;
        const float* q = sp + c * BEAM_STAT + 6 + list * 16 + 2 * r;
        cand[h] = (c < TS_CHUNKS && r < k) ? MaxI{q[0], __float_as_int(q[1])} : none;
    }
    for (int r = 0; r < k; ++r) {
        MaxI x = max_merge(cand[0], cand[1]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x = max_merge(x, MaxI{__shfl_xor(x.v, o, 64), __shfl_xor(x.i, o, 64)});
        const bool ok = x.v > -INFINITY && x.i < a.n_vocab;
        if (lane == 0) {
            a.cand_id[b * 8 + r] = ok ? x.i : -1;
            a.cand_lp[b * 8 + r] = ok ? x.v - lse : -INFINITY;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (ok && cand[h].i == x.i) cand[h] = none;
    }
    if (lane == 0) a.tid[b] = ms.v > -INFINITY ? ms.i : 0;
}

void dec_beam_topk(const BeamArgs& a, int B, hipStream_t st) {
    if (a.k < 1 || a.k > 8) throw std::runtime_error("beam_topk: 1..8 candidates");
    if (a.n_vocab < 1 || a.n_vocab > VJ * TW) throw std::runtime_error("beam_topk: vocabulary above 53248 tokens");
    if (a.stat) {
        hipLaunchKernelGGL(beam_chunk_kernel, dim3(TS_CHUNKS, B), dim3(TS_T), 0, st, a);
        SPT_LAUNCH_CHECK();
        hipLaunchKernelGGL(beam_merge_kernel, dim3(B), dim3(64), 0, st, a);
    } else {
        hipLaunchKernelGGL(beam_topk_kernel, dim3(B), dim3(TW), 0, st, a);
    }
    SPT_LAUNCH_CHECK();
}

void dec_kv_gather(int dtype, const void* src, void* dst, const int* rows, int L, int B, int H, int ctx,
                   const DecState* ds, hipStream_t st) {
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(kv_gather_kernel<bf16>, dim3(2048), dim3(256), 0, st, (const bf16*)src, (bf16*)dst, rows, L, B,
                           H, ctx, ds);
    else
        hipLaunchKernelGGL(kv_gather_kernel<float>, dim3(2048), dim3(256), 0, st, (const float*)src, (float*)dst, rows, L,
                           B, H, ctx, ds);
    SPT_LAUNCH_CHECK();
}

void dec_ts_stats(const TsArgs& a, int B, hipStream_t st) {
    if (a.n_vocab < 1 || a.n_vocab > TS_CHUNKS * TS_T * TS_J) throw std::runtime_error("ts_stats: vocabulary above 53248 tokens");
    if (!a.stat) throw std::runtime_error("ts_stats: no statistics buffer");
    hipLaunchKernelGGL(ts_stats_kernel, dim3(TS_CHUNKS, B), dim3(TS_T), 0, st, a);
    SPT_LAUNCH_CHECK();
}

void dec_finalize_ts(int dtype, const TsArgs& a, int B, hipStream_t st) {
    if (!a.stat) throw std::runtime_error("finalize_ts: no chunk statistics (dec_ts_stats)");
    if (a.n_vocab < 1 || a.n_vocab > VJ * TW) throw std::runtime_error("finalize_ts: vocabulary above 53248 tokens");
    if (dtype == DT_BF16) hipLaunchKernelGGL(finalize_ts_kernel<bf16>, dim3(B), dim3(TW), 0, st, a);
    else hipLaunchKernelGGL(finalize_ts_kernel<float>, dim3(B), dim3(TW), 0, st, a);
    SPT_LAUNCH_CHECK();
}

}  // namespace spt
