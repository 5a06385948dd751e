// engine.h -- the device-resident Whisper engine behind the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <set>
#include <string>
#include <vector>

#include "kernels.h"
#include "vocab.h"

namespace spt {

class GgmlFile;

struct ModelDims {
    std::string name;
    int n_mels = 80, d = 384, n_head = 6, n_enc = 4, n_dec = 4, n_vocab = 51864;
    int n_audio_ctx = 1500, n_text_ctx = 448;
};


struct DecodeRequest {
    std::vector<int> prompt;    // [sot, (lang, task,) notimestamps]: shared by every sequence
    std::vector<int> prefix;    // whisper_full prompt_past ([prev] + prompt tokens), prefilled first
    // per sequence (empty = prompt as given): >= 0 the language token for prompt[1]; -(s + 1)
    // the token detected (whisper_lang_auto_detect) on sequence s of this batch
    std::vector<int> lang_tok;
    int n_steps = 128;
    uint32_t flags = 3;         // SUPPRESS_BLANK | NO_TIMESTAMPS
    const int32_t* forced = nullptr;
    int n_forced = 0;
    // whisper_full decoding (k_sample.hip): timestamps, temperature sampling, per-decoder
    // bookkeeping.  Off: the no-timestamp greedy fast path.  On: tokens as usual, top1 = the
    // token's log-probability (plog), top2 = its timestamp id (tid, as a float).
    bool full = false;
    TsParams ts{};
    std::vector<int> seek, seek_end;           // [B] 10 ms frames
    std::vector<std::vector<int>> row_prefix;  // per-sequence prompt_past (equal lengths); else prefix
    std::vector<int> extra_suppress;           // e.g. the non-speech tokens of the vocabulary
    int blank_tok = 220;                       // " " (suppress_blank)
    int beam_k = 0;                            // > 0: beam search, host-driven (beam_begin / beam_next)
    // per row: the encoded window (cross K/V row of the last encode_windows) it attends to; empty =
    // row b attends to window b.  Rows sharing a window are consecutive runs of equal length (the
    // decoders of one utterance: beam_size / best_of), so one workgroup reads a window's K/V once
    // for all of them.
    std::vector<int> kv_row;
};

// per-row beam candidates of one step (k <= 8 per row)
struct BeamCands {
    std::vector<int> id;     // [B][8], -1 = none
    std::vector<float> lp;   // [B][8] log-probabilities
    std::vector<int> tid;    // [B] most probable timestamp
};

struct Timings {
    double mel_ms = 0, encoder_ms = 0, cross_kv_ms = 0, decode_ms = 0, total_ms = 0, h2d_ms = 0;
    int n_decode_passes = 0, batch = 0;
};

// everything one C-ABI call ran (a whisper_full call: every window batch, temperature fallback
// and beam step), summed; reset by the C ABI at the start of each spt_transcribe* call
struct CallStats {
    int engine_calls = 0, decoder_passes = 0, beam_steps = 0, encoder_windows = 0;
    int pd_passes = 0;     // ABI 12 counters of the persistent decoder pass (deleted in round 6): always 0
    int pd_fallbacks = 0;
    double device_ms = 0, encoder_ms = 0, decode_ms = 0;
};

class Engine {
public:
    // src == nullptr: synthetic weights from `seed`; else the weights, mel filters of a ggml file
    // (dm from ggml_dims(*src)); the file is read during construction only
    // external_weights: allocate the weight arena but leave it unfilled; import_weights() (e.g.
    // the bytes of rank 0's arena after an RCCL broadcast) makes the engine usable
    Engine(const ModelDims& dm, int dtype, int device, int max_batch, uint64_t seed, const GgmlFile* src = nullptr,
           bool external_weights = false);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    const ModelDims& dims() const { return dm_; }
    int dtype() const { return dt_; }
    int max_batch() const { return max_batch_; }
    int max_rows() const { return max_rows_; }  // decoder rows one pass carries (beam search: one group)
    int64_t weight_bytes() const { return wbytes_; }
    bool weights_ready() const { return weights_ready_; }
    // D2D copies of the whole weight arena (device pointers on this engine's device, or any
    // peer-accessible one); the arena layout is a pure function of (dims, dtype, n_mels padding),
    // so two engines of one model exchange their weights byte for byte
    void export_weights(void* dev_dst, int64_t bytes);
    void import_weights(const void* dev_src, int64_t bytes);
    // the arena itself (a collective writes rank 0's bytes straight into it), then
    // commit_weights() marks an external-weights engine usable
    void* weight_arena() const { return warena_; }
    int device() const { return dev_; }
    void commit_weights();
    int64_t workspace_bytes() const { return abytes_; }
    const Timings& timings() const { return tm_; }
    const CallStats& call_stats() const { return cs_; }
    void reset_call_stats() { cs_ = CallStats(); }

    // ---- staged calls: utterances -> encoder windows -> decoder rows (whisper.cpp whisper_full:
    // whisper_pcm_to_mel once per input, whisper_encode_internal once per window at `seek`, then
    // the decoders of every temperature / beam share that window's cross K/V)
    // 1. the log-mel of each WHOLE utterance on the device: 200-sample reflective head from the
    //    utterance itself, (n + 480000) / 160 frames, the utterance's global max - 8 clamp.  Replaces
    //    the previous set.  Host PCM is staged into a device buffer; device PCM is read in place
    //    (utterance u at pcm_dev + u * stride, n[u] <= stride).
    void load_utterances(const float* const* pcm_host, const int* n, int U);
    void load_utterances_device(const float* pcm_dev, int64_t stride, const int* n, int U);
    // 2. encoder rows e < E (<= max_batch): mel frames [seek[e], seek[e] + 3000) of utterance utt[e]
    //    -> conv stem -> encoder -> cross K/V of every decoder layer; kept until the next call
    void encode_windows(const int* utt, const int* seek, int E);
    int encoded_windows() const { return enc_E_; }
    // 3. decode B rows (<= max_batch) over the encoded windows (rq.kv_row).  tokens/top1/top2:
    //    host [B][n_steps]; lang_out (optional, [B]): the language token each row was decoded with
    //    (-1: none); ts_state_out (optional, [B][4], whisper_full mode): has_ts, seek_delta,
    //    result_len, status (0 running, 1 completed, 2 failed) of each row's decoder
    void decode(int B, const DecodeRequest& rq, int* tokens, float* top1, float* top2, int* lang_out = nullptr,
                int* ts_state_out = nullptr);

    // the three stages for B utterances that are one window each (seek 0), decoder row b on window b
    // pcm_dev: B windows at pcm_dev + b * stride (device memory)
    void transcribe_device(const float* pcm_dev, int64_t stride, const int* n_samples, int B, const DecodeRequest& rq,
                           int* tokens, float* top1, float* top2, int* lang_out = nullptr, int* ts_state_out = nullptr);
    void transcribe_host(const float* const* pcm, const int* n_samples, int B, const DecodeRequest& rq, int* tokens,
                         float* top1, float* top2, int* lang_out = nullptr, int* ts_state_out = nullptr);

    // beam search (whisper_full, beam strategy) over the encoded windows: prefix and prompt pass of
    // B decoder rows (rq.beam_k candidates each, rq.kv_row their windows) -> the first step's
    // candidates; then one step per call: row b continues row src[b]'s sequence with tokens[b];
    // rowstate [B][4] = last token, previous token, has_ts, seek_delta; step = index of the token
    // being chosen
    void beam_begin(int B, const DecodeRequest& rq, BeamCands* out, int* lang_out);
    void beam_next(const int* src, const int* tokens, const int* rowstate, int step, BeamCands* out);

    // the normalised log-mel [n_mels][3000] of the window at frame `seek` of one utterance
    void debug_mel(const float* pcm_host, int n, int seek, float* out_host);
    void debug_encode(const float* mel_host, float* out_host);
    bool debug_weight_checksum(int tid, double* out2);
    // re-launch one hot-path kernel on the last call's buffers; returns avg us per launch
    double probe(int kind, int iters, double* work, int* is_flops);

private:
    struct GraphKey {
        int B, B_total, b0, out_cap, n_forced;
        uint32_t flags;
        bool full;
        int share = 0;  // rows per window (0: identity rows, no window map)
        bool operator<(const GraphKey& o) const {
            if (full != o.full) return full < o.full;
            if (B != o.B) return B < o.B;
            if (share != o.share) return share < o.share;
            if (B_total != o.B_total) return B_total < o.B_total;
            if (b0 != o.b0) return b0 < o.b0;
            if (out_cap != o.out_cap) return out_cap < o.out_cap;
            if (n_forced != o.n_forced) return n_forced < o.n_forced;
            return flags < o.flags;
        }
    };
    // An independent slice of the batch decoded on its own stream: its kernels fill
    // the launch gaps of the other group's latency-bound decoder chain.
    struct DecGroup {
        hipStream_t st = nullptr;
        hipEvent_t ev = nullptr;
        int b0 = 0, B = 0;
        float* dx = nullptr;
        void *dq = nullptr, *dao = nullptr, *dff = nullptr;
        void* skv = nullptr;          // self K/V [L][2][B][H][ctx][64]
        float* logits = nullptr;
        void* part = nullptr;         // logits top-2 partials [B][V/16]
        unsigned* arrive = nullptr;
        int *tok_in = nullptr, *out_tok = nullptr, *done = nullptr, *forced = nullptr;
        float *out_t1 = nullptr, *out_t2 = nullptr;
        DecState* ds = nullptr;
        float* dx2 = nullptr;         // second residual buffer (ping-pong with dx)
        float* pend = nullptr;        // pending partial slabs [kMaxPend][R][d]
        float* xpart = nullptr;       // cross-attention chunk partials [R][H][<=4][66]
        int *seek = nullptr, *seek_end = nullptr, *ts_state = nullptr;  // whisper_full decoding
        float* ts_stat = nullptr;     // [B][TS_CHUNKS][6] per-chunk vocabulary statistics (dec_ts_stats)
        float* beam_stat = nullptr;   // [B][TS_CHUNKS][BEAM_STAT] per-chunk statistics and beam candidates
        TsParams* prm = nullptr;
        int *beam_row = nullptr, *beam_step = nullptr, *beam_src = nullptr;  // beam search
        int *cand_id = nullptr, *beam_tid = nullptr;
        float* cand_lp = nullptr;
        int* kvrow = nullptr;         // [B] encoded window of each row (window map)
        int share = 0;                // rows per window of this call (0: identity, no map)
        std::map<GraphKey, hipGraphExec_t> graphs;
        std::vector<int> host_tok;    // host sources of the call's token uploads
        size_t host_used = 0;
    };

    void select() const;
    void release();
    void alloc_weights();
    void generate_weights();
    void load_ggml(const GgmlFile& f);
    void alloc_workspace();
    void upload_tables(const std::vector<float>* filters);
    void run_mel_utts(const float* pcm, const std::vector<int64_t>& pcm_off, const int* n, int U);
    void upload_windows(const int* utt, const int* seek, int E);
    void finish_call_timing();
    void run_encoder(int B);
    void enc_layer(int l, int Bg, int64_t r0, hipStream_t s, int probe = 0, hipEvent_t e0 = nullptr,
                   hipEvent_t e1 = nullptr);
    int enc_groups_cur_ = 1;  // window groups of the encoder run being enqueued (GemmArgs::groups)
    void enqueue_encoder(int B);  // run_encoder, replayed from a per-B graph after the first call
    void run_cross_kv(int B);
    void run_decode(int B, const DecodeRequest& rq, int* tokens, float* top1, float* top2, int* lang_out,
                    int* ts_state_out);
    // E: encoded windows (the cross K/V layout); g.share / g.kvrow: the rows' window map
    void enqueue_decoder_pass(DecGroup& g, int E, int Tq, const DecodeRequest& rq, int out_cap);
    float* enqueue_layers(DecGroup& g, int E, int Tq);
    void enqueue_head(DecGroup& g, int Tq, const DecodeRequest& rq, int out_cap, float* xc, const uint32_t* sup,
                      bool blank);

    ModelDims dm_;
    int dt_, dev_, max_batch_;
    uint64_t seed_;
    int esz_;     // bytes per weight / activation element
    int cp_;      // padded mel channels (conv1 K = 3 * cp_)
    static constexpr int fc2_split_ = 2;  // K split of the fc2 projection (pending slabs)
    // fc2's first split adds the residual into its slab, so the next LayerNorm prologue reads
    // slab 0 + the other slabs instead of x + all of them (SPT_DEC_XFOLD=0: off; read when a pass
    // is captured, by enqueue_layers, and used by the head that follows it)
    bool pend_fold_ = true;
    // the LayerNorm source over the residual xc and np pending slabs at pend (slab stride `slab`)
    void ln_source(GemvArgs& a, float* xc, float* pend, int np, int64_t slab) const;
    int xsplit_ = 1;  // cross-attention key chunks per (b, h) (merged by the output projection)
    int n_groups_ = 1;
    int max_rows_ = 64;  // decoder rows per pass (gemv_max_image_rows); larger batches use more groups  // SPT_DECODE_GROUPS=2 splits the batch over two streams
    hipStream_t st_ = nullptr;
    std::vector<hipEvent_t> ev_;
    // the encoder's window groups (run_encoder): groups 1.. run on these streams beside group 0 on
    // st_; enc_ev_[0] forks them off st_, enc_ev_[i] joins group i back
    static constexpr int kEncGroupsMax = 4;
    std::vector<hipStream_t> enc_st_;
    std::vector<hipEvent_t> enc_ev_;
    int enc_groups(int B) const;
    // probe(): the decoder kernel kind timed in situ by an eager enqueue_layers (-1: none), and
    // its event pair per layer
    int probe_kind_ = -1;
    std::vector<hipEvent_t> probe_ev_;

    // ---- weights (one arena)
    char* warena_ = nullptr;
    int64_t wbytes_ = 0;
    bool weights_ready_ = false;
    void require_weights() const;
    struct EncL { float *ln1_w, *ln1_b; void* qkv_w; float* qkv_b; void* o_w; float* o_b; float *ln2_w, *ln2_b;
                  void* fc1_w; float* fc1_b; void* fc2_w; float* fc2_b; };
    struct DecL { float *ln1_w, *ln1_b; void* qkv_w; float* qkv_b; void* so_w; float* so_b; float *ln2_w, *ln2_b;
                  void* cq_w; float* cq_b; void* co_w; float* co_b; float *ln3_w, *ln3_b; void* fc1_w; float* fc1_b;
                  void* fc2_w; float* fc2_b; };
    void *conv1_w_, *conv2_w_, *ckv_w_, *tok_emb_;
    float *conv1_b_, *conv2_b_, *enc_pos_, *lnp_w_, *lnp_b_, *ckv_b_, *dec_pos_, *lnf_w_, *lnf_b_;
    std::vector<EncL> enc_;
    std::vector<DecL> dec_;
    struct TRef { void* p; int64_t n; int dt; };
    std::map<int, TRef> tref_;
    // (batch size, window groups) -> captured encoder (enqueue_encoder), and the keys whose first,
    // eager encoder call ran
    std::map<std::pair<int, int>, hipGraphExec_t> enc_graphs_;
    std::set<std::pair<int, int>> enc_seen_;

    // ---- tables
    float *hann_ = nullptr, *sinv_ = nullptr, *cosv_ = nullptr, *filt_ = nullptr;
    int* grp_ = nullptr;

    // ---- workspace (one arena)
    char* aarena_ = nullptr;
    int64_t abytes_ = 0;
    int *win_utt_ = nullptr, *win_seek_ = nullptr;  // [max_batch] encoder windows
    void* mel_in_ = nullptr;
    void* y1p_ = nullptr;
    float* x_ = nullptr;
    void *xn_ = nullptr, *qkv_ = nullptr, *ao_ = nullptr, *ff_ = nullptr, *enc_out_ = nullptr;
    void* ckv_ = nullptr;   // cross K/V, per layer [47][B][H][2][32][64] (kernels.h kv_offset)
    uint32_t* suppress_ = nullptr;
    uint32_t* suppress_lang_ = nullptr;  // all but the language tokens (language detection)
    bool suppress_lang_ready_ = false;
    double* scratch_ = nullptr;
    float* zero_ = nullptr;  // [R][d] zeros: the operand of an unused pending slab
    std::vector<DecGroup> groups_;

    std::vector<uint32_t> host_suppress_;
    uint32_t suppress_flags_ = ~0u;
    std::vector<int> suppress_extra_;
    std::vector<int> ts_init_;
    DecodeRequest beam_rq_;      // the request of the beam search in progress
    int beam_B_ = 0;
    int beam_side_ = 0;          // the self-K/V side holding the search's rows: 0 the group's cache, 1 kvtmp_
    void* kvtmp_ = nullptr;      // self-K/V reorder scratch (allocated on first beam search)
    std::vector<int> beam_host_;  // host image of the per-step uploads (beam_row .. beam_src)
    std::vector<int> beam_tok_;   // host source of the step's tokens
    std::vector<char> beam_rd_;   // host image of cand_id .. beam_tid
    void read_cands(int B, BeamCands* out);

    // ---- utterances of load_utterances (grown on demand, outside the arenas)
    float* upcm_ = nullptr;      // staged host PCM
    int64_t upcm_cap_ = 0;       // samples
    float* umel_ = nullptr;      // log10-mel rows of every utterance [rows][n_mels]
    int64_t umel_cap_ = 0;       // rows
    char* uinfo_ = nullptr;      // [U] pcm_off (int64), row_off (int64), n (int), max key (unsigned)
    int uinfo_cap_ = 0;
    MelUtts mu_{};
    unsigned* umax_ = nullptr;
    std::vector<int> un_;        // samples per utterance (host)
    std::vector<int64_t> uhost_; // pcm / row offsets (host)
    std::vector<char> mel_img_;  // host source of the descriptor upload
    std::vector<int> whost_;     // host source of the window upload
    std::vector<int> kvrow_host_;  // host source of the rows' window map upload
    int enc_E_ = 0;              // windows encoded by the last encode_windows
    bool mel_pending_ = false, enc_pending_ = false;  // stages whose events the next decode reads
    void ensure_capacity(void** p, int64_t* cap, int64_t need, size_t esz, const char* what);

    Timings tm_;
    CallStats cs_;
};

// model dimensions of a ggml file's hparams; false + *err if the engine cannot run it
bool ggml_dims(const GgmlFile& f, ModelDims* dm, std::string* err);

// parse "synthetic:<model>[:enc=N][:dec=N][:seed=S]"; returns false if not synthetic
bool parse_synthetic_spec(const std::string& spec, ModelDims* dm, uint64_t* seed, std::string* err);

}  // namespace spt
