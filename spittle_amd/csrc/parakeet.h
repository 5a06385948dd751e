// parakeet.h -- the device-resident Parakeet-V3 (FastConformer encoder + TDT greedy) engine
// behind the spt_parakeet_* C ABI.  Replaces transcribe-rs' ParakeetEngine as Spittle drives it:
// load_model_with_params(path, ParakeetModelParams::int8()) (/root/reference/src-tauri/src/
// managers/transcription.rs:278-297) and transcribe_samples(audio, Some(ParakeetInferenceParams
// { timestamp_granularity: Segment, .. })) (transcription.rs:505-513).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "pk_kernels.h"

namespace spt {

struct PkDims {
    std::string name;
    int n_mels = 128, d = 1024, n_layers = 24, n_heads = 8, ff = 4096, sub_ch = 256, conv_k = 9;
    int pred = 640, n_vocab = 8192, n_dur = 5;
};

// "synthetic:parakeet-tdt-0.6b-v3[:layers=N][:seed=S]" or "synthetic:parakeet-test-small[...]";
// false if the spec is not synthetic
bool parse_parakeet_spec(const std::string& spec, PkDims* dm, uint64_t* seed, std::string* err);

struct PkUtt {                  // one utterance's TDT greedy output
    std::vector<int> tok, frame;  // token ids and the encoder frame (80 ms) each was emitted at
    std::vector<float> top1, top2;  // the token's joint logit and the runner-up's
};

// encoder stage classes of profile_encoder (spt_pk_stage in include/spittle_hip.h)
enum { PK_ST_SUB = 0, PK_ST_POS, PK_ST_LN, PK_ST_FFN, PK_ST_QKVO, PK_ST_ATTN, PK_ST_CONV_PW, PK_ST_CONV_DW,
       PK_ST_JOINT, PK_ST_COUNT };

struct PkTimings {
    double mel_ms = 0, encoder_ms = 0, decode_ms = 0, total_ms = 0, h2d_ms = 0;
    int n_steps = 0, batch = 0, enc_frames = 0;
};

class ParakeetEngine {
public:
    // max_samples: the longest utterance one call takes (longer ones are cut by the caller)
    ParakeetEngine(const PkDims& dm, int dtype, int device, int max_batch, int max_samples, uint64_t seed,
                   bool synthetic_weights = true);
    ~ParakeetEngine();
    ParakeetEngine(const ParakeetEngine&) = delete;
    ParakeetEngine& operator=(const ParakeetEngine&) = delete;

    const PkDims& dims() const { return dm_; }
    int dtype() const { return dt_; }
    int max_batch() const { return max_batch_; }
    int max_samples() const { return max_samples_; }
    // grow the workspace so one pass takes utterances of n samples (the app decodes a whole
    // recording in one pass: transcription.rs:505-513); graphs captured on the old workspace are
    // dropped.  Returns false, with the old workspace kept, if the larger one does not fit in
    // max_bytes (or in device memory).
    bool reserve_samples(int n, int64_t max_bytes);
    int64_t weight_bytes() const { return wbytes_; }
    int64_t workspace_bytes() const { return abytes_; }
    const PkTimings& timings() const { return tm_; }

    // load one weight tensor by id (oracle/po_model.c's table; f32 host data in the tensor's
    // canonical NeMo layout) -- the path real checkpoints take
    void set_tensor(int tid, const float* host, int64_t n);
    bool has_tensor(int tid) const { return table_.count(tid) != 0; }
    std::vector<int> tensor_ids() const {
        std::vector<int> v;
        for (auto& kv : table_) v.push_back(kv.first);
        return v;
    }
    int64_t tensor_numel(int tid) const;

    // B utterances, pcm_dev + b * stride (device); n[b] <= max_samples
    void transcribe_device(const float* pcm_dev, int64_t stride, const int* n, int B, int max_symbols,
                           std::vector<PkUtt>* out);
    void transcribe_host(const float* const* pcm, const int* n, int B, int max_symbols, std::vector<PkUtt>* out);

    void debug_mel(const float* pcm_host, int n, float* out_host);                 // [n_mels][T]
    void debug_encode(const float* mel_host, int T, float* out_host);              // [T3][d] (f32)
    // TDT greedy decoding of a given encoder output [T3][d] (f32 host): the decoder alone
    void debug_decode(const float* enc_host, int T3, int max_symbols, PkUtt* out);
    // the encoder output rows [T3][d] (f32) of batch row b of the last transcribe call; returns T3
    int debug_last_encoder(int b, float* out_host);
    // measurement: re-run the last call's encoder pass `iters` times eagerly (same buffers and
    // shape, bitwise the same output) with a HIP event after every launch; ms[c] = mean time per
    // pass spent in stage class c (PK_ST_*)
    void profile_encoder(int iters, double ms[PK_ST_COUNT]);
    bool debug_weight_checksum(int tid, double* out2);

private:
    struct TSpec {
        int tid; int64_t n; int kind; int exp;      // generator
        int mode; int dt; void* dst;                // placement
        int N, K, ld, row0;
    };
    struct Layer {
        float *ln1_w, *ln1_b; void *ff1_w1; float* ff1_b1; void* ff1_w2; float* ff1_b2;
        float *lna_w, *lna_b; void* qkv_w; float* qkv_b; void* o_w; float* o_b; float *pos_u, *pos_v;
        float *lnc_w, *lnc_b; void* pw1_w; float* pw1_b; float *dw_w, *dw_b, *bn_g, *bn_b, *bn_m, *bn_v;
        void* pw2_w; float* pw2_b;
        float *ln2_w, *ln2_b; void *ff2_w1; float* ff2_b1; void* ff2_w2; float* ff2_b2;
        float *lno_w, *lno_b;
    };
    struct GraphKey {  // decode-step graphs: shape-free in the utterance length (PkState::t3p)
        int B, max_symbols;
        bool operator<(const GraphKey& o) const {
            if (B != o.B) return B < o.B;
            return max_symbols < o.max_symbols;
        }
    };

    void select() const;
    void release();
    void alloc_weights();
    void alloc_workspace();
    void set_frame_limits();  // Tmax_ .. T3max_, cap_ from max_samples_
    void upload_tables();
    void place(const TSpec& t, const float* src_dev);
    void frame_counts(const int* n, int B, std::vector<int>* lens, int* Tp, int* T1p, int* T2p, int* T3p) const;
    void run_mel(const float* pcm_dev, int64_t stride, int B, int Tp);
    void run_encoder(int B, int Tp, int T1p, int T2p, int T3p);
    void encode(int B, int Tp, int T1p, int T2p, int T3p);  // run_encoder, graph-replayed for repeated shapes
    int gemm(int dt, int epi, const void* A, int lda, const void* W, int ldw, int M, int N, int K, const float* bias,
             void* Cp, int ldc, float alpha = 1.0f);
    void run_decode(int B, int T3p, int max_symbols, std::vector<PkUtt>* out);
    void enqueue_step(int B, int max_symbols, int cap, int parity);

    PkDims dm_;
    int dt_, dev_, max_batch_, max_samples_;
    uint64_t seed_;
    int esz_;
    int F1_, F2_, F3_;               // frequency bins after each stride-2 stage
    int Tmax_, T1max_, T2max_, T3max_;
    int P_pad_, joint_pad_, joint_tiles_;  // W^T row lengths (multiples of 64), joint workgroups
    hipStream_t st_ = nullptr;
    std::vector<hipEvent_t> ev_;

    // ---- weights
    char* warena_ = nullptr;
    int64_t wbytes_ = 0;
    std::vector<TSpec> specs_;
    std::map<int, size_t> table_;    // tid -> specs_ index
    float *c0_w_, *c0_b_, *dw1_w_, *dw1_b_, *dw2_w_, *dw2_b_, *pw1_b_, *pw2_b_, *sub_b_;
    void *pw1_w_, *pw2_w_, *sub_w_, *pos_w_;  // pos_w_: every layer's linear_pos [L][d][d]
    std::vector<Layer> L_;
    float* emb_;
    float *lstm_wt_[2], *lstm_bih_[2], *lstm_bhh_[2];
    float *jenc_w_, *jenc_b_, *jpred_wt_, *jpred_b_, *jout_wt_, *jout_b_;

    // ---- tables
    float *win_ = nullptr, *basis_ = nullptr, *fbT_ = nullptr;

    // ---- workspace
    char* aarena_ = nullptr;
    int64_t abytes_ = 0;
    float* pcm_ = nullptr;
    // pinned host staging of transcribe_host's PCM: one DMA instead of a pageable copy per window
    float* pin_ = nullptr;
    size_t pin_cap_ = 0;  // floats
    // pinned read-back of the decode state and of the emitted tokens (rows trimmed to the longest)
    PkState* hst_pin_ = nullptr;
    int hst_cap_ = 0;
    int* res_pin_ = nullptr;
    size_t res_cap_ = 0;  // 4-byte elements
    int *nsamp_ = nullptr, *lens_ = nullptr;
    float *frames_ = nullptr, *spec_ = nullptr, *mel_ = nullptr;
    void *y1_ = nullptr, *y2a_ = nullptr, *y2_ = nullptr, *y3a_ = nullptr, *y3_ = nullptr;
    float* x_ = nullptr;
    void mark(int cls);           // profile_encoder: event after the launch(es) of stage class cls
    std::vector<hipEvent_t> prof_ev_;
    std::vector<int> prof_cls_;
    bool prof_on_ = false;
    int last_dims_[5] = {0, 0, 0, 0, 0};  // the last call's B, Tp, T1p, T2p, T3p
    std::vector<int> last_lens_;  // the last transcribe call's per-row lengths {T, T1, T2, T3}
    int last_T3p_ = 0;
    float* enc_out_ = nullptr;  // the residual buffer holding the last call's encoder output
    void *xn_ = nullptr, *ffh_ = nullptr, *qkv_ = nullptr, *pe_ = nullptr, *pp_ = nullptr, *ctx_ = nullptr;
    void *glu_ = nullptr, *cv_ = nullptr;
    float* fe_ = nullptr;
    float* slab_ = nullptr;          // split-K partial products of the residual GEMMs [ks][M][d]
    PkState* state_ = nullptr;
    float *h_ = nullptr, *c_ = nullptr, *gp_ = nullptr;
    float *xemb_ = nullptr, *fecur_ = nullptr;  // next step's LSTM-0 input rows, current-frame rows
    float4* jpart_ = nullptr;
    float* dur_ = nullptr;
    int *out_tok_ = nullptr, *out_frame_ = nullptr;
    float *out_t1_ = nullptr, *out_t2_ = nullptr;
    int cap_ = 0;
    float* scratch_ = nullptr;       // f32 staging of one weight tensor
    int64_t scratch_n_ = 0;
    double* dsum_ = nullptr;
    std::map<GraphKey, hipGraphExec_t> graphs_;
    std::map<std::pair<int, int>, hipGraphExec_t> enc_graphs_;  // (B, Tp) -> encoder graph
    std::map<std::pair<int, int>, int> enc_seen_;
    std::map<std::pair<int, int>, float*> enc_out_graph_;
    std::vector<PkState> hstate_;

    PkTimings tm_;
};

}  // namespace spt
