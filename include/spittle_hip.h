/*
 * spittle_hip.h -- C ABI of the MI355X-native Whisper transcription backend.
 *
 * This is the drop-in boundary for Spittle's transcription hot path.  In the
 * reference, TranscriptionManager owns a transcribe_rs::engines::whisper::WhisperEngine
 * through `LoadedEngine::Whisper` (/root/reference/src-tauri/src/managers/transcription.rs:29-34)
 * and calls, from different OS threads but serialised by one Mutex
 * (transcription.rs:36-47, 437):
 *
 *   WhisperEngine::new() + load_model(&path)     transcription.rs:261-276  -> spt_ctx_create
 *   transcribe_samples(Vec<f32>, Some(params))   transcription.rs:494-503  -> spt_transcribe
 *   unload_model() / Drop                         transcription.rs:175-208  -> spt_ctx_destroy
 *
 * with WhisperInferenceParams { language, translate, initial_prompt, ..Default }
 * (transcription.rs:445-499) -> spt_infer_params, and TranscriptionResult.text
 * (transcription.rs:537-546) -> spt_result.text.  The Rust binding a maintainer
 * adds (spittle-hip-sys / HipWhisperEngine) is shown in INTEGRATION.md.
 *
 * Conventions (same as the in-tree Swift bridge,
 * src-tauri/swift/apple_intelligence_bridge.h:10-24): plain pointers and sizes,
 * status codes plus a message, library-owned results released by
 * spt_result_free.  Input PCM is borrowed for the duration of the call (16 kHz
 * mono f32 in [-1, 1]).  A context is not thread-affine (every entry point
 * selects its device) but is not re-entrant: callers serialise, as the app does.
 */
#ifndef SPITTLE_HIP_H
#define SPITTLE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPT_ABI_VERSION 12

typedef enum {
    SPT_OK = 0,
    SPT_ERR_INVALID_ARG = 1,   /* bad pointer / size / parameter */
    SPT_ERR_LOAD = 2,          /* model spec or file could not be loaded */
    SPT_ERR_DEVICE = 3,        /* HIP runtime / device failure */
    SPT_ERR_OOM = 4,           /* device allocation failed */
    SPT_ERR_UNSUPPORTED = 5,   /* feature not implemented (e.g. beam search) */
    SPT_ERR_INTERNAL = 6
} spt_status;

typedef enum { SPT_DTYPE_F32 = 0, SPT_DTYPE_BF16 = 1, SPT_DTYPE_F16 = 2 /* Parakeet only */ } spt_dtype;

/* decode flags (spt_infer_params.flags) */
#define SPT_SUPPRESS_BLANK  1u  /* whisper_full_params.suppress_blank (default on) */
#define SPT_NO_TIMESTAMPS   2u  /* whisper_full_params.no_timestamps */
#define SPT_IGNORE_EOT      4u  /* benchmark protocol: keep decoding past <|endoftext|> */
#define SPT_SUPPRESS_NST    8u  /* whisper_full_params.suppress_non_speech_tokens (ggml models) */

typedef struct {
    int32_t dtype;        /* spt_dtype: weights + activations (accumulation is always f32) */
    int32_t device;       /* HIP device ordinal */
    int32_t max_batch;    /* utterance (30 s window) capacity per call */
    uint32_t flags;       /* SPT_MODEL_* (ABI <= 3: reserved, always 0) */
    uint64_t seed;        /* synthetic weights: PRNG seed */
} spt_model_params;

/* spt_model_params.flags */
#define SPT_MODEL_WEIGHTS_EXTERNAL 1u  /* allocate the weight arena but do not generate / dequantise
                                          into it: spt_weights_import fills it (a multi-GPU load
                                          where rank 0 loads and RCCL broadcasts the arena) */

typedef struct {
    const char* language;        /* ISO-639-1 ("en", "zh", ...); NULL or "auto" = auto-detect
                                    (whisper_lang_auto_detect on the utterance's first 30 s) */
    int32_t translate;           /* task <|translate|> instead of <|transcribe|> */
    const char* initial_prompt;  /* jargon prompt text (src-tauri/src/jargon.rs:594); ggml models */
    uint32_t flags;              /* SPT_SUPPRESS_BLANK | SPT_NO_TIMESTAMPS | SPT_SUPPRESS_NST |
                                    SPT_IGNORE_EOT; default SPT_SUPPRESS_BLANK (whisper_full's
                                    defaults: timestamps on) */
    int32_t max_new_tokens;      /* fast path: generated tokens per 30 s window (<= 220);
                                    whisper_full path: whisper_full_params.max_tokens (0 = none) */
    float temperature;           /* initial temperature (0 = greedy) */
    int32_t beam_size;           /* 1: greedy; 2..8: beam search at temperature 0 (one decoder row
                                    per beam: <= max_batch; whisper_full path) */
    const int32_t* forced_tokens;/* test hook (teacher forcing): [batch][n_forced] or NULL */
    int32_t n_forced;
    const int32_t* prompt_tokens;/* whisper_full_params.prompt_tokens: decoded before [sot ...] as
                                    [prev] + the last min(224, n) of them; NULL = none */
    int32_t n_prompt_tokens;
    /* ABI 3: whisper_full's window loop (timestamps, segments, temperature fallback).  A call
     * takes the device-resident no-timestamp greedy fast path when SPT_NO_TIMESTAMPS is set,
     * temperature_inc == 0, temperature == 0 and beam_size <= 1; every other call runs whisper_full. */
    float temperature_inc;       /* fallback step (0.2); 0 = no fallback */
    int32_t best_of;             /* sampled decoders per window at temperature > 0 (5) */
    float entropy_thold;         /* a decoder whose last 32 tokens' entropy is lower fails (2.4) */
    float logprob_thold;         /* fall back when the average log-probability is lower (-1.0) */
    float max_initial_ts;        /* the first timestamp is at most this many seconds (1.0) */
    /* whisper_full_params.no_speech_thold has no counterpart: whisper.cpp 1.7.1 (vendored by
     * whisper-rs-sys 0.11.1, the reference's engine) declares it "TODO: not implemented" and never
     * reads it, so the reference skips no window for no-speech probability [recalled; whisper.cpp
     * is not in /root/reference].  A later whisper.cpp's skip would be added here, not emulated. */
    int32_t reserved0;
    uint64_t seed;               /* temperature sampling stream */
} spt_infer_params;

typedef struct {
    int64_t t0, t1;              /* whisper_full_get_segment_t0 / t1: 10 ms units */
    char* text;                  /* whisper_full_get_segment_text */
    int32_t i0, n_tokens;        /* the segment's tokens in spt_result.tokens */
} spt_segment;

typedef struct {
    char* text;             /* fast path: the text tokens' strings; whisper_full path: the segment
                               texts joined and trimmed (transcribe-rs TranscriptionResult.text);
                               synthetic models spell tokens as "[id]" */
    int32_t* tokens;        /* token ids: fast path every generated token (EOT included, stops
                               after it); whisper_full path each window's chosen decoder's result */
    float* top1;            /* fast path: suppressed logit of the token; whisper_full: its log-prob */
    float* top2;            /* fast path: runner-up suppressed logit; whisper_full: its timestamp id */
    int32_t n_tokens;
    int32_t n_windows;      /* 30 s windows decoded */
    int32_t language;       /* language index decoded with (whisper.cpp order, spt_language_code);
                               -1 for English-only models */
    int32_t n_segments;     /* whisper_full path (0 on the fast path) */
    spt_segment* segments;
    int32_t n_fallbacks;    /* temperature fallbacks taken: decodes repeated at a higher temperature */
    int32_t reserved0;
} spt_result;

typedef struct {
    int32_t n_mels, d, n_head, n_enc, n_dec, n_vocab, n_audio_ctx, n_text_ctx;
    int32_t dtype, max_batch;
    int64_t weight_bytes;
    int64_t workspace_bytes;
} spt_model_info;

/* per-phase device time of the last call, from HIP events on the engine stream; total_ms = the
 * sum of the phases */
typedef struct {
    double mel_ms, encoder_ms, cross_kv_ms, decode_ms, total_ms, h2d_ms;
    int32_t n_decode_passes;
    int32_t batch;
} spt_timings;

typedef struct spt_ctx spt_ctx;

const char* spt_version(void);
void spt_default_model_params(spt_model_params* p);
void spt_default_infer_params(spt_infer_params* p);

/* model_spec: "synthetic:<tiny.en|tiny|base|small|medium|large-v3>[:enc=N][:dec=N][:seed=S]"
 * or the path of a whisper.cpp ggml model file (the catalog's ggml-*.bin; tensor types f32,
 * f16, q4_0, q4_1, q5_0, q5_1, q8_0, q4_K, q5_K, q6_K; dequantised once at load into the engine dtype).
 * Replaces WhisperEngine::load_model(&path) (transcribe-rs; src-tauri/src/managers/
 * transcription.rs:261-276); bad files fail with SPT_ERR_LOAD and a message. */
spt_status spt_ctx_create(const char* model_spec, const spt_model_params* params, spt_ctx** out,
                          char* err, size_t errlen);
void spt_ctx_destroy(spt_ctx* ctx);
const char* spt_last_error(const spt_ctx* ctx);
spt_status spt_ctx_info(const spt_ctx* ctx, spt_model_info* info);

/* one utterance, host PCM (moved Vec<f32> in the app) */
spt_status spt_transcribe(spt_ctx* ctx, const float* pcm16k, size_t n_samples, const spt_infer_params* params,
                          spt_result** out);
/* a batch of utterances, host PCM; out[batch] */
spt_status spt_transcribe_batch(spt_ctx* ctx, const float* const* pcm, const size_t* n_samples, size_t batch,
                                const spt_infer_params* params, spt_result** out);
/* a batch of <= 30 s windows already resident in device memory: pcm_dev[b * stride + i] */
spt_status spt_transcribe_batch_device(spt_ctx* ctx, const float* pcm_dev, size_t stride, const size_t* n_samples,
                                       size_t batch, const spt_infer_params* params, spt_result** out);
void spt_result_free(spt_result* r);
/* ISO-639-1 code of a language index ("en" = 0, "zh" = 1, ...), NULL if out of range */
const char* spt_language_code(int32_t lang_id);

/* whisper_tokenize of the model's vocabulary (ggml models only; SPT_ERR_UNSUPPORTED for
 * synthetic ones).  *n_out = the token count even when it exceeds n_max (then
 * SPT_ERR_INVALID_ARG and nothing is written past n_max). */
spt_status spt_tokenize(spt_ctx* ctx, const char* text, int32_t* tokens, int32_t n_max, int32_t* n_out);
/* whisper_token_to_str: the bytes of token id (owned by the context), NULL without a vocab */
const char* spt_token_to_str(const spt_ctx* ctx, int32_t id);

spt_status spt_get_timings(const spt_ctx* ctx, spt_timings* t);

/* ABI 9: everything the last spt_transcribe* call ran, summed.  spt_timings holds the last engine
 * run only; a whisper_full call (the app's default parameters) runs one decoder run per window
 * batch and temperature, and beam search one decoder pass per step, so its latency reads per
 * decoder pass from here: device_ms / decoder_passes bounds the pass time from above.
 * ABI 11: whisper_full computes the log-mel of each whole utterance once (whisper_pcm_to_mel: its
 * own reflective head, the utterance's global max - 8 clamp) and encodes each 30 s window at
 * `seek` once (whisper_encode_internal), shared by every temperature fallback and by the
 * utterance's beam / best_of decoders: encoder_windows counts those encoder runs.
 * ABI 12: pd_passes / pd_fallbacks counted round 5's opt-in persistent decoder pass; round 6
 * measured it at the persistent-kernel price list's cost, slower than the launch chain at every
 * batch, and deleted it: both counters are always 0 (kept for layout).
 * device_ms (and spt_timings.total_ms) sum the stage intervals (mel, window norm, encoder, cross
 * K/V, decode); host time between the stages is not in them. */
typedef struct {
    int32_t engine_calls;     /* decoder runs (a prompt pass + its steps; ABI <= 10: each with its own
                                 mel + encoder + cross K/V) */
    int32_t decoder_passes;   /* every decoder pass: prompt passes, decode steps, beam steps */
    int32_t beam_steps;       /* host-driven beam steps among them */
    int32_t encoder_windows;  /* ABI 11: 30 s windows encoded (conv stem + encoder + cross K/V): one
                                 per window, shared by every temperature fallback and decoder */
    double device_ms;         /* device time of those runs and steps (HIP events) */
    double encoder_ms;
    double decode_ms;         /* decoder passes incl. prompt prefill and sampling */
    int32_t pd_passes;        /* ABI 12: always 0 (the persistent decoder pass was deleted) */
    int32_t pd_fallbacks;     /* ABI 12: always 0 */
} spt_call_stats;

spt_status spt_get_call_stats(const spt_ctx* ctx, spt_call_stats* s);

/* Multi-GPU load: the weight arena is one device allocation whose layout is a
 * pure function of (model, dtype), spt_model_info.weight_bytes long.  Rank 0 loads the model
 * (file parse + device dequantisation) and exports the arena into a device buffer; the buffer
 * is broadcast over RCCL/xGMI; every other rank, created with SPT_MODEL_WEIGHTS_EXTERNAL on the
 * same model spec, imports it.  Both are synchronous device-to-device copies on the context's
 * device; bytes must equal weight_bytes (else SPT_ERR_INVALID_ARG).  A context created with
 * SPT_MODEL_WEIGHTS_EXTERNAL fails every transcription with SPT_ERR_INVALID_ARG until the
 * import.  The reference loads each engine from disk (transcription.rs:261-276) and has no
 * multi-device path; these two entry points exist for the replica-parallel load only. */
spt_status spt_weights_export(spt_ctx* ctx, void* dev_dst, size_t bytes);
spt_status spt_weights_import(spt_ctx* ctx, const void* dev_src, size_t bytes);
/* ABI 5: the arena itself (device pointer on the context's device, weight_bytes long), so a
 * rank's collective (RCCL broadcast from rank 0) writes straight into it with no staging copy;
 * then spt_weights_commit (synchronises the device) marks an external-weights context usable. */
spt_status spt_weights_arena(spt_ctx* ctx, void** dev_ptr, size_t* bytes);
spt_status spt_weights_commit(spt_ctx* ctx);

/* ABI 5: replica parallelism from ONE host process over several devices, for a
 * host that owns one engine object (the app's TranscriptionManager, transcription.rs:29-47).
 * spt_ctx_create_replicas creates out[i] on devices[i] (distinct ordinals): devices[0] loads the
 * model, one grouped RCCL ncclBroadcast (ncclCommInitAll communicator, xGMI) copies its weight
 * arena into every other context's arena; *bcast_ms (optional) = the broadcast's wall time.
 * Each out[i] is an ordinary context (destroy each with spt_ctx_destroy).
 * spt_transcribe_batch_replicas splits a batch of utterances into n_ctx contiguous balanced
 * shards, transcribes shard i on ctxs[i] in its own host thread (no collective on the data
 * path) and returns out[batch] in input order; on error every result is released and ctxs[0]'s
 * last error names the failing replica. */
spt_status spt_ctx_create_replicas(const char* model_spec, const spt_model_params* params, const int32_t* devices,
                                   int32_t n_devices, spt_ctx** out, double* bcast_ms, char* err, size_t errlen);
spt_status spt_transcribe_batch_replicas(spt_ctx* const* ctxs, int32_t n_ctx, const float* const* pcm,
                                         const size_t* n_samples, size_t batch, const spt_infer_params* params,
                                         spt_result** out);

/* Kernel probe (measurement): re-launch one hot-path kernel `iters` times on the engine
 * stream, on the buffers of the last call.  Decoder kernels (kinds 0-3) are timed between two
 * HIP events after a 512 MB read of other weights (the cold Infinity Cache they meet in the
 * decode loop); kinds 0 and 3 as 8 launches over 8 different layers back to back, like the
 * loop; encoder kernels back to back.  avg_us = mean
 * time per launch; work = algorithmic bytes (HBM-bound kernels) or flops (MFMA-bound kernels)
 * per launch, work_is_flops says which. */
typedef enum {
    SPT_PROBE_DEC_CROSS_ATTN = 0,  /* decoder cross-attention, one layer */
    SPT_PROBE_DEC_SELF_ATTN = 1,   /* decoder self-attention, one layer */
    SPT_PROBE_DEC_LOGITS = 2,      /* final LayerNorm + logits + top-2 partials */
    SPT_PROBE_DEC_FC1 = 3,         /* decoder LayerNorm + fc1 + GELU (weight stream) */
    SPT_PROBE_ENC_FC1_GEMM = 4,    /* encoder fc1 GEMM + bias + GELU */
    SPT_PROBE_ENC_ATTN = 5         /* encoder flash attention, one layer */
} spt_probe_kind;
spt_status spt_probe_kernel(spt_ctx* ctx, int32_t kind, int32_t iters, double* avg_us, double* work,
                            int32_t* work_is_flops);

/* test hooks (parity against the CPU restatement) */
/* normalised log-mel of one window [n_mels][3000] (f32) */
spt_status spt_debug_mel(spt_ctx* ctx, const float* pcm16k, size_t n_samples, float* out);
/* ABI 11: the normalised log-mel [n_mels][3000] the encoder takes for the window at frame `seek` of
 * an utterance of any length: frames [seek, seek + 3000) of the utterance's whole log-mel */
spt_status spt_debug_mel_at(spt_ctx* ctx, const float* pcm16k, size_t n_samples, int32_t seek, float* out);
/* encoder output [1500][d] (f32) from a host mel [n_mels][3000] */
spt_status spt_debug_encode(spt_ctx* ctx, const float* mel, float* out);
/* sum|w| and sum w of the weight tensor with a given id (oracle/wo_model.c table) */
spt_status spt_debug_weight_checksum(spt_ctx* ctx, int32_t tensor_id, double* out2);
/* host-only (no device): whisper_tokenize with the vocabulary of a ggml file */
spt_status spt_debug_ggml_tokenize(const char* model_path, const char* text, int32_t* tokens, int32_t n_max,
                                   int32_t* n_out);
/* host-only: the host reference dequantisation of n elements of one ggml type to f32 */
spt_status spt_debug_ggml_dequant(int32_t ggml_type, const void* src, int64_t n, float* dst);

/* ================================================================================================
 * ABI 6: Parakeet-V3 (NeMo FastConformer-TDT), the app's other local engine;
 * ABI 8: spt_parakeet_create takes the app's model directory (the int8 ONNX export) natively.
 *
 * In the reference TranscriptionManager owns a transcribe_rs ParakeetEngine through
 * LoadedEngine::Parakeet and calls (src-tauri/src/managers/transcription.rs):
 *
 *   ParakeetEngine::new() + load_model_with_params(&path, ParakeetModelParams::int8())
 *                                                   :278-297  -> spt_parakeet_create (+ set_tensor)
 *   transcribe_samples(audio, Some(ParakeetInferenceParams { timestamp_granularity: Segment, .. }))
 *                                                   :505-513  -> spt_parakeet_transcribe
 *   unload_model() / Drop                            :175-208  -> spt_parakeet_destroy
 *
 * and reads TranscriptionResult.text (:537-546).  The encoder runs in fp16 (SPT_DTYPE_F16, the
 * BASELINE config) or f32; the prediction network and joint always in f32.  Weights come from a
 * synthetic spec or tensor by tensor through spt_parakeet_set_tensor (the id table of
 * oracle/po_model.c, NeMo layouts; spittle_amd.parakeet.load_nemo maps a .nemo checkpoint).
 * ============================================================================================== */
typedef struct spt_pk_ctx spt_pk_ctx;

typedef struct {
    int32_t dtype;        /* SPT_DTYPE_F16 (default) or SPT_DTYPE_F32 (bf16 also accepted) */
    int32_t device;
    int32_t max_batch;    /* utterances (chunks) per device pass, <= 64 */
    float max_seconds;    /* workspace size: the longest utterance one pass takes before it grows.
                             A longer recording grows the workspace to its length and is decoded
                             whole (up to 20 min / 96 GiB of workspace); only past that is it cut
                             into chunks (multiples of 80 ms) whose results are concatenated */
    uint64_t seed;        /* synthetic weights */
    uint32_t flags;       /* SPT_PK_WEIGHTS_EMPTY: zero weights, to be filled by set_tensor */
    int32_t reserved0;
} spt_pk_model_params;

#define SPT_PK_WEIGHTS_EMPTY 1u

typedef enum { SPT_PK_TS_TOKEN = 0, SPT_PK_TS_WORD = 1, SPT_PK_TS_SEGMENT = 2 } spt_pk_granularity;

typedef struct {
    int32_t max_symbols;            /* TDT greedy: tokens per encoder frame (NeMo default 10; <= 16) */
    int32_t timestamp_granularity;  /* an spt_pk_granularity; the app asks for SPT_PK_TS_SEGMENT */
} spt_pk_infer_params;

typedef struct {
    double start, end;     /* seconds */
    char* text;
    int32_t i0, n_tokens;  /* the unit's tokens in spt_pk_result.tokens */
} spt_pk_segment;

typedef struct {
    char* text;            /* the pieces joined ("▁" -> space) and trimmed; "[id]" without a vocabulary */
    int32_t* tokens;
    int32_t* frames;       /* encoder frame (80 ms) of each token, utterance-relative */
    float* logit;          /* the token's joint logit */
    float* runner_up;      /* the best other token's (blank included) */
    int32_t n_tokens;
    int32_t n_segments;
    spt_pk_segment* segments;  /* timestamp units of the requested granularity */
    int32_t n_chunks;
    int32_t reserved0;
} spt_pk_result;

typedef struct {
    int32_t n_mels, d, n_layers, n_heads, ff, sub_ch, conv_k, pred, n_vocab, n_dur;
    int32_t dtype, max_batch, max_samples, reserved0;
    int64_t weight_bytes, workspace_bytes;
} spt_pk_model_info;

typedef struct {
    double mel_ms, encoder_ms, decode_ms, total_ms, h2d_ms;
    int32_t n_steps;       /* TDT joint evaluations (graph-replayed decode steps) */
    int32_t batch;
    int32_t enc_frames;    /* padded encoder frames of the pass */
    int32_t reserved0;
} spt_pk_timings;

void spt_parakeet_default_model_params(spt_pk_model_params* p);
void spt_parakeet_default_infer_params(spt_pk_infer_params* p);
/* model_spec: the app's model directory (below; the weights are dequantised and placed, vocab.txt
 * becomes the vocabulary), or "synthetic:parakeet-tdt-0.6b-v3[:layers=N][:seed=S]" /
 * "synthetic:parakeet-test-small[...]" (seeded weights; real ones through spt_parakeet_set_tensor) */
spt_status spt_parakeet_create(const char* model_spec, const spt_pk_model_params* params, spt_pk_ctx** out,
                               char* err, size_t errlen);

/* The model directory the app downloads (parakeet-tdt-0.6b-v3-int8, the onnx-asr export that
 * transcribe-rs reads: encoder-model[.int8].onnx, decoder_joint-model[.int8].onnx, vocab.txt;
 * model_catalog.json:229-241) is also what spt_parakeet_create takes as model_spec -- this is the
 * same loader without a device: parse, dequantise (int8 / uint8 + scale + zero point, per tensor or
 * per channel), map onto the engine's tensor ids (NeMo layouts), infer the dimensions.
 * info->reserved0 receives the number of dequantised initializers.  Host memory only. */
typedef struct spt_pk_onnx spt_pk_onnx;
spt_status spt_parakeet_onnx_open(const char* dir, spt_pk_onnx** out, spt_pk_model_info* info, char* err, size_t errlen);
/* a tensor's f32 values (NeMo layout) by engine tensor id: its element count, or -1 */
int64_t spt_parakeet_onnx_tensor(const spt_pk_onnx* h, int32_t tensor_id, const float** data);
/* vocab.txt's piece for a token id (NULL past the vocabulary or without vocab.txt) */
const char* spt_parakeet_onnx_piece(const spt_pk_onnx* h, int32_t token_id);
void spt_parakeet_onnx_close(spt_pk_onnx* h);
void spt_parakeet_destroy(spt_pk_ctx* ctx);
const char* spt_parakeet_last_error(const spt_pk_ctx* ctx);
spt_status spt_parakeet_info(const spt_pk_ctx* ctx, spt_pk_model_info* info);
/* element count of tensor id (SPT_ERR_INVALID_ARG if unknown) and its upload (f32, NeMo layout) */
spt_status spt_parakeet_tensor_numel(const spt_pk_ctx* ctx, int32_t tensor_id, int64_t* n);
spt_status spt_parakeet_set_tensor(spt_pk_ctx* ctx, int32_t tensor_id, const float* data, int64_t n);
/* SentencePiece pieces by id (UTF-8, "▁" marks a word start); copied */
spt_status spt_parakeet_set_vocab(spt_pk_ctx* ctx, const char* const* pieces, int32_t n);
spt_status spt_parakeet_transcribe(spt_pk_ctx* ctx, const float* pcm16k, size_t n_samples,
                                   const spt_pk_infer_params* params, spt_pk_result** out);
spt_status spt_parakeet_transcribe_batch(spt_pk_ctx* ctx, const float* const* pcm, const size_t* n_samples,
                                         size_t batch, const spt_pk_infer_params* params, spt_pk_result** out);
/* batch <= max_batch chunks already in device memory (pcm_dev[b * stride + i], n <= max samples) */
spt_status spt_parakeet_transcribe_batch_device(spt_pk_ctx* ctx, const float* pcm_dev, size_t stride,
                                                const size_t* n_samples, size_t batch,
                                                const spt_pk_infer_params* params, spt_pk_result** out);
void spt_parakeet_result_free(spt_pk_result* r);
spt_status spt_parakeet_get_timings(const spt_pk_ctx* ctx, spt_pk_timings* t);
/* ABI 10: encoder stage profile (measurement).  Re-runs the last call's encoder pass `iters` times
 * eagerly, on the same buffers and shape (bitwise the same output), with a HIP event on the engine
 * stream after every stage's launches; ms[c] = mean time per pass spent in stage class c.
 * n >= SPT_PK_STAGE_COUNT. */
typedef enum {
    SPT_PK_STAGE_SUBSAMPLING = 0, /* conv stem: conv0, two depthwise + pointwise stages, linear */
    SPT_PK_STAGE_POS = 1,         /* relative positions + every layer's linear_pos (one GEMM) */
    SPT_PK_STAGE_LAYERNORM = 2,   /* 5 LayerNorms per layer (pending split-K products folded in) */
    SPT_PK_STAGE_FFN = 3,         /* both half-FFNs' GEMMs (SiLU up-projection, split-K down) */
    SPT_PK_STAGE_QKV_OUT = 4,     /* attention q/k/v and output GEMMs */
    SPT_PK_STAGE_ATTN = 5,        /* relative-position attention */
    SPT_PK_STAGE_CONV_PW = 6,     /* convolution module pointwise GEMMs */
    SPT_PK_STAGE_CONV_DW = 7,     /* GLU + depthwise conv + BatchNorm + SiLU */
    SPT_PK_STAGE_JOINT_ENC = 8,   /* the joint's encoder projection */
    SPT_PK_STAGE_COUNT = 9
} spt_pk_stage;
spt_status spt_parakeet_profile_encoder(spt_pk_ctx* ctx, int32_t iters, double* ms, int32_t n);
/* test hooks: normalised log-mel [n_mels][max(1, n / 160)] (n / 160 valid frames, NeMo get_seq_len); encoder output [T3][d] of a mel
 * [n_mels][T]; sum|w| and sum w of a tensor as stored (transposed tensors: SPT_ERR_UNSUPPORTED) */
spt_status spt_parakeet_debug_mel(spt_pk_ctx* ctx, const float* pcm16k, size_t n_samples, float* out);
spt_status spt_parakeet_debug_encode(spt_pk_ctx* ctx, const float* mel, int32_t T, float* out);
/* the encoder output [T3][d] (f32) of batch row b of the last transcribe call (the production
 * path: graph-replayed or eager); out holds the T3 rows of spt_pk_model_info.max_samples (which grows
 * with the longest recording decoded); *T3 receives the row's count */
spt_status spt_parakeet_debug_last_encoder(spt_pk_ctx* ctx, int32_t b, float* out, int32_t* T3);
/* TDT greedy decoding of a given encoder output [T3][d] (f32): the decoder alone */
spt_status spt_parakeet_debug_decode(spt_pk_ctx* ctx, const float* enc, int32_t T3, int32_t max_symbols,
                                     spt_pk_result** out);
spt_status spt_parakeet_debug_weight_checksum(spt_pk_ctx* ctx, int32_t tensor_id, double* out2);

/* ================================================================================================
 * ABI 7: the capture-side resampler.
 *
 * Replaces FrameResampler (src-tauri/src/audio_toolkit/audio/resampler.rs:7-104): rubato 0.16.2
 * FftFixedIn<f32>(in_hz, out_hz, RESAMPLER_CHUNK_SIZE = 1024, 1, 1) behind 1024-sample input
 * chunks, its output cut into frames of frame_samples (the recorder's 30 ms = 480 samples at
 * 16 kHz, recorder.rs:264-268).  spt_resample runs one whole capture stream as
 * FrameResampler::new + push(all samples) + finish (recorder.rs:330, 355): the concatenated
 * frames, including finish's zero padding of the last input chunk and of the last frame.
 * in_hz == out_hz: frames of the input, as FrameResampler does without rubato.
 * ============================================================================================== */
typedef struct spt_resampler spt_resampler;
spt_status spt_resampler_create(int32_t in_hz, int32_t out_hz, int32_t frame_samples, int32_t device,
                                spt_resampler** out, char* err, size_t errlen);
/* rubato's unit sizes (0 when in_hz == out_hz) */
spt_status spt_resampler_info(const spt_resampler* r, int32_t* fft_size_in, int32_t* fft_size_out);
/* samples spt_resample writes for an n-sample stream (a multiple of frame_samples) */
size_t spt_resample_output_len(const spt_resampler* r, size_t n_samples);
/* pcm: host samples (borrowed); out: host buffer of at least spt_resample_output_len samples */
spt_status spt_resample(spt_resampler* r, const float* pcm, size_t n_samples, float* out, size_t out_cap,
                        size_t* n_out);
const char* spt_resampler_last_error(const spt_resampler* r);
void spt_resampler_destroy(spt_resampler* r);

/* ================================================================================================
 * ABI 8: the capture-side voice-activity gate.  The recorder's consumer thread
 * pushes every 480-sample (30 ms) frame from the FrameResampler through
 *   SmoothedVad::new(Box::new(SileroVad::new("resources/models/silero_vad_v4.onnx", 0.3)), 15, 15, 2)
 * (src-tauri/src/managers/audio.rs:132-134, 295-307) and appends what it returns as Speech to the
 * recording (audio_toolkit/audio/recorder.rs:284-301); Cmd::Start resets the smoothing (:343-349).
 *
 *   spt_vad_create(model_path, params)  = SileroVad::new + SmoothedVad::new  (the model file the app
 *                                         ships is read natively: ONNX graph, 16 kHz branch)
 *   spt_vad_push(pcm, n)                = push_frame for each 480-sample frame in order (a trailing
 *                                         partial frame is kept as Speech, like the recorder's
 *                                         unwrap_or); result: the kept samples, each frame's speech
 *                                         probability and VadFrame kind (0 Noise, 1 Speech(frame),
 *                                         2 Speech(prefill + frame))
 *   spt_vad_reset(v, 0)                 = SmoothedVad::reset (the Silero LSTM state carries, as in the
 *                                         app); reset_model_state = 1 also zeroes it (a new SileroVad)
 *
 * The network runs on the device: every frame's convolutional front end at once, then the
 * two-layer LSTM recurrence over the frames in one workgroup (its state kept between calls).
 * ============================================================================================== */
typedef struct spt_vad spt_vad;
typedef struct {
    float threshold;          /* speech when prob > threshold (0.3) */
    int32_t prefill_frames;   /* 15 */
    int32_t hangover_frames;  /* 15 */
    int32_t onset_frames;     /* 2 */
    int32_t device;
    int32_t reserved0;
} spt_vad_params;
typedef struct {
    float* samples;           /* the kept audio (Speech frames, prefill at onsets), n_samples long */
    size_t n_samples;
    float* prob;              /* per whole frame: Silero's speech probability */
    uint8_t* kind;            /* per frame (a trailing partial frame included): 0 Noise, 1 Speech, 2 onset */
    int32_t n_frames;
    int32_t reserved0;
    double device_ms;         /* front end + recurrence on the device */
} spt_vad_result;
void spt_vad_default_params(spt_vad_params* p);
spt_status spt_vad_create(const char* model_path, const spt_vad_params* params, spt_vad** out, char* err,
                          size_t errlen);
spt_status spt_vad_push(spt_vad* v, const float* pcm, size_t n_samples, spt_vad_result** out);
void spt_vad_result_free(spt_vad_result* r);
spt_status spt_vad_reset(spt_vad* v, int32_t reset_model_state);
const char* spt_vad_last_error(const spt_vad* v);
void spt_vad_destroy(spt_vad* v);

#ifdef __cplusplus
}
#endif
#endif
