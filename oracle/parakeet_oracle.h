/*
 * parakeet_oracle.h -- CPU restatement of Spittle's Parakeet-V3 transcription path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in spittle_amd/ links, loads or calls this library.
 * Only tests/ and bench.py's cpu_baseline leg may use it, as the checker / CPU baseline.
 *
 * Reference path: TranscriptionManager (/root/reference/src-tauri/src/managers/transcription.rs)
 * loads `ParakeetEngine::load_model_with_params(path, ParakeetModelParams::int8())` (:278-297)
 * and calls `transcribe_samples(audio, Some(ParakeetInferenceParams { timestamp_granularity:
 * Segment, .. }))` (:505-513) -- transcribe-rs 0.2.3 (Cargo.lock:7471-7490) running the
 * catalog's parakeet-tdt-0.6b-v3-int8 ONNX export (model_catalog.json) through ONNX Runtime.
 * Neither the crate nor the ONNX graphs nor the weights exist in /root/reference or offline,
 * so the model is restated from NVIDIA NeMo's published FastConformer-TDT definition
 * [upstream, recalled]:
 *   preprocessor  NeMo FilterbankFeatures: pre-emphasis 0.97, STFT n_fft 512, hop 160,
 *                 400-sample symmetric Hann centred in the 512 window, centre padding of
 *                 256 zeros, power spectrum, 128 slaney mel bands (0-8 kHz), log(x + 2^-24),
 *                 per-feature normalisation over the n / 160 valid frames (unbiased std + 1e-5);
 *   encoder       ConvSubsampling "dw_striding" x8 (conv 3x3 s2 -> ReLU -> [dw 3x3 s2 ->
 *                 pw 1x1 -> ReLU] x 2 -> flatten (channel-major) -> linear), x * sqrt(d),
 *                 relative sinusoidal positions; 24 Conformer layers: 1/2 FFN (Swish), rel-pos
 *                 MHSA (Transformer-XL, per-layer pos_bias_u / pos_bias_v, linear_pos without
 *                 bias), conv module (pw -> GLU -> depthwise k9 -> BatchNorm -> Swish -> pw),
 *                 1/2 FFN, LayerNorm out; LayerNorm eps 1e-5;
 *   decoder       RNNT prediction network: embedding (blank row zero), 2-layer LSTM;
 *                 joint: ReLU(enc.Wf + pred.Wg) -> linear to vocab + blank + 5 durations;
 *   search        TDT greedy: argmax token and duration per joint evaluation, duration
 *                 0 keeps the frame (max_symbols per frame), a blank always advances.
 * The ONNX int8 export is not reproduced (its quantisation is not observable offline): this is
 * the fp32 model; parity against the real engine is "parity unpinned".
 *
 * Synthetic weights: the splitmix64 scheme of whisper_oracle.h (power-of-two scales, exact in
 * f32; the encoder's matrices optionally bf16- or fp16-rounded), tensor ids below, shared with
 * spittle_amd/csrc/parakeet.cpp.
 */
#ifndef PARAKEET_ORACLE_H
#define PARAKEET_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int n_mels;       /* 128 */
    int d;            /* 1024 */
    int n_layers;     /* 24 */
    int n_heads;      /* 8 */
    int ff;           /* 4096 */
    int sub_ch;       /* 256: subsampling conv channels */
    int conv_k;       /* 9 */
    int pred;         /* 640: prediction-network and joint width */
    int n_vocab;      /* 8192 (blank = n_vocab) */
    int n_dur;        /* 5: durations 0..4 */
} po_dims;

enum { PO_W_F32 = 0, PO_W_BF16 = 1, PO_W_F16 = 2 };  /* rounding of the encoder's linear-layer matrices */

typedef struct po_model po_model;

po_model* po_create(const po_dims* dims, uint64_t seed, int wdtype);
void po_destroy(po_model* m);
void po_set_threads(int n);

/* valid frames of the preprocessor for n samples: n / 160 (NeMo get_seq_len) */
int po_n_frames(int n_samples);
/* encoder frames after the x8 subsampling of T mel frames */
int po_n_enc_frames(int T);
/* normalised log-mel [n_mels][T] of n samples (16 kHz mono); returns T */
int po_mel(const float* pcm, int n_samples, int n_mels, float* out);
/* encoder output [T3][d] of a mel [n_mels][T]; returns T3 */
int po_encode(po_model* m, const float* mel, int T, float* out);
/* TDT greedy over enc [T3][d]: tokens, their frames and (optional) top-1/top-2 token logits of
 * the joint evaluation that emitted them; returns the count (<= cap) */
int po_decode(po_model* m, const float* enc, int T3, int max_symbols, int* tokens, int* frames, float* top1,
              float* top2, int cap);
/* po_decode plus gmin[i]: the smallest top-1/top-2 margin of any token or duration decision since
 * emission i - 1 (inclusive of emission i); gmin[n] covers the evaluations after the last one
 * (cap must exceed the count) -- the decision margin a GPU run's first disagreement is held to */
int po_decode_gaps(po_model* m, const float* enc, int T3, int max_symbols, int* tokens, int* frames, float* top1,
                   float* top2, float* gmin, int cap);
/* a weight tensor by id (contract with the engine): its element count, or -1 */
int64_t po_tensor(po_model* m, int tid, const float** data);
/* replace a weight tensor (the values a loaded model file holds); 0, or -1 on an unknown id / size */
int po_set_tensor(po_model* m, int tid, const float* data, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
