//! Raw bindings to `include/spittle_hip.h` (ABI 12), the C boundary of the MI355X-native Whisper
//! and Parakeet-V3 backend.  One item per declaration of the header, same names, same layouts (x86-64 SysV; the
//! layouts are checked field by field against gcc by tests/test_capi.py).  Safe wrappers live in
//! the `spittle-hip` crate.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub const SPT_ABI_VERSION: c_int = 12;
pub const SPT_PK_STAGE_COUNT: c_int = 9;

pub type spt_status = c_int;
pub const SPT_OK: spt_status = 0;
pub const SPT_ERR_INVALID_ARG: spt_status = 1;
pub const SPT_ERR_LOAD: spt_status = 2;
pub const SPT_ERR_DEVICE: spt_status = 3;
pub const SPT_ERR_OOM: spt_status = 4;
pub const SPT_ERR_UNSUPPORTED: spt_status = 5;
pub const SPT_ERR_INTERNAL: spt_status = 6;

pub type spt_dtype = c_int;
pub const SPT_DTYPE_F32: spt_dtype = 0;
pub const SPT_DTYPE_BF16: spt_dtype = 1;
pub const SPT_DTYPE_F16: spt_dtype = 2;

pub const SPT_SUPPRESS_BLANK: u32 = 1;
pub const SPT_NO_TIMESTAMPS: u32 = 2;
pub const SPT_IGNORE_EOT: u32 = 4;
pub const SPT_SUPPRESS_NST: u32 = 8;

pub const SPT_MODEL_WEIGHTS_EXTERNAL: u32 = 1;

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct spt_model_params {
    pub dtype: i32,
    pub device: i32,
    pub max_batch: i32,
    pub flags: u32,
    pub seed: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct spt_infer_params {
    pub language: *const c_char,
    pub translate: i32,
    pub initial_prompt: *const c_char,
    pub flags: u32,
    pub max_new_tokens: i32,
    pub temperature: f32,
    pub beam_size: i32,
    pub forced_tokens: *const i32,
    pub n_forced: i32,
    pub prompt_tokens: *const i32,
    pub n_prompt_tokens: i32,
    pub temperature_inc: f32,
    pub best_of: i32,
    pub entropy_thold: f32,
    pub logprob_thold: f32,
    pub max_initial_ts: f32,
    pub reserved0: i32,
    pub seed: u64,
}

#[repr(C)]
#[derive(Debug)]
pub struct spt_segment {
    pub t0: i64,
    pub t1: i64,
    pub text: *mut c_char,
    pub i0: i32,
    pub n_tokens: i32,
}

#[repr(C)]
#[derive(Debug)]
pub struct spt_result {
    pub text: *mut c_char,
    pub tokens: *mut i32,
    pub top1: *mut f32,
    pub top2: *mut f32,
    pub n_tokens: i32,
    pub n_windows: i32,
    pub language: i32,
    pub n_segments: i32,
    pub segments: *mut spt_segment,
    pub n_fallbacks: i32,
    pub reserved0: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct spt_model_info {
    pub n_mels: i32,
    pub d: i32,
    pub n_head: i32,
    pub n_enc: i32,
    pub n_dec: i32,
    pub n_vocab: i32,
    pub n_audio_ctx: i32,
    pub n_text_ctx: i32,
    pub dtype: i32,
    pub max_batch: i32,
    pub weight_bytes: i64,
    pub workspace_bytes: i64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct spt_call_stats {
    pub engine_calls: i32,
    pub decoder_passes: i32,
    pub beam_steps: i32,
    /// ABI 11: 30 s windows encoded (one per window, shared by fallbacks and decoders)
    pub encoder_windows: i32,
    pub device_ms: f64,
    pub encoder_ms: f64,
    pub decode_ms: f64,
    /// ABI 12: always 0 (the persistent decoder pass was deleted in round 6)
    pub pd_passes: i32,
    /// ABI 12: always 0
    pub pd_fallbacks: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct spt_timings {
    pub mel_ms: f64,
    pub encoder_ms: f64,
    pub cross_kv_ms: f64,
    pub decode_ms: f64,
    pub total_ms: f64,
    pub h2d_ms: f64,
    pub n_decode_passes: i32,
    pub batch: i32,
}

/// Opaque context (one loaded model on one device).
#[repr(C)]
pub struct spt_ctx {
    _private: [u8; 0],
}

pub type spt_probe_kind = c_int;
pub const SPT_PROBE_DEC_CROSS_ATTN: spt_probe_kind = 0;
pub const SPT_PROBE_DEC_SELF_ATTN: spt_probe_kind = 1;
pub const SPT_PROBE_DEC_LOGITS: spt_probe_kind = 2;
pub const SPT_PROBE_DEC_FC1: spt_probe_kind = 3;
pub const SPT_PROBE_ENC_FC1_GEMM: spt_probe_kind = 4;
pub const SPT_PROBE_ENC_ATTN: spt_probe_kind = 5;

extern "C" {
    pub fn spt_version() -> *const c_char;
    pub fn spt_default_model_params(p: *mut spt_model_params);
    pub fn spt_default_infer_params(p: *mut spt_infer_params);

    pub fn spt_ctx_create(
        model_spec: *const c_char,
        params: *const spt_model_params,
        out: *mut *mut spt_ctx,
        err: *mut c_char,
        errlen: usize,
    ) -> spt_status;
    pub fn spt_ctx_destroy(ctx: *mut spt_ctx);
    pub fn spt_last_error(ctx: *const spt_ctx) -> *const c_char;
    pub fn spt_ctx_info(ctx: *const spt_ctx, info: *mut spt_model_info) -> spt_status;

    pub fn spt_transcribe(
        ctx: *mut spt_ctx,
        pcm16k: *const f32,
        n_samples: usize,
        params: *const spt_infer_params,
        out: *mut *mut spt_result,
    ) -> spt_status;
    pub fn spt_transcribe_batch(
        ctx: *mut spt_ctx,
        pcm: *const *const f32,
        n_samples: *const usize,
        batch: usize,
        params: *const spt_infer_params,
        out: *mut *mut spt_result,
    ) -> spt_status;
    pub fn spt_transcribe_batch_device(
        ctx: *mut spt_ctx,
        pcm_dev: *const f32,
        stride: usize,
        n_samples: *const usize,
        batch: usize,
        params: *const spt_infer_params,
        out: *mut *mut spt_result,
    ) -> spt_status;
    pub fn spt_result_free(r: *mut spt_result);
    pub fn spt_language_code(lang_id: i32) -> *const c_char;

    pub fn spt_tokenize(
        ctx: *mut spt_ctx,
        text: *const c_char,
        tokens: *mut i32,
        n_max: i32,
        n_out: *mut i32,
    ) -> spt_status;
    pub fn spt_token_to_str(ctx: *const spt_ctx, id: i32) -> *const c_char;

    pub fn spt_get_timings(ctx: *const spt_ctx, t: *mut spt_timings) -> spt_status;
    // ---- ABI 9: the whole last call (every window, fallback and beam step)
    pub fn spt_get_call_stats(ctx: *const spt_ctx, s: *mut spt_call_stats) -> spt_status;

    pub fn spt_weights_export(ctx: *mut spt_ctx, dev_dst: *mut c_void, bytes: usize) -> spt_status;
    pub fn spt_weights_import(ctx: *mut spt_ctx, dev_src: *const c_void, bytes: usize) -> spt_status;
    pub fn spt_weights_arena(ctx: *mut spt_ctx, dev_ptr: *mut *mut c_void, bytes: *mut usize) -> spt_status;
    pub fn spt_weights_commit(ctx: *mut spt_ctx) -> spt_status;

    pub fn spt_ctx_create_replicas(
        model_spec: *const c_char,
        params: *const spt_model_params,
        devices: *const i32,
        n_devices: i32,
        out: *mut *mut spt_ctx,
        bcast_ms: *mut f64,
        err: *mut c_char,
        errlen: usize,
    ) -> spt_status;
    pub fn spt_transcribe_batch_replicas(
        ctxs: *const *mut spt_ctx,
        n_ctx: i32,
        pcm: *const *const f32,
        n_samples: *const usize,
        batch: usize,
        params: *const spt_infer_params,
        out: *mut *mut spt_result,
    ) -> spt_status;

    pub fn spt_probe_kernel(
        ctx: *mut spt_ctx,
        kind: i32,
        iters: i32,
        avg_us: *mut f64,
        work: *mut f64,
        work_is_flops: *mut i32,
    ) -> spt_status;

    pub fn spt_debug_mel(ctx: *mut spt_ctx, pcm16k: *const f32, n_samples: usize, out: *mut f32) -> spt_status;
    pub fn spt_debug_mel_at(ctx: *mut spt_ctx, pcm16k: *const f32, n_samples: usize, seek: i32, out: *mut f32) -> spt_status;
    pub fn spt_debug_encode(ctx: *mut spt_ctx, mel: *const f32, out: *mut f32) -> spt_status;
    pub fn spt_debug_weight_checksum(ctx: *mut spt_ctx, tensor_id: i32, out2: *mut f64) -> spt_status;
    pub fn spt_debug_ggml_tokenize(
        model_path: *const c_char,
        text: *const c_char,
        tokens: *mut i32,
        n_max: i32,
        n_out: *mut i32,
    ) -> spt_status;
    pub fn spt_debug_ggml_dequant(ggml_type: i32, src: *const c_void, n: i64, dst: *mut f32) -> spt_status;

    // ---- ABI 6: Parakeet-V3
    pub fn spt_parakeet_default_model_params(p: *mut spt_pk_model_params);
    pub fn spt_parakeet_default_infer_params(p: *mut spt_pk_infer_params);
    pub fn spt_parakeet_create(
        model_spec: *const c_char,
        params: *const spt_pk_model_params,
        out: *mut *mut spt_pk_ctx,
        err: *mut c_char,
        errlen: usize,
    ) -> spt_status;
    pub fn spt_parakeet_destroy(ctx: *mut spt_pk_ctx);
    pub fn spt_parakeet_last_error(ctx: *const spt_pk_ctx) -> *const c_char;
    pub fn spt_parakeet_info(ctx: *const spt_pk_ctx, info: *mut spt_pk_model_info) -> spt_status;
    pub fn spt_parakeet_tensor_numel(ctx: *const spt_pk_ctx, tensor_id: i32, n: *mut i64) -> spt_status;
    pub fn spt_parakeet_set_tensor(ctx: *mut spt_pk_ctx, tensor_id: i32, data: *const f32, n: i64) -> spt_status;
    pub fn spt_parakeet_set_vocab(ctx: *mut spt_pk_ctx, pieces: *const *const c_char, n: i32) -> spt_status;
    pub fn spt_parakeet_transcribe(
        ctx: *mut spt_pk_ctx,
        pcm16k: *const f32,
        n_samples: usize,
        params: *const spt_pk_infer_params,
        out: *mut *mut spt_pk_result,
    ) -> spt_status;
    pub fn spt_parakeet_transcribe_batch(
        ctx: *mut spt_pk_ctx,
        pcm: *const *const f32,
        n_samples: *const usize,
        batch: usize,
        params: *const spt_pk_infer_params,
        out: *mut *mut spt_pk_result,
    ) -> spt_status;
    pub fn spt_parakeet_transcribe_batch_device(
        ctx: *mut spt_pk_ctx,
        pcm_dev: *const f32,
        stride: usize,
        n_samples: *const usize,
        batch: usize,
        params: *const spt_pk_infer_params,
        out: *mut *mut spt_pk_result,
    ) -> spt_status;
    pub fn spt_parakeet_result_free(r: *mut spt_pk_result);
    pub fn spt_parakeet_get_timings(ctx: *const spt_pk_ctx, t: *mut spt_pk_timings) -> spt_status;
    // ---- ABI 10: encoder stage profile (ms[SPT_PK_STAGE_COUNT], spt_pk_stage order)
    pub fn spt_parakeet_profile_encoder(ctx: *mut spt_pk_ctx, iters: i32, ms: *mut f64, n: i32) -> spt_status;
    pub fn spt_parakeet_debug_mel(ctx: *mut spt_pk_ctx, pcm16k: *const f32, n_samples: usize, out: *mut f32) -> spt_status;
    pub fn spt_parakeet_debug_encode(ctx: *mut spt_pk_ctx, mel: *const f32, t: i32, out: *mut f32) -> spt_status;
    pub fn spt_parakeet_debug_last_encoder(ctx: *mut spt_pk_ctx, b: i32, out: *mut f32, t3: *mut i32) -> spt_status;
    pub fn spt_parakeet_debug_decode(
        ctx: *mut spt_pk_ctx,
        enc: *const f32,
        t3: i32,
        max_symbols: i32,
        out: *mut *mut spt_pk_result,
    ) -> spt_status;
    pub fn spt_parakeet_debug_weight_checksum(ctx: *mut spt_pk_ctx, tensor_id: i32, out2: *mut f64) -> spt_status;

    // ---- ABI 7: capture-side resampler (audio_toolkit/audio/resampler.rs FrameResampler)
    pub fn spt_resampler_create(
        in_hz: i32,
        out_hz: i32,
        frame_samples: i32,
        device: i32,
        out: *mut *mut spt_resampler,
        err: *mut c_char,
        errlen: usize,
    ) -> spt_status;
    pub fn spt_resampler_info(r: *const spt_resampler, fft_size_in: *mut i32, fft_size_out: *mut i32) -> spt_status;
    pub fn spt_resample_output_len(r: *const spt_resampler, n_samples: usize) -> usize;
    pub fn spt_resample(
        r: *mut spt_resampler,
        pcm: *const f32,
        n_samples: usize,
        out: *mut f32,
        out_cap: usize,
        n_out: *mut usize,
    ) -> spt_status;
    pub fn spt_resampler_last_error(r: *const spt_resampler) -> *const c_char;
    pub fn spt_resampler_destroy(r: *mut spt_resampler);

    // ---- ABI 8: the app's Parakeet model directory without a device (spt_parakeet_create also
    // takes the directory itself)
    pub fn spt_parakeet_onnx_open(
        dir: *const c_char,
        out: *mut *mut spt_pk_onnx,
        info: *mut spt_pk_model_info,
        err: *mut c_char,
        errlen: usize,
    ) -> spt_status;
    pub fn spt_parakeet_onnx_tensor(h: *const spt_pk_onnx, tensor_id: i32, data: *mut *const f32) -> i64;
    pub fn spt_parakeet_onnx_piece(h: *const spt_pk_onnx, token_id: i32) -> *const c_char;
    pub fn spt_parakeet_onnx_close(h: *mut spt_pk_onnx);

    // ---- ABI 8: voice-activity gate (audio_toolkit/vad: SmoothedVad over SileroVad)
    pub fn spt_vad_default_params(p: *mut spt_vad_params);
    pub fn spt_vad_create(
        model_path: *const c_char,
        params: *const spt_vad_params,
        out: *mut *mut spt_vad,
        err: *mut c_char,
        errlen: usize,
    ) -> spt_status;
    pub fn spt_vad_push(v: *mut spt_vad, pcm: *const f32, n_samples: usize, out: *mut *mut spt_vad_result) -> spt_status;
    pub fn spt_vad_result_free(r: *mut spt_vad_result);
    pub fn spt_vad_reset(v: *mut spt_vad, reset_model_state: i32) -> spt_status;
    pub fn spt_vad_last_error(v: *const spt_vad) -> *const c_char;
    pub fn spt_vad_destroy(v: *mut spt_vad);
}

/// Opaque parsed Parakeet model directory (ABI 8).
#[repr(C)]
pub struct spt_pk_onnx {
    _private: [u8; 0],
}

/// Opaque voice-activity gate (ABI 8).
#[repr(C)]
pub struct spt_vad {
    _private: [u8; 0],
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct spt_vad_params {
    pub threshold: f32,
    pub prefill_frames: i32,
    pub hangover_frames: i32,
    pub onset_frames: i32,
    pub device: i32,
    pub reserved0: i32,
}

#[repr(C)]
pub struct spt_vad_result {
    pub samples: *mut f32,
    pub n_samples: usize,
    pub prob: *mut f32,
    pub kind: *mut u8,
    pub n_frames: i32,
    pub reserved0: i32,
    pub device_ms: f64,
}

/// Opaque capture-side resampler context (ABI 7).
#[repr(C)]
pub struct spt_resampler {
    _private: [u8; 0],
}

// ---- ABI 6: Parakeet-V3 types
pub const SPT_PK_WEIGHTS_EMPTY: u32 = 1;
pub type spt_pk_granularity = c_int;
pub const SPT_PK_TS_TOKEN: spt_pk_granularity = 0;
pub const SPT_PK_TS_WORD: spt_pk_granularity = 1;
pub const SPT_PK_TS_SEGMENT: spt_pk_granularity = 2;

#[repr(C)]
pub struct spt_pk_ctx {
    _private: [u8; 0],
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct spt_pk_model_params {
    pub dtype: i32,
    pub device: i32,
    pub max_batch: i32,
    pub max_seconds: f32,
    pub seed: u64,
    pub flags: u32,
    pub reserved0: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct spt_pk_infer_params {
    pub max_symbols: i32,
    pub timestamp_granularity: i32,
}

#[repr(C)]
pub struct spt_pk_segment {
    pub start: f64,
    pub end: f64,
    pub text: *mut c_char,
    pub i0: i32,
    pub n_tokens: i32,
}

#[repr(C)]
pub struct spt_pk_result {
    pub text: *mut c_char,
    pub tokens: *mut i32,
    pub frames: *mut i32,
    pub logit: *mut f32,
    pub runner_up: *mut f32,
    pub n_tokens: i32,
    pub n_segments: i32,
    pub segments: *mut spt_pk_segment,
    pub n_chunks: i32,
    pub reserved0: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct spt_pk_model_info {
    pub n_mels: i32,
    pub d: i32,
    pub n_layers: i32,
    pub n_heads: i32,
    pub ff: i32,
    pub sub_ch: i32,
    pub conv_k: i32,
    pub pred: i32,
    pub n_vocab: i32,
    pub n_dur: i32,
    pub dtype: i32,
    pub max_batch: i32,
    pub max_samples: i32,
    pub reserved0: i32,
    pub weight_bytes: i64,
    pub workspace_bytes: i64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct spt_pk_timings {
    pub mel_ms: f64,
    pub encoder_ms: f64,
    pub decode_ms: f64,
    pub total_ms: f64,
    pub h2d_ms: f64,
    pub n_steps: i32,
    pub batch: i32,
    pub enc_frames: i32,
    pub reserved0: i32,
}
