//! `HipWhisperEngine` and `HipParakeetEngine`: the `transcribe_rs::TranscriptionEngine` surfaces
//! Spittle binds to, backed by the MI355X-native library (`libspittle_hip.so`, C ABI 12), plus `HipFrameResampler` and
//! `HipSmoothedVad` (the capture-side resampler and voice-activity gate).
//!
//! What it replaces in the app (/root/reference/src-tauri/src/managers/transcription.rs):
//!
//! | app call site | transcribe-rs `WhisperEngine` | here |
//! |---|---|---|
//! | `:29-34` `LoadedEngine::Whisper(WhisperEngine)` | engine type | `HipWhisperEngine` (feature swap) |
//! | `:261-276` | `WhisperEngine::new()` + `load_model(&path)` | `new()` + `load_model` (ggml `.bin` from the catalog) |
//! | `:494-503` | `transcribe_samples(audio, Some(WhisperInferenceParams { language, translate, initial_prompt, ..Default::default() }))` | same call |
//! | `:175-208` | `unload_model()` / `Drop` | same |
//!
//! The trait and parameter types come from transcribe-rs 0.2.3 itself, so the app's code at
//! those sites compiles unchanged.  The trait's shape (associated `InferenceParams` /
//! `ModelParams`, `load_model_with_params`, `transcribe_samples(Vec<f32>, Option<_>)`) is
//! restated from the published crate, which is not vendored in the reference
//! [upstream, unverifiable offline].
//!
//! Threading: the app loads from a spawned thread, transcribes from a tokio worker and unloads
//! from the idle watcher, serialised by one Mutex (transcription.rs:36-47, 437).  A context
//! selects its device on every entry point, so the engine is `Send`; it is not `Sync`.

use std::error::Error;
use std::ffi::{CStr, CString};
use std::os::raw::c_char;
use std::path::Path;

use spittle_hip_sys as sys;
use transcribe_rs::engines::parakeet::{ParakeetInferenceParams, TimestampGranularity};
use transcribe_rs::engines::whisper::WhisperInferenceParams;
use transcribe_rs::{TranscriptionEngine, TranscriptionResult, TranscriptionSegment};

/// Device-side model parameters (`spt_model_params`).  The defaults are what the app needs:
/// bf16 weights on device 0, one utterance (and up to 7 more 30 s windows of it) per call.
#[derive(Clone, Copy, Debug)]
pub struct HipModelParams {
    pub bf16: bool,
    pub device: i32,
    pub max_batch: i32,
}

impl Default for HipModelParams {
    fn default() -> Self {
        Self { bf16: true, device: 0, max_batch: 8 }
    }
}

fn model_params(p: &HipModelParams) -> sys::spt_model_params {
    let mut mp = std::mem::MaybeUninit::<sys::spt_model_params>::uninit();
    // SAFETY: spt_default_model_params fills every field of the struct
    let mut mp = unsafe {
        sys::spt_default_model_params(mp.as_mut_ptr());
        mp.assume_init()
    };
    mp.dtype = if p.bf16 { sys::SPT_DTYPE_BF16 } else { sys::SPT_DTYPE_F32 };
    mp.device = p.device;
    mp.max_batch = p.max_batch;
    mp
}

fn status_error(what: &str, st: sys::spt_status, msg: String) -> Box<dyn Error> {
    format!("{what} failed (status {st}): {msg}").into()
}

/// The request's parameters, with the CStrings their pointers borrow kept alive beside them.
struct Request {
    ip: sys::spt_infer_params,
    _language: Option<CString>,
    _prompt: Option<CString>,
}

/// whisper_full's defaults (`spt_default_infer_params`) plus the fields the app sets
/// (transcription.rs:445-499): language (None or "auto" = auto-detect), translate,
/// initial_prompt (the jargon prompt, jargon.rs:594), and the two suppression switches
/// `WhisperInferenceParams` carries.
fn request(params: Option<WhisperInferenceParams>) -> Result<Request, Box<dyn Error>> {
    let params = params.unwrap_or_default();
    let language = params.language.clone().map(CString::new).transpose()?;
    let prompt = params.initial_prompt.clone().map(CString::new).transpose()?;
    let mut ip = std::mem::MaybeUninit::<sys::spt_infer_params>::uninit();
    // SAFETY: spt_default_infer_params fills every field of the struct
    let mut ip = unsafe {
        sys::spt_default_infer_params(ip.as_mut_ptr());
        ip.assume_init()
    };
    ip.language = language.as_ref().map_or(std::ptr::null(), |s| s.as_ptr());
    ip.translate = params.translate as i32;
    ip.initial_prompt = prompt.as_ref().map_or(std::ptr::null(), |s| s.as_ptr());
    if params.suppress_non_speech_tokens {
        ip.flags |= sys::SPT_SUPPRESS_NST;
    }
    if !params.suppress_blank {
        ip.flags &= !sys::SPT_SUPPRESS_BLANK;
    }
    Ok(Request { ip, _language: language, _prompt: prompt })
}

/// Copy a library-owned result into transcribe-rs' type and release it.
///
/// SAFETY: `r` must be a result returned by the library and not yet freed.
unsafe fn take_result(r: *mut sys::spt_result) -> TranscriptionResult {
    let res = &*r;
    let text = if res.text.is_null() { String::new() } else { CStr::from_ptr(res.text).to_string_lossy().into_owned() };
    let segments = (0..res.n_segments.max(0) as usize)
        .map(|i| {
            let s = &*res.segments.add(i);
            TranscriptionSegment {
                // whisper_full_get_segment_t0 / t1 are in 10 ms units
                start: s.t0 as f32 / 100.0,
                end: s.t1 as f32 / 100.0,
                text: if s.text.is_null() { String::new() } else { CStr::from_ptr(s.text).to_string_lossy().into_owned() },
            }
        })
        .collect();
    sys::spt_result_free(r);
    TranscriptionResult { text, segments: Some(segments) }
}

/// One Whisper model on one MI355X.
pub struct HipWhisperEngine {
    ctx: *mut sys::spt_ctx,
}

// SAFETY: a context is not thread-affine (every entry point selects its device); the app
// serialises all calls through one Mutex, which is what `Send` without `Sync` expresses.
unsafe impl Send for HipWhisperEngine {}

impl HipWhisperEngine {
    pub fn new() -> Self {
        Self { ctx: std::ptr::null_mut() }
    }

    fn last_error(&self) -> String {
        // SAFETY: spt_last_error accepts any context pointer (a static string for null)
        unsafe { CStr::from_ptr(sys::spt_last_error(self.ctx)).to_string_lossy().into_owned() }
    }

    fn need(&self) -> Result<(), Box<dyn Error>> {
        if self.ctx.is_null() {
            return Err("Model is not loaded for transcription.".into());
        }
        Ok(())
    }

    /// Several utterances in one call (each <= 30 s window is a batch row).
    pub fn transcribe_batch(
        &mut self,
        batch: &[Vec<f32>],
        params: Option<WhisperInferenceParams>,
    ) -> Result<Vec<TranscriptionResult>, Box<dyn Error>> {
        self.need()?;
        let rq = request(params)?;
        let ptrs: Vec<*const f32> = batch.iter().map(|a| a.as_ptr()).collect();
        let lens: Vec<usize> = batch.iter().map(|a| a.len()).collect();
        let mut out = vec![std::ptr::null_mut::<sys::spt_result>(); batch.len()];
        // SAFETY: every pointer is valid for its length for the duration of the call
        let st = unsafe {
            sys::spt_transcribe_batch(self.ctx, ptrs.as_ptr(), lens.as_ptr(), batch.len(), &rq.ip, out.as_mut_ptr())
        };
        if st != sys::SPT_OK {
            return Err(status_error("transcription", st, self.last_error()));
        }
        // SAFETY: on success every out[i] is a live library result
        Ok(out.into_iter().map(|r| unsafe { take_result(r) }).collect())
    }
}

impl Default for HipWhisperEngine {
    fn default() -> Self {
        Self::new()
    }
}

impl TranscriptionEngine for HipWhisperEngine {
    type InferenceParams = WhisperInferenceParams;
    type ModelParams = HipModelParams;

    fn load_model_with_params(&mut self, model_path: &Path, params: HipModelParams) -> Result<(), Box<dyn Error>> {
        self.unload_model();
        // the catalog's ggml-*.bin (managers/model.rs:804-847)
        let spec = CString::new(model_path.to_string_lossy().as_bytes())?;
        let mp = model_params(&params);
        let mut err = vec![0 as c_char; 1024];
        let mut ctx = std::ptr::null_mut();
        // SAFETY: valid C strings and out-pointers for the duration of the call
        let st = unsafe { sys::spt_ctx_create(spec.as_ptr(), &mp, &mut ctx, err.as_mut_ptr(), err.len()) };
        if st != sys::SPT_OK {
            // SAFETY: the library NUL-terminates err
            let msg = unsafe { CStr::from_ptr(err.as_ptr()) }.to_string_lossy().into_owned();
            return Err(status_error("model load", st, msg));
        }
        self.ctx = ctx;
        Ok(())
    }

    fn unload_model(&mut self) {
        if !self.ctx.is_null() {
            // SAFETY: the context came from spt_ctx_create and is destroyed once
            unsafe { sys::spt_ctx_destroy(self.ctx) };
            self.ctx = std::ptr::null_mut();
        }
    }

    /// The app's call (transcription.rs:501-503).  `samples` (16 kHz mono f32) is borrowed for
    /// the call and copied to the device; the result's `text` is whisper_full's segment texts
    /// joined and trimmed, `segments` carries their times.
    fn transcribe_samples(
        &mut self,
        samples: Vec<f32>,
        params: Option<WhisperInferenceParams>,
    ) -> Result<TranscriptionResult, Box<dyn Error>> {
        self.need()?;
        let rq = request(params)?;
        let mut out = std::ptr::null_mut();
        // SAFETY: samples outlives the call; out receives a library-owned result
        let st = unsafe { sys::spt_transcribe(self.ctx, samples.as_ptr(), samples.len(), &rq.ip, &mut out) };
        if st != sys::SPT_OK {
            return Err(status_error("transcription", st, self.last_error()));
        }
        // SAFETY: a successful call returns a live result
        Ok(unsafe { take_result(out) })
    }
}

impl Drop for HipWhisperEngine {
    fn drop(&mut self) {
        self.unload_model();
    }
}

/// One model replicated over several MI355X of a node: device 0 loads it, one
/// RCCL broadcast over xGMI fills the others; a batch of utterances is split into contiguous
/// shards, one per device, transcribed concurrently.
pub struct HipWhisperReplicas {
    ctxs: Vec<*mut sys::spt_ctx>,
    /// wall time of the weight broadcast at load, ms
    pub broadcast_ms: f64,
}

// SAFETY: as for HipWhisperEngine
unsafe impl Send for HipWhisperReplicas {}

impl HipWhisperReplicas {
    pub fn load(model_path: &Path, params: HipModelParams, devices: &[i32]) -> Result<Self, Box<dyn Error>> {
        let spec = CString::new(model_path.to_string_lossy().as_bytes())?;
        let mp = model_params(&params);
        let mut ctxs = vec![std::ptr::null_mut(); devices.len()];
        let mut ms = 0.0f64;
        let mut err = vec![0 as c_char; 1024];
        // SAFETY: buffers sized for devices.len() contexts
        let st = unsafe {
            sys::spt_ctx_create_replicas(
                spec.as_ptr(),
                &mp,
                devices.as_ptr(),
                devices.len() as i32,
                ctxs.as_mut_ptr(),
                &mut ms,
                err.as_mut_ptr(),
                err.len(),
            )
        };
        if st != sys::SPT_OK {
            // SAFETY: the library NUL-terminates err
            let msg = unsafe { CStr::from_ptr(err.as_ptr()) }.to_string_lossy().into_owned();
            return Err(status_error("replica load", st, msg));
        }
        Ok(Self { ctxs, broadcast_ms: ms })
    }

    pub fn transcribe_batch(
        &mut self,
        batch: &[Vec<f32>],
        params: Option<WhisperInferenceParams>,
    ) -> Result<Vec<TranscriptionResult>, Box<dyn Error>> {
        let rq = request(params)?;
        let ptrs: Vec<*const f32> = batch.iter().map(|a| a.as_ptr()).collect();
        let lens: Vec<usize> = batch.iter().map(|a| a.len()).collect();
        let mut out = vec![std::ptr::null_mut::<sys::spt_result>(); batch.len()];
        // SAFETY: every pointer is valid for its length for the duration of the call
        let st = unsafe {
            sys::spt_transcribe_batch_replicas(
                self.ctxs.as_ptr(),
                self.ctxs.len() as i32,
                ptrs.as_ptr(),
                lens.as_ptr(),
                batch.len(),
                &rq.ip,
                out.as_mut_ptr(),
            )
        };
        if st != sys::SPT_OK {
            // SAFETY: ctxs[0] is live; it carries the failing replica's message
            let msg = unsafe { CStr::from_ptr(sys::spt_last_error(self.ctxs[0])) }.to_string_lossy().into_owned();
            return Err(status_error("replica transcription", st, msg));
        }
        // SAFETY: on success every out[i] is a live library result
        Ok(out.into_iter().map(|r| unsafe { take_result(r) }).collect())
    }
}

impl Drop for HipWhisperReplicas {
    fn drop(&mut self) {
        for c in self.ctxs.drain(..) {
            // SAFETY: each context is destroyed once
            unsafe { sys::spt_ctx_destroy(c) };
        }
    }
}

/// Device-side Parakeet parameters (`spt_pk_model_params`).  `int8()` mirrors the app's
/// `ParakeetModelParams::int8()` (transcription.rs:281); the network runs with an fp16 encoder.
#[derive(Clone, Copy, Debug)]
pub struct HipParakeetModelParams {
    pub fp16: bool,
    pub device: i32,
    pub max_batch: i32,
    pub max_seconds: f32,
}

impl HipParakeetModelParams {
    pub fn int8() -> Self {
        Self { fp16: true, device: 0, max_batch: 8, max_seconds: 30.0 }
    }
}

impl Default for HipParakeetModelParams {
    fn default() -> Self {
        Self::int8()
    }
}

/// Parakeet-V3 (FastConformer-TDT) on one MI355X.  What it replaces: `LoadedEngine::Parakeet`
/// (transcription.rs:278-297 load, :505-513 `transcribe_samples` with
/// `TimestampGranularity::Segment`).  The model path is a synthetic spec; a NeMo checkpoint is
/// mapped onto the context tensor by tensor with `set_tensor`.
pub struct HipParakeetEngine {
    ctx: *mut sys::spt_pk_ctx,
}

// SAFETY: as for HipWhisperEngine (calls serialised by the app's Mutex; not thread-affine)
unsafe impl Send for HipParakeetEngine {}

impl HipParakeetEngine {
    pub fn new() -> Self {
        Self { ctx: std::ptr::null_mut() }
    }

    fn last_error(&self) -> String {
        // SAFETY: accepts any context pointer (a static string for null)
        unsafe { CStr::from_ptr(sys::spt_parakeet_last_error(self.ctx)).to_string_lossy().into_owned() }
    }

    /// One weight tensor (f32, NeMo layout) by the id table of oracle/po_model.c.
    pub fn set_tensor(&mut self, tensor_id: i32, data: &[f32]) -> Result<(), Box<dyn Error>> {
        // SAFETY: data is valid for its length during the call
        let st = unsafe { sys::spt_parakeet_set_tensor(self.ctx, tensor_id, data.as_ptr(), data.len() as i64) };
        if st != sys::SPT_OK {
            return Err(status_error("set_tensor", st, self.last_error()));
        }
        Ok(())
    }
}

impl Default for HipParakeetEngine {
    fn default() -> Self {
        Self::new()
    }
}

fn granularity(g: &TimestampGranularity) -> i32 {
    match g {
        TimestampGranularity::Token => sys::SPT_PK_TS_TOKEN,
        TimestampGranularity::Word => sys::SPT_PK_TS_WORD,
        TimestampGranularity::Segment => sys::SPT_PK_TS_SEGMENT,
    }
}

impl TranscriptionEngine for HipParakeetEngine {
    type InferenceParams = ParakeetInferenceParams;
    type ModelParams = HipParakeetModelParams;

    fn load_model_with_params(&mut self, model_path: &Path, params: HipParakeetModelParams) -> Result<(), Box<dyn Error>> {
        self.unload_model();
        let spec = CString::new(model_path.to_string_lossy().as_bytes())?;
        let mut mp = std::mem::MaybeUninit::<sys::spt_pk_model_params>::uninit();
        // SAFETY: fills every field
        let mut mp = unsafe {
            sys::spt_parakeet_default_model_params(mp.as_mut_ptr());
            mp.assume_init()
        };
        mp.dtype = if params.fp16 { sys::SPT_DTYPE_F16 } else { sys::SPT_DTYPE_F32 };
        mp.device = params.device;
        mp.max_batch = params.max_batch;
        mp.max_seconds = params.max_seconds;
        let mut err = vec![0 as c_char; 1024];
        let mut ctx = std::ptr::null_mut();
        // SAFETY: valid C strings and out-pointers for the duration of the call
        let st = unsafe { sys::spt_parakeet_create(spec.as_ptr(), &mp, &mut ctx, err.as_mut_ptr(), err.len()) };
        if st != sys::SPT_OK {
            // SAFETY: the library NUL-terminates err
            let msg = unsafe { CStr::from_ptr(err.as_ptr()) }.to_string_lossy().into_owned();
            return Err(status_error("model load", st, msg));
        }
        self.ctx = ctx;
        Ok(())
    }

    fn unload_model(&mut self) {
        if !self.ctx.is_null() {
            // SAFETY: created by spt_parakeet_create, destroyed once
            unsafe { sys::spt_parakeet_destroy(self.ctx) };
            self.ctx = std::ptr::null_mut();
        }
    }

    fn transcribe_samples(
        &mut self,
        samples: Vec<f32>,
        params: Option<ParakeetInferenceParams>,
    ) -> Result<TranscriptionResult, Box<dyn Error>> {
        if self.ctx.is_null() {
            return Err("Model is not loaded for transcription.".into());
        }
        let mut ip = sys::spt_pk_infer_params { max_symbols: 10, timestamp_granularity: sys::SPT_PK_TS_SEGMENT };
        // SAFETY: fills every field
        unsafe { sys::spt_parakeet_default_infer_params(&mut ip) };
        if let Some(p) = params.as_ref() {
            ip.timestamp_granularity = granularity(&p.timestamp_granularity);
        }
        let mut out = std::ptr::null_mut();
        // SAFETY: samples outlives the call; out receives a library-owned result
        let st = unsafe { sys::spt_parakeet_transcribe(self.ctx, samples.as_ptr(), samples.len(), &ip, &mut out) };
        if st != sys::SPT_OK {
            return Err(status_error("transcription", st, self.last_error()));
        }
        // SAFETY: a successful call returns a live result, read then freed once
        unsafe {
            let res = &*out;
            let text = if res.text.is_null() { String::new() } else { CStr::from_ptr(res.text).to_string_lossy().into_owned() };
            let segments = (0..res.n_segments.max(0) as usize)
                .map(|i| {
                    let s = &*res.segments.add(i);
                    TranscriptionSegment {
                        start: s.start as f32,
                        end: s.end as f32,
                        text: if s.text.is_null() { String::new() } else { CStr::from_ptr(s.text).to_string_lossy().into_owned() },
                    }
                })
                .collect();
            sys::spt_parakeet_result_free(out);
            Ok(TranscriptionResult { text, segments: Some(segments) })
        }
    }
}

impl Drop for HipParakeetEngine {
    fn drop(&mut self) {
        self.unload_model();
    }
}

/// The capture-side resampler (ABI 7): `FrameResampler` of
/// /root/reference/src-tauri/src/audio_toolkit/audio/resampler.rs:7-104 over the device.
/// `process_stream` = `FrameResampler::new(in_hz, out_hz, frame_dur)` + `push(all)` + `finish`
/// (recorder.rs:264-268, 330, 355): the concatenated frames of one recorded stream.  The app's
/// streaming `push` per capture buffer stays on the host; a recording-level caller (or a batch
/// re-import of a file) hands the whole stream over at once.
pub struct HipFrameResampler {
    r: *mut sys::spt_resampler,
}

// SAFETY: the context selects its device on every call and holds no thread-local state
unsafe impl Send for HipFrameResampler {}

impl HipFrameResampler {
    pub fn new(in_hz: u32, out_hz: u32, frame_dur: std::time::Duration, device: i32) -> Result<Self, Box<dyn Error>> {
        let frame_samples = (out_hz as f64 * frame_dur.as_secs_f64()).round() as i32;
        if frame_samples <= 0 {
            return Err("frame duration too short".into());
        }
        let mut r = std::ptr::null_mut();
        let mut err = vec![0 as c_char; 512];
        // SAFETY: out-pointer and error buffer are valid for the call
        let st = unsafe {
            sys::spt_resampler_create(in_hz as i32, out_hz as i32, frame_samples, device, &mut r, err.as_mut_ptr(), err.len())
        };
        if st != sys::SPT_OK {
            // SAFETY: the library NUL-terminates the message inside the buffer
            let msg = unsafe { CStr::from_ptr(err.as_ptr()) }.to_string_lossy().into_owned();
            return Err(status_error("resampler", st, msg));
        }
        Ok(Self { r })
    }

    pub fn process_stream(&mut self, samples: &[f32]) -> Result<Vec<f32>, Box<dyn Error>> {
        // SAFETY: a live context; the length query has no other effect
        let need = unsafe { sys::spt_resample_output_len(self.r, samples.len()) };
        let mut out = vec![0f32; need];
        let mut n_out = 0usize;
        // SAFETY: both buffers outlive the call and `out` holds `need` samples
        let st = unsafe { sys::spt_resample(self.r, samples.as_ptr(), samples.len(), out.as_mut_ptr(), out.len(), &mut n_out) };
        if st != sys::SPT_OK {
            // SAFETY: the message lives in the context until its next call
            let msg = unsafe { CStr::from_ptr(sys::spt_resampler_last_error(self.r)) }.to_string_lossy().into_owned();
            return Err(status_error("resample", st, msg));
        }
        out.truncate(n_out);
        Ok(out)
    }
}

impl Drop for HipFrameResampler {
    fn drop(&mut self) {
        // SAFETY: created by spt_resampler_create, destroyed once
        unsafe { sys::spt_resampler_destroy(self.r) };
    }
}

/// The capture-side voice-activity gate (ABI 8): `SmoothedVad::new(Box::new(SileroVad::new(path,
/// 0.3)), 15, 15, 2)` of /root/reference/src-tauri/src/managers/audio.rs:132-134 in one object,
/// the Silero network on the device.  `push_frame` has the app's `VoiceActivityDetector` shape
/// (audio_toolkit/vad/mod.rs); the app-side adapter is three lines.
pub struct HipSmoothedVad {
    v: *mut sys::spt_vad,
    last: Vec<f32>,
}

/// `VadFrame` of audio_toolkit/vad/mod.rs
pub enum HipVadFrame<'a> {
    Speech(&'a [f32]),
    Noise,
}

// SAFETY: the context selects its device on every call and holds no thread-local state
unsafe impl Send for HipSmoothedVad {}

impl HipSmoothedVad {
    pub fn new<P: AsRef<Path>>(model_path: P, threshold: f32, prefill: usize, hangover: usize, onset: usize,
                               device: i32) -> Result<Self, Box<dyn Error>> {
        let path = CString::new(model_path.as_ref().to_string_lossy().as_bytes())?;
        let mut p = sys::spt_vad_params { threshold, prefill_frames: prefill as i32, hangover_frames: hangover as i32,
                                          onset_frames: onset as i32, device, reserved0: 0 };
        if !(0.0..=1.0).contains(&threshold) {
            return Err("threshold must be between 0.0 and 1.0".into());
        }
        let mut v = std::ptr::null_mut();
        let mut err = vec![0 as c_char; 512];
        // SAFETY: every pointer is valid for the call
        let st = unsafe { sys::spt_vad_create(path.as_ptr(), &mut p, &mut v, err.as_mut_ptr(), err.len()) };
        if st != sys::SPT_OK {
            // SAFETY: the library NUL-terminates the message inside the buffer
            let msg = unsafe { CStr::from_ptr(err.as_ptr()) }.to_string_lossy().into_owned();
            return Err(status_error("vad", st, msg));
        }
        Ok(Self { v, last: Vec::new() })
    }

    /// One 30 ms frame (or a whole recorded stream, frame after frame): the kept samples.
    pub fn push_frame<'a>(&'a mut self, frame: &'a [f32]) -> Result<HipVadFrame<'a>, Box<dyn Error>> {
        let mut r = std::ptr::null_mut();
        // SAFETY: the frame outlives the call; the result is library-owned and freed below
        let st = unsafe { sys::spt_vad_push(self.v, frame.as_ptr(), frame.len(), &mut r) };
        if st != sys::SPT_OK {
            // SAFETY: the message lives in the context until its next call
            let msg = unsafe { CStr::from_ptr(sys::spt_vad_last_error(self.v)) }.to_string_lossy().into_owned();
            return Err(status_error("vad push", st, msg));
        }
        // SAFETY: r is a valid result until spt_vad_result_free
        let (kept, speech) = unsafe {
            let res = &*r;
            let kept = if res.n_samples > 0 { std::slice::from_raw_parts(res.samples, res.n_samples).to_vec() } else { Vec::new() };
            (kept, res.n_frames > 0 && *res.kind != 0)
        };
        // SAFETY: freed once
        unsafe { sys::spt_vad_result_free(r) };
        self.last = kept;
        Ok(if speech { HipVadFrame::Speech(&self.last) } else { HipVadFrame::Noise })
    }

    /// `SmoothedVad::reset` (the Silero state carries over, as in the app)
    pub fn reset(&mut self) {
        // SAFETY: a live context
        unsafe { sys::spt_vad_reset(self.v, 0) };
    }
}

impl Drop for HipSmoothedVad {
    fn drop(&mut self) {
        // SAFETY: created by spt_vad_create, destroyed once
        unsafe { sys::spt_vad_destroy(self.v) };
    }
}
