"""Host-side mirror of transcribe-rs' Whisper engine surface, over the C ABI.

Reference interface (transcribe-rs 0.2.3, used by
/root/reference/src-tauri/src/managers/transcription.rs):
  * ``WhisperEngine::new()`` / ``load_model(&path)``        (transcription.rs:261-276)
  * ``transcribe_samples(Vec<f32>, Option<WhisperInferenceParams>)
     -> Result<TranscriptionResult>``                        (transcription.rs:494-503)
  * ``unload_model()``                                       (transcription.rs:175-208)
  * ``WhisperInferenceParams { language, translate, initial_prompt, ..Default }``
                                                             (transcription.rs:445-499)
  * ``TranscriptionResult { text, segments }``; the app uses ``.text``
                                                             (transcription.rs:537-546)

Same names, same meaning, same error behaviour (an exception carrying the
status and message where the Rust engine returns ``Err(Box<dyn Error>)``).
Everything below the boundary runs on the GPU (libspittle_hip.so); there is no
CPU path here.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

from . import _lib as L


class TranscriptionError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{L.STATUS_NAMES.get(status, status)}: {message}")
        self.status = status
        self.message = message


@dataclass
class WhisperModelParams:
    dtype: str = "bf16"          # "bf16" | "f32"
    device: int = 0
    max_batch: int = 8
    seed: int = 1234             # synthetic weights
    # allocate the weight arena but leave it empty: import_weights() fills it (multi-GPU load,
    # rank 0's arena broadcast over RCCL; spittle_amd.dist.broadcast_weights)
    external_weights: bool = False


@dataclass
class WhisperInferenceParams:
    language: Optional[str] = None      # None / "auto" = auto-detect (settings "auto")
    translate: bool = False
    initial_prompt: Optional[str] = None
    # whisper_full_params.prompt_tokens: token ids decoded before [sot ...] (what initial_prompt
    # becomes after tokenization)
    prompt_tokens: Optional[Sequence[int]] = None
    # whisper_full_params the app leaves at their defaults (whisper_full_default_params)
    suppress_blank: bool = True
    suppress_non_speech_tokens: bool = False
    no_timestamps: bool = False
    max_new_tokens: int = 220           # fast path: tokens per window; whisper_full: max_tokens
    temperature: float = 0.0
    temperature_inc: float = 0.2        # fallback step; 0 = none
    best_of: int = 5
    entropy_thold: float = 2.4
    logprob_thold: float = -1.0
    max_initial_ts: float = 1.0
    beam_size: int = 1
    seed: int = 0
    # benchmark / test hooks
    ignore_eot: bool = False
    forced_tokens: Optional[np.ndarray] = None  # [batch][n] teacher forcing


@dataclass
class TranscriptionSegment:
    start: float            # seconds (whisper_full_get_segment_t0 / 100, as transcribe-rs)
    end: float
    text: str
    i0: int = 0             # the segment's tokens: TranscriptionResult.tokens[i0:i0 + n_tokens]
    n_tokens: int = 0


@dataclass
class TranscriptionResult:
    text: str
    segments: list = field(default_factory=list)
    tokens: list = field(default_factory=list)
    top1: Optional[np.ndarray] = None
    top2: Optional[np.ndarray] = None
    n_windows: int = 0
    language: Optional[str] = None      # ISO-639-1 code decoded with (detected or given)
    n_fallbacks: int = 0                # temperature fallbacks taken (repeated decodes)


def _infer_params(p: Optional[WhisperInferenceParams], keep: list) -> L.InferParams:
    p = p or WhisperInferenceParams()
    ip = L.InferParams()
    ip.language = p.language.encode() if p.language else None
    ip.translate = int(bool(p.translate))
    ip.initial_prompt = p.initial_prompt.encode() if p.initial_prompt else None
    ip.flags = (L.SPT_SUPPRESS_BLANK if p.suppress_blank else 0) | \
               (L.SPT_NO_TIMESTAMPS if p.no_timestamps else 0) | (L.SPT_IGNORE_EOT if p.ignore_eot else 0) | \
               (L.SPT_SUPPRESS_NST if p.suppress_non_speech_tokens else 0)
    ip.max_new_tokens = int(p.max_new_tokens)
    ip.temperature = float(p.temperature)
    ip.beam_size = int(p.beam_size)
    ip.temperature_inc = float(p.temperature_inc)
    ip.best_of = int(p.best_of)
    ip.entropy_thold = float(p.entropy_thold)
    ip.logprob_thold = float(p.logprob_thold)
    ip.max_initial_ts = float(p.max_initial_ts)
    ip.seed = int(p.seed)
    if p.forced_tokens is not None:
        f = np.ascontiguousarray(p.forced_tokens, dtype=np.int32)
        keep.append(f)
        ip.forced_tokens = f.ctypes.data_as(C.POINTER(C.c_int32))
        ip.n_forced = int(f.shape[-1])
    if p.prompt_tokens is not None and len(p.prompt_tokens) > 0:
        t = np.ascontiguousarray(np.asarray(p.prompt_tokens, dtype=np.int32).reshape(-1))
        keep.append(t)
        ip.prompt_tokens = t.ctypes.data_as(C.POINTER(C.c_int32))
        ip.n_prompt_tokens = int(t.size)
    return ip


def _take_result(rp) -> TranscriptionResult:
    r = rp.contents
    n = r.n_tokens
    toks = [r.tokens[i] for i in range(n)]
    t1 = np.ctypeslib.as_array(r.top1, shape=(n,)).copy() if n else np.zeros(0, np.float32)
    t2 = np.ctypeslib.as_array(r.top2, shape=(n,)).copy() if n else np.zeros(0, np.float32)
    lib = L.load()
    code = lib.spt_language_code(r.language) if r.language >= 0 else None
    segs = []
    for i in range(r.n_segments):
        s = r.segments[i]
        segs.append(TranscriptionSegment(start=s.t0 / 100.0, end=s.t1 / 100.0,
                                         text=(s.text or b"").decode("utf-8", "replace"), i0=s.i0, n_tokens=s.n_tokens))
    res = TranscriptionResult(text=(r.text or b"").decode("utf-8", "replace"), segments=segs, tokens=toks, top1=t1,
                              top2=t2, n_windows=r.n_windows, language=code.decode() if code else None,
                              n_fallbacks=r.n_fallbacks)
    lib.spt_result_free(rp)
    return res


class WhisperEngine:
    """transcribe_rs::engines::whisper::WhisperEngine, MI355X-native."""

    def __init__(self, params: Optional[WhisperModelParams] = None):
        self._lib = L.load()
        self._ctx = None
        self.params = params or WhisperModelParams()
        self.model_path = None

    # -- lifecycle ----------------------------------------------------------
    def load_model(self, model_path: str) -> None:
        """`model_path`: a whisper.cpp ggml .bin file (f32/f16/q4_0/q4_1/q5_0/q5_1/q8_0 tensors)
        or ``synthetic:<name>[:enc=N][:dec=N][:seed=S]``."""
        self.unload_model()
        mp = L.ModelParams()
        self._lib.spt_default_model_params(C.byref(mp))
        mp.dtype = L.SPT_DTYPE_BF16 if self.params.dtype == "bf16" else L.SPT_DTYPE_F32
        mp.device = int(self.params.device)
        mp.max_batch = int(self.params.max_batch)
        mp.seed = int(self.params.seed)
        mp.flags = L.SPT_MODEL_WEIGHTS_EXTERNAL if self.params.external_weights else 0
        ctx = C.c_void_p()
        err = C.create_string_buffer(1024)
        st = self._lib.spt_ctx_create(str(model_path).encode(), C.byref(mp), C.byref(ctx), err, 1024)
        if st != L.SPT_OK:
            raise TranscriptionError(st, err.value.decode())
        self._ctx = ctx
        self.model_path = model_path

    def unload_model(self) -> None:
        if self._ctx:
            self._lib.spt_ctx_destroy(self._ctx)
            self._ctx = None

    def is_loaded(self) -> bool:
        return bool(self._ctx)

    def __del__(self):
        try:
            self.unload_model()
        except Exception:
            pass

    def _check(self, st: int):
        if st != L.SPT_OK:
            raise TranscriptionError(st, self._lib.spt_last_error(self._ctx).decode())

    def _need(self):
        if not self._ctx:
            raise TranscriptionError(L.SPT_ERR_INVALID_ARG, "Model is not loaded for transcription.")

    # -- inference ----------------------------------------------------------
    def transcribe_samples(self, samples, params: Optional[WhisperInferenceParams] = None) -> TranscriptionResult:
        return self.transcribe_batch([samples], params)[0]

    def transcribe_batch(self, batch: Sequence, params: Optional[WhisperInferenceParams] = None):
        self._need()
        keep: list = []
        ip = _infer_params(params, keep)
        arrs = [np.ascontiguousarray(np.asarray(s, dtype=np.float32).reshape(-1)) for s in batch]
        n = len(arrs)
        ptrs = (C.POINTER(C.c_float) * n)(*[a.ctypes.data_as(C.POINTER(C.c_float)) for a in arrs])
        lens = (C.c_size_t * n)(*[a.size for a in arrs])
        out = (C.POINTER(L.Result) * n)()
        self._check(self._lib.spt_transcribe_batch(self._ctx, ptrs, lens, n, C.byref(ip), out))
        return [_take_result(out[i]) for i in range(n)]

    def transcribe_batch_device(self, dev_ptr: int, stride: int, lengths: Sequence[int],
                                params: Optional[WhisperInferenceParams] = None):
        """Windows (<= 30 s each) already resident in device memory at dev_ptr + b*stride floats."""
        self._need()
        keep: list = []
        ip = _infer_params(params, keep)
        n = len(lengths)
        lens = (C.c_size_t * n)(*[int(x) for x in lengths])
        out = (C.POINTER(L.Result) * n)()
        self._check(self._lib.spt_transcribe_batch_device(self._ctx, C.c_void_p(dev_ptr), int(stride), lens, n,
                                                          C.byref(ip), out))
        return [_take_result(out[i]) for i in range(n)]

    # -- introspection / test hooks -----------------------------------------
    def export_weights(self, dev_ptr: int, nbytes: int) -> None:
        """Copy the device weight arena (info()["weight_bytes"] bytes) to device memory at dev_ptr."""
        self._need()
        self._check(self._lib.spt_weights_export(self._ctx, C.c_void_p(dev_ptr), C.c_size_t(nbytes)))

    def import_weights(self, dev_ptr: int, nbytes: int) -> None:
        """Fill the weight arena of an external-weights engine from device memory at dev_ptr."""
        self._need()
        self._check(self._lib.spt_weights_import(self._ctx, C.c_void_p(dev_ptr), C.c_size_t(nbytes)))

    def weights_arena(self) -> tuple:
        """(device pointer, bytes) of the weight arena: a collective writes straight into it."""
        self._need()
        ptr, n = C.c_void_p(), C.c_size_t()
        self._check(self._lib.spt_weights_arena(self._ctx, C.byref(ptr), C.byref(n)))
        return int(ptr.value or 0), int(n.value)

    def commit_weights(self) -> None:
        """Mark an external-weights engine usable once its arena holds the model's bytes."""
        self._need()
        self._check(self._lib.spt_weights_commit(self._ctx))

    def info(self) -> dict:
        self._need()
        mi = L.ModelInfo()
        self._check(self._lib.spt_ctx_info(self._ctx, C.byref(mi)))
        return {k: getattr(mi, k) for k, _ in mi._fields_}

    def timings(self) -> dict:
        self._need()
        t = L.Timings()
        self._check(self._lib.spt_get_timings(self._ctx, C.byref(t)))
        return {k: getattr(t, k) for k, _ in t._fields_}

    def call_stats(self) -> dict:
        """What the last transcribe* call ran in total (engine calls, decoder passes, device ms)."""
        self._need()
        t = L.CallStats()
        self._check(self._lib.spt_get_call_stats(self._ctx, C.byref(t)))
        return {k: getattr(t, k) for k, _ in t._fields_ if k != "reserved0"}

    def debug_mel(self, samples, seek: int = 0) -> np.ndarray:
        """The normalised log-mel [n_mels][3000] the encoder takes for the window at frame `seek`
        (frames seek .. seek + 2999 of the whole utterance's log-mel)."""
        self._need()
        x = np.ascontiguousarray(np.asarray(samples, np.float32).reshape(-1))
        out = np.empty((self.info()["n_mels"], 3000), np.float32)
        self._check(self._lib.spt_debug_mel_at(self._ctx, x.ctypes.data_as(C.POINTER(C.c_float)), x.size, int(seek),
                                               out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def debug_encode(self, mel) -> np.ndarray:
        self._need()
        info = self.info()
        m = np.ascontiguousarray(mel, dtype=np.float32)
        assert m.shape == (info["n_mels"], 3000)
        out = np.empty((info["n_audio_ctx"], info["d"]), np.float32)
        self._check(self._lib.spt_debug_encode(self._ctx, m.ctypes.data_as(C.POINTER(C.c_float)),
                                               out.ctypes.data_as(C.POINTER(C.c_float))))
        return out

    def probe(self, kernel: str, iters: int = 50) -> dict:
        """Time one hot-path kernel (HIP events, engine stream) on the last call's buffers."""
        self._need()
        us, work, fl = C.c_double(), C.c_double(), C.c_int32()
        self._check(self._lib.spt_probe_kernel(self._ctx, L.PROBES[kernel], int(iters), C.byref(us), C.byref(work),
                                               C.byref(fl)))
        return {"avg_us": us.value, "work": work.value, "work_is_flops": bool(fl.value)}

    def tokenize(self, text: str) -> list[int]:
        """whisper_tokenize with the loaded ggml model's vocabulary (greedy longest match)."""
        self._need()
        raw = text.encode("utf-8")
        n = C.c_int32()
        buf = (C.c_int32 * max(1, len(raw) + 1))()
        self._check(self._lib.spt_tokenize(self._ctx, raw, buf, len(raw) + 1, C.byref(n)))
        return [buf[i] for i in range(n.value)]

    def token_to_str(self, token: int) -> Optional[bytes]:
        """whisper_token_to_str: the token's bytes (None for synthetic models / bad ids)."""
        self._need()
        return self._lib.spt_token_to_str(self._ctx, int(token))

    def weight_checksum(self, tensor_id: int):
        self._need()
        o = (C.c_double * 2)()
        self._check(self._lib.spt_debug_weight_checksum(self._ctx, int(tensor_id), o))
        return float(o[0]), float(o[1])
