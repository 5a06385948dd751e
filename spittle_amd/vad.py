"""Host mirror of Spittle's capture-side voice-activity gate over the HIP implementation
(spt_vad_*, ABI 8).

Reference (src-tauri/src/audio_toolkit/vad/, managers/audio.rs:132-134, 295-307):
  * ``SileroVad::new(model_path, 0.3)``  -- vad/silero.rs:19-31 (the model file that ships with
    the app, resources/models/silero_vad_v4.onnx, run by vad-rs with its LSTM state carried)
  * ``SmoothedVad::new(Box::new(silero), 15, 15, 2)`` -- vad/smoothed.rs:20-41
  * ``push_frame(&[f32; 480]) -> VadFrame::{Speech(&[f32]), Noise}`` -- smoothed.rs:43-104
  * ``reset()``  -- smoothed.rs:106-112 (the smoothing only; SileroVad has no reset)
The network and the smoothing both run inside libspittle_hip.so (the network on the device);
there is no CPU path here.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib as L
from .engine import TranscriptionError

FRAME = 480  # 30 ms at 16 kHz


@dataclass
class VadFrame:
    """Speech(samples) or Noise (samples is None)."""
    samples: Optional[np.ndarray]

    def is_speech(self) -> bool:
        return self.samples is not None


@dataclass
class VadStreamResult:
    samples: np.ndarray     # the audio the recorder keeps (Speech frames, prefill at onsets)
    prob: np.ndarray        # per whole frame: Silero's speech probability
    kind: np.ndarray        # per frame: 0 Noise, 1 Speech(frame), 2 Speech(prefill + frame)
    device_ms: float


class SileroVad:
    """The inner detector's parameters (vad/silero.rs); it runs inside SmoothedVad's context."""

    def __init__(self, model_path: str, threshold: float):
        if not 0.0 <= threshold <= 1.0:
            raise ValueError("threshold must be between 0.0 and 1.0")
        self.model_path, self.threshold = str(model_path), float(threshold)


class SmoothedVad:
    def __init__(self, inner: SileroVad, prefill_frames: int = 15, hangover_frames: int = 15, onset_frames: int = 2,
                 device: int = 0):
        self._lib = L.load()
        p = L.VadParams()
        self._lib.spt_vad_default_params(C.byref(p))
        p.threshold, p.prefill_frames, p.hangover_frames, p.onset_frames, p.device = (
            inner.threshold, prefill_frames, hangover_frames, onset_frames, device)
        err = C.create_string_buffer(512)
        self._v = C.c_void_p()
        st = self._lib.spt_vad_create(inner.model_path.encode(), C.byref(p), C.byref(self._v), err, 512)
        if st != L.SPT_OK:
            raise TranscriptionError(st, err.value.decode())

    def push_stream(self, pcm) -> VadStreamResult:
        """push_frame over every 480-sample frame of pcm, in order (one device call)."""
        a = np.ascontiguousarray(np.asarray(pcm, dtype=np.float32).ravel())
        out = C.POINTER(L.VadResult)()
        st = self._lib.spt_vad_push(self._need(), a.ctypes.data_as(C.POINTER(C.c_float)), a.size, C.byref(out))
        if st != L.SPT_OK:
            raise TranscriptionError(st, self._lib.spt_vad_last_error(self._v).decode())
        r = out.contents
        nf = a.size // FRAME
        res = VadStreamResult(np.ctypeslib.as_array(r.samples, shape=(r.n_samples,)).copy() if r.n_samples else
                              np.zeros(0, np.float32),
                              np.ctypeslib.as_array(r.prob, shape=(nf,)).copy() if nf else np.zeros(0, np.float32),
                              np.ctypeslib.as_array(r.kind, shape=(r.n_frames,)).copy() if r.n_frames else
                              np.zeros(0, np.uint8), float(r.device_ms))
        self._lib.spt_vad_result_free(out)
        return res

    def push_frame(self, frame) -> VadFrame:
        r = self.push_stream(frame)
        return VadFrame(r.samples if r.kind.size and r.kind[0] else None)

    def is_voice(self, frame) -> bool:
        return self.push_frame(frame).is_speech()

    def reset(self, model_state: bool = False) -> None:
        """SmoothedVad::reset; model_state=True also zeroes the Silero LSTM state (a new SileroVad)."""
        self._lib.spt_vad_reset(self._need(), 1 if model_state else 0)

    def close(self) -> None:
        if self._v:
            self._lib.spt_vad_destroy(self._v)
            self._v = C.c_void_p()

    def _need(self):
        if not self._v:
            raise TranscriptionError(L.SPT_ERR_INVALID_ARG, "VAD closed")
        return self._v

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
