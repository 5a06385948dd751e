"""Host mirror of Spittle's FrameResampler over the HIP resampler (ABI 7).

/root/reference/src-tauri/src/audio_toolkit/audio/resampler.rs:7-104: FrameResampler::new(in_hz,
out_hz, frame_dur) over rubato FftFixedIn (1024-sample input chunks), push / finish with an emit
callback per frame.  The recorder (recorder.rs:264-268, 330, 355) pushes every capture buffer and
finishes on Stop; `process_stream` is that whole sequence for one recorded stream, computed on the
GPU in one call (spt_resample): every rubato unit is one row of an f32 GEMM against the unit's
fixed linear map, then an overlap-add.  No CPU fallback: without libspittle_hip.so this raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class ResamplerError(RuntimeError):
    pass


class FrameResampler:
    def __init__(self, in_hz: int, out_hz: int, frame_dur_s: float = 0.030, device: int = 0):
        self.frame_samples = int(round(out_hz * frame_dur_s))
        if self.frame_samples <= 0:
            raise ResamplerError("frame duration too short")  # resampler.rs:18 assert
        self._lib = L.load()
        self._r = C.c_void_p()
        err = C.create_string_buffer(512)
        st = self._lib.spt_resampler_create(int(in_hz), int(out_hz), self.frame_samples, int(device),
                                            C.byref(self._r), err, 512)
        if st != L.SPT_OK:
            raise ResamplerError(f"spt_resampler_create: {L.STATUS_NAMES.get(st, st)}: {err.value.decode()}")
        self.in_hz, self.out_hz = in_hz, out_hz

    @property
    def fft_sizes(self) -> tuple[int, int]:
        a, b = C.c_int32(), C.c_int32()
        self._lib.spt_resampler_info(self._r, C.byref(a), C.byref(b))
        return a.value, b.value

    def output_len(self, n_samples: int) -> int:
        return int(self._lib.spt_resample_output_len(self._r, int(n_samples)))

    def process_stream(self, pcm) -> np.ndarray:
        """FrameResampler::new + push(pcm) + finish: the concatenated 30 ms frames."""
        x = np.ascontiguousarray(pcm, dtype=np.float32)
        out = np.empty(max(self.output_len(len(x)), 1), dtype=np.float32)
        n_out = C.c_size_t()
        fp = C.POINTER(C.c_float)
        st = self._lib.spt_resample(self._r, x.ctypes.data_as(fp), len(x), out.ctypes.data_as(fp), len(out),
                                    C.byref(n_out))
        if st != L.SPT_OK:
            raise ResamplerError(f"spt_resample: {L.STATUS_NAMES.get(st, st)}: "
                                 f"{self._lib.spt_resampler_last_error(self._r).decode()}")
        return out[: n_out.value]

    def close(self) -> None:
        if self._r:
            self._lib.spt_resampler_destroy(self._r)
            self._r = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
