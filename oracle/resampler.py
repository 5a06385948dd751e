"""CPU restatement of Spittle's capture-side resampler.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's cpu_baseline leg, as the checker /
the reported CPU baseline.  spittle_amd/ never imports it.

What it follows:
* `FrameResampler` -- /root/reference/src-tauri/src/audio_toolkit/audio/resampler.rs:
  new (:16-35: chunk_in = RESAMPLER_CHUNK_SIZE = 1024 (:5), frame_samples =
  round(out_hz * frame_dur), rubato only when in_hz != out_hz), push (:37-64: fill a 1024-sample
  chunk, process it, emit the output as frames), finish (:66-86: zero-pad the partial chunk to
  1024 and process it, then zero-pad the pending partial frame), emit_frames (:88-103).
  The recorder feeds every capture buffer through push and calls finish on Stop
  (/root/reference/src-tauri/src/audio_toolkit/audio/recorder.rs:264-268, 330, 355).
* `rubato::FftFixedIn<f32>::new(in_hz, out_hz, 1024, 1, 1)` -- rubato 0.16.2
  (/root/reference/src-tauri/Cargo.lock:5384-5386; the crate is not vendored, so its algorithm
  is restated from its published source **[upstream, recalled]**):
  - fft sizes: g = gcd(in, out); fft_chunks = ceil(chunk / (in / g)); fft_size_in =
    fft_chunks * in / g, fft_size_out = fft_chunks * out / g;
  - each unit takes fft_size_in input frames (a saved-frames buffer carries the remainder of a
    1024-frame chunk to the next call), zero-pads them to 2 * fft_size_in, real FFT, multiplies by
    the filter spectrum, keeps bins [0, new_len) (new_len = fft_size_out when downsampling,
    fft_size_in + 1 when upsampling; the rest zero), unnormalised inverse real FFT of size
    2 * fft_size_out, first half + the previous unit's second half (overlap-add) is the output;
  - filter: fft_size_in taps of a Blackman-Harris^2-windowed sinc centred at fft_size_in / 2,
    normalised to unit sum, divided by 2 * fft_size_in; relative cutoff
    0.4^(16 / n) (n = fft_size_in) scaled by fft_size_out / fft_size_in when downsampling.
    The cutoff constant is the recalled part: parity against rubato itself is **unpinned** (no
    crate, no fixtures offline).  The GPU path takes the same filter definition
    (spittle_amd/csrc/resample.cpp), so GPU-vs-oracle parity checks the arithmetic exactly.
Computed in float64 (rubato runs in f32; the difference is at f32 rounding level).
"""
from __future__ import annotations

from math import ceil, gcd

import numpy as np

CHUNK_IN = 1024  # resampler.rs:5 RESAMPLER_CHUNK_SIZE


def fft_sizes(in_hz: int, out_hz: int, chunk_in: int = CHUNK_IN, sub_chunks: int = 1) -> tuple[int, int]:
    g = gcd(in_hz, out_hz)
    fft_chunks = int(ceil((chunk_in // sub_chunks) / (in_hz // g)))
    return fft_chunks * in_hz // g, fft_chunks * out_hz // g


def cutoff(fft_size_in: int, fft_size_out: int) -> float:
    c = 0.4 ** (16.0 / fft_size_in)
    return c * fft_size_out / fft_size_in if fft_size_in > fft_size_out else c


def blackman_harris2(n: int) -> np.ndarray:
    x = np.arange(n, dtype=np.float64) / n
    w = 0.35875 - 0.48829 * np.cos(2 * np.pi * x) + 0.14128 * np.cos(4 * np.pi * x) - 0.01168 * np.cos(6 * np.pi * x)
    return w * w


def filter_taps(fft_size_in: int, fft_size_out: int) -> np.ndarray:
    """The time-domain filter of one unit: [fft_size_in] (zero-padded to 2 * fft_size_in)."""
    n = fft_size_in
    fc = cutoff(fft_size_in, fft_size_out)
    arg = (np.arange(n, dtype=np.float64) - (n // 2)) * fc
    y = blackman_harris2(n) * np.sinc(arg)  # np.sinc(x) = sin(pi x) / (pi x)
    return y / y.sum() / (2 * n)


class FftFixedIn:
    """rubato FftFixedIn, one channel: fixed input chunk, variable output."""

    def __init__(self, in_hz: int, out_hz: int, chunk_in: int = CHUNK_IN):
        self.chunk_in = chunk_in
        self.nin, self.nout = fft_sizes(in_hz, out_hz, chunk_in)
        h = np.zeros(2 * self.nin)
        h[: self.nin] = filter_taps(self.nin, self.nout)
        self.hf = np.fft.rfft(h)  # [nin + 1]
        self.new_len = self.nout if self.nin > self.nout else self.nin + 1
        self.overlap = np.zeros(self.nout)
        self.saved = np.zeros(0)

    def _unit(self, x: np.ndarray) -> np.ndarray:
        xp = np.zeros(2 * self.nin)
        xp[: self.nin] = x
        spec = np.fft.rfft(xp) * self.hf
        of = np.zeros(self.nout + 1, dtype=np.complex128)
        of[: self.new_len] = spec[: self.new_len]
        y = np.fft.irfft(of, n=2 * self.nout) * (2 * self.nout)  # realfft's inverse is unnormalised
        out = y[: self.nout] + self.overlap
        self.overlap = y[self.nout:].copy()
        return out

    def process(self, chunk: np.ndarray) -> np.ndarray:
        assert len(chunk) == self.chunk_in
        buf = np.concatenate([self.saved, np.asarray(chunk, dtype=np.float64)])
        n_units = len(buf) // self.nin
        outs = [self._unit(buf[u * self.nin:(u + 1) * self.nin]) for u in range(n_units)]
        self.saved = buf[n_units * self.nin:]
        return np.concatenate(outs) if outs else np.zeros(0)


class FrameResampler:
    """resampler.rs FrameResampler: push / finish with an emit callback per frame."""

    def __init__(self, in_hz: int, out_hz: int, frame_dur_s: float):
        self.frame_samples = int(round(out_hz * frame_dur_s))
        assert self.frame_samples > 0, "frame duration too short"
        self.chunk_in = CHUNK_IN
        self.resampler = FftFixedIn(in_hz, out_hz, CHUNK_IN) if in_hz != out_hz else None
        self.in_buf: list[float] = []
        self.pending: list[float] = []

    def push(self, src, emit) -> None:
        src = list(np.asarray(src, dtype=np.float64))
        if self.resampler is None:
            self._emit_frames(src, emit)
            return
        while src:
            take = min(self.chunk_in - len(self.in_buf), len(src))
            self.in_buf.extend(src[:take])
            src = src[take:]
            if len(self.in_buf) == self.chunk_in:
                self._emit_frames(list(self.resampler.process(np.array(self.in_buf))), emit)
                self.in_buf = []

    def finish(self, emit) -> None:
        if self.resampler is not None and self.in_buf:
            self.in_buf.extend([0.0] * (self.chunk_in - len(self.in_buf)))
            self._emit_frames(list(self.resampler.process(np.array(self.in_buf))), emit)
            self.in_buf = []
        if self.pending:
            self.pending.extend([0.0] * (self.frame_samples - len(self.pending)))
            emit(np.array(self.pending))
            self.pending = []

    def _emit_frames(self, data, emit) -> None:
        while data:
            take = min(self.frame_samples - len(self.pending), len(data))
            self.pending.extend(data[:take])
            data = data[take:]
            if len(self.pending) == self.frame_samples:
                emit(np.array(self.pending))
                self.pending = []


def resample_stream(pcm, in_hz: int, out_hz: int, frame_dur_s: float = 0.030, push_sizes=None) -> np.ndarray:
    """One capture stream through FrameResampler (push in `push_sizes` pieces, then finish): the
    concatenated frames, i.e. what the recorder accumulates without a VAD."""
    r = FrameResampler(in_hz, out_hz, frame_dur_s)
    frames: list[np.ndarray] = []
    pcm = np.asarray(pcm, dtype=np.float64)
    if push_sizes is None:
        r.push(pcm, frames.append)
    else:
        i = 0
        for s in push_sizes:
            r.push(pcm[i:i + s], frames.append)
            i += s
        assert i == len(pcm)
    r.finish(frames.append)
    return np.concatenate(frames) if frames else np.zeros(0)


def resample_fast(pcm, in_hz: int, out_hz: int, frame_dur_s: float = 0.030) -> np.ndarray:
    """The same result computed block-parallel (every unit is independent given its predecessor's
    overlap), as the GPU path does; vectorised for large inputs."""
    pcm = np.asarray(pcm, dtype=np.float64)
    n = len(pcm)
    fs = int(round(out_hz * frame_dur_s))
    if in_hz == out_hz:
        nf = -(-n // fs)
        out = np.zeros(nf * fs)
        out[:n] = pcm
        return out
    r = FftFixedIn(in_hz, out_hz)
    n_proc = -(-n // CHUNK_IN) * CHUNK_IN
    n_units = n_proc // r.nin
    xp = np.zeros(max(n_units * r.nin, 1))
    m = min(n, n_units * r.nin)
    xp[:m] = pcm[:m]
    blocks = np.zeros((n_units, 2 * r.nin))
    blocks[:, : r.nin] = xp[: n_units * r.nin].reshape(n_units, r.nin)
    spec = np.fft.rfft(blocks, axis=1) * r.hf[None, :]
    of = np.zeros((n_units, r.nout + 1), dtype=np.complex128)
    of[:, : r.new_len] = spec[:, : r.new_len]
    y = np.fft.irfft(of, n=2 * r.nout, axis=1) * (2 * r.nout)
    out = y[:, : r.nout].copy()
    out[1:] += y[:-1, r.nout:]
    out = out.reshape(-1)
    nf = -(-len(out) // fs)
    res = np.zeros(nf * fs)
    res[: len(out)] = out
    return res
