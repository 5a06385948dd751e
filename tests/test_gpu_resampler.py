"""GPU parity of the capture-side resampler (spt_resample, ABI 7) against the CPU restatement of
FrameResampler over rubato FftFixedIn (oracle/resampler.py; reference
/root/reference/src-tauri/src/audio_toolkit/audio/resampler.rs:7-104, recorder.rs:264-268, 330, 355).

Bar: output length exact (finish's padding of the last input chunk and of the last 30 ms frame),
samples within 2e-5 absolute of the f64 oracle for |x| <= 1 input (the GPU forms each rubato unit
as one exact-f32 MFMA GEMM row against the unit's linear map built in f64 and rounded to f32; the
oracle runs numpy FFTs in f64).  Identity rates are bitwise.  Parity with rubato itself is unpinned.
"""
import numpy as np
import pytest

from oracle import resampler as R

pytestmark = pytest.mark.gpu


def _rs(fin, fout=16000, frame=0.030):
    from spittle_amd.resampler import FrameResampler
    return FrameResampler(fin, fout, frame)


@pytest.mark.parametrize("fin", [48000, 44100, 22050, 8000, 32000])
def test_resample_matches_oracle(fin):
    r = _rs(fin)
    assert r.fft_sizes == R.fft_sizes(fin, 16000)
    rng = np.random.default_rng(fin)
    for n in (1, 1023, 1024, 1025, 4097, 3 * fin + 77):
        x = np.clip(0.3 * rng.standard_normal(n) + 0.4 * np.sin(np.arange(n) * 0.01), -1, 1).astype(np.float32)
        y = r.process_stream(x)
        ref = R.resample_fast(x.astype(np.float64), fin, 16000)
        assert len(y) == len(ref) == r.output_len(n), (fin, n)
        err = np.abs(y - ref).max() if len(y) else 0.0
        assert err < 2e-5, (fin, n, err)


def test_identity_rate_and_empty():
    r = _rs(16000)
    assert r.fft_sizes == (0, 0)
    x = np.random.default_rng(1).standard_normal(1000).astype(np.float32)
    y = r.process_stream(x)
    assert len(y) == 1440 and np.array_equal(y[:1000], x) and not y[1000:].any()
    assert len(r.process_stream(np.zeros(0, np.float32))) == 0
    assert len(_rs(48000).process_stream(np.zeros(0, np.float32))) == 0


def test_long_stream_and_reuse():
    """10 minutes at 48 kHz in one call (28 k rubato units in one GEMM), then a short call on the
    same context (workspace reuse): both equal the oracle."""
    r = _rs(48000)
    rng = np.random.default_rng(5)
    x = np.clip(0.2 * rng.standard_normal(48000 * 600), -1, 1).astype(np.float32)
    y = r.process_stream(x)
    ref = R.resample_fast(x.astype(np.float64), 48000, 16000)
    assert len(y) == len(ref)
    assert np.abs(y - ref).max() < 2e-5
    x2 = x[:5000]
    assert np.abs(r.process_stream(x2) - R.resample_fast(x2.astype(np.float64), 48000, 16000)).max() < 2e-5


def test_upsample_and_frame_sizes():
    r = _rs(8000, 16000, 0.020)  # 320-sample frames
    x = np.sin(np.arange(12345) * 0.05).astype(np.float32)
    y = r.process_stream(x)
    ref = R.resample_fast(x.astype(np.float64), 8000, 16000, 0.020)
    assert len(y) == len(ref) and len(y) % 320 == 0
    assert np.abs(y - ref).max() < 2e-5


def test_errors():
    from spittle_amd.resampler import FrameResampler, ResamplerError
    with pytest.raises(ResamplerError):
        FrameResampler(10, 16000)
    with pytest.raises(ResamplerError):
        FrameResampler(48000, 16000, 0.00001)
