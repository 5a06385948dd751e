"""CPU: the resampler oracle (oracle/resampler.py) -- rubato FftFixedIn + FrameResampler restated.

Known answers: rubato's unit sizes for the capture rates the app meets (48 / 44.1 / 22.05 / 8 kHz
-> 16 kHz, 1024-sample chunks); properties: the streaming form (FrameResampler push in arbitrary
pieces + finish, resampler.rs:37-86) equals the block-parallel form the GPU uses, output lengths
follow finish's padding rules, a pass-band tone keeps its amplitude, a stop-band tone is removed,
the map is linear.  Parity with rubato itself is unpinned (the crate is not in /root/reference).
"""
import numpy as np
import pytest

from oracle import resampler as R


@pytest.mark.parametrize("fin,exp", [(48000, (1026, 342)), (44100, (1323, 480)), (22050, (1323, 960)),
                                     (8000, (1024, 2048)), (32000, (1024, 512))])
def test_fft_sizes(fin, exp):
    assert R.fft_sizes(fin, 16000) == exp


@pytest.mark.parametrize("fin", [48000, 44100, 8000, 16000])
@pytest.mark.parametrize("n", [0, 1, 700, 1024, 5000, 20011])
def test_stream_equals_block_parallel(fin, n):
    rng = np.random.default_rng(n + fin)
    x = rng.standard_normal(n) * 0.3
    sizes, i = [], 0
    while i < n:
        s = min(int(rng.integers(1, 1500)), n - i)
        sizes.append(s)
        i += s
    a = R.resample_stream(x, fin, 16000, push_sizes=sizes)
    b = R.resample_fast(x, fin, 16000)
    assert len(a) == len(b) and len(a) % 480 == 0
    if fin != 16000 and n:
        nin, nout = R.fft_sizes(fin, 16000)
        units = (-(-n // 1024) * 1024) // nin
        assert len(a) == -(-(units * nout) // 480) * 480
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-12)


def test_tones_and_linearity():
    t = np.arange(48000 * 2) / 48000.0
    passband = np.sin(2 * np.pi * 1000 * t)
    stopband = np.sin(2 * np.pi * 12000 * t)  # above the 8 kHz output Nyquist
    y = R.resample_fast(passband, 48000, 16000)[3000:28000]
    assert abs(np.sqrt(np.mean(y ** 2)) - np.sqrt(0.5)) < 1e-3
    z = R.resample_fast(stopband, 48000, 16000)[3000:28000]
    assert np.sqrt(np.mean(z ** 2)) < 1e-3
    rng = np.random.default_rng(3)
    a, b = rng.standard_normal(9000), rng.standard_normal(9000)
    np.testing.assert_allclose(R.resample_fast(2 * a - b, 44100, 16000),
                               2 * R.resample_fast(a, 44100, 16000) - R.resample_fast(b, 44100, 16000), atol=1e-12)
