"""Synthetic benchmark input: one 16 kHz mono f32 chunk,
clip(0.1 N(0,1) + sum_k 0.3 sin(2 pi f_k t + phi_k), -1, 1) with
f_k ~ U(100, 4000) Hz and phi_k ~ U(0, 2 pi) drawn from numpy PCG64(1000 + i).
(oracle/oracle.py carries the same generator for the tests.)"""
import numpy as np


def synth_audio(i: int, n_samples: int = 480000) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(1000 + i))
    f = rng.uniform(100.0, 4000.0, 3)
    ph = rng.uniform(0.0, 2 * np.pi, 3)
    noise = rng.standard_normal(n_samples)
    t = np.arange(n_samples) / 16000.0
    x = 0.1 * noise
    for k in range(3):
        x = x + 0.3 * np.sin(2 * np.pi * f[k] * t + ph[k])
    return np.clip(x, -1.0, 1.0).astype(np.float32)


def synth_speech(i: int, seconds: float = 6.0) -> np.ndarray:
    """Speech-like 16 kHz audio for the voice-activity gate: vowel segments (a glottal harmonic
    series with slow pitch drift, shaped by three formant resonances, raised-cosine envelopes)
    separated by pauses, over a faint noise floor -- seeded by PCG64(2000 + i)."""
    sr = 16000
    rng = np.random.Generator(np.random.PCG64(2000 + i))
    n = int(seconds * sr)
    x = np.zeros(n)
    vowels = [((700, 130), (1220, 150), (2600, 200)), ((300, 100), (2300, 200), (3000, 250)),
              ((500, 120), (900, 140), (2500, 200)), ((400, 110), (1900, 180), (2700, 220))]
    pos = int(rng.uniform(0.2, 0.6) * sr)
    while pos < n - sr // 4:
        dur = int(rng.uniform(0.25, 0.8) * sr)
        dur = min(dur, n - pos)
        t = np.arange(dur) / sr
        f0 = rng.uniform(100, 220)
        ph = 2 * np.pi * np.cumsum(f0 * (1 + 0.05 * np.sin(2 * np.pi * rng.uniform(2, 5) * t))) / sr
        form = vowels[int(rng.integers(len(vowels)))]
        seg = np.zeros(dur)
        for k in range(1, 40):
            amp = sum(np.exp(-((k * f0 - F) / B) ** 2) for F, B in form) / np.sqrt(k)
            seg += amp * np.sin(k * ph)
        env = np.sqrt(0.5 * (1 - np.cos(2 * np.pi * t / (dur / sr))))
        x[pos:pos + dur] += rng.uniform(0.15, 0.4) * seg / (np.abs(seg).max() + 1e-9) * env
        pos += dur + int(rng.uniform(0.05, 0.9) * sr)
    x += 0.003 * rng.standard_normal(n)
    return np.clip(x, -1.0, 1.0).astype(np.float32)
