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
