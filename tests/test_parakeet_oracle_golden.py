"""The Parakeet-V3 CPU oracle (oracle/po_model.c) against HF transformers' independent Parakeet
port (ParakeetFeatureExtractor, ParakeetEncoder, ParakeetForTDT.generate), through the committed
fixtures tests/golden/parakeet_*.npz (written by tests/golden/make_golden_parakeet.py).

Cases: test-small dims (d 256, 2 layers; 1 s, 2 s + 77 samples, 3 s) and the full
parakeet-tdt-0.6b-v3 shape (24 layers, d 1024, 8 heads; 2 s and 1.27 s).  Reference call:
/root/reference/src-tauri/src/managers/transcription.rs:505-513."""
import os

import numpy as np
import pytest

from oracle import parakeet as P
from oracle.oracle import synth_audio

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["parakeet_small", "parakeet_v3_full"]

# bars (measured: mel 4.0e-4, encoder on HF's mel 7.9e-6, encoder on the oracle's mel 1.5e-5)
MEL_TOL = 1e-3      # torch.stft in f32 vs the oracle's f64 DFT, through log and normalisation
ENC_TOL = 5e-5      # post-LayerNorm rows, O(1)
ENC_OWN_TOL = 2e-4  # the same, fed the oracle's own mel


@pytest.fixture(scope="module", params=CASES)
def case(request):
    P.set_threads(8)
    g = dict(np.load(os.path.join(GOLD, request.param + ".npz")))
    dims = P.dims_for(str(g["config"]), n_layers=int(g["n_layers"]))
    return request.param, g, dims, P.Model(dims, seed=int(g["seed"]))


def _clips(g):
    return [(i, int(s), int(n)) for i, (s, n) in enumerate(zip(g["audio_seeds"], g["audio_lens"]))]


def test_mel_matches_hf(case):
    _, g, dims, _ = case
    for i, s, n in _clips(g):
        mo = P.mel(synth_audio(s, n), dims.n_mels)
        mg = g[f"mel_{i}"]
        assert mo.shape == mg.shape == (dims.n_mels, n // 160)
        assert np.abs(mo - mg).max() < MEL_TOL


def test_encoder_matches_hf(case):
    _, g, dims, m = case
    for i, s, n in _clips(g):
        eg = g[f"enc_{i}"]
        eo = m.encode(g[f"mel_{i}"])
        assert eo.shape == eg.shape == (P.n_enc_frames(n // 160), dims.d)
        assert np.abs(eo - eg).max() < ENC_TOL
        eo2 = m.encode(P.mel(synth_audio(s, n), dims.n_mels))
        assert np.abs(eo2 - eg).max() < ENC_OWN_TOL


def test_tdt_greedy_matches_hf(case):
    """Tokens and their frames identical.  HF's TDT search has no max-symbols guard; every fixture
    finished with fewer than 10 symbols on any frame, where the oracle's guard (10) never fires."""
    _, g, dims, m = case
    for i, _, _ in _clips(g):
        tg, fg = g[f"tokens_{i}"], g[f"frames_{i}"]
        assert int(g[f"finished_{i}"]) == 1 and len(tg) > 0
        assert np.unique(fg, return_counts=True)[1].max() < 10
        tk, fr, t1, t2 = m.decode(g[f"enc_{i}"], max_symbols=10)
        assert np.array_equal(tk, tg) and np.array_equal(fr, fg)
        # and from the oracle's own encoder output, where no decision is within the drift
        tk2, fr2, a1, a2 = m.decode(m.encode(g[f"mel_{i}"]), max_symbols=10)
        assert np.array_equal(tk2, tg) and np.array_equal(fr2, fg)


def test_fixture_provenance():
    for c in CASES:
        g = np.load(os.path.join(GOLD, c + ".npz"))
        assert str(g["config"]) in P.CONFIGS
        assert len(g["audio_seeds"]) == len(g["audio_lens"]) >= 2
