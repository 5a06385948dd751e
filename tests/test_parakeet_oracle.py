"""The Parakeet-V3 CPU oracle (oracle/po_model.c) against an independent PyTorch restatement
(tests/pk_torch.py: torch.stft, conv2d, NeMo's rel_shift, torch.nn.LSTM).  Parity with the
real ONNX engine is unpinned (no export or weights offline); this pins the restatement's
arithmetic against PyTorch's building blocks."""
import numpy as np
import pytest
import torch

from oracle import parakeet as P
from oracle.oracle import synth_audio

pk = pytest.importorskip("tests.pk_torch")


@pytest.fixture(scope="module")
def small():
    torch.set_num_threads(4)
    P.set_threads(4)
    d = P.dims_for("test-small")
    return d, P.Model(d, seed=11)


@pytest.mark.parametrize("n", [16000, 16000 * 3 + 77, 4000])
def test_mel_matches_torch_stft(n):
    pcm = synth_audio(5, n)
    mo = P.mel(pcm)
    assert mo.shape == (128, n // 160)
    mt = pk.mel(pcm).numpy()
    assert np.abs(mo - mt).max() < 1e-3


def test_encoder_matches_torch(small):
    d, m = small
    mo = P.mel(synth_audio(3, 16000 * 3))
    eo = m.encode(mo)
    assert eo.shape == (P.n_enc_frames(mo.shape[1]), d.d)
    et = pk.encode(m, d, torch.from_numpy(mo)).numpy()
    assert np.abs(eo - et).max() < 1e-4


def test_tdt_greedy_matches_torch(small):
    d, m = small
    eo = m.encode(P.mel(synth_audio(4, 16000 * 2)))
    toks, frames, t1, t2 = m.decode(eo)
    tt, ft = pk.tdt_greedy(m, d, torch.from_numpy(eo))
    assert list(toks) == tt and list(frames) == ft
    assert len(toks) > 0
    assert np.all(t1 >= t2)
    assert np.all(np.diff(frames) >= 0)


def test_max_symbols_per_frame(small):
    d, m = small
    eo = m.encode(P.mel(synth_audio(6, 16000)))
    for ms in (1, 2):
        toks, frames, _, _ = m.decode(eo, max_symbols=ms)
        _, counts = np.unique(frames, return_counts=True)
        assert counts.max() <= ms


def test_frame_counts():
    # NeMo get_seq_len / HF ParakeetFeatureExtractor: n // 160 valid frames
    assert P.n_frames(16000) == 100 and P.n_enc_frames(100) == 13
    assert P.n_frames(480000) == 3000 and P.n_enc_frames(3000) == 375
    assert P.n_frames(0) == 0 and P.n_enc_frames(0) == 0
    assert P.n_frames(159) == 0 and P.n_frames(160) == 1 and P.n_enc_frames(1) == 1


def test_weight_rounding_modes():
    d = P.dims_for("test-small")
    w32 = P.Model(d, seed=2, wdtype=P.W_F32).tensor(1002)
    wh = P.Model(d, seed=2, wdtype=P.W_F16).tensor(1002)
    wb = P.Model(d, seed=2, wdtype=P.W_BF16).tensor(1002)
    assert np.array_equal(wh, w32.astype(np.float16).astype(np.float32))
    bf = (w32.view(np.uint32) + 0x7FFF + ((w32.view(np.uint32) >> 16) & 1)) & 0xFFFF0000
    assert np.array_equal(wb, bf.astype(np.uint32).view(np.float32))
    # non-matrix tensors are never rounded
    assert np.array_equal(P.Model(d, seed=2, wdtype=P.W_F16).tensor(1023), P.Model(d, seed=2).tensor(1023))
