"""GPU parity of the voice-activity gate (spt_vad_*, ABI 8) against the oracle (oracle/silero.py
interpreting the reference's own silero_vad_v4.onnx, pinned in test_vad_oracle.py; golden vectors
tests/golden/silero_vad.npz).

Bars: per-frame speech probability within 2e-4 of the oracle (f32 on the device, f64 sums in the
oracle); the VadFrame kinds equal wherever no probability lies within 2e-4 of the threshold (0.3);
the kept audio then bit-identical to the oracle's SmoothedVad output (it is a copy of input
frames).  Reference: SmoothedVad::new(Box::new(SileroVad::new(path, 0.3)), 15, 15, 2)
(/root/reference/src-tauri/src/managers/audio.rs:132-134), recorder.rs:284-301."""
import os

import numpy as np
import pytest

from oracle import silero as S
from spittle_amd.synth import synth_speech

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MODEL = os.path.join(GOLD, "silero_vad_v4.onnx")
TOL = 2e-4


def _gate(**kw):
    from spittle_amd.vad import SileroVad, SmoothedVad
    return SmoothedVad(SileroVad(MODEL, 0.3), 15, 15, 2, **kw)


def _frames(x):
    return [x[i * 480:(i + 1) * 480] for i in range(x.size // 480)]


@pytest.mark.parametrize("k", [0, 1, 2])
def test_stream_matches_oracle(k):
    g = np.load(os.path.join(GOLD, "silero_vad.npz"))
    x = synth_speech(int(g[f"seed_{k}"]), float(g[f"seconds_{k}"]))
    x = x[:x.size // 480 * 480]  # whole 30 ms frames, as the FrameResampler delivers them
    gate = _gate()
    r = gate.push_stream(x)
    po = g[f"prob_{k}"]
    assert r.prob.shape == po.shape
    assert np.abs(r.prob - po).max() < TOL, np.abs(r.prob - po).max()
    near = np.abs(po - 0.3) < TOL
    assert not near.any()  # the fixtures have no decision inside the tolerance
    assert np.array_equal(r.kind, g[f"kind_{k}"])
    kept = S.gate_stream(list(po > np.float32(0.3)), _frames(x))
    assert r.samples.size == int(g[f"kept_len_{k}"]) and np.array_equal(r.samples, kept)
    gate.close()


def test_stream_in_pieces_equals_one_call():
    """push_frame one frame at a time (the recorder's order) and odd-sized pieces give the same
    probabilities and kept audio as one call: the LSTM state and the smoothing carry over."""
    x = synth_speech(7, 3.0)
    a = _gate().push_stream(x)
    b = _gate()
    probs, kept = [], []
    for f in _frames(x)[:40]:
        r = b.push_stream(f)
        probs += list(r.prob)
        kept.append(r.samples)
    r = b.push_stream(x[40 * 480:])
    probs += list(r.prob)
    kept.append(r.samples)
    assert np.array_equal(np.asarray(probs, np.float32), a.prob)
    assert np.array_equal(np.concatenate(kept), a.samples)


def test_reset_keeps_the_model_state():
    """Cmd::Start resets the SmoothedVad only (recorder.rs:343-349); SileroVad has no reset, so a
    second recording starts with the first one's LSTM state, unless the model state is reset too."""
    x = synth_speech(8, 2.0)
    g = _gate()
    g.push_stream(x)
    g.reset()
    carried = g.push_stream(x)
    g.reset(model_state=True)
    fresh = g.push_stream(x)
    first = _gate().push_stream(x)
    assert np.array_equal(fresh.prob, first.prob)
    assert not np.array_equal(carried.prob, first.prob)
    v = S.SileroVad(MODEL, 0.3)
    po = [v.prob(f) for f in _frames(x)] + [v.prob(f) for f in _frames(x)]
    assert np.abs(carried.prob - np.asarray(po[len(po) // 2:], np.float32)).max() < TOL


def test_partial_frame_and_errors():
    from spittle_amd import TranscriptionError
    from spittle_amd.vad import SileroVad, SmoothedVad
    g = _gate()
    x = synth_speech(9, 1.0)[:480 * 5 + 100]
    r = g.push_stream(x)
    assert r.prob.size == 5 and r.kind.size == 6 and r.kind[-1] == 1  # kept like the recorder's unwrap_or
    assert np.array_equal(r.samples[-100:], x[-100:])
    assert g.push_stream(np.zeros(0, np.float32)).samples.size == 0
    with pytest.raises(ValueError):
        SileroVad(MODEL, 1.5)
    with pytest.raises(TranscriptionError, match="Failed to create VAD"):
        SmoothedVad(SileroVad("/nonexistent/silero_vad_v4.onnx", 0.3))
