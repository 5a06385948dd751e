"""The voice-activity gate's oracle (oracle/silero.py): the numpy interpreter of the reference's own
model graph (resources/models/silero_vad_v4.onnx, committed as tests/golden/silero_vad_v4.onnx)
against an independent torch restatement (tests/vad_torch.py) and the committed golden vectors;
the SmoothedVad restatement against known answers worked from vad/smoothed.rs:43-104.  The C++
SmoothedVad is checked bit-exactly against this restatement on the GPU (test_gpu_vad.py)."""
import hashlib
import os

import numpy as np
import pytest

from oracle import silero as S
from spittle_amd.synth import synth_speech

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MODEL = os.path.join(GOLD, "silero_vad_v4.onnx")
SHA = "a35ebf52fd3ce5f1469b2a36158dba761bc47b973ea3382b3186ca15b1f5af28"


def test_model_is_the_reference_file():
    assert hashlib.sha256(open(MODEL, "rb").read()).hexdigest() == SHA
    ref = "/root/reference/src-tauri/resources/models/silero_vad_v4.onnx"
    if os.path.exists(ref):
        assert hashlib.sha256(open(ref, "rb").read()).hexdigest() == SHA


def test_interpreter_matches_torch_restatement():
    vt = pytest.importorskip("tests.vad_torch")
    x = synth_speech(5, 2.0)
    rng = np.random.default_rng(1)
    frames = [x[i * 480:(i + 1) * 480] for i in range(x.size // 480)] + \
             [rng.standard_normal(480).astype(np.float32) * 0.05 for _ in range(4)]
    v, t = S.SileroVad(MODEL, 0.3), vt.TorchSilero(MODEL)
    for f in frames:
        assert abs(v.prob(f) - t.prob(f)) < 1e-5
    assert np.abs(v.h[:, 0] - t.h.numpy()).max() < 1e-5 and np.abs(v.c[:, 0] - t.cs.numpy()).max() < 1e-5


def test_golden_vectors_reproduce():
    g = np.load(os.path.join(GOLD, "silero_vad.npz"))
    seed, sec = int(g["seed_2"]), float(g["seconds_2"])
    x = synth_speech(seed, sec)
    v = S.SileroVad(MODEL, 0.3)
    probs = np.array([v.prob(x[i * 480:(i + 1) * 480]) for i in range(x.size // 480)], np.float32)
    assert np.abs(probs - g["prob_2"]).max() < 1e-6
    assert (probs > 0.3).sum() > 10 and (probs <= 0.3).sum() > 10  # both decisions occur


def _kinds(decisions, prefill=15, hangover=15, onset=2):
    frames = [np.full(480, i, np.float32) for i in range(len(decisions))]
    it = iter(decisions)
    sv = S.SmoothedVad(lambda _f: next(it), prefill, hangover, onset)
    outs = [sv.push_frame(f) for f in frames]
    return [0 if o.size == 0 else (1 if o.size == 480 else 2) for o in outs], outs


def test_smoothed_vad_known_answers():
    T, F = True, False
    # one voiced frame is not an onset (onset 2); two are: the second emits prefill + itself
    k, outs = _kinds([F, T, F, T, T, T])
    assert k == [0, 0, 0, 0, 2, 1]
    assert outs[4].size == 5 * 480 and outs[4][0] == 0 and outs[4][-1] == 4  # frames 0..4 (buffer <= 16)
    # hangover: 15 silent frames still kept, the 16th ends the speech
    k, _ = _kinds([T, T] + [F] * 17)
    assert k == [0, 2] + [1] * 15 + [0, 0]
    # the prefill buffer holds prefill + 1 = 16 frames at most
    k, outs = _kinds([F] * 30 + [T, T])
    assert k[-1] == 2 and outs[-1].size == 16 * 480 and outs[-1][0] == 16
    # voice during hangover re-arms it
    k, _ = _kinds([T, T] + [F] * 10 + [T] + [F] * 16)
    assert k[:13] == [0, 2] + [1] * 11 and k[13:28] == [1] * 15 and k[28] == 0
    # reset clears the buffer, counters and state
    it = iter([T, T, T, F, T, T])
    sv = S.SmoothedVad(lambda _f: next(it))
    r = [sv.push_frame(np.zeros(480, np.float32)).size for _ in range(3)]
    sv.reset()
    r += [sv.push_frame(np.zeros(480, np.float32)).size for _ in range(3)]
    assert r == [0, 960, 480, 0, 0, 1440]  # after reset the pre-roll holds the silent frame 3 too
