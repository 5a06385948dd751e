"""The app's real Whisper call at the app's model width: whisper_full with timestamps on and
temperature fallback off, large-v3 dimensions (d 1280, 20 heads, 128 mels, 51866 tokens) in bf16,
2 encoder + 2 decoder layers, for B = 1 and B = 4 and 8 / 20 / 45 s inputs, and beam search
(beam 5) -- against the oracle's whisper_full restatement (oracle/whisper_full.py over the fp32 C
model on identically bf16-rounded weights).

Reference call: /root/reference/src-tauri/src/managers/transcription.rs:494-503 (whisper params
with timestamps on: the transcribe-rs default) -> whisper_full.

Bars (bf16 activations at every GEMM input vs the oracle's f32):
  * tokens, timestamp ids and segments equal up to the oracle's first decision whose margin
    (argmax gap, timestamp-mass rule gap, beam candidate gap) is below GAP_BF16;
  * on that agreed prefix the chosen tokens' log-probabilities within PLOG_BF16;
  * a case whose oracle's first decision is already under the bar compares nothing and fails
    (the non-empty-prefix guard of test_gpu_full._compare).
Measured values per case: gpurun_out/full_large_v3.json."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from oracle import whisper_full as W

pytestmark = pytest.mark.gpu

SEED = 1234
SPEC = "synthetic:large-v3:enc=2:dec=2"
GAP_BF16 = 0.1     # measured largest |logit error| of the 2+2 bf16 model: ~0.05
PLOG_BF16 = 0.05   # measured max 0.027 (b4, 8 s)
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
_REC = {}


@pytest.fixture(scope="module")
def large():
    from spittle_amd import WhisperEngine, WhisperModelParams
    O.set_threads(16)
    e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=8, seed=SEED))
    e.load_model(SPEC)
    om = O.Model(O.dims_for("large-v3", 2, 2), SEED, O.W_BF16)
    yield e, om
    e.unload_model()
    om.close()
    os.makedirs(OUT, exist_ok=True)
    json.dump(_REC, open(os.path.join(OUT, "full_large_v3.json"), "w"), indent=1)


def _params(**kw):
    from spittle_amd import WhisperInferenceParams
    kw.setdefault("language", "en")
    kw.setdefault("temperature_inc", 0.0)
    return WhisperInferenceParams(**kw)


def _audio(seconds, seed):
    n = int(seconds * 16000)
    return np.concatenate([O.synth_audio(seed + k) for k in range((n + 479999) // 480000)])[:n]


def _check(name, r, om, x, p):
    wins, segs, toks, kept = W.transcribe(om, x, p)
    steps = [s for _, w in wins for s in w.steps]
    gaps = [s.margin for s in steps]
    k = next((i for i, g in enumerate(gaps) if g <= GAP_BF16), None)
    got = list(r.tokens)
    n = len(toks)
    rec = {"oracle_tokens": n, "gpu_tokens": len(got), "oracle_windows": len(wins), "gpu_windows": r.n_windows,
           "first_small_margin_step": k, "smallest_margin": float(min(gaps)) if gaps else None}
    if k is None:
        assert got == toks, name
        assert [(int(round(s.start * 100)), int(round(s.end * 100)), s.text) for s in r.segments] == \
               [(a, b, t) for a, b, t, _, _ in segs], name
        m = n
    else:
        assert min(k, n) > 0, (name, "the oracle's first decision is already under the bar: nothing to compare")
        m = min(k, n)
        assert got[:m] == toks[:m], name
    dplog = [abs(float(r.top1[i]) - kept[i].plog) for i in range(m)]
    # the timestamp id (best timestamp token of a step) reaches the output only through a
    # timestamp token, where it is that token; elsewhere its own near-ties are not decisions
    beg = O.special_tokens(om.dims.n_vocab)["beg"]
    tid_ts = all(int(r.top2[i]) == kept[i].tid for i in range(m) if toks[i] >= beg)
    rec.update({"compared_tokens": m, "max_plog_diff": max(dplog) if dplog else 0.0,
                "tids_equal_all_steps": all(int(r.top2[i]) == kept[i].tid for i in range(m)),
                "tids_equal_at_timestamps": tid_ts, "exact": k is None, "whole_output_equal": got == toks})
    _REC[name] = rec
    assert max(dplog, default=0.0) < PLOG_BF16, (name, max(dplog))
    assert tid_ts, name
    return rec


@pytest.mark.parametrize("seconds,seed", [(8, 160), (20, 161), (45, 162)])
def test_large_v3_timestamps_b1(large, seconds, seed):
    e, om = large
    x = _audio(seconds, seed)
    r = e.transcribe_samples(x, _params(max_new_tokens=32))
    _check(f"b1_{seconds}s", r, om, x, W.Params(max_tokens=32))
    assert r.n_windows >= (2 if seconds > 30 else 1)


def test_large_v3_timestamps_b4(large):
    """Four utterances of different lengths (so different seek paths) in one call: each against
    its own oracle run."""
    e, om = large
    xs = [_audio(8, 170), _audio(20, 171), _audio(45, 172), _audio(12.5, 173)]
    rs = e.transcribe_batch(xs, _params(max_new_tokens=32))
    for i, (x, r) in enumerate(zip(xs, rs)):
        _check(f"b4_{i}_{len(x) / 16000:g}s", r, om, x, W.Params(max_tokens=32))


@pytest.mark.parametrize("seconds,seed", [(20, 191), (45, 206)])
def test_large_v3_beam5(large, seconds, seed):
    """Beam 5: the oracle's margin for a step is the smallest gap among the ranked candidates
    (5th vs 6th included), which bf16 random-weight logits make small within a few steps; the
    inputs are ones whose first steps are decided by more than GAP_BF16 (seeds chosen by scanning
    180-211 with the oracle), so the compared prefix is 5 and 2 tokens; the whole output is
    recorded ("whole_output_equal")."""
    e, om = large
    x = _audio(seconds, seed)
    r = e.transcribe_samples(x, _params(beam_size=5, max_new_tokens=16))
    _check(f"beam5_{seconds}s", r, om, x, W.Params(max_tokens=16, beam_size=5))


def _loud_then_quiet(seconds, seed):
    x = _audio(seconds, seed).copy()
    x[x.size // 2:] *= np.float32(0.03)  # the second half 30 dB quieter
    return x


@pytest.mark.parametrize("seconds,seed", [(45, 310), (75, 312)])
def test_large_v3_loud_then_quiet(large, seconds, seed):
    """The app's call on a loud-then-quiet dictation over 30 s: every window's frames come from one
    log-mel of the whole utterance (whisper_pcm_to_mel's global max - 8 clamp), at large-v3 width,
    against the oracle's whole-input restatement."""
    e, om = large
    x = _loud_then_quiet(seconds, seed)
    r = e.transcribe_samples(x, _params(max_new_tokens=24))
    rec = _check(f"loud_quiet_{seconds}s", r, om, x, W.Params(max_tokens=24))
    assert r.n_windows >= 2 and rec["oracle_windows"] >= 2
    assert e.call_stats()["encoder_windows"] == r.n_windows


def test_large_v3_beam5_shared_window_bitwise(large, monkeypatch):
    """Beam 5 at large-v3 width in bf16: the five decoders read one shared window (one workgroup
    per (window, head) for all five queries), bitwise the result of five private copies."""
    e, _ = large
    x = _audio(20, 191)
    a = e.transcribe_samples(x, _params(beam_size=5, max_new_tokens=16))
    monkeypatch.setenv("SPT_NO_WINDOW_SHARE", "1")
    b = e.transcribe_samples(x, _params(beam_size=5, max_new_tokens=16))
    monkeypatch.delenv("SPT_NO_WINDOW_SHARE")
    assert a.tokens == b.tokens and np.array_equal(np.asarray(a.top1), np.asarray(b.top1))


@pytest.mark.parametrize("vw", ["0", "3"])
def test_large_v3_beam5_cross_attention_strategies_bitwise(large, vw, monkeypatch):
    """Beam 5 at large-v3 width in bf16: the default one-query single-wave workgroups with the
    partial merge, the 8-wave kernel with five queries per workgroup (SPT_XATTN_VW=0) and the
    single-wave five-query kernel (3) give bitwise the same result (a new engine captures its
    passes under the switch)."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e, _ = large
    x = _audio(20, 193)
    a = e.transcribe_samples(x, _params(beam_size=5, max_new_tokens=12))
    monkeypatch.setenv("SPT_XATTN_VW", vw)
    e2 = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=8, seed=SEED))
    try:
        e2.load_model(SPEC)
        b = e2.transcribe_samples(x, _params(beam_size=5, max_new_tokens=12))
    finally:
        e2.unload_model()
    assert a.tokens == b.tokens and np.array_equal(np.asarray(a.top1), np.asarray(b.top1))


def test_large_v3_fc2_residual_fold_bitwise(large, monkeypatch):
    """Greedy and beam 5 at large-v3 width in bf16: fc2's residual fold into slab 0 (default)
    gives bitwise the unfolded passes' result (SPT_DEC_XFOLD=0, a new engine's captures)."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e, _ = large
    x = _audio(20, 194)
    a = [e.transcribe_samples(x, _params(max_new_tokens=24)), e.transcribe_samples(x, _params(beam_size=5, max_new_tokens=12))]
    monkeypatch.setenv("SPT_DEC_XFOLD", "0")
    e2 = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=8, seed=SEED))
    try:
        e2.load_model(SPEC)
        b = [e2.transcribe_samples(x, _params(max_new_tokens=24)), e2.transcribe_samples(x, _params(beam_size=5, max_new_tokens=12))]
    finally:
        e2.unload_model()
    for ra, rb in zip(a, b):
        assert ra.tokens == rb.tokens and np.array_equal(np.asarray(ra.top1), np.asarray(rb.top1))


def test_large_v3_beam5_dedup_batch_geometry():
    """Beam 5 at large-v3 width in bf16 (38 rows per pass): the same utterance alone, beside 1, 3
    and 6 others (one engine call of 10, 20, 35 rows) and in a call of 9 utterances split over two
    engine calls (max_batch 40: 7 utterances per beam call) -- bitwise-equal tokens and
    log-probabilities, so whisper.cpp's exact-equality candidate dedup sees the same scores in every
    pass geometry."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=40, seed=SEED))
    e.load_model(SPEC)
    try:
        p = _params(beam_size=5, max_new_tokens=12)
        x = _audio(20, 191)
        others = [_audio(5 + i, 220 + i) for i in range(8)]
        runs = [("alone", e.transcribe_samples(x, p))]
        for k, pos in ((1, 0), (3, 3), (6, 2)):
            xs = others[:k][:pos] + [x] + others[:k][pos:]
            runs.append((f"with{k}@{pos}", e.transcribe_batch(xs, p)[pos]))
        xs = others[:7] + [x] + others[7:]  # calls of 7 and 2 utterances, x in the second
        runs.append(("split_calls", e.transcribe_batch(xs, p)[7]))
        ref = runs[0][1]
        for name, r in runs[1:]:
            assert r.tokens == ref.tokens, name
            assert np.array_equal(np.asarray(r.top1), np.asarray(ref.top1)), name
            assert np.array_equal(np.asarray(r.top2), np.asarray(ref.top2)), name
    finally:
        e.unload_model()
