"""The persistent decoder pass (spittle_amd/csrc/k_pdec.hip): every decoder layer of a one-token
pass as ONE launch, its stages handing data-tagged granules to each other inside the launch.  Each
unit repeats the per-stage kernels' arithmetic operation for operation (gemv_kernel's K chains and
their summation order, AttnWave's online softmax over the same key blocks, attn_merge), so the pass
must be BITWISE the launch chain's (SPT_PERSISTENT=0): tokens, top-1 and top-2 logits, on the fast
path (B = 1 / 5 / 8), on whisper_full's best_of and beam search (beam 5: 5 rows per step) and at
full large-v3 depth.  Every comparison also checks that the persistent pass ran (pd_passes) and
never gave up (pd_fallbacks)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 1234


def _engine(spec, max_batch, persistent, monkeypatch):
    from spittle_amd import WhisperEngine, WhisperModelParams
    monkeypatch.setenv("SPT_PERSISTENT", "1" if persistent else "0")  # read when the context is created
    e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=max_batch, seed=SEED))
    e.load_model(spec)
    return e


def _fast(n):
    from spittle_amd import WhisperInferenceParams
    return WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                                  max_new_tokens=n)


def _full(**kw):
    from spittle_amd import WhisperInferenceParams
    kw.setdefault("language", "en")
    kw.setdefault("temperature_inc", 0.0)
    return WhisperInferenceParams(**kw)


def _both(spec, max_batch, xs, p, monkeypatch):
    """(chain results, persistent results, the persistent call's stats)"""
    e = _engine(spec, max_batch, False, monkeypatch)
    try:
        ref = e.transcribe_batch(xs, p)
        assert e.call_stats()["pd_passes"] == 0
    finally:
        e.unload_model()
    e = _engine(spec, max_batch, True, monkeypatch)
    try:
        got = e.transcribe_batch(xs, p)
        cs = e.call_stats()
    finally:
        e.unload_model()
    return ref, got, cs


def _assert_bitwise(ref, got):
    for i, (a, b) in enumerate(zip(ref, got)):
        assert a.tokens == b.tokens, (i, a.tokens, b.tokens)
        assert np.array_equal(np.asarray(a.top1), np.asarray(b.top1)), i
        assert np.array_equal(np.asarray(a.top2), np.asarray(b.top2)), i
        assert a.text == b.text


@pytest.mark.parametrize("spec", ["synthetic:tiny", "synthetic:large-v3:enc=2:dec=2"])
@pytest.mark.parametrize("B", [1, 5, 8])
def test_fast_path_bitwise(spec, B, monkeypatch):
    xs = [O.synth_audio(200 + i, (9 + 2 * i) * 16000) for i in range(B)]
    n = 24
    ref, got, cs = _both(spec, 8, xs, _fast(n), monkeypatch)
    assert cs["pd_passes"] == n - 1 and cs["pd_fallbacks"] == 0, cs  # every step after the prompt pass
    _assert_bitwise(ref, got)


@pytest.mark.parametrize("kind", ["beam5", "best_of5"])
def test_whisper_full_bitwise(kind, monkeypatch):
    """whisper_full over two utterances (12 s, 35 s: two windows): beam 5 (a host-driven step of 5
    rows per utterance on one shared window) and best_of 5 under forced temperature fallback."""
    xs = [O.synth_audio(210, 12 * 16000), O.synth_audio(211, 35 * 16000)]
    kw = dict(beam_size=5, max_new_tokens=10) if kind == "beam5" else \
        dict(temperature_inc=0.2, logprob_thold=10.0, best_of=5, max_new_tokens=10, seed=21)
    ref, got, cs = _both("synthetic:large-v3:enc=2:dec=2", 8, xs, _full(**kw), monkeypatch)
    assert cs["pd_passes"] > 0 and cs["pd_fallbacks"] == 0, cs
    _assert_bitwise(ref, got)
    for a, b in zip(ref, got):
        assert [(s.start, s.end, s.text) for s in a.segments] == [(s.start, s.end, s.text) for s in b.segments]


def test_language_detection_bitwise(monkeypatch):
    """language auto-detection is a one-token pass on [sot] (persistent), then the prompt pass"""
    from spittle_amd import WhisperInferenceParams
    xs = [O.synth_audio(220 + i, 8 * 16000) for i in range(3)]
    p = WhisperInferenceParams(language=None, no_timestamps=True, temperature_inc=0.0, ignore_eot=True, max_new_tokens=6)
    ref, got, cs = _both("synthetic:large-v3:enc=2:dec=2", 4, xs, p, monkeypatch)
    assert cs["pd_passes"] > 0 and cs["pd_fallbacks"] == 0, cs
    _assert_bitwise(ref, got)
    assert [r.language for r in ref] == [r.language for r in got]


@pytest.mark.parametrize("B", [1, 8])
def test_full_depth_large_v3_bitwise(B, monkeypatch):
    """the benchmark's model: large-v3, 32 + 32 layers, bf16; B = 1 (the app) and B = 8 (C3)"""
    xs = [O.synth_audio(1000 + i) for i in range(B)]
    n = 16
    ref, got, cs = _both("synthetic:large-v3", 8, xs, _fast(n), monkeypatch)
    assert cs["pd_passes"] == n - 1 and cs["pd_fallbacks"] == 0, cs
    _assert_bitwise(ref, got)


@pytest.mark.parametrize("case", ["fast_b1", "fast_b8", "beam5", "best_of5"])
def test_forced_give_up_reruns_bitwise(case, monkeypatch):
    """The give-up path: SPT_PD_FORCE_GIVEUP=k makes the k-th persistent launch of every
    call set the error word, as a pass starved of CUs would.  The fast path then re-runs the whole
    call on the launch chain (Engine::decode), a beam search re-runs the step and continues on the
    chain (beam_next); the persistent attempt's later launches leave at once.  Tokens, top-1 / top-2
    and segments must still be the chain's bit for bit, with pd_fallbacks counted and no give-up
    counted as a persistent pass."""
    monkeypatch.setenv("SPT_PD_FORCE_GIVEUP", "3")
    if case.startswith("fast"):
        B = 1 if case == "fast_b1" else 8
        xs = [O.synth_audio(230 + i, (10 + i) * 16000) for i in range(B)]
        p = _fast(12)
    else:
        xs = [O.synth_audio(240, 12 * 16000), O.synth_audio(241, 35 * 16000)]
        kw = dict(beam_size=5, max_new_tokens=10) if case == "beam5" else \
            dict(temperature_inc=0.2, logprob_thold=10.0, best_of=5, max_new_tokens=10, seed=22)
        p = _full(**kw)
    ref, got, cs = _both("synthetic:large-v3:enc=2:dec=2", 8, xs, p, monkeypatch)
    assert cs["pd_fallbacks"] >= 1, cs
    if case.startswith("fast"):
        assert cs["pd_passes"] == 0, cs  # the re-run call ran on the chain only
    _assert_bitwise(ref, got)
    for a, b in zip(ref, got):
        assert [(s.start, s.end, s.text) for s in a.segments] == [(s.start, s.end, s.text) for s in b.segments]
