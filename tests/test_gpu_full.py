"""GPU parity of whisper_full (timestamps, segments, seek loop, fallback) against the oracle's
restatement (oracle/whisper_full.py) on synthetic tiny.en weights, f32 engine.

Bars: tokens, timestamp ids and segments identical up to the first step where the oracle's
decision gap (argmax gap, or the timestamp-mass rule's gap) is below 2e-3 -- the f32 logits of
the two sides agree to ~1e-4; log-probabilities within 2e-3.  Temperature sampling is checked
for structure and determinism (its draws come from the device stream)."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import whisper_full as W

pytestmark = pytest.mark.gpu

SEED = 1234
GAP = 2e-3


@pytest.fixture(scope="module")
def tiny():
    from spittle_amd import WhisperEngine, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=8, seed=SEED))
    e.load_model("synthetic:tiny.en")
    om = O.Model(O.dims_for("tiny.en"), SEED, O.W_F32)
    yield e, om
    e.unload_model()
    om.close()


def _params(**kw):
    from spittle_amd import WhisperInferenceParams
    kw.setdefault("language", "en")
    kw.setdefault("temperature_inc", 0.0)
    kw.setdefault("max_new_tokens", 0)
    return WhisperInferenceParams(**kw)


def _compare(r, wins, segs, toks):
    """GPU result vs oracle: equal until the oracle's first small-gap step."""
    steps = []
    for _, w in wins:
        steps += w.steps
    gaps = [s.margin for s in steps]
    exact = all(g > GAP for g in gaps)
    n = len(toks)
    got = list(r.tokens)
    if exact:
        assert got == toks
        assert [(int(round(s.start * 100)), int(round(s.end * 100)), s.text) for s in r.segments] == \
               [(a, b, t) for a, b, t, _, _ in segs]
        return True
    # compare the prefix before the first uncertain decision; an input whose very first decision
    # is uncertain would compare nothing, so it is a bad test input, not a pass
    k = next(i for i, g in enumerate(gaps) if g <= GAP)
    assert min(k, n) > 0, "the oracle's first decision is already uncertain: nothing to compare"
    assert got[:min(k, n)] == toks[:min(k, n)]
    return False


@pytest.mark.parametrize("seconds,seed", [(8, 60), (20, 61), (29.5, 62)])
def test_single_window_timestamps(tiny, seconds, seed):
    e, om = tiny
    x = O.synth_audio(seed, int(seconds * 16000))
    p = W.Params(max_tokens=40)
    r = e.transcribe_samples(x, _params(max_new_tokens=40))
    wins, segs, toks, kept = W.transcribe(om, x, p)
    exact = _compare(r, wins, segs, toks)
    if exact:
        for i, s in enumerate(kept):
            assert abs(r.top1[i] - s.plog) < GAP and int(r.top2[i]) == s.tid, i
    # segments are ordered in time and refer to text tokens
    for s in r.segments:
        assert s.end >= s.start and s.text
    assert r.text == "".join(s.text for s in r.segments).strip()


def test_multi_window_seek(tiny):
    """45 s: the second window starts where the first one's last timestamp (seek_delta) ends."""
    e, om = tiny
    x = np.concatenate([O.synth_audio(70), O.synth_audio(71)[:240000]])
    p = W.Params(max_tokens=24)
    r = e.transcribe_samples(x, _params(max_new_tokens=24))
    wins, segs, toks, _ = W.transcribe(om, x, p)
    if _compare(r, wins, segs, toks):
        assert r.n_windows == len(wins)
    assert r.n_windows >= 2


@pytest.mark.parametrize("seconds,seed", [(75, 72), (100, 74)])
def test_long_input_seek_loop(tiny, seconds, seed):
    """Inputs of 3-4+ windows: the seek loop, prompt_past conditioning across windows and segment
    times relative to each window's seek, against the oracle's whisper_full restatement."""
    e, om = tiny
    n = int(seconds * 16000)
    x = np.concatenate([O.synth_audio(seed + k) for k in range((n + 479999) // 480000)])[:n]
    p = W.Params(max_tokens=16)
    r = e.transcribe_samples(x, _params(max_new_tokens=16))
    wins, segs, toks, _ = W.transcribe(om, x, p)
    assert len(wins) >= 3
    if _compare(r, wins, segs, toks):
        assert r.n_windows == len(wins)
    assert r.n_windows >= 3


def test_too_short_and_empty(tiny):
    e, _ = tiny
    for n in (0, 100, 15000):  # < 1 s: whisper_full decodes nothing
        r = e.transcribe_samples(np.ones(n, np.float32) * 0.1, _params())
        assert r.text == "" and r.segments == [] and r.n_windows == 0


@pytest.mark.parametrize("n", [16159, 16160, 16320, 480000, 480001, 496000])
def test_window_boundary_lengths(tiny, n):
    """Input lengths at the seek loop's edges (oracle/whisper_full.py:281-287): the one-second
    threshold (16160 samples decode nothing, 16320 one window), exactly 30 s, 30 s + 1 sample,
    and 31 s, whose second window starts within 5 s of the end (prompt_past cleared) -- the same
    window count and tokens as the oracle (full.cpp's seek loop)."""
    e, om = tiny
    x = np.concatenate([O.synth_audio(95), O.synth_audio(96)])[:n]
    p = W.Params(max_tokens=16)
    r = e.transcribe_samples(x, _params(max_new_tokens=16))
    wins, segs, toks, _ = W.transcribe(om, x, p)
    if not wins:
        assert r.n_windows == 0 and r.text == "" and r.segments == []
        return
    if _compare(r, wins, segs, toks):
        assert r.n_windows == len(wins)


def _long_audio(n, seed):
    return np.concatenate([O.synth_audio(seed + k) for k in range((n + 479999) // 480000)])[:n]


@pytest.mark.parametrize("n,seed", [(15000, 130), (480001, 131), (45 * 16000, 133), (75 * 16000, 136)])
def test_fast_path_follows_seek_loop(tiny, n, seed):
    """The fast path's protocol (no timestamps, greedy, temperature_inc 0: capi.cpp full_mode() is
    false) on inputs that are not one window: whisper_full's window rules hold (VERDICT r4 missing 3,
    reference transcription.rs:494-503 hands the whole utterance to whisper_full).  Under one second
    nothing is decoded; 480 001 samples are ONE window (seek + 100 >= seek_end after it); 45 / 75 s
    take the seek loop with each later window conditioned on the earlier tokens (prompt_past).
    Window count and tokens equal to the oracle's whisper_full run at no_timestamps."""
    e, om = tiny
    x = _long_audio(n, seed)
    r = e.transcribe_samples(x, _params(no_timestamps=True, max_new_tokens=16))
    wins, segs, toks, _ = W.transcribe(om, x, W.Params(no_timestamps=True, max_tokens=16))
    if not wins:
        assert r.n_windows == 0 and r.text == "" and r.tokens == [] and r.segments == []
        return
    if _compare(r, wins, segs, toks):
        assert r.n_windows == len(wins)
    if n == 480001:
        assert len(wins) == 1 and r.n_windows == 1
    if n >= 45 * 16000:
        assert r.n_windows >= 2 and len(wins) >= 2


def test_fast_path_one_window_unchanged(tiny):
    """A 30 s window (the benchmark's input) stays on the device-resident fast path (no segments,
    one decoder pass per token) and decodes the tokens of whisper_full's single window."""
    e, om = tiny
    x = O.synth_audio(137)
    r = e.transcribe_samples(x, _params(no_timestamps=True, max_new_tokens=16))
    assert r.n_windows == 1 and r.segments == []  # the fast path's result carries no segments
    wins, _, toks, _ = W.transcribe(om, x, W.Params(no_timestamps=True, max_tokens=16))
    gaps = [s.margin for _, w in wins for s in w.steps]
    got = list(r.tokens)
    k = min(next((i for i, g in enumerate(gaps) if g <= GAP), len(gaps)), len(got))
    assert k > 0 and got[:k] == toks[:k]


def test_best_of_rows_not_dividing_pass_rows(monkeypatch):
    """a batch whose windows of best_of rows do not fit the decode groups whole (f32
    medium width: 23 rows per pass, 3 groups at max_batch 64; best_of 6 over 10 windows = 60 rows ->
    4 windows = 24 rows in the largest group) decodes with one row per window run instead of
    failing, and gives bitwise the result of private window copies (SPT_NO_WINDOW_SHARE=1)."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=64, seed=SEED))
    e.load_model("synthetic:medium.en:enc=1:dec=3")
    try:
        xs = [O.synth_audio(140 + i, 2 * 16000 + 160 * i) for i in range(10)]
        kw = dict(temperature_inc=0.5, logprob_thold=10.0, best_of=6, max_new_tokens=4, seed=5)
        a = e.transcribe_batch(xs, _params(**kw))
        monkeypatch.setenv("SPT_NO_WINDOW_SHARE", "1")
        b = e.transcribe_batch(xs, _params(**kw))
        monkeypatch.delenv("SPT_NO_WINDOW_SHARE")
        for ra, rb in zip(a, b):
            assert ra.n_fallbacks == 2 * ra.n_windows and ra.n_windows == 1
            assert ra.tokens == rb.tokens and np.array_equal(np.asarray(ra.top1), np.asarray(rb.top1))
    finally:
        e.unload_model()


def _beam_geometry_runs(e, x, others, p):
    """the beam-5 result for x alone, beside 1, 3 and 7 other utterances (x first, last and in the
    middle), as (tokens, plog) per placement"""
    runs = [("alone", e.transcribe_samples(x, p))]
    for k in (1, 3, 7):
        batch = others[:k]
        pos = {1: 0, 3: 3, 7: 4}[k]
        xs = batch[:pos] + [x] + batch[pos:]
        runs.append((f"with{k}@{pos}", e.transcribe_batch(xs, p)[pos]))
    return runs


def test_beam_dedup_batch_geometry():
    """whisper.cpp's beam search deduplicates candidates by exact score equality, which needs
    identical decoder rows to compute bitwise-equal scores in every pass geometry.
    The same beam-5 utterance alone, beside 1, 3 and 7 others (one engine call of 10, 20, 40 rows)
    and in a call of 14 utterances split over two engine calls (max_batch 64: 12 beam-5 utterances
    per call): bitwise-equal tokens and log-probabilities everywhere."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=64, seed=SEED))
    e.load_model("synthetic:tiny.en")
    try:
        p = _params(beam_size=5, max_new_tokens=12)
        x = O.synth_audio(91, 20 * 16000)
        others = [O.synth_audio(150 + i, (6 + i) * 16000) for i in range(13)]
        runs = _beam_geometry_runs(e, x, others, p)
        xs = others[:12] + [x] + others[12:]  # 14 utterances: calls of 12 and 2 (x in the second)
        runs.append(("split_calls", e.transcribe_batch(xs, p)[12]))
        ref = runs[0][1]
        for name, r in runs[1:]:
            assert r.tokens == ref.tokens, name
            assert np.array_equal(np.asarray(r.top1), np.asarray(ref.top1)), name
            assert np.array_equal(np.asarray(r.top2), np.asarray(ref.top2)), name
    finally:
        e.unload_model()


def test_temperature_fallback(tiny):
    """logprob_thold above any average log-probability forces every fallback: 0, 0.2, ..., 1.0
    (5 fallbacks), best_of = 5 sampled decoders per window at temperature > 0; the same seed
    reproduces the same result."""
    e, _ = tiny
    x = O.synth_audio(80, 10 * 16000)
    kw = dict(temperature_inc=0.2, logprob_thold=10.0, best_of=5, max_new_tokens=16, seed=7)
    a = e.transcribe_samples(x, _params(**kw))
    b = e.transcribe_samples(x, _params(**kw))
    assert a.n_fallbacks == 5 * a.n_windows and a.n_windows >= 1
    assert a.tokens == b.tokens and a.text == b.text
    V = 51864
    assert all(0 <= t < V for t in a.tokens)
    assert np.all(np.asarray(a.top1) <= 1e-6)
    c = e.transcribe_samples(x, _params(**{**kw, "seed": 8}))
    assert c.n_fallbacks == a.n_fallbacks


def test_no_timestamps_fallback_path(tiny):
    """no_timestamps with fallback enabled runs whisper_full: one segment per window spanning
    the window, [notimestamps] in the prompt, no timestamp tokens generated."""
    e, om = tiny
    x = O.synth_audio(81, 12 * 16000)
    r = e.transcribe_samples(x, _params(no_timestamps=True, temperature_inc=0.2, max_new_tokens=20))
    sp = O.special_tokens(51864)
    assert all(t < sp["beg"] for t in r.tokens)
    if r.n_fallbacks == 0:
        p = W.Params(no_timestamps=True, max_tokens=20)
        wins, segs, toks, _ = W.transcribe(om, x, p)
        _compare(r, wins, segs, toks)


@pytest.mark.parametrize("beam,seconds,seed", [(3, 8, 90), (5, 20, 91)])
def test_beam_search(tiny, beam, seconds, seed):
    """beam_size > 1 (WHISPER_SAMPLING_BEAM_SEARCH at temperature 0): each live decoder proposes
    its beam_size best candidates, the utterance's candidates are ranked by cumulative
    log-probability, decoders take them in order, K/V rows follow their source decoder; the best
    non-failed decoder by average log-probability wins."""
    e, om = tiny
    x = O.synth_audio(seed, int(seconds * 16000))
    r = e.transcribe_samples(x, _params(beam_size=beam, max_new_tokens=16))
    wins, segs, toks, kept = W.transcribe(om, x, W.Params(max_tokens=16, beam_size=beam))
    if _compare(r, wins, segs, toks):
        for i, s in enumerate(kept):
            assert abs(r.top1[i] - s.plog) < GAP and int(r.top2[i]) == s.tid, i
    g = e.transcribe_samples(x, _params(beam_size=1, max_new_tokens=16))
    assert g.n_windows >= 1 and r.n_windows >= 1


def test_beam_search_multi_window(tiny):
    """beam_size 4 over 45 s: the winning decoder's tokens set each window's seek and the next
    window's prompt, as in the oracle's seek loop."""
    e, om = tiny
    x = np.concatenate([O.synth_audio(92), O.synth_audio(93)[:240000]])
    r = e.transcribe_samples(x, _params(beam_size=4, max_new_tokens=16))
    wins, segs, toks, _ = W.transcribe(om, x, W.Params(max_tokens=16, beam_size=4))
    assert len(wins) >= 2
    if _compare(r, wins, segs, toks):
        assert r.n_windows == len(wins)
    assert r.n_windows >= 2


def test_beam_needs_rows():
    from spittle_amd import TranscriptionError, WhisperEngine, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=2, seed=SEED))
    e.load_model("synthetic:tiny.en:enc=1:dec=1")
    with pytest.raises(TranscriptionError, match="beam_size exceeds"):
        e.transcribe_samples(O.synth_audio(1, 32000), _params(beam_size=3))
    e.unload_model()


def test_full_batch_invariance(tiny):
    """whisper_full over a batch of utterances (different lengths, so different seek paths)
    gives each utterance the result it gets alone."""
    e, _ = tiny
    xs = [O.synth_audio(100, 9 * 16000), O.synth_audio(101, 40 * 16000), O.synth_audio(102, 3 * 16000)]
    p = _params(max_new_tokens=12)
    batch = e.transcribe_batch(xs, p)
    for x, rb in zip(xs, batch):
        ra = e.transcribe_samples(x, p)
        assert ra.tokens == rb.tokens and ra.text == rb.text and ra.n_windows == rb.n_windows
        assert [(s.start, s.end, s.text) for s in ra.segments] == [(s.start, s.end, s.text) for s in rb.segments]


def test_full_language_autodetect():
    """language=None on the whisper_full path detects once per utterance (first window) and
    reports the same language as the fast path's detection."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=4, seed=SEED))
    e.load_model("synthetic:tiny:enc=2:dec=3")
    xs = [O.synth_audio(110 + i, 12 * 16000) for i in range(2)]
    full = e.transcribe_batch(xs, _params(language=None, max_new_tokens=8))
    fast = e.transcribe_batch(xs, _params(language=None, no_timestamps=True, ignore_eot=True, max_new_tokens=2))
    for a, b in zip(full, fast):
        assert a.language is not None and a.language == b.language
    e.unload_model()


def _loud_then_quiet(seconds, seed):
    n = int(seconds * 16000)
    x = np.concatenate([O.synth_audio(seed + k) for k in range((n + 479999) // 480000)])[:n].copy()
    x[n // 2:] *= np.float32(0.03)  # the second half 30 dB quieter
    return x


@pytest.mark.parametrize("seconds,seed", [(45, 300), (75, 302)])
def test_loud_then_quiet_whole_input_mel(tiny, seconds, seed):
    """whisper.cpp's whisper_full takes every window's frames from ONE log-mel of the whole input
    (global max - 8 clamp, real preceding samples at each window start; transcription.rs:494-503
    hands it the whole utterance).  A loud-then-quiet dictation over 30 s makes the later windows'
    mel differ from a per-window mel; the oracle restates the whole-input mel, and the device must
    match it window by window."""
    e, om = tiny
    x = _loud_then_quiet(seconds, seed)
    p = W.Params(max_tokens=16)
    r = e.transcribe_samples(x, _params(max_new_tokens=16))
    wins, segs, toks, _ = W.transcribe(om, x, p)
    assert len(wins) >= 2
    if _compare(r, wins, segs, toks):
        assert r.n_windows == len(wins)
    assert r.n_windows >= 2
    cs = e.call_stats()
    assert cs["encoder_windows"] == r.n_windows, cs  # one encoder run per window


def test_one_encoder_run_per_window_with_fallback(tiny):
    """Temperature fallback re-decodes a window at each temperature (best_of 5 sampled decoders
    at t > 0) over the SAME encoded window: one encoder run per window, several decoder runs."""
    e, _ = tiny
    x = O.synth_audio(84, 30 * 16000)
    r = e.transcribe_samples(x, _params(temperature_inc=0.2, logprob_thold=10.0, best_of=5, max_new_tokens=8, seed=3))
    cs = e.call_stats()
    assert r.n_fallbacks == 5 * r.n_windows
    assert cs["encoder_windows"] == r.n_windows, cs
    assert cs["engine_calls"] >= 6 * r.n_windows, cs
    # ABI 12's persistent-pass counters stay in the struct for layout; the pass was deleted in r6
    assert cs["pd_passes"] == 0 and cs["pd_fallbacks"] == 0, cs


@pytest.mark.parametrize("vw", ["0", "3"])
@pytest.mark.parametrize("kind", ["beam5", "fallback_best_of5"])
def test_cross_attention_strategies_bitwise(tiny, kind, vw, monkeypatch):
    """The decoders of one utterance on one shared window run, by default, one query per
    single-wave workgroup with the 8 partials merged by attn_part_merge_kernel (r4).  The 8-wave
    kernel with five queries per workgroup (SPT_XATTN_VW=0) and the single-wave kernel with five
    queries per workgroup (SPT_XATTN_VW=3) must give bitwise the same result: every strategy runs
    the same per-lane keys, block order and pinned arithmetic (contraction off, explicit fmaf)."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e, _ = tiny
    xs = [O.synth_audio(87, 12 * 16000), O.synth_audio(88, 35 * 16000)]
    kw = dict(beam_size=5, max_new_tokens=10) if kind == "beam5" else \
        dict(temperature_inc=0.2, logprob_thold=10.0, best_of=5, max_new_tokens=10, seed=13)
    ref = e.transcribe_batch(xs, _params(**kw))
    monkeypatch.setenv("SPT_XATTN_VW", vw)
    e2 = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=8, seed=SEED))  # captures under vw
    try:
        e2.load_model("synthetic:tiny.en")
        got = e2.transcribe_batch(xs, _params(**kw))
    finally:
        e2.unload_model()
    for a, b in zip(ref, got):
        assert a.tokens == b.tokens and a.text == b.text
        assert np.array_equal(np.asarray(a.top1), np.asarray(b.top1))


@pytest.mark.parametrize("kind", ["greedy", "beam5"])
def test_fc2_residual_fold_bitwise(tiny, kind, monkeypatch):
    """fc2's first K split adds the residual into its slab (r6), so the next LayerNorm prologue sums
    slab 0 + slab 1 instead of x + slab 0 + slab 1: the same additions in the same order, so the
    result is bitwise that of the unfolded passes (SPT_DEC_XFOLD=0, a new engine's captures)."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e, _ = tiny
    xs = [O.synth_audio(89, 12 * 16000), O.synth_audio(90, 35 * 16000)]
    kw = dict(beam_size=5, max_new_tokens=10) if kind == "beam5" else dict(max_new_tokens=24)
    ref = e.transcribe_batch(xs, _params(**kw))
    monkeypatch.setenv("SPT_DEC_XFOLD", "0")
    e2 = WhisperEngine(WhisperModelParams(dtype="f32", max_batch=8, seed=SEED))
    try:
        e2.load_model("synthetic:tiny.en")
        got = e2.transcribe_batch(xs, _params(**kw))
    finally:
        e2.unload_model()
    for a, b in zip(ref, got):
        assert a.tokens == b.tokens and a.text == b.text
        assert np.array_equal(np.asarray(a.top1), np.asarray(b.top1))


@pytest.mark.parametrize("kind", ["beam5", "fallback_best_of5"])
def test_shared_window_bitwise_equal_to_copies(tiny, kind, monkeypatch):
    """The decoders of one utterance (beam 5, best_of 5) read one shared encoded window; the
    result is bitwise the one they get when each decoder row encodes its own copy (every engine
    call before ABI 11; SPT_NO_WINDOW_SHARE=1)."""
    e, _ = tiny
    xs = [O.synth_audio(85, 12 * 16000), O.synth_audio(86, 40 * 16000)]
    kw = dict(beam_size=5, max_new_tokens=12) if kind == "beam5" else \
        dict(temperature_inc=0.2, logprob_thold=10.0, best_of=5, max_new_tokens=12, seed=11)
    shared = e.transcribe_batch(xs, _params(**kw))
    cs = e.call_stats()
    monkeypatch.setenv("SPT_NO_WINDOW_SHARE", "1")
    copies = e.transcribe_batch(xs, _params(**kw))
    cs2 = e.call_stats()
    monkeypatch.delenv("SPT_NO_WINDOW_SHARE")
    for a, b in zip(shared, copies):
        assert a.tokens == b.tokens and a.text == b.text
        assert np.array_equal(np.asarray(a.top1), np.asarray(b.top1))
        assert [(s.start, s.end, s.text) for s in a.segments] == [(s.start, s.end, s.text) for s in b.segments]
    assert cs["encoder_windows"] < cs2["encoder_windows"], (cs, cs2)
