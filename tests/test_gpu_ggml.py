"""GPU parity of ggml model files (whisper.cpp's .bin models, the format Spittle's catalog
ships): files written by oracle/ggml.py from the oracle's weights -- as f32, f16 and every
supported quantisation -- are loaded through spt_ctx_create(path), dequantised on the device
and transcribed; the oracle runs with the dequantised values the file holds.

Tolerances: weights bit-exact (checksums to 1e-10 relative); f32 engine: greedy tokens equal
wherever the oracle's top-1/top-2 gap > 2e-3, logits within 2e-3 (as tests/test_gpu_parity.py);
bf16 engine: encoder relative L2 error < 3e-2.  Text: the vocabulary strings of the text tokens,
byte for byte (whisper_full's segment text)."""
import numpy as np
import pytest

from oracle import ggml as G
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 1234
FLAGS = O.SUPPRESS_BLANK | O.NO_TIMESTAMPS | O.IGNORE_EOT


def _bf16(x):
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def _engine_dtype_tids(dims):
    """tensors the engine stores in its own dtype (bf16-rounded in a bf16 engine)"""
    return {tid for tid, name, ne in G.tensor_table(dims) if len(ne) >= 2 and name not in G._F32_ALWAYS}


class ModelFile:
    def __init__(self, tmp, cfg, wtype, n_enc=None, n_dec=None, **kw):
        self.dims = O.dims_for(cfg, n_enc, n_dec) if isinstance(cfg, str) else cfg
        base = O.Model(self.dims, SEED, O.W_F32)
        self.sp = O.special_tokens(self.dims.n_vocab)
        self.vocab = G.synth_vocab(self.sp["eot"])
        codes = [c.decode() for c in (_lib().spt_language_code(i) for i in range(100))]
        self.full_vocab = self.vocab + G.special_names(self.dims.n_vocab, len(self.vocab), self.sp, codes)
        tag = cfg if isinstance(cfg, str) else f"d{cfg.d}"
        self.path = str(tmp / f"ggml-{tag}-{wtype}.bin")
        self.deq = G.write_model(self.path, self.dims, O.mel_filters(self.dims.n_mels), self.vocab, base.tensors(),
                                 wtype, **kw)
        base.close()

    def oracle(self, dtype="f32"):
        om = O.Model(self.dims, SEED, O.W_BF16 if dtype == "bf16" else O.W_F32)
        rnd = _engine_dtype_tids(self.dims) if dtype == "bf16" else set()
        for tid, v in self.deq.items():
            om.set_tensor(tid, _bf16(v) if tid in rnd else v)
        return om


def _lib():
    from spittle_amd import _lib as L
    return L.load()


def _engine(path, dtype="f32", max_batch=2):
    from spittle_amd import WhisperEngine, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype=dtype, max_batch=max_batch, seed=SEED))
    e.load_model(path)
    return e


def _params(**kw):
    from spittle_amd import WhisperInferenceParams
    kw.setdefault("language", "en")
    kw.setdefault("no_timestamps", True)  # the device-resident greedy protocol (no fallback)
    kw.setdefault("temperature_inc", 0.0)
    return WhisperInferenceParams(**kw)


def _check_greedy(got, top1, tk, t1, t2, gap_tol=2e-3, logit_tol=2e-3):
    for s in range(len(tk)):
        if got[s] != tk[s]:
            assert (t1 - t2)[s] < gap_tol, (s, got, tk)
            return
        assert abs(top1[s] - t1[s]) < logit_tol, (s, top1[s], t1[s])


@pytest.fixture(scope="module")
def tiny_f32(tmp_path_factory):
    return ModelFile(tmp_path_factory.mktemp("g"), "tiny.en", G.F32)


def test_f32_file_equals_synthetic_model(tiny_f32):
    """A file holding exactly the synthetic weights transcribes exactly like the synthetic model."""
    e = _engine(tiny_f32.path)
    s = _engine("synthetic:tiny.en")
    x = O.synth_audio(2)
    p = _params(ignore_eot=True, max_new_tokens=24)
    a, b = e.transcribe_samples(x, p), s.transcribe_samples(x, p)
    assert a.tokens == b.tokens
    assert np.abs(np.asarray(a.top1) - np.asarray(b.top1)).max() < 1e-5
    for tid in (1, 3, 7, 10, 102, 104, 5013, 5014, 5015):
        assert e.weight_checksum(tid) == pytest.approx(s.weight_checksum(tid), rel=1e-12)
    e.unload_model()
    s.unload_model()


@pytest.mark.parametrize("wtype", [G.F16, G.Q8_0, G.Q5_0, G.Q5_1, G.Q4_0, G.Q4_1])
def test_quantized_file_f32(tmp_path, wtype):
    mf = ModelFile(tmp_path, "tiny.en", wtype, 2, 2)
    e = _engine(mf.path)
    for tid in (1, 3, 10, 100 + 2, 100 + 13, 5000 + 13, 5000 + 14, 5032 + 22):
        w = mf.deq[tid].astype(np.float64)
        a, s = e.weight_checksum(tid)
        assert a == pytest.approx(np.abs(w).sum(), rel=1e-10, abs=1e-9), tid
        assert s == pytest.approx(w.sum(), rel=1e-8, abs=1e-6), tid
    om = mf.oracle()
    x = O.synth_audio(3)
    n = 16
    r = e.transcribe_samples(x, _params(ignore_eot=True, max_new_tokens=n))
    enc = om.encode(O.mel(x, 80))
    assert np.abs(e.debug_encode(O.mel(x, 80)) - enc).max() < 2e-3
    tk, t1, t2 = om.decode(enc, O.default_prompt(mf.dims.n_vocab), n, FLAGS)
    _check_greedy(np.array(r.tokens), r.top1, tk, t1, t2)
    e.unload_model()


@pytest.mark.parametrize("wtype", [G.Q5_K, G.Q4_K, G.Q6_K])
def test_k_quant_file_f32(tmp_path, wtype):
    """K-quants (256-element super-blocks: the catalog's breeze-asr-q5_k) need rows that are
    multiples of 256: base geometry (512 wide, 8 heads), 2 + 2 layers, f32 engine."""
    mf = ModelFile(tmp_path, O.Dims(80, 512, 8, 2, 2, 51865, 1500, 448), wtype)
    e = _engine(mf.path)
    for tid in (10, 102, 111, 113, 5013, 5054):
        w = mf.deq[tid].astype(np.float64)
        a, s = e.weight_checksum(tid)
        assert a == pytest.approx(np.abs(w).sum(), rel=1e-10), tid
        assert s == pytest.approx(w.sum(), rel=1e-8, abs=1e-6), tid
    om = mf.oracle()
    x = O.synth_audio(8)
    n = 8
    r = e.transcribe_samples(x, _params(ignore_eot=True, max_new_tokens=n))
    enc = om.encode(O.mel(x, 80))
    tk, t1, t2 = om.decode(enc, O.default_prompt(mf.dims.n_vocab), n, FLAGS)
    _check_greedy(np.array(r.tokens), r.top1, tk, t1, t2)
    e.unload_model()


def test_f16_file_bf16_engine(tmp_path):
    """bf16 engine, large-v3 geometry (128 mels, 1280 wide, 2 + 2 layers), f16 file."""
    mf = ModelFile(tmp_path, "large-v3", G.F16, 2, 2)
    e = _engine(mf.path, "bf16")
    for tid in (1, 10, 102, 5013):
        w = _bf16(mf.deq[tid]).astype(np.float64)
        a, _ = e.weight_checksum(tid)
        assert a == pytest.approx(np.abs(w).sum(), rel=1e-10), tid
    om = mf.oracle("bf16")
    mel = O.mel(O.synth_audio(4), 128)
    g, o = e.debug_encode(mel), om.encode(mel)
    assert np.linalg.norm(g - o) / np.linalg.norm(o) < 3e-2
    e.unload_model()


def test_text_is_vocabulary_strings(tiny_f32):
    e = _engine(tiny_f32.path)
    r = e.transcribe_samples(O.synth_audio(5), _params(ignore_eot=True, max_new_tokens=20))
    eot = tiny_f32.sp["eot"]
    want = b"".join(tiny_f32.full_vocab[t] for t in r.tokens if t < eot)
    assert r.text == want.decode("utf-8", "replace")
    for t in (0, 300, eot, eot + 1, tiny_f32.dims.n_vocab - 1):
        assert e.token_to_str(t) == tiny_f32.full_vocab[t]
    assert e.token_to_str(tiny_f32.dims.n_vocab) is None
    e.unload_model()


def test_initial_prompt(tiny_f32):
    """initial_prompt (Spittle's custom-words prompt) is tokenised with whisper_tokenize and
    decoded as prompt_past: same tokens as passing those ids as prompt_tokens, and the oracle's
    greedy decode with [prev] + tokens ahead of [sot]."""
    e = _engine(tiny_f32.path)
    text = "Spittle, Kubernetes, PostgreSQL, gRPC, MI355X"
    ids = G.tokenize(tiny_f32.full_vocab, text.encode())
    assert e.tokenize(text) == ids
    x = O.synth_audio(6)
    n = 12
    a = e.transcribe_samples(x, _params(initial_prompt=text, ignore_eot=True, max_new_tokens=n))
    b = e.transcribe_samples(x, _params(prompt_tokens=ids, ignore_eot=True, max_new_tokens=n))
    assert a.tokens == b.tokens
    om = tiny_f32.oracle()
    enc = om.encode(O.mel(x, 80))
    tk, t1, t2 = om.decode(enc, O.default_prompt(tiny_f32.dims.n_vocab, past=ids), n, FLAGS)
    _check_greedy(np.array(a.tokens), a.top1, tk, t1, t2)
    e.unload_model()


def test_f32_engine_width_limit(tmp_path):
    """The f32 engine (a parity mode) stages LayerNorm'd decoder rows of at most 1024 f32 values;
    wider models load in bf16 -- and a wider f32 request fails at load, not mid-transcription."""
    from spittle_amd import TranscriptionError
    with pytest.raises(TranscriptionError, match="f32 engine"):
        _engine("synthetic:large-v3:enc=1:dec=1", "f32")


def test_missing_or_misshapen_tensor(tmp_path):
    from spittle_amd import TranscriptionError
    mf = ModelFile(tmp_path, "tiny.en", G.Q8_0, 1, 1, skip=("decoder.blocks.0.cross_attn.value.bias",))
    with pytest.raises(TranscriptionError, match="lacks tensor decoder.blocks.0.cross_attn.value.bias"):
        _engine(mf.path)
    mf = ModelFile(tmp_path, "tiny.en", G.F16, 1, 1, override={"encoder.blocks.0.mlp.0.weight": (G.F16, [384, 384])})
    with pytest.raises(TranscriptionError, match="encoder.blocks.0.mlp.0.weight has 147456 elements"):
        _engine(mf.path)


NST = ["\"", "#", "(", ")", "*", "+", "/", ":", ";", "<", "=", ">", "@", "[", "\\", "]", "^", "_", "`", "{", "|",
       "}", "~", "「", "」", "『", "』", "<<", ">>", "<<<", ">>>", "--", "---", "-(", "-[", "('", "(\"", "((", "))",
       "(((", ")))", "[[", "]]", "{{", "}}", "♪♪", "♪♪♪", "♩", "♪", "♫", "♬", "♭", "♮", "♯"]


def test_whisper_full_with_vocabulary(tiny_f32):
    """The whisper_full path on a ggml model: suppress_non_speech_tokens keeps every non-speech
    token (whisper_process_logits' list, with and without a leading space, plus " -" and " '")
    out of the result; initial_prompt equals passing its tokens; segment texts are vocabulary
    strings and the result text is their trimmed concatenation."""
    e = _engine(tiny_f32.path)
    ids = {}
    for i, w in enumerate(tiny_f32.full_vocab):
        ids[w] = i  # later duplicates win, as in the loader
    nst = set()
    for t in NST:
        for w in (t.encode(), b" " + t.encode()):
            if w in ids:
                nst.add(ids[w])
    for w in (b" -", b" '"):
        if w in ids:
            nst.add(ids[w])
    assert len(nst) > 10
    from spittle_amd import WhisperInferenceParams
    x = O.synth_audio(120, 15 * 16000)
    base = dict(language="en", temperature_inc=0.0, max_new_tokens=30)
    r = e.transcribe_samples(x, WhisperInferenceParams(suppress_non_speech_tokens=True, **base))
    assert not (set(r.tokens) & nst)
    prompt = "Kubernetes, PostgreSQL, gRPC"
    a = e.transcribe_samples(x, WhisperInferenceParams(initial_prompt=prompt, **base))
    b = e.transcribe_samples(x, WhisperInferenceParams(prompt_tokens=e.tokenize(prompt), **base))
    assert a.tokens == b.tokens and a.text == b.text
    eot = tiny_f32.sp["eot"]
    for s in a.segments:
        toks = a.tokens[s.i0:s.i0 + s.n_tokens]
        assert s.text == b"".join(tiny_f32.full_vocab[t] for t in toks if t < eot).decode("utf-8", "replace")
    assert a.text == "".join(s.text for s in a.segments).strip()
    e.unload_model()


@pytest.fixture(scope="module")
def turbo(tmp_path_factory):
    """ggml-large-v3-turbo.bin's geometry (/root/reference/src-tauri/resources/model_catalog.json:
    169-173): large-v3 width (d 1280, 20 heads, 128 mels, 51866 tokens) with 4 decoder layers, as
    an f16 file; 2 encoder layers here (turbo's encoder is large-v3's 32, covered at full depth by
    test_gpu_fullsize)."""
    O.set_threads(16)
    mf = ModelFile(tmp_path_factory.mktemp("turbo"), "large-v3", G.F16, 2, 4)
    e = _engine(mf.path, "bf16", max_batch=8)
    om = mf.oracle("bf16")
    yield mf, e, om
    e.unload_model()
    om.close()


def _long_audio(seconds, seed):
    n = int(seconds * 16000)
    return np.concatenate([O.synth_audio(seed + k) for k in range((n + 479999) // 480000)])[:n]


@pytest.mark.parametrize("seconds,seed", [(20, 400), (45, 404)])
def test_turbo_file_whisper_full(turbo, seconds, seed):
    """The app's call (whisper_full, timestamps on, fallback off) on the turbo geometry: tokens,
    timestamp ids and segments equal to the oracle's whisper_full on the file's values rounded as
    the bf16 engine holds them (bars of test_gpu_full_large: decisions over 0.1, log-probabilities
    within 0.05; the seeds' oracle decisions all clear 0.1)."""
    from oracle import whisper_full as W
    from spittle_amd import WhisperInferenceParams
    mf, e, om = turbo
    assert e.info()["n_dec"] == 4 and e.info()["n_enc"] == 2
    x = _long_audio(seconds, seed)
    r = e.transcribe_samples(x, WhisperInferenceParams(language="en", temperature_inc=0.0, max_new_tokens=24))
    wins, segs, toks, kept = W.transcribe(om, x, W.Params(max_tokens=24))
    assert min(s.margin for _, w in wins for s in w.steps) > 0.1  # the seed's decisions clear the bar
    assert list(r.tokens) == toks and r.n_windows == len(wins)
    assert max(abs(float(r.top1[i]) - kept[i].plog) for i in range(len(toks))) < 0.05
    # segment times as the oracle's, texts the vocabulary strings of their text tokens
    eot = mf.sp["eot"]
    assert [(int(round(s.start * 100)), int(round(s.end * 100))) for s in r.segments] == [(a, b) for a, b, _, _, _ in segs]
    for s, (_, _, _, i0, n) in zip(r.segments, segs):
        assert s.text == b"".join(mf.full_vocab[t] for t in toks[i0:i0 + n] if t < eot).decode("utf-8", "replace")


def test_turbo_file_fast_path_batch(turbo):
    """The benchmark protocol on the turbo geometry (B = 8 windows, greedy, no timestamps):
    teacher-forced on the oracle's tokens, top-1 logits within 0.1; batch-invariant (bitwise)."""
    mf, e, om = turbo
    xs = [O.synth_audio(410 + i) for i in range(8)]
    n = 12
    rs = e.transcribe_batch(xs, _params(ignore_eot=True, max_new_tokens=n))
    for i in (0, 5):
        enc = om.encode(O.mel(xs[i], 128))
        tk, t1, t2 = om.decode(enc, O.default_prompt(mf.dims.n_vocab), n, FLAGS)
        got = np.array(rs[i].tokens)
        k = next((s for s in range(n) if (t1 - t2)[s] < 0.2), n)
        assert list(got[:k]) == list(tk[:k]), (i, got, tk)
        assert np.abs(np.asarray(rs[i].top1[:k]) - t1[:k]).max() < 0.1
        alone = e.transcribe_samples(xs[i], _params(ignore_eot=True, max_new_tokens=n))
        assert alone.tokens == rs[i].tokens and np.array_equal(alone.top1, rs[i].top1)
