"""ggml model files on the CPU: the host parser and dequantisation of the C ABI library
against oracle/ggml.py (and hand-derived known-answer blocks), the whisper tokenizer against
its restatement, and the load-time error paths that fail before any device is touched.

Bars: dequantisation bit-exact (integer codes times an f16 scale, f32 arithmetic, no
contraction on either side); tokenisation identical token lists."""
import ctypes as C
import struct

import numpy as np
import pytest

from oracle import ggml as G
from oracle import oracle as O


def _lib():
    from spittle_amd import _lib as L
    return L.load()


def _host_dequant(raw: bytes, t: int, n: int) -> np.ndarray:
    out = np.empty(n, np.float32)
    buf = C.create_string_buffer(raw, len(raw))
    st = _lib().spt_debug_ggml_dequant(t, buf, n, out.ctypes.data_as(C.POINTER(C.c_float)))
    assert st == 0, st
    return out


def _f16(v: float) -> bytes:
    return np.float16(v).tobytes()


# ---------------------------------------------------------------- known-answer blocks
def test_known_answer_blocks():
    """Blocks assembled by hand from the published layouts (ggml-quants.h block_q*)."""
    qs = bytes([0x10] + [0x00] * 15)  # element 0 code 0, element 16 code 1, the rest 0
    # q4_0: (q - 8) * d, d = 0.5
    v = G.dequantize(_f16(0.5) + qs, G.Q4_0, 32)
    assert v[0] == -4.0 and v[16] == -3.5 and v[1] == -4.0
    # q4_1: q * d + m, d = 2, m = -1
    v = G.dequantize(_f16(2.0) + _f16(-1.0) + qs, G.Q4_1, 32)
    assert v[0] == -1.0 and v[16] == 1.0
    # q5_0: fifth bit of element j in qh bit j (j < 16) / bit j - 16 + 16 (j >= 16); (q - 16) * d
    qh = struct.pack("<I", (1 << 0) | (1 << 16))
    v = G.dequantize(_f16(0.25) + qh + qs, G.Q5_0, 32)
    assert v[0] == 0.0 and v[16] == 0.25 and v[1] == -4.0
    # q5_1
    v = G.dequantize(_f16(1.0) + _f16(0.5) + qh + qs, G.Q5_1, 32)
    assert v[0] == 16.5 and v[16] == 17.5 and v[2] == 0.5
    # q8_0: int8 * d
    v = G.dequantize(_f16(0.125) + bytes([0x7F, 0x80] + [0x01] * 30), G.Q8_0, 32)
    assert v[0] == 15.875 and v[1] == -16.0 and v[2] == 0.125
    for raw, t in ((_f16(0.5) + qs, G.Q4_0), (_f16(0.25) + qh + qs, G.Q5_0),
                   (_f16(1.0) + _f16(0.5) + qh + qs, G.Q5_1), (_f16(2.0) + _f16(-1.0) + qs, G.Q4_1)):
        assert np.array_equal(_host_dequant(raw, t, 32), G.dequantize(raw, t, 32))


@pytest.mark.parametrize("t", [G.F32, G.F16, G.Q4_0, G.Q4_1, G.Q5_0, G.Q5_1, G.Q8_0])
def test_host_dequant_matches_restatement(t):
    rng = np.random.default_rng(t)
    x = (rng.standard_normal(32 * 257) * np.exp(rng.uniform(-6, 3, 32 * 257))).astype(np.float32)
    raw = G.quantize(x, t)
    assert len(raw) == (x.size // G.BLOCK[t][0]) * G.BLOCK[t][1]
    ref = G.dequantize(raw, t, x.size)
    assert np.array_equal(_host_dequant(raw, t, x.size), ref)
    # random bytes too (every code / high bit pattern), finite f16 scales
    blk, nbytes = G.BLOCK[t]
    if blk == 32:
        junk = bytearray(rng.integers(0, 256, 64 * nbytes, dtype=np.uint8).tobytes())
        for b in range(64):
            junk[b * nbytes:b * nbytes + 2] = _f16(float(rng.uniform(-2, 2)))
            if t in (G.Q4_1, G.Q5_1):
                junk[b * nbytes + 2:b * nbytes + 4] = _f16(float(rng.uniform(-2, 2)))
        raw = bytes(junk)
        assert np.array_equal(_host_dequant(raw, t, 64 * 32), G.dequantize(raw, t, 64 * 32))


def test_quantizer_round_trip_error():
    x = np.random.default_rng(0).uniform(-1, 1, 32 * 64).astype(np.float32)
    for t, tol in ((G.F16, 1e-3), (G.Q8_0, 1 / 127), (G.Q5_1, 2 / 31), (G.Q5_0, 1 / 16 + 1e-3),
                   (G.Q4_1, 2 / 15), (G.Q4_0, 1 / 8 + 1e-3)):
        y = G.dequantize(G.quantize(x, t), t, x.size)
        assert np.abs(x - y).max() <= tol, t


def test_unsupported_type_rejected():
    assert _lib().spt_debug_ggml_dequant(12, b"\0" * 256, 256, (C.c_float * 256)()) != 0  # q4_K


# ---------------------------------------------------------------- files and tokenizer
def _vocab_file(tmp_path, n_vocab=51864, seed=7):
    dims = O.dims_for("tiny.en", 1, 1)
    sp = O.special_tokens(n_vocab)
    vocab = G.synth_vocab(sp["eot"], seed)
    path = str(tmp_path / "vocab_only.bin")
    # header + filters + vocabulary only: enough for the host-side tokenizer hook
    with open(path, "wb") as f:
        f.write(struct.pack("<I", G.MAGIC))
        f.write(struct.pack("<11i", n_vocab, 1500, dims.d, dims.n_head, 1, 448, dims.d, dims.n_head, 1, 80, 1))
        f.write(struct.pack("<ii", 80, 201))
        f.write(O.mel_filters(80).tobytes())
        f.write(struct.pack("<i", len(vocab)))
        for w in vocab:
            f.write(struct.pack("<I", len(w)) + w)
    full = vocab + G.special_names(n_vocab, len(vocab), sp, _codes())
    return path, full


def _codes():
    lib = _lib()
    return [lib.spt_language_code(i).decode() for i in range(100)]


def _c_tokenize(path, text: bytes):
    n = C.c_int32()
    buf = (C.c_int32 * (len(text) + 1))()
    st = _lib().spt_debug_ggml_tokenize(path.encode(), text, buf, len(text) + 1, C.byref(n))
    assert st == 0, st
    return [buf[i] for i in range(n.value)]


TEXTS = [
    "Hello world, this is a test.",
    "It's the model's turn; they'll say we've done it, I'm sure you'd agree.",
    "numbers 12345 and 3.14159 and 1,000,000",
    "   leading   and trailing spaces   ",
    "tabs\tand\nnewlines\r\n mixed \t ",
    "Spittle, Kubernetes, PostgreSQL, gRPC, MI355X, gfx950",
    "café naïve über straße — “quoted” ‘single’ 日本語のテキスト",
    "!!!???... ((parens)) [brackets] {braces} <angles> @#$%^&*",
    "a",
    "",
    " ",
    "x" * 300,
]


@pytest.mark.parametrize("text", TEXTS)
def test_tokenizer_matches_restatement(tmp_path, text):
    path, full = _vocab_file(tmp_path)
    raw = text.encode()
    assert _c_tokenize(path, raw) == G.tokenize(full, raw)


def test_tokenizer_round_trip(tmp_path):
    """Every byte is a token (the 256 single-byte entries), so the tokens spell the text back."""
    path, full = _vocab_file(tmp_path)
    for text in TEXTS:
        raw = text.encode()
        toks = _c_tokenize(path, raw)
        assert b"".join(full[t] for t in toks) == raw
        if len(raw) > 3:
            assert len(toks) < len(raw)  # longest match merges pieces


def test_tokenizer_greedy_longest_match(tmp_path):
    """Longest entry from the left, not BPE merges: ' abc' with entries ' ab', 'bc', 'c'."""
    path = str(tmp_path / "v.bin")
    vocab = [bytes([i]) if i else b"<NUL>" for i in range(256)] + [b" ab", b"bc", b" abc", b"abcd"]
    vocab += [b"pad%d" % i for i in range(50256 - len(vocab))]
    with open(path, "wb") as f:
        f.write(struct.pack("<I", G.MAGIC) + struct.pack("<11i", 51864, 1500, 384, 6, 1, 448, 384, 6, 1, 80, 1))
        f.write(struct.pack("<ii", 80, 201) + np.zeros((80, 201), np.float32).tobytes())
        f.write(struct.pack("<i", len(vocab)) + b"".join(struct.pack("<I", len(w)) + w for w in vocab))
    assert _c_tokenize(path, b" abcd") == [258, ord("d")]  # ' abc' then 'd' (the piece is ' abcd')
    assert _c_tokenize(path, b"abcd") == [259]
    assert _c_tokenize(path, b" abc abcd") == [258, 258, ord("d")]


# ---------------------------------------------------------------- load errors (no device needed)
def _ctx_create(path):
    from spittle_amd import _lib as L
    lib = _lib()
    ctx = C.c_void_p()
    err = C.create_string_buffer(512)
    st = lib.spt_ctx_create(path.encode(), None, C.byref(ctx), err, 512)
    return st, err.value.decode()


def test_bad_files_fail_to_load(tmp_path):
    from spittle_amd import _lib as L
    p = tmp_path / "bad.bin"
    p.write_bytes(b"GGUF" + b"\0" * 100)
    st, msg = _ctx_create(str(p))
    assert st == L.SPT_ERR_LOAD and "magic" in msg
    path, _ = _vocab_file(tmp_path)
    data = open(path, "rb").read()
    p.write_bytes(data[: len(data) // 2])  # truncated vocabulary
    st, msg = _ctx_create(str(p))
    assert st == L.SPT_ERR_LOAD and "truncated" in msg
    # a tensor of an unsupported type (q4_K)
    tail = struct.pack("<iii", 2, 4, 12) + struct.pack("<2i", 256, 4) + b"abcd" + b"\0" * 576
    p.write_bytes(data + tail)
    st, msg = _ctx_create(str(p))
    assert st == L.SPT_ERR_LOAD and "unsupported ggml type 12" in msg
    # a tensor whose data runs past the end of the file
    tail = struct.pack("<iii", 1, 4, 0) + struct.pack("<i", 64) + b"abcd" + b"\0" * 100
    p.write_bytes(data + tail)
    st, msg = _ctx_create(str(p))
    assert st == L.SPT_ERR_LOAD and "truncated tensor data" in msg
    # unsupported model geometry: head dim 96
    bad = bytearray(data)
    bad[4 + 3 * 4:4 + 4 * 4] = struct.pack("<i", 4)
    p.write_bytes(bytes(bad))
    st, msg = _ctx_create(str(p))
    assert st == L.SPT_ERR_LOAD and "head" in msg
    st, msg = _ctx_create(str(tmp_path / "missing.bin"))
    assert st == L.SPT_ERR_LOAD and "not found" in msg
