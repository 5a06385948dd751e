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


@pytest.mark.parametrize("t", [G.F32, G.F16, G.Q4_0, G.Q4_1, G.Q5_0, G.Q5_1, G.Q8_0, G.Q4_K, G.Q5_K, G.Q6_K])
def test_host_dequant_matches_restatement(t):
    rng = np.random.default_rng(t)
    x = (rng.standard_normal(256 * 33) * np.exp(rng.uniform(-6, 3, 256 * 33))).astype(np.float32)
    raw = G.quantize(x, t)
    assert len(raw) == (x.size // G.BLOCK[t][0]) * G.BLOCK[t][1]
    ref = G.dequantize(raw, t, x.size)
    assert np.array_equal(_host_dequant(raw, t, x.size), ref)
    # random bytes too (every code / high bit pattern), finite f16 scales
    blk, nbytes = G.BLOCK[t]
    if blk > 1:
        junk = bytearray(rng.integers(0, 256, 64 * nbytes, dtype=np.uint8).tobytes())
        halves = {G.Q4_1: (0, 2), G.Q5_1: (0, 2), G.Q4_K: (0, 2), G.Q5_K: (0, 2), G.Q6_K: (208,)}.get(t, (0,))
        for b in range(64):
            for o in halves:
                junk[b * nbytes + o:b * nbytes + o + 2] = _f16(float(rng.uniform(-2, 2)))
        raw = bytes(junk)
        assert np.array_equal(_host_dequant(raw, t, 64 * blk), G.dequantize(raw, t, 64 * blk))


def test_known_answer_k_blocks():
    """q4_K / q6_K blocks assembled by hand (ggml-quants.h block_q4_K, block_q6_K)."""
    # q4_K: d = 1, dmin = 0.5; sub-block 0 scale 2 min 1, sub-block 5 scale 17 (4 + 16) min 33 (1 + 32)
    sc = bytearray(12)
    sc[0], sc[4] = 2, 1
    sc[1] |= 1 << 6           # high bits of sub-block 5's scale (scales[j - 4] >> 6)
    sc[5] |= 2 << 6           # high bits of sub-block 5's min (scales[j] >> 6, j = 5)
    sc[9] = 1 | (1 << 4)      # low nibbles of sub-block 5's scale / min
    qs = bytearray(128)
    qs[0] = 0x3 | (0x7 << 4)  # element 0: 3 (sub-block 0), element 32: 7 (sub-block 1)
    qs[64 + 5] = 0x9 << 4     # element 128 + 32 + 5 = 165 (sub-block 5, high nibble): 9
    raw = _f16(1.0) + _f16(0.5) + bytes(sc) + bytes(qs)
    v = G.dequantize(raw, G.Q4_K, 256)
    assert v[0] == 2 * 3 - 0.5 and v[1] == -0.5
    assert v[165] == 17 * 9 - 0.5 * 33
    assert np.array_equal(_host_dequant(raw, G.Q4_K, 256), v)
    # q6_K: d = 0.25; 16-element sub-block 0 has scale 4, sub-block 9 (elements 144..159) -2;
    # codes are 6 bits minus 32
    ql, qh, s6 = bytearray(128), bytearray(64), bytearray(16)
    s6[0], s6[9] = 4, 0xFE
    ql[0], qh[0] = 0xF, 0x3  # element 0: 0xF | 3 << 4 = 63
    ql[64 + 16] = 0x5        # element 128 + 16 = 144 (second half, l = 16): low nibble 5
    raw = bytes(ql) + bytes(qh) + bytes(s6) + _f16(0.25)
    v = G.dequantize(raw, G.Q6_K, 256)
    assert v[0] == 0.25 * 4 * 31 and v[144] == 0.25 * -2 * (5 - 32) and v[1] == 0.25 * 4 * -32
    assert np.array_equal(_host_dequant(raw, G.Q6_K, 256), v)


def test_quantizer_round_trip_error():
    x = np.random.default_rng(0).uniform(-1, 1, 256 * 8).astype(np.float32)
    for t, tol in ((G.F16, 1e-3), (G.Q8_0, 1 / 127), (G.Q5_1, 2 / 31), (G.Q5_0, 1 / 16 + 1e-3),
                   (G.Q4_1, 2 / 15), (G.Q4_0, 1 / 8 + 1e-3), (G.Q6_K, 0.02), (G.Q5_K, 0.04), (G.Q4_K, 0.08)):
        y = G.dequantize(G.quantize(x, t), t, x.size)
        assert np.abs(x - y).max() <= tol, t


def test_unsupported_type_rejected():
    assert _lib().spt_debug_ggml_dequant(10, b"\0" * 256, 256, (C.c_float * 256)()) != 0  # q2_K


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
    # a tensor of an unsupported type (q3_K)
    tail = struct.pack("<iii", 2, 4, 11) + struct.pack("<2i", 256, 4) + b"abcd" + b"\0" * 440
    p.write_bytes(data + tail)
    st, msg = _ctx_create(str(p))
    assert st == L.SPT_ERR_LOAD and "unsupported ggml type 11" in msg
    # a K-quant row that is not a multiple of the 256-element block
    tail = struct.pack("<iii", 2, 4, 13) + struct.pack("<2i", 384, 2) + b"abcd" + b"\0" * 528
    p.write_bytes(data + tail)
    st, msg = _ctx_create(str(p))
    assert st == L.SPT_ERR_LOAD and "multiple of the block" in msg
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
