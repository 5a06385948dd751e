"""ggml model files and the whisper tokenizer, restated for the tests.

TEST INFRASTRUCTURE ONLY (like the rest of oracle/): the product reads ggml files with
spittle_amd/csrc/ggml_file.cpp and dequantises on the device (k_init.hip ggml_dequant); this
module writes such files from the oracle's weights and is the checker for both.

What it restates (whisper.cpp / ggml, ~v1.7.x, the version whisper-rs-sys 0.11.1 vendors;
/root/reference/src-tauri/Cargo.lock:8156-8174 -- not vendored in /root/reference, so the
formats are restated from their published source):
  * the legacy whisper ggml container (models/convert-pt-to-ggml.py writes it,
    whisper_model_load reads it): magic, 11 int32 hparams, mel filters, vocabulary, tensors;
  * ggml-quants.c quantize_row_*_ref / dequantize_row_* for q4_0, q4_1, q5_0, q5_1, q8_0
    (32-element blocks, f16 scale d [and offset m]);
  * whisper.cpp tokenize(): GPT-2 pre-tokenisation regex, then greedy longest match.
Parity: the block formats are also pinned by hand-derived known-answer blocks in
tests/test_ggml.py; relative to whisper.cpp itself they are "parity unpinned" (no ggml
binary or model file exists in /root/reference to run or read).
"""
from __future__ import annotations

import re
import struct

import numpy as np

MAGIC = 0x67676D6C
F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q4_K, Q5_K, Q6_K = 0, 1, 2, 3, 6, 7, 8, 12, 13, 14
BLOCK = {F32: (1, 4), F16: (1, 2), Q4_0: (32, 18), Q4_1: (32, 20), Q5_0: (32, 22), Q5_1: (32, 24),
         Q8_0: (32, 34), Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210)}
# file-level ftype (ggml_ftype) of a model whose 2-D weights are of a given tensor type
FTYPE = {F32: 0, F16: 1, Q4_0: 2, Q4_1: 3, Q8_0: 7, Q5_0: 8, Q5_1: 9, Q4_K: 12, Q5_K: 13, Q6_K: 14}


# ----------------------------------------------------------------------------- quantisation
def _f16(x):
    return np.asarray(x, np.float32).astype(np.float16)


def _rnd(v):
    return np.sign(v) * np.floor(np.abs(v) + 0.5)


def _pack_k4_scales(sc: np.ndarray, mn: np.ndarray) -> np.ndarray:
    """inverse of get_scale_min_k4: 8 six-bit scale and min codes -> 12 bytes"""
    q = np.zeros((sc.shape[0], 12), np.uint8)
    for j in range(4):
        q[:, j] = (sc[:, j] & 63) | ((sc[:, j + 4] >> 4) << 6)
        q[:, j + 4] = (mn[:, j] & 63) | ((mn[:, j + 4] >> 4) << 6)
        q[:, j + 8] = (sc[:, j + 4] & 0xF) | ((mn[:, j + 4] & 0xF) << 4)
    return q


def _quantize_k(x: np.ndarray, t: int) -> bytes:
    """A valid (not ggml's iterative, error-minimising) encoding of the K-quant formats: the
    tests only need well-formed blocks to compare the loader with dequantize()."""
    b = x.reshape(-1, 256).astype(np.float32)
    nb = b.shape[0]
    if t == Q6_K:
        sub = b.reshape(nb, 16, 16)
        s = np.abs(sub).max(axis=2) / 31.0
        d = (s.max(axis=1) / 127.0).astype(np.float32)
        d16 = _f16(d)
        dq = d16.astype(np.float32)
        sc = np.clip(_rnd(s / np.where(dq > 0, dq, 1)[:, None]), -128, 127).astype(np.int8)
        step = dq[:, None] * sc.astype(np.float32)
        q = np.clip(_rnd(sub / np.where(step != 0, step, 1)[:, :, None]), -32, 31).astype(np.int32) + 32
        q = q.reshape(nb, 256)
        out = np.zeros((nb, 210), np.uint8)
        for h in range(2):
            e = q[:, 128 * h:128 * h + 128]
            out[:, 64 * h:64 * h + 32] = (e[:, 0:32] & 0xF) | ((e[:, 64:96] & 0xF) << 4)
            out[:, 64 * h + 32:64 * h + 64] = (e[:, 32:64] & 0xF) | ((e[:, 96:128] & 0xF) << 4)
            out[:, 128 + 32 * h:128 + 32 * h + 32] = ((e[:, 0:32] >> 4) | ((e[:, 32:64] >> 4) << 2) |
                                                     ((e[:, 64:96] >> 4) << 4) | ((e[:, 96:128] >> 4) << 6))
        out[:, 192:208] = sc.view(np.uint8)
        out[:, 208:210] = d16.view(np.uint8).reshape(nb, 2)
        return out.tobytes()
    qmax = 15 if t == Q4_K else 31
    sub = b.reshape(nb, 8, 32)
    lo = np.minimum(sub.min(axis=2), 0.0)
    s = (sub.max(axis=2) - lo) / qmax
    d16, m16 = _f16(s.max(axis=1) / 63.0), _f16(-lo.min(axis=1) / 63.0)
    d, dmin = d16.astype(np.float32), m16.astype(np.float32)
    sc = np.clip(np.ceil(s / np.where(d > 0, d, 1)[:, None]), 0, 63).astype(np.int32)
    mn = np.clip(_rnd(-lo / np.where(dmin > 0, dmin, 1)[:, None]), 0, 63).astype(np.int32)
    step = d[:, None] * sc
    q = np.clip(_rnd((sub + (dmin[:, None] * mn)[:, :, None]) / np.where(step > 0, step, 1)[:, :, None]), 0, qmax)
    q = q.astype(np.int32).reshape(nb, 4, 2, 32)  # [group][low/high sub-block][l]
    out = np.zeros((nb, 144 if t == Q4_K else 176), np.uint8)
    out[:, 0:2] = d16.view(np.uint8).reshape(nb, 2)
    out[:, 2:4] = m16.view(np.uint8).reshape(nb, 2)
    out[:, 4:16] = _pack_k4_scales(sc, mn)
    o = 16
    if t == Q5_K:
        qh = np.zeros((nb, 32), np.int32)
        for g in range(4):
            qh |= ((q[:, g, 0] >> 4) & 1) << (2 * g)
            qh |= ((q[:, g, 1] >> 4) & 1) << (2 * g + 1)
        out[:, 16:48] = qh.astype(np.uint8)
        o = 48
    ql = (q[:, :, 0] & 0xF) | ((q[:, :, 1] & 0xF) << 4)
    out[:, o:o + 128] = ql.reshape(nb, 128).astype(np.uint8)
    return out.tobytes()


def _dequantize_k(a: np.ndarray, t: int, n: int) -> np.ndarray:
    """dequantize_row_q4_K / q5_K / q6_K (products rounded one at a time)"""
    _, nbytes = BLOCK[t]
    b = a[: (n // 256) * nbytes].reshape(-1, nbytes)
    nb = b.shape[0]
    if t == Q6_K:
        ql, qh = b[:, 0:128].astype(np.int32), b[:, 128:192].astype(np.int32)
        sc = b[:, 192:208].view(np.int8).astype(np.float32)
        d = b[:, 208:210].copy().view(np.float16).astype(np.float32)[:, 0]
        q = np.zeros((nb, 256), np.int32)
        for h in range(2):
            a_, b_, c = ql[:, 64 * h:64 * h + 32], ql[:, 64 * h + 32:64 * h + 64], qh[:, 32 * h:32 * h + 32]
            q[:, 128 * h:128 * h + 32] = (a_ & 0xF) | (((c >> 0) & 3) << 4)
            q[:, 128 * h + 32:128 * h + 64] = (b_ & 0xF) | (((c >> 2) & 3) << 4)
            q[:, 128 * h + 64:128 * h + 96] = (a_ >> 4) | (((c >> 4) & 3) << 4)
            q[:, 128 * h + 96:128 * h + 128] = (b_ >> 4) | (((c >> 6) & 3) << 4)
        ds = (d[:, None] * sc).astype(np.float32)  # [nb][16]: d * sc, then * q
        v = np.repeat(ds, 16, axis=1) * (q - 32).astype(np.float32)
        return v.astype(np.float32).ravel()
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
    dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
    s = b[:, 4:16].astype(np.int32)
    sc, mn = np.zeros((nb, 8), np.int32), np.zeros((nb, 8), np.int32)
    for j in range(8):
        if j < 4:
            sc[:, j], mn[:, j] = s[:, j] & 63, s[:, j + 4] & 63
        else:
            sc[:, j] = (s[:, j + 4] & 0xF) | ((s[:, j - 4] >> 6) << 4)
            mn[:, j] = (s[:, j + 4] >> 4) | ((s[:, j] >> 6) << 4)
    o = 48 if t == Q5_K else 16
    ql = b[:, o:o + 128].astype(np.int32).reshape(nb, 4, 32)
    q = np.stack([ql & 0xF, ql >> 4], axis=2)  # [nb][4][2][32]
    if t == Q5_K:
        qh = b[:, 16:48].astype(np.int32)
        for g in range(4):
            q[:, g, 0] += ((qh >> (2 * g)) & 1) * 16
            q[:, g, 1] += ((qh >> (2 * g + 1)) & 1) * 16
    dd = (d[:, None] * sc.astype(np.float32)).astype(np.float32).reshape(nb, 4, 2, 1)
    mm = (dmin[:, None] * mn.astype(np.float32)).astype(np.float32).reshape(nb, 4, 2, 1)
    v = (dd * q.astype(np.float32)).astype(np.float32) - mm
    return v.astype(np.float32).ravel()


def quantize(x: np.ndarray, t: int) -> bytes:
    """ggml-quants.c quantize_row_*_ref of a flat f32 array (length % 32 == 0 for q types;
    % 256 for the K types, whose encoder here is a simple valid one, see _quantize_k)."""
    x = np.ascontiguousarray(x, np.float32).ravel()
    if t in (Q4_K, Q5_K, Q6_K):
        return _quantize_k(x, t)
    if t == F32:
        return x.tobytes()
    if t == F16:
        return _f16(x).tobytes()
    b = x.reshape(-1, 32)
    nb = b.shape[0]
    if t in (Q4_0, Q5_0):
        imax = np.argmax(np.abs(b), axis=1)
        mx = b[np.arange(nb), imax]
        d = mx / (-8.0 if t == Q4_0 else -16.0)
        idd = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0).astype(np.float32)
        off = 8.5 if t == Q4_0 else 16.5
        q = np.minimum(15 if t == Q4_0 else 31, (b * idd[:, None] + off).astype(np.int8).astype(np.int32))
        dh, mh = _f16(d), None
    elif t in (Q4_1, Q5_1):
        mn, mx = b.min(axis=1), b.max(axis=1)
        d = (mx - mn) / (15.0 if t == Q4_1 else 31.0)
        idd = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0).astype(np.float32)
        q = ((b - mn[:, None]) * idd[:, None] + 0.5).astype(np.uint8).astype(np.int32)
        q = np.minimum(q, 15 if t == Q4_1 else 31)
        dh, mh = _f16(d), _f16(mn)
    elif t == Q8_0:
        amax = np.abs(b).max(axis=1)
        d = (amax / 127.0).astype(np.float32)
        idd = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0).astype(np.float32)
        v = b * idd[:, None]
        q = (np.sign(v) * np.floor(np.abs(v) + 0.5)).astype(np.int8)  # roundf: half away from zero
        out = np.zeros((nb, 34), np.uint8)
        out[:, 0:2] = _f16(d).view(np.uint8).reshape(nb, 2)
        out[:, 2:] = q.view(np.uint8)
        return out.tobytes()
    else:
        raise ValueError(f"unsupported type {t}")
    _, bytes_ = BLOCK[t]
    out = np.zeros((nb, bytes_), np.uint8)
    out[:, 0:2] = dh.view(np.uint8).reshape(nb, 2)
    o = 2
    if mh is not None:
        out[:, 2:4] = mh.view(np.uint8).reshape(nb, 2)
        o = 4
    if t in (Q5_0, Q5_1):
        hb = ((q >> 4) & 1).astype(np.uint32)
        qh = (hb << np.arange(32, dtype=np.uint32)[None, :]).sum(axis=1).astype(np.uint32)
        out[:, o:o + 4] = qh.view(np.uint8).reshape(nb, 4)
        o += 4
    lo, hi = q[:, :16] & 0xF, q[:, 16:] & 0xF
    out[:, o:o + 16] = (lo | (hi << 4)).astype(np.uint8)
    return out.tobytes()


def dequantize(raw: bytes, t: int, n: int) -> np.ndarray:
    """ggml-quants.c dequantize_row_*: f32 values (f32 products, then + m, no fused multiply-add)."""
    a = np.frombuffer(raw, np.uint8)
    if t == F32:
        return a.view(np.float32)[:n].copy()
    if t == F16:
        return a.view(np.float16)[:n].astype(np.float32)
    if t in (Q4_K, Q5_K, Q6_K):
        return _dequantize_k(a, t, n)
    _, bytes_ = BLOCK[t]
    b = a[: (n // 32) * bytes_].reshape(-1, bytes_)
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
    if t == Q8_0:
        q = b[:, 2:34].view(np.int8).astype(np.float32)
        return (q * d[:, None]).astype(np.float32).ravel()
    o, m = 2, None
    if t in (Q4_1, Q5_1):
        m = b[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
        o = 4
    qh = None
    if t in (Q5_0, Q5_1):
        qh = b[:, o:o + 4].copy().view(np.uint32)[:, 0]
        o += 4
    qs = b[:, o:o + 16].astype(np.int32)
    x = np.concatenate([qs & 0xF, qs >> 4], axis=1)
    if qh is not None:
        bits = ((qh[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1).astype(np.int32)
        x = x | (bits << 4)
    if t == Q4_0:
        x = x - 8
    elif t == Q5_0:
        x = x - 16
    v = x.astype(np.float32) * d[:, None]
    if m is not None:
        v = (v + m[:, None]).astype(np.float32)
    return v.astype(np.float32).ravel()


# ----------------------------------------------------------------------------- whisper tensors
def tensor_table(dims) -> list[tuple[int, str, list[int]]]:
    """(oracle tensor id, whisper.cpp name, ggml ne[] fastest-first) of every model tensor
    (ids: oracle/wo_model.c build_table; names / shapes: whisper_model_load)."""
    d, nm, V = dims.d, dims.n_mels, dims.n_vocab
    t = [(1, "encoder.conv1.weight", [3, nm, d]), (2, "encoder.conv1.bias", [1, d]),
         (3, "encoder.conv2.weight", [3, d, d]), (4, "encoder.conv2.bias", [1, d]),
         (5, "encoder.ln_post.weight", [d]), (6, "encoder.ln_post.bias", [d]),
         (7, "encoder.positional_embedding", [d, dims.n_audio_ctx])]
    for l in range(dims.n_enc):
        b, p = 100 + 32 * l, f"encoder.blocks.{l}."
        t += [(b + 0, p + "attn_ln.weight", [d]), (b + 1, p + "attn_ln.bias", [d]),
              (b + 2, p + "attn.query.weight", [d, d]), (b + 3, p + "attn.query.bias", [d]),
              (b + 4, p + "attn.key.weight", [d, d]), (b + 5, p + "attn.value.weight", [d, d]),
              (b + 6, p + "attn.value.bias", [d]), (b + 7, p + "attn.out.weight", [d, d]),
              (b + 8, p + "attn.out.bias", [d]), (b + 9, p + "mlp_ln.weight", [d]), (b + 10, p + "mlp_ln.bias", [d]),
              (b + 11, p + "mlp.0.weight", [d, 4 * d]), (b + 12, p + "mlp.0.bias", [4 * d]),
              (b + 13, p + "mlp.2.weight", [4 * d, d]), (b + 14, p + "mlp.2.bias", [d])]
    t += [(10, "decoder.token_embedding.weight", [d, V]), (11, "decoder.positional_embedding", [d, dims.n_text_ctx]),
          (12, "decoder.ln.weight", [d]), (13, "decoder.ln.bias", [d])]
    for l in range(dims.n_dec):
        b, p = 5000 + 32 * l, f"decoder.blocks.{l}."
        t += [(b + 0, p + "attn_ln.weight", [d]), (b + 1, p + "attn_ln.bias", [d]),
              (b + 2, p + "attn.query.weight", [d, d]), (b + 3, p + "attn.query.bias", [d]),
              (b + 4, p + "attn.key.weight", [d, d]), (b + 5, p + "attn.value.weight", [d, d]),
              (b + 6, p + "attn.value.bias", [d]), (b + 7, p + "attn.out.weight", [d, d]),
              (b + 8, p + "attn.out.bias", [d]), (b + 9, p + "cross_attn_ln.weight", [d]),
              (b + 10, p + "cross_attn_ln.bias", [d]), (b + 11, p + "cross_attn.query.weight", [d, d]),
              (b + 12, p + "cross_attn.query.bias", [d]), (b + 13, p + "cross_attn.key.weight", [d, d]),
              (b + 14, p + "cross_attn.value.weight", [d, d]), (b + 15, p + "cross_attn.value.bias", [d]),
              (b + 16, p + "cross_attn.out.weight", [d, d]), (b + 17, p + "cross_attn.out.bias", [d]),
              (b + 18, p + "mlp_ln.weight", [d]), (b + 19, p + "mlp_ln.bias", [d]),
              (b + 20, p + "mlp.0.weight", [d, 4 * d]), (b + 21, p + "mlp.0.bias", [4 * d]),
              (b + 22, p + "mlp.2.weight", [4 * d, d]), (b + 23, p + "mlp.2.bias", [d])]
    return t


_F32_ALWAYS = {"encoder.conv1.bias", "encoder.conv2.bias", "encoder.positional_embedding",
               "decoder.positional_embedding"}


def tensor_type(name: str, ne: list[int], wtype: int) -> int:
    """convert-pt-to-ggml.py + whisper_model_quantize: 1-D tensors, conv biases and positional
    embeddings f32; the 3-D conv kernels f16 (never quantised); other 2-D weights wtype."""
    if len(ne) < 2 or name in _F32_ALWAYS:
        return F32
    if len(ne) == 3:
        return F16 if wtype != F32 else F32
    return wtype


def write_model(path: str, dims, filters: np.ndarray, vocab: list[bytes], tensors: dict[int, np.ndarray],
                wtype: int = F16, skip: tuple = (), override: dict | None = None) -> dict[int, np.ndarray]:
    """Write a whisper ggml file; returns the dequantised values of every tensor as the file
    holds them (what an exact loader must reproduce).  skip: names to leave out; override:
    name -> (type, ne) to write a tensor with another type / shape (error-path tests)."""
    override = override or {}
    out = {}
    with open(path, "wb") as f:
        hp = [dims.n_vocab, dims.n_audio_ctx, dims.d, dims.n_head, dims.n_enc, dims.n_text_ctx, dims.d, dims.n_head,
              dims.n_dec, dims.n_mels, FTYPE.get(wtype, 1) + (2000 if wtype not in (F32, F16) else 0)]
        f.write(struct.pack("<I", MAGIC))
        f.write(struct.pack("<11i", *hp))
        filters = np.ascontiguousarray(filters, np.float32)
        f.write(struct.pack("<ii", filters.shape[0], filters.shape[1]))
        f.write(filters.tobytes())
        f.write(struct.pack("<i", len(vocab)))
        for w in vocab:
            f.write(struct.pack("<I", len(w)))
            f.write(w)
        for tid, name, ne in tensor_table(dims):
            if name in skip:
                continue
            ty = tensor_type(name, ne, wtype)
            data = tensors[tid]
            if name in override:
                ty, ne = override[name]
                data = np.resize(data, int(np.prod(ne)))
            raw = quantize(data, ty)
            nb = name.encode()
            f.write(struct.pack("<iii", len(ne), len(nb), ty))
            f.write(struct.pack(f"<{len(ne)}i", *ne))
            f.write(nb)
            f.write(raw)
            out[tid] = dequantize(raw, ty, int(np.prod(ne)))
    return out


def synth_vocab(n: int, seed: int = 7) -> list[bytes]:
    """A deterministic stand-in vocabulary of n byte strings: the 256 single bytes (NUL spelled
    out, since result text is a C string), then words with and without a leading space, digit
    runs, punctuation runs and multi-byte UTF-8 pieces, so greedy longest matching is exercised."""
    rng = np.random.default_rng(seed)
    v = [bytes([i]) if i else b"<NUL>" for i in range(256)]
    letters = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
    utf8 = ["é", "ü", "ß", "ñ", "日本", "語", "ö", "ç", "—", "’"]
    while len(v) < n:
        k = int(rng.integers(0, 6))
        if k <= 2:
            w = bytes(letters[int(i)] for i in rng.integers(0, 52, int(rng.integers(2, 7))))
            v.append((b" " if k == 0 else b"") + w)
        elif k == 3:
            v.append((b" " if rng.integers(0, 2) else b"") + bytes(str(int(rng.integers(0, 1000))), "ascii"))
        elif k == 4:
            v.append(bytes(b".,;:!?'\"-()"[int(i)] for i in rng.integers(0, 11, int(rng.integers(1, 3)))))
        else:
            v.append(((" " if rng.integers(0, 2) else "") + utf8[int(rng.integers(0, len(utf8)))]).encode())
    return v[:n]


# ----------------------------------------------------------------------------- tokenizer
# whisper.cpp tokenize(): std::regex (ECMAScript, "C" locale) of GPT-2's pre-tokenisation
# pattern.  In bytes mode Python's re has the same classes: \s = [ \t\n\v\f\r], bytes >= 0x80
# are neither alpha nor digit; alternatives are tried in order as in ECMAScript.
_PAT = re.compile(rb"'s|'t|'re|'ve|'m|'ll|'d| ?[A-Za-z]+| ?[0-9]+| ?[^\sA-Za-z0-9]+|\s+(?!\S)|\s+")


def special_names(n_vocab: int, n_file: int, sp: dict, lang_codes: list[str]) -> list[bytes]:
    """whisper_model_load's names of the ids past the file's vocabulary."""
    out = []
    for i in range(n_file, n_vocab):
        if i > sp["beg"]:
            w = f"[_TT_{i - sp['beg']}]"
        elif i == sp["eot"]:
            w = "[_EOT_]"
        elif i == sp["sot"]:
            w = "[_SOT_]"
        elif i == sp["translate"]:
            w = "[_TRANSLATE_]"
        elif i == sp["transcribe"]:
            w = "[_TRANSCRIBE_]"
        elif i == sp["solm"]:
            w = "[_SOLM_]"
        elif i == sp["prev"]:
            w = "[_PREV_]"
        elif i == sp["nosp"]:
            w = "[_NOSP_]"
        elif i == sp["not"]:
            w = "[_NOT_]"
        elif i == sp["beg"]:
            w = "[_BEG_]"
        elif sp["sot"] < i <= sp["sot"] + sp["n_langs"]:
            w = f"[_LANG_{lang_codes[i - sp['sot'] - 1]}]"
        else:
            w = f"[_extra_token_{i}]"
        out.append(w.encode())
    return out


def tokenize(vocab: list[bytes], text: bytes) -> list[int]:
    """whisper_tokenize: pieces of the pattern, each covered by the longest vocabulary entries
    from the left; a byte no entry starts is skipped ("unknown token")."""
    to_id = {}
    for i, w in enumerate(vocab):
        to_id[w] = i  # later duplicates win (token_to_id[word] = i in whisper_model_load)
    out = []
    for m in _PAT.finditer(text):
        w = m.group(0)
        i, n = 0, len(w)
        while i < n:
            for j in range(n, i, -1):
                t = to_id.get(w[i:j])
                if t is not None:
                    out.append(t)
                    i = j
                    break
            else:
                i += 1
    return out
