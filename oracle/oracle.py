"""ctypes wrapper for the CPU oracle (oracle/libwhisper_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / the reported CPU baseline.
spittle_amd/ never imports this module.

The C sources restate whisper.cpp's log-mel / encoder / decoder / greedy path
(see oracle/whisper_oracle.h for the upstream functions and the reference
call site /root/reference/src-tauri/src/managers/transcription.rs:494-503).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libwhisper_oracle.so")

MEL_WHISPER_CPP, MEL_HF = 0, 1
GELU_TANH, GELU_ERF = 0, 1
W_F32, W_BF16 = 0, 1
SUPPRESS_BLANK, NO_TIMESTAMPS, IGNORE_EOT = 1, 2, 4

# dims: (n_mels, d, n_head, n_enc, n_dec, n_vocab, n_audio_ctx, n_text_ctx)
CONFIGS = {
    "tiny.en": (80, 384, 6, 4, 4, 51864, 1500, 448),
    "tiny": (80, 384, 6, 4, 4, 51865, 1500, 448),
    "small": (80, 768, 12, 12, 12, 51865, 1500, 448),
    "large-v3": (128, 1280, 20, 32, 32, 51866, 1500, 448),
}


class Dims(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ("n_mels", "d", "n_head", "n_enc", "n_dec", "n_vocab", "n_audio_ctx", "n_text_ctx")]


def dims_for(name: str, n_enc: int | None = None, n_dec: int | None = None) -> Dims:
    v = list(CONFIGS[name])
    if n_enc is not None:
        v[3] = n_enc
    if n_dec is not None:
        v[4] = n_dec
    return Dims(*v)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        fp = C.POINTER(C.c_float)
        ip = C.POINTER(C.c_int32)
        L.wo_model_new.restype = C.c_void_p
        L.wo_model_new.argtypes = [C.POINTER(Dims), C.c_uint64, C.c_int]
        L.wo_model_free.argtypes = [C.c_void_p]
        L.wo_tensor_count.argtypes = [C.c_void_p]
        L.wo_tensor_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int64),
                                     C.POINTER(fp)]
        L.wo_set_threads.argtypes = [C.c_int]
        L.wo_mel_filters.argtypes = [C.c_int, fp]
        L.wo_tables.argtypes = [fp, fp, fp]
        L.wo_mel.argtypes = [C.c_int, fp, C.c_int, C.c_int, fp]
        L.wo_mel_len.argtypes = [C.c_int]
        L.wo_mel_full.argtypes = [C.c_int, fp, C.c_int, fp]
        L.wo_encode.argtypes = [C.c_void_p, fp, C.c_int, fp]
        L.wo_decode.argtypes = [C.c_void_p, fp, ip, C.c_int, C.c_int, C.c_uint32, C.c_int, ip, ip, fp, fp]
        L.wo_decode_logits.argtypes = [C.c_void_p, fp, ip, C.c_int, C.c_int, fp]
        L.wo_special_tokens.argtypes = [C.c_int, ip]
        L.wo_lang_detect.argtypes = [C.c_void_p, fp, C.c_int, fp]
        L.wo_tensor_set.argtypes = [C.c_void_p, C.c_int, fp, C.c_int64]
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def set_threads(n: int) -> None:
    lib().wo_set_threads(int(n))


def mel(pcm: np.ndarray, n_mels: int, mode: int = MEL_WHISPER_CPP) -> np.ndarray:
    pcm = np.ascontiguousarray(pcm, dtype=np.float32)
    out = np.empty((n_mels, 3000), np.float32)
    rc = lib().wo_mel(n_mels, _f(pcm), int(pcm.size), mode, _f(out))
    if rc != 0:
        raise ValueError(f"wo_mel failed rc={rc}")
    return out


def mel_full(pcm: np.ndarray, n_mels: int) -> np.ndarray:
    """whisper.cpp's log-mel of a whole input of any length: [n_mels][(n + 480000) // 160], clamped
    at the input's global max - 8 (whisper_pcm_to_mel, once per whisper_full call)."""
    pcm = np.ascontiguousarray(pcm, dtype=np.float32)
    n_len = lib().wo_mel_len(int(pcm.size))
    out = np.empty((n_mels, n_len), np.float32)
    rc = lib().wo_mel_full(n_mels, _f(pcm), int(pcm.size), _f(out))
    if rc != 0:
        raise ValueError(f"wo_mel_full failed rc={rc}")
    return out


def mel_window(full: np.ndarray, seek: int) -> np.ndarray:
    """whisper_encode_internal's input: frames [seek, seek + 3000) of a whole-input log-mel, zero
    past its end."""
    out = np.zeros((full.shape[0], 3000), np.float32)
    i1 = min(full.shape[1], seek + 3000)
    if i1 > seek:
        out[:, :i1 - seek] = full[:, seek:i1]
    return out


def mel_filters(n_mels: int) -> np.ndarray:
    out = np.empty((n_mels, 201), np.float32)
    lib().wo_mel_filters(n_mels, _f(out))
    return out


def tables():
    h, s, c = (np.empty(400, np.float32) for _ in range(3))
    lib().wo_tables(_f(h), _f(s), _f(c))
    return h, s, c


def special_tokens(n_vocab: int) -> dict:
    o = np.empty(10, np.int32)
    lib().wo_special_tokens(n_vocab, _i(o))
    keys = ("eot", "sot", "translate", "transcribe", "solm", "prev", "nosp", "not", "beg", "n_langs")
    return dict(zip(keys, (int(x) for x in o)))


def default_prompt(n_vocab: int, lang_id: int = 0, translate: bool = False, past=None) -> list[int]:
    """[sot, lang, task, notimestamps] for multilingual, [sot, notimestamps] for .en
    (whisper_full's prompt_init with no_timestamps); with `past` (prompt tokens) whisper_full
    prepends [prev] + the last min(n_text_ctx / 2 = 224, len) of them."""
    sp = special_tokens(n_vocab)
    p = []
    if past is not None and len(past) > 0:
        p = [sp["prev"]] + [int(t) for t in list(past)[-224:]]
    p.append(sp["sot"])
    if sp["n_langs"] > 0:
        p += [sp["sot"] + 1 + lang_id, sp["translate"] if translate else sp["transcribe"]]
    p.append(sp["not"])
    return p


class Model:
    def __init__(self, dims: Dims, seed: int = 1234, wdtype: int = W_F32):
        self.dims = dims
        self._p = lib().wo_model_new(C.byref(dims), C.c_uint64(seed), wdtype)
        if not self._p:
            raise RuntimeError("wo_model_new failed")

    def close(self):
        if self._p:
            lib().wo_model_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tensors(self) -> dict[int, np.ndarray]:
        out = {}
        L = lib()
        for i in range(L.wo_tensor_count(self._p)):
            tid, n, ptr = C.c_int(), C.c_int64(), C.POINTER(C.c_float)()
            L.wo_tensor_info(self._p, i, C.byref(tid), C.byref(n), C.byref(ptr))
            out[tid.value] = np.ctypeslib.as_array(ptr, shape=(n.value,)).copy()
        return out

    def set_tensor(self, tid: int, data: np.ndarray) -> None:
        a = np.ascontiguousarray(data, dtype=np.float32).ravel()
        rc = lib().wo_tensor_set(self._p, int(tid), _f(a), C.c_int64(a.size))
        if rc != 0:
            raise ValueError(f"wo_tensor_set({tid}) failed rc={rc}")

    def encode(self, mel_: np.ndarray, gelu: int = GELU_TANH) -> np.ndarray:
        mel_ = np.ascontiguousarray(mel_, dtype=np.float32)
        assert mel_.shape == (self.dims.n_mels, 3000)
        out = np.empty((self.dims.n_audio_ctx, self.dims.d), np.float32)
        lib().wo_encode(self._p, _f(mel_), gelu, _f(out))
        return out

    def decode(self, enc: np.ndarray, prompt, n_steps: int, flags: int = SUPPRESS_BLANK | NO_TIMESTAMPS,
               gelu: int = GELU_TANH, forced=None):
        enc = np.ascontiguousarray(enc, dtype=np.float32)
        pr = np.asarray(prompt, np.int32)
        toks = np.empty(n_steps, np.int32)
        t1 = np.empty(n_steps, np.float32)
        t2 = np.empty(n_steps, np.float32)
        fz = None if forced is None else np.ascontiguousarray(forced, dtype=np.int32)
        rc = lib().wo_decode(self._p, _f(enc), _i(pr), int(pr.size), int(n_steps), flags, gelu,
                             _i(fz) if fz is not None else None, _i(toks), _f(t1), _f(t2))
        if rc < 0:
            raise ValueError("wo_decode failed")
        return toks, t1, t2

    def detect_language(self, enc: np.ndarray, gelu: int = GELU_TANH):
        """whisper_lang_auto_detect: (language index, softmax probabilities over languages);
        (-1, None) for an English-only vocabulary."""
        enc = np.ascontiguousarray(enc, dtype=np.float32)
        n = special_tokens(self.dims.n_vocab)["n_langs"]
        probs = np.zeros(max(n, 1), np.float32)
        lid = lib().wo_lang_detect(self._p, _f(enc), gelu, _f(probs))
        return lid, (probs[:n] if n > 0 else None)

    def logits(self, enc: np.ndarray, toks, gelu: int = GELU_TANH) -> np.ndarray:
        enc = np.ascontiguousarray(enc, dtype=np.float32)
        t = np.asarray(toks, np.int32)
        out = np.empty(self.dims.n_vocab, np.float32)
        lib().wo_decode_logits(self._p, _f(enc), _i(t), int(t.size), gelu, _f(out))
        return out


def synth_audio(i: int, n_samples: int = 480000) -> np.ndarray:
    """BASELINE.md §3 input: clip(0.1 N(0,1) + sum_k 0.3 sin(2 pi f_k t + phi_k), -1, 1),
    f_k ~ U(100, 4000) Hz, phi_k ~ U(0, 2 pi), numpy PCG64(seed = 1000 + i)."""
    rng = np.random.Generator(np.random.PCG64(1000 + i))
    f = rng.uniform(100.0, 4000.0, 3)
    ph = rng.uniform(0.0, 2 * np.pi, 3)
    noise = rng.standard_normal(n_samples)
    t = np.arange(n_samples) / 16000.0
    x = 0.1 * noise
    for k in range(3):
        x = x + 0.3 * np.sin(2 * np.pi * f[k] * t + ph[k])
    return np.clip(x, -1.0, 1.0).astype(np.float32)
