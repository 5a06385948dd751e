"""ctypes wrapper for the Parakeet-V3 CPU oracle (oracle/libparakeet_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / the reported CPU baseline.  spittle_amd/ never imports it.

The C source restates the FastConformer-TDT model transcribe-rs' ParakeetEngine runs
(oracle/parakeet_oracle.h lists the NeMo modules; reference call site
/root/reference/src-tauri/src/managers/transcription.rs:278-297, 505-513).
Parity with the real engine is unpinned: no ONNX export or weights exist offline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libparakeet_oracle.so")

W_F32, W_BF16, W_F16 = 0, 1, 2
FIELDS = ("n_mels", "d", "n_layers", "n_heads", "ff", "sub_ch", "conv_k", "pred", "n_vocab", "n_dur")
# parakeet-tdt-0.6b-v3 (NeMo FastConformer-TDT, 24 layers, d 1024) and a small test shape
CONFIGS = {
    "parakeet-tdt-0.6b-v3": (128, 1024, 24, 8, 4096, 256, 9, 640, 8192, 5),
    # the catalog's English-only parakeet-tdt-0.6b-v2 (model_catalog.json:214-217): v3's network with
    # a 1024-piece vocabulary [upstream, recalled]
    "parakeet-tdt-0.6b-v2": (128, 1024, 24, 8, 4096, 256, 9, 640, 1024, 5),
    "test-small": (128, 256, 2, 4, 1024, 128, 9, 128, 1024, 5),  # engine spec "synthetic:parakeet-test-small"
}


class Dims(C.Structure):
    _fields_ = [(n, C.c_int) for n in FIELDS]


def dims_for(name: str, **over) -> Dims:
    v = dict(zip(FIELDS, CONFIGS[name]))
    v.update(over)
    return Dims(*(v[k] for k in FIELDS))


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
        L.po_create.restype = C.c_void_p
        L.po_create.argtypes = [C.POINTER(Dims), C.c_uint64, C.c_int]
        L.po_destroy.argtypes = [C.c_void_p]
        L.po_set_threads.argtypes = [C.c_int]
        L.po_n_frames.argtypes = [C.c_int]
        L.po_n_enc_frames.argtypes = [C.c_int]
        L.po_mel.argtypes = [fp, C.c_int, C.c_int, fp]
        L.po_encode.argtypes = [C.c_void_p, fp, C.c_int, fp]
        L.po_decode.argtypes = [C.c_void_p, fp, C.c_int, C.c_int, ip, ip, fp, fp, C.c_int]
        L.po_decode_gaps.argtypes = [C.c_void_p, fp, C.c_int, C.c_int, ip, ip, fp, fp, fp, C.c_int]
        L.po_set_tensor.argtypes = [C.c_void_p, C.c_int, fp, C.c_int64]
        L.po_tensor.restype = C.c_int64
        L.po_tensor.argtypes = [C.c_void_p, C.c_int, C.POINTER(fp)]
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def set_threads(n: int) -> None:
    lib().po_set_threads(int(n))


def n_frames(n_samples: int) -> int:
    return lib().po_n_frames(int(n_samples))


def n_enc_frames(T: int) -> int:
    return lib().po_n_enc_frames(int(T))


def mel(pcm: np.ndarray, n_mels: int = 128) -> np.ndarray:
    pcm = np.ascontiguousarray(pcm, dtype=np.float32)
    T = n_frames(pcm.size)
    out = np.empty((n_mels, T), np.float32)
    lib().po_mel(_f(pcm), int(pcm.size), n_mels, _f(out))
    return out


class Model:
    def __init__(self, dims: Dims, seed: int = 1234, wdtype: int = W_F32):
        self.dims = dims
        self._p = lib().po_create(C.byref(dims), C.c_uint64(seed), wdtype)
        if not self._p:
            raise RuntimeError("po_create failed")

    def close(self):
        if self._p:
            lib().po_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tensor(self, tid: int) -> np.ndarray:
        ptr = C.POINTER(C.c_float)()
        n = lib().po_tensor(self._p, int(tid), C.byref(ptr))
        if n < 0:
            raise KeyError(tid)
        return np.ctypeslib.as_array(ptr, shape=(n,)).copy()

    def set_tensor(self, tid: int, data: np.ndarray) -> None:
        a = np.ascontiguousarray(data, dtype=np.float32).ravel()
        if lib().po_set_tensor(self._p, int(tid), _f(a), a.size) != 0:
            raise KeyError(tid)

    def encode(self, mel_: np.ndarray) -> np.ndarray:
        mel_ = np.ascontiguousarray(mel_, dtype=np.float32)
        assert mel_.shape[0] == self.dims.n_mels
        T = mel_.shape[1]
        out = np.empty((max(T, 1) * self.dims.d,), np.float32)  # subsampling output fits in T rows
        T3 = lib().po_encode(self._p, _f(mel_), int(T), _f(out))
        return out[:T3 * self.dims.d].reshape(T3, self.dims.d).copy()

    def decode(self, enc: np.ndarray, max_symbols: int = 10, cap: int | None = None):
        enc = np.ascontiguousarray(enc, dtype=np.float32)
        T3 = enc.shape[0]
        cap = cap if cap is not None else T3 * max_symbols + 1
        toks = np.empty(cap, np.int32)
        frames = np.empty(cap, np.int32)
        t1 = np.empty(cap, np.float32)
        t2 = np.empty(cap, np.float32)
        n = lib().po_decode(self._p, _f(enc), int(T3), int(max_symbols), _i(toks), _i(frames), _f(t1), _f(t2), cap)
        n = min(n, cap)
        return toks[:n].copy(), frames[:n].copy(), t1[:n].copy(), t2[:n].copy()

    def decode_gaps(self, enc: np.ndarray, max_symbols: int = 10):
        """decode() plus the decision margins: gmin[i] is the smallest top-1/top-2 margin of any
        token or duration decision leading to emission i; gmin[n] covers the evaluations after
        the last emission."""
        enc = np.ascontiguousarray(enc, dtype=np.float32)
        T3 = enc.shape[0]
        cap = T3 * max_symbols + 2
        toks, frames = np.empty(cap, np.int32), np.empty(cap, np.int32)
        t1, t2, g = np.empty(cap, np.float32), np.empty(cap, np.float32), np.empty(cap, np.float32)
        n = lib().po_decode_gaps(self._p, _f(enc), int(T3), int(max_symbols), _i(toks), _i(frames), _f(t1), _f(t2),
                                 _f(g), cap)
        return toks[:n].copy(), frames[:n].copy(), t1[:n].copy(), t2[:n].copy(), g[:n + 1].copy()


def first_disagreement(tok, frm, otok, ofrm, gmin) -> tuple[int, float]:
    """Index of the first (token, frame) pair where a run departs from the oracle's, and the
    oracle's smallest decision margin up to that point (inf when the runs agree throughout)."""
    n = min(len(tok), len(otok))
    i = next((k for k in range(n) if tok[k] != otok[k] or frm[k] != ofrm[k]), n)
    if i == len(tok) == len(otok):
        return i, float("inf")
    return i, float(np.min(gmin[:i + 1]))
