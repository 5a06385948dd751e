"""CPU-only checks of the C-ABI boundary: the library loads, exports every symbol
include/spittle_hip.h declares, and its host-only entry points behave (no GPU
compute here)."""
import ctypes as C
import os
import re

import pytest

from spittle_amd import _lib as L

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "spittle_hip.h")).read()
    return sorted(set(re.findall(r"\b(spt_[a-z_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert _header_symbols() == sorted(L.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = L.load()
    for name in _header_symbols():
        assert hasattr(lib, name), name


def test_version_and_defaults():
    lib = L.load()
    assert b"gfx950" in lib.spt_version()
    mp = L.ModelParams()
    lib.spt_default_model_params(C.byref(mp))
    assert (mp.dtype, mp.device, mp.max_batch, mp.seed) == (L.SPT_DTYPE_BF16, 0, 8, 1234)
    ip = L.InferParams()
    lib.spt_default_infer_params(C.byref(ip))
    assert ip.language == b"en" and ip.beam_size == 1 and ip.max_new_tokens == 220
    assert ip.flags == L.SPT_SUPPRESS_BLANK | L.SPT_NO_TIMESTAMPS


def test_struct_layouts_match_header():
    # sizes of the ABI structs as the C compiler lays them out (x86-64 SysV)
    assert C.sizeof(L.ModelParams) == 24
    assert C.sizeof(L.InferParams) == 72
    assert C.sizeof(L.Result) == 48
    assert C.sizeof(L.ModelInfo) == 56
    assert C.sizeof(L.Timings) == 56


def test_language_codes():
    lib = L.load()
    assert lib.spt_language_code(0) == b"en" and lib.spt_language_code(1) == b"zh"
    assert lib.spt_language_code(99) == b"yue"
    assert lib.spt_language_code(100) is None and lib.spt_language_code(-1) is None


def test_create_errors_are_reported_not_raised():
    lib = L.load()
    ctx = C.c_void_p()
    err = C.create_string_buffer(256)
    st = lib.spt_ctx_create(b"/nonexistent/ggml-large-v3.bin", None, C.byref(ctx), err, 256)
    assert st == L.SPT_ERR_LOAD and b"not found" in err.value and not ctx.value
    st = lib.spt_ctx_create(b"synthetic:no-such-model", None, C.byref(ctx), err, 256)
    assert st == L.SPT_ERR_LOAD and b"unknown synthetic model" in err.value
    st = lib.spt_ctx_create(None, None, C.byref(ctx), err, 256)
    assert st == L.SPT_ERR_INVALID_ARG


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is not None, reason="device-visible env")
def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = L.load()
    ctx = C.c_void_p()
    err = C.create_string_buffer(256)
    st = lib.spt_ctx_create(b"synthetic:tiny.en", None, C.byref(ctx), err, 256)
    assert st == L.SPT_ERR_DEVICE and not ctx.value


def test_engine_mirror_surface():
    from spittle_amd import WhisperEngine, WhisperInferenceParams
    e = WhisperEngine()
    assert not e.is_loaded()
    with pytest.raises(Exception, match="not loaded"):
        e.transcribe_samples([0.0] * 10, WhisperInferenceParams(language="en"))
    p = WhisperInferenceParams()
    assert p.language is None and p.translate is False and p.initial_prompt is None
