"""CPU-only checks of the C-ABI boundary: the library loads, exports every symbol
include/spittle_hip.h declares, and its host-only entry points behave (no GPU
compute here)."""
import ctypes as C
import os
import re

import pytest

from spittle_amd import _lib as L

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "spittle_hip.h")


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "spittle_hip.h")).read()
    return sorted(set(re.findall(r"\b(spt_[a-z_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert _header_symbols() == sorted(L.EXPORTS)


def test_rust_sys_crate_mirrors_header():
    """rust/spittle-hip-sys declares every header entry point exactly once (no cargo in this
    image, so the extern block is checked as text: a duplicate item is rustc error E0428)."""
    src = open(os.path.join(ROOT, "rust", "spittle-hip-sys", "src", "lib.rs")).read()
    names = re.findall(r"\bpub fn (spt_[a-z_0-9]+)\s*\(", src)
    dups = sorted({n for n in names if names.count(n) > 1})
    assert not dups, f"declared more than once: {dups}"
    hdr = set(_header_symbols())
    assert set(names) == hdr, (sorted(hdr - set(names)), sorted(set(names) - hdr))


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
    # whisper_full_default_params: timestamps on, temperature fallback 0.2 / best_of 5
    assert ip.flags == L.SPT_SUPPRESS_BLANK
    assert (ip.temperature, ip.best_of, ip.logprob_thold, ip.max_initial_ts) == (0.0, 5, -1.0, 1.0)
    assert abs(ip.temperature_inc - 0.2) < 1e-7 and abs(ip.entropy_thold - 2.4) < 1e-6


def test_struct_layouts_match_header(tmp_path):
    """Every ctypes mirror has the size and field offsets gcc gives the header's structs."""
    import subprocess
    structs = {"spt_model_params": L.ModelParams, "spt_infer_params": L.InferParams, "spt_result": L.Result,
               "spt_segment": L.Segment, "spt_model_info": L.ModelInfo, "spt_timings": L.Timings,
               "spt_pk_model_params": L.PkModelParams, "spt_pk_infer_params": L.PkInferParams,
               "spt_pk_segment": L.PkSegment, "spt_pk_result": L.PkResult, "spt_pk_model_info": L.PkModelInfo,
               "spt_pk_timings": L.PkTimings}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for line in filter(None, got):
        cname, field, val = line.split()
        py = structs[cname]
        want = C.sizeof(py) if field == "size" else getattr(py, field).offset
        assert int(val) == want, (cname, field, val, want)


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
