"""The C boundary as a C program sees it (tests/native/capi_smoke.c): the header compiles as
C11 with -Wall -Werror, the program links against libspittle_hip.so, and -- on a GPU -- it runs
the exact sequence the Rust binding performs (rust/spittle-hip: create -> transcribe -> read
-> free -> destroy, twice, plus the error paths; the resampler, the Parakeet model directory and
the voice-activity gate sessions)."""
import os
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIBDIR = os.path.join(ROOT, "spittle_amd")


def _build(tmp_path):
    exe = str(tmp_path / "capi_smoke")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-O1",
                    os.path.join(ROOT, "tests", "native", "capi_smoke.c"), "-I", os.path.join(ROOT, "include"),
                    "-L", LIBDIR, "-lspittle_hip", f"-Wl,-rpath,{LIBDIR}", "-lm", "-o", exe],
                   check=True, capture_output=True, timeout=120)
    return exe


def _model_dir(tmp_path):
    """the catalog's parakeet-tdt-0.6b-v3-int8 layout (tests/onnx_parakeet.py), test-small dims"""
    from oracle import parakeet as P
    from tests import onnx_parakeet
    d = P.dims_for("test-small")
    path = str(tmp_path / "parakeet-tdt-0.6b-v3-int8")
    onnx_parakeet.write_dir(path, P.Model(d, seed=3), d, quant="int8")
    return path


def test_c_program_compiles_and_links(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe, "synthetic:tiny", "--link-only", _model_dir(tmp_path)], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    assert "ABI 12" in r.stdout
    assert "parakeet dir: d 256, layers 2, heads 4, vocab 1024" in r.stdout


@pytest.mark.gpu
def test_c_program_runs_the_binding_sequence(tmp_path):
    exe = _build(tmp_path)
    vad_model = os.path.join(ROOT, "tests", "golden", "silero_vad_v4.onnx")
    r = subprocess.run([exe, "synthetic:tiny", "--run", _model_dir(tmp_path), vad_model], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "parakeet: " in r.stdout and "vad: " in r.stdout and "capi_smoke ok" in r.stdout
