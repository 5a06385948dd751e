"""The C boundary as a C program sees it (tests/native/capi_smoke.c): the header compiles as
C11 with -Wall -Werror, the program links against libspittle_hip.so, and -- on a GPU -- it runs
the exact sequence the Rust binding performs (rust/spittle-hip: create -> transcribe -> read
-> free -> destroy, twice, plus the error paths)."""
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


def test_c_program_compiles_and_links(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe, "synthetic:tiny", "--link-only"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "ABI 7" in r.stdout


@pytest.mark.gpu
def test_c_program_runs_the_binding_sequence(tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe, "synthetic:tiny"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi_smoke ok" in r.stdout
