"""The host code that parses untrusted input -- the ggml model-file reader (ggml_file.cpp), the
tokenizer (vocab.cpp) and the host block dequantisers (ggml_quant.h) -- built standalone with
AddressSanitizer + UndefinedBehaviorSanitizer (g++, no device code; tests/native/host_fuzz.cpp)
and fed a valid small model file plus truncated, bit-flipped and size-inflated variants.  Every
variant must be parsed or rejected cleanly: exit 0, no sanitizer report.  (run
ASan on the C++ host code; the app hands the engine whatever .bin file sits in its models dir,
/root/reference/src-tauri/src/managers/model.rs:267-382.)"""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from oracle import ggml as G
from oracle import oracle as O

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
CSRC = os.path.join(ROOT, "spittle_amd", "csrc")
TEXT = "Technical dictation. Common terms: Kubernetes, gRPC, MI355X -- café 日本語 x" * 3


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("asan") / "host_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
           os.path.join(ROOT, "tests", "native", "host_fuzz.cpp"), os.path.join(CSRC, "ggml_file.cpp"),
           os.path.join(CSRC, "vocab.cpp"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return out


def _model_bytes() -> bytes:
    """A small well-formed file: header, filters, a vocabulary, 8 tensors of assorted types."""
    rng = np.random.default_rng(3)
    sp = O.special_tokens(51864)
    vocab = G.synth_vocab(sp["eot"], 7)
    out = [struct.pack("<I", G.MAGIC), struct.pack("<11i", 51864, 1500, 384, 6, 1, 448, 384, 6, 1, 80, 1),
           struct.pack("<ii", 80, 201), O.mel_filters(80).tobytes(), struct.pack("<i", len(vocab))]
    out += [struct.pack("<I", len(w)) + w for w in vocab]
    types = [G.F32, G.F16, G.Q4_0, G.Q4_1, G.Q5_0, G.Q8_0, G.Q4_K, G.Q6_K]
    for i, t in enumerate(types):
        ne = [256, 3] if t not in (G.F32, G.F16) else [64, 2]
        x = rng.standard_normal(ne[0] * ne[1]).astype(np.float32)
        name = f"t{i}".encode()
        out.append(struct.pack("<iii", 2, len(name), t) + struct.pack("<2i", *ne) + name + G.quantize(x, t))
    return b"".join(out)


def _run(harness, tmp_path, data: bytes, tag: str):
    p = tmp_path / f"{tag}.bin"
    p.write_bytes(data)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness, str(p), TEXT], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, \
        (tag, r.returncode, r.stderr[-2000:])
    return r.stdout


def test_valid_file_parses_clean(harness, tmp_path):
    out = _run(harness, tmp_path, _model_bytes(), "valid")
    assert out.startswith("parsed: 8 tensors") and "8 dequantised" in out


def test_truncations(harness, tmp_path):
    data = _model_bytes()
    cuts = sorted(set(list(range(0, 64)) + list(range(64, len(data), max(1, len(data) // 150))) + [len(data) - 1]))
    for n in cuts:
        out = _run(harness, tmp_path, data[:n], f"cut{n}")
        assert out.startswith("rejected") or out.startswith("parsed"), (n, out)


def test_inflated_and_corrupt_headers(harness, tmp_path):
    data = bytearray(_model_bytes())
    first = data.index(struct.pack("<iii", 2, 2, G.F32))  # the first tensor header
    cases = {
        "ne_huge": (first + 12, struct.pack("<2i", 0x7FFFFFFF, 0x7FFFFFFF)),
        "ne_neg": (first + 12, struct.pack("<2i", -5, 3)),
        "ne_zero": (first + 12, struct.pack("<2i", 0, 3)),
        "dims_4_huge": (first, struct.pack("<i", 4)),
        "dims_9": (first, struct.pack("<i", 9)),
        "name_len_huge": (first + 4, struct.pack("<i", 0x7FFFFFF0)),
        "type_bad": (first + 8, struct.pack("<i", 99)),
        "n_vocab_neg": (4 + 48 + 8 + 80 * 201 * 4, struct.pack("<i", -1)),
        "n_vocab_huge": (4 + 48 + 8 + 80 * 201 * 4, struct.pack("<i", 999999)),
        "tok_len_huge": (4 + 48 + 8 + 80 * 201 * 4 + 4, struct.pack("<I", 0xFFFFFFF0)),
        "n_mel_huge": (4 + 48, struct.pack("<ii", 511, 4095)),
    }
    for tag, (off, patch) in cases.items():
        d = bytearray(data)
        d[off:off + len(patch)] = patch
        out = _run(harness, tmp_path, bytes(d), tag)
        assert out.startswith("rejected") or out.startswith("parsed"), (tag, out)
    # the four-dimensional product that used to overflow int64 before any bound was applied
    d = bytearray(data[:first]) + struct.pack("<iii", 4, 2, G.F32) + struct.pack("<4i", *([0x7FFFFFFF] * 4)) + b"t0"
    out = _run(harness, tmp_path, bytes(d) + b"\0" * 64, "overflow4")
    assert out.startswith("rejected") and "truncated tensor data" in out


def test_random_bit_flips(harness, tmp_path):
    data = _model_bytes()
    rng = np.random.default_rng(11)
    for k in range(60):
        d = bytearray(data)
        for _ in range(int(rng.integers(1, 8))):
            i = int(rng.integers(0, len(d)))
            d[i] ^= 1 << int(rng.integers(0, 8))
        _run(harness, tmp_path, bytes(d), f"flip{k}")
