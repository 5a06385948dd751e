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


# ---------------------------------------------------------------------------------------------
# The ONNX readers: the Parakeet model directory the app downloads (onnx_pb.cpp + pk_onnx.cpp) and
# the Silero VAD model it ships (vad_model.cpp), under the same sanitizers (tests/native/onnx_fuzz.cpp).

VAD_ONNX = os.path.join(ROOT, "tests", "golden", "silero_vad_v4.onnx")


@pytest.fixture(scope="module")
def onnx_harness(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("asan_onnx") / "onnx_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
           os.path.join(ROOT, "tests", "native", "onnx_fuzz.cpp"), os.path.join(CSRC, "onnx_pb.cpp"),
           os.path.join(CSRC, "pk_onnx.cpp"), os.path.join(CSRC, "vad_model.cpp"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    return out


def _onnx_run(harness, mode: str, path: str, tag: str) -> str:
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness, mode, path], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, \
        (tag, r.returncode, r.stderr[-2000:])
    assert r.stdout.startswith("parsed") or r.stdout.startswith("rejected"), (tag, r.stdout)
    return r.stdout


@pytest.fixture(scope="module")
def pk_dir(tmp_path_factory):
    """A small valid model directory in the export's layout (int8, tests/onnx_parakeet.py)."""
    onnx_parakeet = pytest.importorskip("tests.onnx_parakeet")
    from oracle import parakeet as P
    d = P.dims_for("test-small", d=64, n_layers=1, n_heads=2, ff=128, sub_ch=16, pred=32, n_vocab=64)
    path = str(tmp_path_factory.mktemp("pkdir"))
    onnx_parakeet.write_dir(path, P.Model(d, seed=3), d, quant="int8")
    return path


def _variant_dir(src: str, dst, name: str, data: bytes) -> str:
    """a copy of the model directory with one file replaced"""
    dst = str(dst)
    if os.path.exists(dst):
        shutil.rmtree(dst)
    shutil.copytree(src, dst)
    with open(os.path.join(dst, name), "wb") as f:
        f.write(data)
    return dst


def test_onnx_valid_files_parse_clean(onnx_harness, pk_dir):
    out = _onnx_run(onnx_harness, "parakeet", pk_dir, "valid")
    assert "d 64, layers 1, 64 pieces" in out and "quantised" in out
    out = _onnx_run(onnx_harness, "vad", VAD_ONNX, "vad")
    assert out.startswith("parsed: blob"), out


def test_onnx_truncations(onnx_harness, pk_dir, tmp_path):
    for name in ("encoder-model.int8.onnx", "decoder_joint-model.int8.onnx"):
        data = open(os.path.join(pk_dir, name), "rb").read()
        cuts = sorted(set(list(range(0, 24)) + list(range(24, len(data), max(1, len(data) // 60))) + [len(data) - 1]))
        for n in cuts:
            out = _onnx_run(onnx_harness, "parakeet", _variant_dir(pk_dir, tmp_path / "v", name, data[:n]), f"{name}:{n}")
            assert out.startswith("rejected"), (name, n, out)
    data = open(VAD_ONNX, "rb").read()
    for n in sorted(set(list(range(0, 16)) + list(range(16, len(data), max(1, len(data) // 80))))):
        p = tmp_path / "vad.onnx"
        p.write_bytes(data[:n])
        assert _onnx_run(onnx_harness, "vad", str(p), f"vad:{n}").startswith("rejected"), n


def test_onnx_oversized_varints_and_lengths(onnx_harness, pk_dir, tmp_path):
    from tests.onnx_parakeet import _int, _key, _ld, _str, _varint
    name = "encoder-model.int8.onnx"
    data = open(os.path.join(pk_dir, name), "rb").read()
    cases = {
        "varint_11_bytes": b"\xff" * 11 + data,
        "graph_len_2^40": _key(7, 2) + _varint(1 << 40) + data,
        "graph_len_past_end": _key(7, 2) + _varint(len(data) + 5) + data,
        "wire_type_group": bytes([(7 << 3) | 3]) + data,
        "deep_subgraphs": _ld(7, _ld(1, _ld(5, _ld(6, _ld(1, _ld(5, _ld(6, b"\xff" * 9))))))) + data,
    }
    # tensors whose fields lie: dims inflated / overflowing / negative, raw_data shorter than the dims,
    # a float attribute carried as a 1-byte varint, an external-data file that does not exist
    def graph_with(init=b"", node=b""):
        return _ld(7, (_ld(1, node) if node else b"") + (_ld(5, init) if init else b""))
    raw = np.arange(3, dtype=np.float32).tobytes()
    cases["raw_short"] = graph_with(_int(1, 1000) + _int(2, 1) + _str(8, "w") + _ld(9, raw))
    cases["dims_product_overflow"] = graph_with(b"".join(_int(1, 1 << 33) for _ in range(4)) + _int(2, 1) + _str(8, "w") + _ld(9, raw))
    cases["dim_negative"] = graph_with(_int(1, (1 << 64) - 3) + _int(2, 1) + _str(8, "w") + _ld(9, raw))
    cases["float_attr_as_varint"] = graph_with(node=_str(4, "Conv") + _ld(5, _str(1, "alpha") + _int(2, 1)))
    cases["packed_float_ragged"] = graph_with(_int(1, 2) + _int(2, 1) + _str(8, "w") + _ld(4, b"\0" * 7))
    cases["dtype_as_string"] = graph_with(_int(1, 2) + _ld(2, b"xx") + _str(8, "w") + _ld(9, raw[:8]))
    ext = _ld(13, _str(1, "location") + _str(2, "missing.data")) + _int(14, 1)
    cases["external_missing"] = graph_with(_int(1, 4) + _int(2, 1) + _str(8, "w") + ext)
    ext_out = _ld(13, _str(1, "location") + _str(2, "../x.data")) + _int(14, 1)
    cases["external_outside_dir"] = graph_with(_int(1, 4) + _int(2, 1) + _str(8, "w") + ext_out)
    for tag, blob in cases.items():
        out = _onnx_run(onnx_harness, "parakeet", _variant_dir(pk_dir, tmp_path / "v", name, blob), tag)
        assert out.startswith("rejected"), (tag, out)
        p = tmp_path / "vad.onnx"
        p.write_bytes(blob)
        _onnx_run(onnx_harness, "vad", str(p), "vad-" + tag)


def test_onnx_external_data_offsets(onnx_harness, pk_dir, tmp_path):
    """external data: a range past the end of its file, and the file removed"""
    onnx_parakeet = pytest.importorskip("tests.onnx_parakeet")
    from oracle import parakeet as P
    d = P.dims_for("test-small", d=64, n_layers=1, n_heads=2, ff=128, sub_ch=16, pred=32, n_vocab=64)
    path = tmp_path / "ext"
    onnx_parakeet.write_dir(str(path), P.Model(d, seed=3), d, quant="int8", external=True)
    assert _onnx_run(onnx_harness, "parakeet", str(path), "ext-valid").startswith("parsed")
    data_file = [f for f in os.listdir(path) if f.endswith(".data")][0]
    blob = (path / data_file).read_bytes()
    (path / data_file).write_bytes(blob[: len(blob) // 2])
    assert _onnx_run(onnx_harness, "parakeet", str(path), "ext-short").startswith("rejected")
    os.remove(path / data_file)
    assert _onnx_run(onnx_harness, "parakeet", str(path), "ext-missing").startswith("rejected")


def test_onnx_random_bit_flips(onnx_harness, pk_dir, tmp_path):
    rng = np.random.default_rng(17)
    for name in ("encoder-model.int8.onnx", "decoder_joint-model.int8.onnx"):
        data = open(os.path.join(pk_dir, name), "rb").read()
        for k in range(60):
            d = bytearray(data)
            for _ in range(int(rng.integers(1, 8))):
                i = int(rng.integers(0, len(d)))
                d[i] ^= 1 << int(rng.integers(0, 8))
            _onnx_run(onnx_harness, "parakeet", _variant_dir(pk_dir, tmp_path / "v", name, bytes(d)), f"{name}:flip{k}")
    data = open(VAD_ONNX, "rb").read()
    for k in range(60):
        d = bytearray(data)
        for _ in range(int(rng.integers(1, 8))):
            i = int(rng.integers(0, len(d)))
            d[i] ^= 1 << int(rng.integers(0, 8))
        p = tmp_path / "vad.onnx"
        p.write_bytes(bytes(d))
        _onnx_run(onnx_harness, "vad", str(p), f"vad:flip{k}")
