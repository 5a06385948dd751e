"""The native loader of the app's Parakeet model directory (spittle_amd/csrc/onnx_pb.cpp +
pk_onnx.cpp, through the host-only spt_parakeet_onnx_* ABI: no device needed).

The directory is the catalog's parakeet-tdt-0.6b-v3-int8 layout (/root/reference/src-tauri/
resources/model_catalog.json:229-241) that ParakeetEngine::load_model_with_params receives
(/root/reference/src-tauri/src/managers/transcription.rs:278-297), written by tests/onnx_parakeet.py
from the oracle's tensors in the torch.onnx + quantize_dynamic layout [upstream, recalled: parity
with the real export is unpinned].  Every tensor must come back exactly as (q - zero_point) * scale
in f32, in NeMo's layout, with the dimensions inferred from the tensors alone."""
import os

import numpy as np
import pytest

from oracle import parakeet as P

onnx_parakeet = pytest.importorskip("tests.onnx_parakeet")

VARIANTS = {
    "int8": dict(quant="int8"),
    "uint8_per_channel_folded_bn_anon_bias": dict(quant="uint8pc", fold_bn=True, anon_pos_bias=True),
    "qdq_external_data": dict(quant="int8", qdq=True, external=True, lstm_quant=False),
    "float": dict(quant=""),
}


@pytest.fixture(scope="module")
def small():
    d = P.dims_for("test-small")
    return d, P.Model(d, seed=21)


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_loader_recovers_every_tensor(tmp_path, small, variant):
    from spittle_amd.parakeet import OnnxModelDir, is_onnx_dir
    d, m = small
    exp = onnx_parakeet.write_dir(str(tmp_path), m, d, **VARIANTS[variant])
    assert is_onnx_dir(str(tmp_path))
    h = OnnxModelDir(str(tmp_path))
    dims = h.dims()
    for k in ("n_mels", "d", "n_layers", "n_heads", "ff", "sub_ch", "conv_k", "pred", "n_vocab", "n_dur"):
        assert dims[k] == getattr(d, k), k
    n_q = h.n_quantized
    assert (n_q > 0) == bool(VARIANTS[variant]["quant"])
    for tid, want in exp.items():
        got = h.tensor(tid)
        assert got is not None, tid
        assert got.size == m.tensor(tid).size, tid
        assert np.array_equal(got, want), (variant, tid, np.abs(got - want).max())
    # the quantised matrices really are the dequantised values, not the originals
    if VARIANTS[variant]["quant"]:
        assert not np.array_equal(h.tensor(1002), m.tensor(1002))
        assert np.abs(h.tensor(1002) - m.tensor(1002)).max() < 0.05 * np.abs(m.tensor(1002)).max()
    assert h.piece(0) == onnx_parakeet.vocab_piece(0) and h.piece(d.n_vocab - 1) == onnx_parakeet.vocab_piece(d.n_vocab - 1)
    assert h.piece(d.n_vocab) is None
    h.close()


def test_loader_errors(tmp_path, small):
    from spittle_amd import TranscriptionError
    from spittle_amd.parakeet import OnnxModelDir
    d, m = small
    with pytest.raises(TranscriptionError, match="not a Parakeet model directory"):
        OnnxModelDir(str(tmp_path))
    onnx_parakeet.write_dir(str(tmp_path), m, d, quant="int8")
    enc = tmp_path / "encoder-model.int8.onnx"
    blob = enc.read_bytes()
    for cut in (len(blob) // 3, len(blob) - 7):  # truncated protobuf
        enc.write_bytes(blob[:cut])
        with pytest.raises(TranscriptionError):
            OnnxModelDir(str(tmp_path))
    enc.write_bytes(blob)
    os.remove(tmp_path / "decoder_joint-model.int8.onnx")
    with pytest.raises(TranscriptionError, match="decoder_joint"):
        OnnxModelDir(str(tmp_path))
    onnx_parakeet.write_dir(str(tmp_path), m, d, quant="int8")
    (tmp_path / "vocab.txt").write_text("a 0\n")
    with pytest.raises(TranscriptionError, match="token ids present"):
        OnnxModelDir(str(tmp_path))


@pytest.mark.parametrize("fault,msg", [("transposed_ff1", "shape"), ("third_pos_bias", "third unnamed"),
                                       ("conflicting_q", "second, different value")])
def test_loader_rejects_ambiguous_graphs(tmp_path, small, fault, msg):
    """A graph that maps a weight in the wrong orientation, has an unexpected unnamed pos-bias
    operand, or gives one role two different values fails to load with the tensor named, instead of
    loading a silently wrong model."""
    from spittle_amd import TranscriptionError
    from spittle_amd.parakeet import OnnxModelDir
    d, m = small
    onnx_parakeet.write_dir(str(tmp_path), m, d, quant="int8", anon_pos_bias=True, faults=(fault,))
    with pytest.raises(TranscriptionError, match=msg):
        OnnxModelDir(str(tmp_path))


def test_loader_full_shape_dims(tmp_path):
    """parakeet-tdt-0.6b-v3's own shape (24 layers, d 1024, 8 heads, 8192 tokens + 5 durations),
    written int8 as the catalog model is: dimensions and a sample of tensors."""
    from spittle_amd.parakeet import OnnxModelDir
    d = P.dims_for("parakeet-tdt-0.6b-v3")
    m = P.Model(d, seed=5)
    exp = onnx_parakeet.write_dir(str(tmp_path), m, d, quant="int8")
    h = OnnxModelDir(str(tmp_path))
    assert h.dims() == {k: getattr(d, k) for k in h.dims()}
    for tid in (1, 11, 1002, 1017, 1023, 1000 + 64 * 23 + 35, 90001, 90006, 90013):
        assert np.array_equal(h.tensor(tid), exp[tid]), tid
    h.close()


def test_nemo_rejects_durations_other_than_range(tmp_path):
    """load_nemo refuses a TDT checkpoint whose duration table is not 0..n-1 before it touches a
    device: the decoder advances by the duration head's argmax index (k_pk.hip joint_fin)."""
    import io
    import tarfile

    import yaml
    from spittle_amd import ParakeetEngine, ParakeetModelParams, TranscriptionError
    from spittle_amd.parakeet import load_nemo
    cfg = {"encoder": {"d_model": 64, "n_layers": 1, "n_heads": 2}, "decoder": {"prednet": {"pred_hidden": 32}},
           "joint": {"num_classes": 30}, "model_defaults": {"tdt_durations": [0, 1, 2, 4, 8]}}
    path = str(tmp_path / "m.nemo")
    with tarfile.open(path, "w") as tf:
        for name, data in (("model_config.yaml", yaml.safe_dump(cfg).encode()), ("model_weights.ckpt", b"")):
            ti = tarfile.TarInfo("./" + name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))
    with pytest.raises(TranscriptionError, match="tdt_durations"):
        load_nemo(ParakeetEngine(), path, ParakeetModelParams())
