"""Generate the golden fixtures that pin the CPU oracle (run in the build
container only; the GPU box never imports transformers or this script).

Independent implementation used as the pin: HF transformers 5.15
WhisperFeatureExtractor._np_extract_fbank_features (numpy log-mel) and
WhisperModel (PyTorch CPU) built from a LOCAL WhisperConfig (no download) whose
weights are the oracle's seeded synthetic tensors.  activation_function is
"gelu_new" (tanh form), the GELU whisper.cpp's ggml_gelu uses, so the oracle's
default mode is pinned directly.

The reference itself (whisper.cpp behind transcribe-rs / whisper-rs, see
/root/reference/src-tauri/Cargo.lock:7471-7490,8156-8174) is not vendored and
cannot run here, and the reference's tests never exercise inference
(src-tauri/src/managers/transcription_mock.rs:1-3), so these HF fixtures are
the only available pin.

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from oracle import oracle as O  # noqa: E402

ENC_ROWS = [0, 1, 749, 1499]
MEL_COLS = list(range(0, 40)) + list(range(1480, 1520)) + list(range(2960, 3000))
N_STEPS = 24


def hf_name_map(n_enc: int, n_dec: int) -> dict[int, str]:
    m = {1: "encoder.conv1.weight", 2: "encoder.conv1.bias", 3: "encoder.conv2.weight",
         4: "encoder.conv2.bias", 5: "encoder.layer_norm.weight", 6: "encoder.layer_norm.bias",
         7: "encoder.embed_positions.weight", 10: "decoder.embed_tokens.weight",
         11: "decoder.embed_positions.weight", 12: "decoder.layer_norm.weight",
         13: "decoder.layer_norm.bias"}
    enc = ["self_attn_layer_norm.weight", "self_attn_layer_norm.bias", "self_attn.q_proj.weight",
           "self_attn.q_proj.bias", "self_attn.k_proj.weight", "self_attn.v_proj.weight",
           "self_attn.v_proj.bias", "self_attn.out_proj.weight", "self_attn.out_proj.bias",
           "final_layer_norm.weight", "final_layer_norm.bias", "fc1.weight", "fc1.bias",
           "fc2.weight", "fc2.bias"]
    dec = ["self_attn_layer_norm.weight", "self_attn_layer_norm.bias", "self_attn.q_proj.weight",
           "self_attn.q_proj.bias", "self_attn.k_proj.weight", "self_attn.v_proj.weight",
           "self_attn.v_proj.bias", "self_attn.out_proj.weight", "self_attn.out_proj.bias",
           "encoder_attn_layer_norm.weight", "encoder_attn_layer_norm.bias",
           "encoder_attn.q_proj.weight", "encoder_attn.q_proj.bias", "encoder_attn.k_proj.weight",
           "encoder_attn.v_proj.weight", "encoder_attn.v_proj.bias", "encoder_attn.out_proj.weight",
           "encoder_attn.out_proj.bias", "final_layer_norm.weight", "final_layer_norm.bias",
           "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"]
    for l in range(n_enc):
        for i, n in enumerate(enc):
            m[100 + 32 * l + i] = f"encoder.layers.{l}.{n}"
    for l in range(n_dec):
        for i, n in enumerate(dec):
            m[5000 + 32 * l + i] = f"decoder.layers.{l}.{n}"
    return m


def build_hf(dims, tensors):
    from transformers import WhisperConfig, WhisperModel
    cfg = WhisperConfig(vocab_size=dims.n_vocab, num_mel_bins=dims.n_mels, d_model=dims.d,
                        encoder_layers=dims.n_enc, decoder_layers=dims.n_dec,
                        encoder_attention_heads=dims.n_head, decoder_attention_heads=dims.n_head,
                        encoder_ffn_dim=4 * dims.d, decoder_ffn_dim=4 * dims.d,
                        max_source_positions=dims.n_audio_ctx, max_target_positions=dims.n_text_ctx,
                        activation_function="gelu_new", dropout=0.0, attention_dropout=0.0,
                        activation_dropout=0.0)
    torch.manual_seed(0)
    model = WhisperModel(cfg).eval()
    sd = model.state_dict()
    names = hf_name_map(dims.n_enc, dims.n_dec)
    new = {}
    for tid, arr in tensors.items():
        n = names[tid]
        new[n] = torch.from_numpy(arr.reshape(tuple(sd[n].shape)))
    missing = set(sd) - set(new)
    assert not missing, missing
    model.load_state_dict(new, strict=True)
    return model


def suppress_np(lg: np.ndarray, n_vocab: int, first: bool) -> np.ndarray:
    sp = O.special_tokens(n_vocab)
    lg = lg.copy()
    if first:
        lg[sp["eot"]] = -np.inf
        lg[220] = -np.inf
    lg[sp["not"]] = -np.inf
    lg[sp["beg"]:] = -np.inf
    for k in ("sot", "nosp", "solm", "translate", "transcribe", "prev"):
        lg[sp[k]] = -np.inf
    lg[sp["sot"] + 1: sp["sot"] + 1 + sp["n_langs"]] = -np.inf
    return lg


@torch.no_grad()
def make(name: str, cfg: str, n_enc=None, n_dec=None, seed=1234, audio=0):
    from transformers import WhisperFeatureExtractor
    dims = O.dims_for(cfg, n_enc, n_dec)
    om = O.Model(dims, seed, O.W_F32)
    tensors = om.tensors()
    x = O.synth_audio(audio)

    fe = WhisperFeatureExtractor(feature_size=dims.n_mels)
    mel_hf = fe._np_extract_fbank_features(x[None, :].astype(np.float32), "cpu")[0].astype(np.float32)
    filt_hf = np.asarray(fe.mel_filters, np.float32).T.copy()  # [n_mels][201]

    mel_cpp = O.mel(x, dims.n_mels, O.MEL_WHISPER_CPP)  # encoder input for both sides
    model = build_hf(dims, tensors)
    enc = model.encoder(torch.from_numpy(mel_cpp)[None]).last_hidden_state[0].numpy()

    prompt = O.default_prompt(dims.n_vocab)
    enc_t = torch.from_numpy(enc)[None]
    toks = list(prompt)
    out_tok, top1, top2 = [], [], []
    step0_top_ids = step0_top_vals = None
    for s in range(N_STEPS):
        h = model.decoder(input_ids=torch.tensor([toks]), encoder_hidden_states=enc_t).last_hidden_state
        lg = (h[0, -1] @ model.decoder.embed_tokens.weight.T).numpy().astype(np.float32)
        if s == 0:
            order = np.argsort(-lg)[:16]
            step0_top_ids, step0_top_vals = order.astype(np.int32), lg[order]
        sl = suppress_np(lg, dims.n_vocab, s == 0)
        o = np.argsort(-sl)[:2]
        out_tok.append(int(o[0]))
        top1.append(float(sl[o[0]]))
        top2.append(float(sl[o[1]]))
        toks.append(int(o[0]))

    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(
        path,
        dims=np.array([dims.n_mels, dims.d, dims.n_head, dims.n_enc, dims.n_dec, dims.n_vocab,
                       dims.n_audio_ctx, dims.n_text_ctx], np.int32),
        seed=np.int64(seed), audio=np.int32(audio),
        mel_hf_cols=np.int32(MEL_COLS), mel_hf=mel_hf[:, MEL_COLS],
        mel_hf_sum=np.float64(mel_hf.astype(np.float64).sum()),
        mel_filters_hf=filt_hf,
        enc_rows_idx=np.int32(ENC_ROWS), enc_rows=enc[ENC_ROWS],
        enc_sum=np.float64(enc.astype(np.float64).sum()),
        enc_sumsq=np.float64((enc.astype(np.float64) ** 2).sum()),
        prompt=np.int32(prompt), tokens=np.int32(out_tok), top1=np.float32(top1),
        top2=np.float32(top2), step0_top_ids=step0_top_ids, step0_top_vals=step0_top_vals,
    )
    print(name, "->", path, "tokens", out_tok[:8], "gaps", np.round(np.array(top1) - np.array(top2), 3)[:8])


if __name__ == "__main__":
    torch.set_num_threads(8)
    make("tiny_en_full", "tiny.en")
    make("large_v3_l2", "large-v3", n_enc=2, n_dec=2, audio=1)
