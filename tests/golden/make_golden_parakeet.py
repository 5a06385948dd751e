"""Generate the golden fixtures that pin the Parakeet-V3 CPU oracle (oracle/po_model.c) to an
independent implementation (run in the build container only; the GPU box never imports
transformers or this script).

TEST INFRASTRUCTURE.  The pin is HF transformers 5.15's Parakeet port, built from a LOCAL config
(no download) whose weights are the oracle's seeded synthetic tensors:

* features  ``ParakeetFeatureExtractor.__call__`` (transformers/models/parakeet/
            feature_extraction_parakeet.py:129-284): pre-emphasis with a time mask, torch.stft
            (centre, constant padding, symmetric Hann 400 in 512), log(x + 2^-24), per-feature
            normalisation over ``n // 160`` valid frames (unbiased, std + 1e-5), the rest zeroed.
            Its constructor needs librosa (absent here), so the object is built without it and
            given the slaney filterbank from ``transformers.audio_utils.mel_filter_bank`` --
            librosa.filters.mel(norm="slaney") restated by HF in f64, rounded to f32 as librosa
            returns it.
* encoder   ``ParakeetEncoder`` (modeling_parakeet.py:549-641): dw_striding subsampling with
            per-stage length masks, x sqrt(d), interleaved sin/cos relative positions,
            ``ParakeetEncoderBlock`` x L (rel-pos attention with bias_u / bias_v and
            ``_rel_shift``, conv module with BatchNorm in eval mode).
* decoding  ``ParakeetForTDT.generate`` (generation_parakeet.py:271-299): greedy, token argmax
            over vocab + blank, duration argmax, a blank with duration 0 advances one frame.
            HF applies no max-symbols-per-frame guard to TDT; the oracle is called with a bound
            no utterance reaches, so the two searches are the same rule.

Convention switches between HF's port and the r1/r2 restatement (both recorded in DESIGN.md §9.2):
* valid frames: HF (= NeMo ``FilterbankFeatures.get_seq_len``) counts ``n // 160`` frames and
  zeroes the last STFT frame; r2's oracle used ``n // 160 + 1``.  Oracle and GPU now follow HF.
* the start-of-decoding token is the blank (decoder_start_token_id = blank), whose embedding row
  is zero in both (NeMo ``blank_as_pad``).

Reference call being pinned: /root/reference/src-tauri/src/managers/transcription.rs:505-513
(``ParakeetEngine::transcribe_samples``).  Parity against the ONNX int8 engine itself stays
unpinned (no export or weights offline).

Usage:  python tests/golden/make_golden_parakeet.py   (writes tests/golden/parakeet_*.npz)
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from oracle import parakeet as P  # noqa: E402
from oracle.oracle import synth_audio  # noqa: E402

# (fixture name, oracle config, layer override, weight seed, [(audio seed, n samples)])
CASES = [
    ("parakeet_small", "test-small", None, 11, [(3, 16000 * 3), (4, 16000 * 2 + 77), (5, 16000)]),
    ("parakeet_v3_full", "parakeet-tdt-0.6b-v3", None, 1234, [(7, 16000 * 2), (8, 16000 + 4321)]),
]


def hf_name_map(dims) -> dict[int, str]:
    m = {1: "encoder.subsampling.layers.0.weight", 2: "encoder.subsampling.layers.0.bias",
         3: "encoder.subsampling.layers.2.weight", 4: "encoder.subsampling.layers.2.bias",
         5: "encoder.subsampling.layers.3.weight", 6: "encoder.subsampling.layers.3.bias",
         7: "encoder.subsampling.layers.5.weight", 8: "encoder.subsampling.layers.5.bias",
         9: "encoder.subsampling.layers.6.weight", 10: "encoder.subsampling.layers.6.bias",
         11: "encoder.subsampling.linear.weight", 12: "encoder.subsampling.linear.bias",
         90000: "decoder.embedding.weight",
         90009: "encoder_projector.weight", 90010: "encoder_projector.bias",
         90011: "decoder.decoder_projector.weight", 90012: "decoder.decoder_projector.bias",
         90013: "joint.head.weight", 90014: "joint.head.bias"}
    for j in range(2):
        for k, n in enumerate(("weight_ih", "weight_hh", "bias_ih", "bias_hh")):
            m[90001 + 4 * j + k] = f"decoder.lstm.{n}_l{j}"
    per = {0: "norm_feed_forward1.weight", 1: "norm_feed_forward1.bias",
           2: "feed_forward1.linear1.weight", 3: "feed_forward1.linear1.bias",
           4: "feed_forward1.linear2.weight", 5: "feed_forward1.linear2.bias",
           6: "norm_self_att.weight", 7: "norm_self_att.bias",
           8: "self_attn.q_proj.weight", 9: "self_attn.q_proj.bias",
           10: "self_attn.k_proj.weight", 11: "self_attn.k_proj.bias",
           12: "self_attn.v_proj.weight", 13: "self_attn.v_proj.bias",
           14: "self_attn.o_proj.weight", 15: "self_attn.o_proj.bias",
           16: "self_attn.relative_k_proj.weight", 17: "self_attn.bias_u", 18: "self_attn.bias_v",
           19: "norm_conv.weight", 20: "norm_conv.bias",
           21: "conv.pointwise_conv1.weight", 22: "conv.pointwise_conv1.bias",
           23: "conv.depthwise_conv.weight", 24: "conv.depthwise_conv.bias",
           25: "conv.norm.weight", 26: "conv.norm.bias", 27: "conv.norm.running_mean", 28: "conv.norm.running_var",
           29: "conv.pointwise_conv2.weight", 30: "conv.pointwise_conv2.bias",
           31: "norm_feed_forward2.weight", 32: "norm_feed_forward2.bias",
           33: "feed_forward2.linear1.weight", 34: "feed_forward2.linear1.bias",
           35: "feed_forward2.linear2.weight", 36: "feed_forward2.linear2.bias",
           37: "norm_out.weight", 38: "norm_out.bias"}
    for l in range(dims.n_layers):
        for i, n in per.items():
            m[1000 + 64 * l + i] = f"encoder.layers.{l}.{n}"
    return m


def build_hf(model: P.Model, dims):
    from transformers import ParakeetForTDT, ParakeetTDTConfig

    enc = dict(hidden_size=dims.d, num_hidden_layers=dims.n_layers, num_attention_heads=dims.n_heads,
               intermediate_size=dims.ff, conv_kernel_size=dims.conv_k, subsampling_conv_channels=dims.sub_ch,
               num_mel_bins=dims.n_mels, dropout=0.0, layerdrop=0.0, activation_dropout=0.0,
               attention_dropout=0.0)
    cfg = ParakeetTDTConfig(vocab_size=dims.n_vocab + 1, blank_token_id=dims.n_vocab, pad_token_id=dims.n_vocab,
                            decoder_hidden_size=dims.pred, num_decoder_layers=2,
                            durations=list(range(dims.n_dur)), encoder_config=enc, max_symbols_per_step=10)
    cfg._attn_implementation = "eager"
    hf = ParakeetForTDT(cfg).eval()
    sd = hf.state_dict()
    names = hf_name_map(dims)
    with torch.no_grad():
        for tid, name in names.items():
            t = torch.from_numpy(model.tensor(tid)).reshape(sd[name].shape)
            sd[name].copy_(t)
    missing = [k for k in sd if k not in names.values() and not k.endswith("num_batches_tracked")]
    assert not missing, missing
    return hf


def feature_extractor(n_mels: int):
    from transformers.audio_utils import mel_filter_bank
    from transformers.models.parakeet.feature_extraction_parakeet import ParakeetFeatureExtractor
    from transformers.feature_extraction_sequence_utils import SequenceFeatureExtractor

    fe = ParakeetFeatureExtractor.__new__(ParakeetFeatureExtractor)
    SequenceFeatureExtractor.__init__(fe, feature_size=n_mels, sampling_rate=16000, padding_value=0.0)
    fe.hop_length, fe.n_fft, fe.win_length, fe.preemphasis = 160, 512, 400, 0.97
    fb = mel_filter_bank(num_frequency_bins=257, num_mel_filters=n_mels, min_frequency=0.0, max_frequency=8000.0,
                         sampling_rate=16000, norm="slaney", mel_scale="slaney")
    fe.mel_filters = torch.from_numpy(fb.T.astype(np.float32))   # librosa layout [n_mels][257], f32
    return fe


def run_case(name, cfg, layers, seed, clips):
    over = {} if layers is None else {"n_layers": layers}
    dims = P.dims_for(cfg, **over)
    model = P.Model(dims, seed=seed)
    hf = build_hf(model, dims)
    fe = feature_extractor(dims.n_mels)
    out = {"seed": np.int64(seed), "config": np.array(cfg), "n_layers": np.int64(dims.n_layers),
           "audio_seeds": np.array([s for s, _ in clips], np.int64),
           "audio_lens": np.array([n for _, n in clips], np.int64)}
    for i, (s, n) in enumerate(clips):
        # one utterance per call, trimmed to its valid frames: HF's eager attention turns a fully
        # masked (padding) query row into NaN, which the next layer's keys spread to every row
        feats = fe([synth_audio(s, n)], sampling_rate=16000, return_tensors="pt", return_attention_mask=True)
        T = int(feats.attention_mask[0].sum())
        x, am = feats.input_features[:, :T], feats.attention_mask[:, :T]
        with torch.no_grad():
            enc = hf.get_audio_features(input_features=x, attention_mask=am)
            gen = hf.generate(input_features=x, attention_mask=am, decoder_start_token_id=dims.n_vocab)
        seq, dur = gen.sequences[0].numpy(), gen.durations[0].numpy()
        T3 = int(enc.attention_mask[0].sum())
        assert T3 == enc.last_hidden_state.shape[1]
        out[f"mel_{i}"] = x[0].numpy().T.astype(np.float32).copy()            # [n_mels][T]
        out[f"enc_{i}"] = enc.last_hidden_state[0].numpy().astype(np.float32).copy()
        toks, frames, f = [], [], 0
        for k in range(1, seq.shape[0]):
            if f >= T3:
                break
            if int(seq[k]) != dims.n_vocab:
                toks.append(int(seq[k]))
                frames.append(f)
            f += int(dur[k])
        # generate() stops at max_length = max_symbols_per_step x T3 steps; an utterance whose
        # search sits on one frame (duration-0 tokens) is cut there: the fixture is then a prefix
        out[f"finished_{i}"] = np.int64(f >= T3)
        out[f"tokens_{i}"] = np.array(toks, np.int32)
        out[f"frames_{i}"] = np.array(frames, np.int32)
        print(f"{name}[{i}] n={n}: T={T} T3={T3} tokens={len(toks)} finished={f >= T3}")
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    P.set_threads(8)
    for case in CASES:
        run_case(*case)


if __name__ == "__main__":
    main()
