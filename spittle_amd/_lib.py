"""ctypes binding of the C ABI in include/spittle_hip.h (libspittle_hip.so, in-tree).

The product path has no CPU fallback: if the HIP library is missing this module
raises, loudly, at import of the engine.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libspittle_hip.so")

# status codes
SPT_OK, SPT_ERR_INVALID_ARG, SPT_ERR_LOAD, SPT_ERR_DEVICE, SPT_ERR_OOM, SPT_ERR_UNSUPPORTED, SPT_ERR_INTERNAL = range(7)
STATUS_NAMES = {0: "OK", 1: "INVALID_ARG", 2: "LOAD", 3: "DEVICE", 4: "OOM", 5: "UNSUPPORTED", 6: "INTERNAL"}
SPT_DTYPE_F32, SPT_DTYPE_BF16, SPT_DTYPE_F16 = 0, 1, 2
SPT_SUPPRESS_BLANK, SPT_NO_TIMESTAMPS, SPT_IGNORE_EOT, SPT_SUPPRESS_NST = 1, 2, 4, 8

# every symbol include/spittle_hip.h declares
EXPORTS = [
    "spt_version", "spt_default_model_params", "spt_default_infer_params", "spt_ctx_create",
    "spt_ctx_destroy", "spt_last_error", "spt_ctx_info", "spt_transcribe", "spt_transcribe_batch",
    "spt_transcribe_batch_device", "spt_result_free", "spt_get_timings", "spt_get_call_stats", "spt_debug_mel",
    "spt_debug_mel_at", "spt_debug_encode", "spt_debug_weight_checksum", "spt_probe_kernel", "spt_language_code",
    "spt_tokenize", "spt_token_to_str", "spt_debug_ggml_tokenize", "spt_debug_ggml_dequant",
    "spt_weights_export", "spt_weights_import", "spt_weights_arena", "spt_weights_commit",
    "spt_ctx_create_replicas", "spt_transcribe_batch_replicas",
    # ABI 6: Parakeet-V3
    "spt_parakeet_default_model_params", "spt_parakeet_default_infer_params", "spt_parakeet_create",
    "spt_parakeet_destroy", "spt_parakeet_last_error", "spt_parakeet_info", "spt_parakeet_tensor_numel",
    "spt_parakeet_set_tensor", "spt_parakeet_set_vocab", "spt_parakeet_transcribe", "spt_parakeet_transcribe_batch",
    "spt_parakeet_transcribe_batch_device", "spt_parakeet_result_free", "spt_parakeet_get_timings",
    "spt_parakeet_debug_mel", "spt_parakeet_debug_encode", "spt_parakeet_debug_decode", "spt_parakeet_debug_last_encoder",
    "spt_parakeet_debug_weight_checksum", "spt_parakeet_onnx_open", "spt_parakeet_onnx_tensor",
    "spt_parakeet_onnx_piece", "spt_parakeet_onnx_close",
    # ABI 7: capture-side resampler
    "spt_resampler_create", "spt_resampler_info", "spt_resample_output_len", "spt_resample",
    "spt_resampler_last_error", "spt_resampler_destroy",
    # ABI 8: voice-activity gate
    "spt_vad_default_params", "spt_vad_create", "spt_vad_push", "spt_vad_result_free", "spt_vad_reset",
    "spt_vad_last_error", "spt_vad_destroy",
    # ABI 10: Parakeet encoder stage profile
    "spt_parakeet_profile_encoder",
]
SPT_PK_WEIGHTS_EMPTY = 1
SPT_PK_TS_TOKEN, SPT_PK_TS_WORD, SPT_PK_TS_SEGMENT = 0, 1, 2
SPT_MODEL_WEIGHTS_EXTERNAL = 1
# spt_pk_stage: encoder stage classes of spt_parakeet_profile_encoder, in order
PK_STAGES = ("subsampling", "pos", "layernorm", "ffn", "qkv_out", "attn", "conv_pw", "conv_dw", "joint_enc")
PROBES = {"dec_cross_attn": 0, "dec_self_attn": 1, "dec_logits": 2, "dec_fc1": 3, "enc_fc1_gemm": 4,
          "enc_attn": 5}


class ModelParams(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("device", C.c_int32), ("max_batch", C.c_int32),
                ("flags", C.c_uint32), ("seed", C.c_uint64)]


class InferParams(C.Structure):
    _fields_ = [("language", C.c_char_p), ("translate", C.c_int32), ("initial_prompt", C.c_char_p),
                ("flags", C.c_uint32), ("max_new_tokens", C.c_int32), ("temperature", C.c_float),
                ("beam_size", C.c_int32), ("forced_tokens", C.POINTER(C.c_int32)), ("n_forced", C.c_int32),
                ("prompt_tokens", C.POINTER(C.c_int32)), ("n_prompt_tokens", C.c_int32),
                ("temperature_inc", C.c_float), ("best_of", C.c_int32), ("entropy_thold", C.c_float),
                ("logprob_thold", C.c_float), ("max_initial_ts", C.c_float), ("reserved0", C.c_int32),
                ("seed", C.c_uint64)]


class Segment(C.Structure):
    _fields_ = [("t0", C.c_int64), ("t1", C.c_int64), ("text", C.c_char_p), ("i0", C.c_int32),
                ("n_tokens", C.c_int32)]


class Result(C.Structure):
    _fields_ = [("text", C.c_char_p), ("tokens", C.POINTER(C.c_int32)), ("top1", C.POINTER(C.c_float)),
                ("top2", C.POINTER(C.c_float)), ("n_tokens", C.c_int32), ("n_windows", C.c_int32),
                ("language", C.c_int32), ("n_segments", C.c_int32), ("segments", C.POINTER(Segment)),
                ("n_fallbacks", C.c_int32), ("reserved0", C.c_int32)]


class ModelInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("n_mels", "d", "n_head", "n_enc", "n_dec", "n_vocab", "n_audio_ctx",
                                          "n_text_ctx", "dtype", "max_batch")] + \
               [("weight_bytes", C.c_int64), ("workspace_bytes", C.c_int64)]


class Timings(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("mel_ms", "encoder_ms", "cross_kv_ms", "decode_ms", "total_ms",
                                           "h2d_ms")] + [("n_decode_passes", C.c_int32), ("batch", C.c_int32)]


class CallStats(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("engine_calls", "decoder_passes", "beam_steps", "encoder_windows")] + \
               [(n, C.c_double) for n in ("device_ms", "encoder_ms", "decode_ms")] + \
               [(n, C.c_int32) for n in ("pd_passes", "pd_fallbacks")]


class PkModelParams(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("device", C.c_int32), ("max_batch", C.c_int32), ("max_seconds", C.c_float),
                ("seed", C.c_uint64), ("flags", C.c_uint32), ("reserved0", C.c_int32)]


class PkInferParams(C.Structure):
    _fields_ = [("max_symbols", C.c_int32), ("timestamp_granularity", C.c_int32)]


class PkSegment(C.Structure):
    _fields_ = [("start", C.c_double), ("end", C.c_double), ("text", C.c_char_p), ("i0", C.c_int32),
                ("n_tokens", C.c_int32)]


class PkResult(C.Structure):
    _fields_ = [("text", C.c_char_p), ("tokens", C.POINTER(C.c_int32)), ("frames", C.POINTER(C.c_int32)),
                ("logit", C.POINTER(C.c_float)), ("runner_up", C.POINTER(C.c_float)), ("n_tokens", C.c_int32),
                ("n_segments", C.c_int32), ("segments", C.POINTER(PkSegment)), ("n_chunks", C.c_int32),
                ("reserved0", C.c_int32)]


class PkModelInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("n_mels", "d", "n_layers", "n_heads", "ff", "sub_ch", "conv_k", "pred",
                                          "n_vocab", "n_dur", "dtype", "max_batch", "max_samples", "reserved0")] + \
               [("weight_bytes", C.c_int64), ("workspace_bytes", C.c_int64)]


class PkTimings(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("mel_ms", "encoder_ms", "decode_ms", "total_ms", "h2d_ms")] + \
               [(n, C.c_int32) for n in ("n_steps", "batch", "enc_frames", "reserved0")]


class VadParams(C.Structure):
    _fields_ = [("threshold", C.c_float), ("prefill_frames", C.c_int32), ("hangover_frames", C.c_int32),
                ("onset_frames", C.c_int32), ("device", C.c_int32), ("reserved0", C.c_int32)]


class VadResult(C.Structure):
    _fields_ = [("samples", C.POINTER(C.c_float)), ("n_samples", C.c_size_t), ("prob", C.POINTER(C.c_float)),
                ("kind", C.POINTER(C.c_uint8)), ("n_frames", C.c_int32), ("reserved0", C.c_int32),
                ("device_ms", C.c_double)]


_lib = None


def load():
    """Load libspittle_hip.so (built by __graft_entry__.build / make -C spittle_amd/csrc)."""
    global _lib
    if _lib is not None:
        return _lib
    path = LIB_PATH
    if os.environ.get("SPT_DEBUG_LIB"):  # bounds-checked developer build (make -C spittle_amd/csrc dbg)
        path = os.path.join(os.path.dirname(LIB_PATH), "libspittle_hip_dbg.so")
    if not os.path.exists(path):
        raise ImportError(f"spittle_amd: HIP library not built: {path} (run `make -C spittle_amd/csrc`)")
    L = C.CDLL(path)
    vp, fp = C.c_void_p, C.POINTER(C.c_float)
    L.spt_version.restype = C.c_char_p
    L.spt_default_model_params.argtypes = [C.POINTER(ModelParams)]
    L.spt_default_infer_params.argtypes = [C.POINTER(InferParams)]
    L.spt_ctx_create.argtypes = [C.c_char_p, C.POINTER(ModelParams), C.POINTER(vp), C.c_char_p, C.c_size_t]
    L.spt_ctx_create.restype = C.c_int
    L.spt_ctx_destroy.argtypes = [vp]
    L.spt_last_error.argtypes = [vp]
    L.spt_last_error.restype = C.c_char_p
    L.spt_ctx_info.argtypes = [vp, C.POINTER(ModelInfo)]
    L.spt_transcribe.argtypes = [vp, fp, C.c_size_t, C.POINTER(InferParams), C.POINTER(C.POINTER(Result))]
    L.spt_transcribe_batch.argtypes = [vp, C.POINTER(fp), C.POINTER(C.c_size_t), C.c_size_t,
                                       C.POINTER(InferParams), C.POINTER(C.POINTER(Result))]
    L.spt_transcribe_batch_device.argtypes = [vp, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.c_size_t,
                                              C.POINTER(InferParams), C.POINTER(C.POINTER(Result))]
    L.spt_result_free.argtypes = [C.POINTER(Result)]
    L.spt_language_code.argtypes = [C.c_int32]
    L.spt_language_code.restype = C.c_char_p
    ip = C.POINTER(C.c_int32)
    L.spt_tokenize.argtypes = [vp, C.c_char_p, ip, C.c_int32, ip]
    L.spt_token_to_str.argtypes = [vp, C.c_int32]
    L.spt_token_to_str.restype = C.c_char_p
    L.spt_debug_ggml_tokenize.argtypes = [C.c_char_p, C.c_char_p, ip, C.c_int32, ip]
    L.spt_debug_ggml_dequant.argtypes = [C.c_int32, C.c_void_p, C.c_int64, fp]
    L.spt_get_timings.argtypes = [vp, C.POINTER(Timings)]
    L.spt_get_call_stats.argtypes = [vp, C.POINTER(CallStats)]
    L.spt_debug_mel.argtypes = [vp, fp, C.c_size_t, fp]
    L.spt_debug_mel_at.argtypes = [vp, fp, C.c_size_t, C.c_int32, fp]
    L.spt_debug_encode.argtypes = [vp, fp, fp]
    L.spt_debug_weight_checksum.argtypes = [vp, C.c_int32, C.POINTER(C.c_double)]
    L.spt_probe_kernel.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                   C.POINTER(C.c_int32)]
    L.spt_weights_export.argtypes = [vp, C.c_void_p, C.c_size_t]
    L.spt_weights_import.argtypes = [vp, C.c_void_p, C.c_size_t]
    L.spt_weights_arena.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_size_t)]
    L.spt_weights_commit.argtypes = [vp]
    L.spt_ctx_create_replicas.argtypes = [C.c_char_p, C.POINTER(ModelParams), C.POINTER(C.c_int32), C.c_int32,
                                          C.POINTER(vp), C.POINTER(C.c_double), C.c_char_p, C.c_size_t]
    L.spt_transcribe_batch_replicas.argtypes = [C.POINTER(vp), C.c_int32, C.POINTER(fp), C.POINTER(C.c_size_t),
                                                C.c_size_t, C.POINTER(InferParams), C.POINTER(C.POINTER(Result))]
    # ABI 6: Parakeet-V3
    PR = C.POINTER(C.POINTER(PkResult))
    L.spt_parakeet_default_model_params.argtypes = [C.POINTER(PkModelParams)]
    L.spt_parakeet_default_infer_params.argtypes = [C.POINTER(PkInferParams)]
    L.spt_parakeet_create.argtypes = [C.c_char_p, C.POINTER(PkModelParams), C.POINTER(vp), C.c_char_p, C.c_size_t]
    L.spt_parakeet_onnx_open.argtypes = [C.c_char_p, C.POINTER(vp), C.POINTER(PkModelInfo), C.c_char_p, C.c_size_t]
    L.spt_parakeet_onnx_tensor.restype = C.c_int64
    L.spt_parakeet_onnx_tensor.argtypes = [vp, C.c_int32, C.POINTER(C.POINTER(C.c_float))]
    L.spt_parakeet_onnx_piece.restype = C.c_char_p
    L.spt_parakeet_onnx_piece.argtypes = [vp, C.c_int32]
    L.spt_parakeet_onnx_close.argtypes = [vp]
    L.spt_parakeet_destroy.argtypes = [vp]
    L.spt_parakeet_last_error.argtypes = [vp]
    L.spt_parakeet_last_error.restype = C.c_char_p
    L.spt_parakeet_info.argtypes = [vp, C.POINTER(PkModelInfo)]
    L.spt_parakeet_tensor_numel.argtypes = [vp, C.c_int32, C.POINTER(C.c_int64)]
    L.spt_parakeet_set_tensor.argtypes = [vp, C.c_int32, fp, C.c_int64]
    L.spt_parakeet_set_vocab.argtypes = [vp, C.POINTER(C.c_char_p), C.c_int32]
    L.spt_parakeet_transcribe.argtypes = [vp, fp, C.c_size_t, C.POINTER(PkInferParams), PR]
    L.spt_parakeet_transcribe_batch.argtypes = [vp, C.POINTER(fp), C.POINTER(C.c_size_t), C.c_size_t,
                                                C.POINTER(PkInferParams), PR]
    L.spt_parakeet_transcribe_batch_device.argtypes = [vp, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.c_size_t,
                                                       C.POINTER(PkInferParams), PR]
    L.spt_parakeet_result_free.argtypes = [C.POINTER(PkResult)]
    L.spt_parakeet_get_timings.argtypes = [vp, C.POINTER(PkTimings)]
    L.spt_parakeet_profile_encoder.argtypes = [vp, C.c_int32, C.POINTER(C.c_double), C.c_int32]
    L.spt_parakeet_debug_mel.argtypes = [vp, fp, C.c_size_t, fp]
    L.spt_parakeet_debug_encode.argtypes = [vp, fp, C.c_int32, fp]
    L.spt_parakeet_debug_decode.argtypes = [vp, fp, C.c_int32, C.c_int32, PR]
    L.spt_parakeet_debug_last_encoder.argtypes = [vp, C.c_int32, fp, C.POINTER(C.c_int32)]
    L.spt_parakeet_debug_weight_checksum.argtypes = [vp, C.c_int32, C.POINTER(C.c_double)]
    L.spt_resampler_create.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.POINTER(vp), C.c_char_p,
                                       C.c_size_t]
    L.spt_resampler_create.restype = C.c_int
    L.spt_resampler_info.argtypes = [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    L.spt_resampler_info.restype = C.c_int
    L.spt_resample_output_len.argtypes = [vp, C.c_size_t]
    L.spt_resample_output_len.restype = C.c_size_t
    L.spt_resample.argtypes = [vp, fp, C.c_size_t, fp, C.c_size_t, C.POINTER(C.c_size_t)]
    L.spt_resample.restype = C.c_int
    L.spt_resampler_last_error.argtypes = [vp]
    L.spt_resampler_last_error.restype = C.c_char_p
    L.spt_resampler_destroy.argtypes = [vp]
    L.spt_resampler_destroy.restype = None
    L.spt_vad_default_params.argtypes = [C.POINTER(VadParams)]
    L.spt_vad_default_params.restype = None
    L.spt_vad_create.argtypes = [C.c_char_p, C.POINTER(VadParams), C.POINTER(vp), C.c_char_p, C.c_size_t]
    L.spt_vad_create.restype = C.c_int
    L.spt_vad_push.argtypes = [vp, fp, C.c_size_t, C.POINTER(C.POINTER(VadResult))]
    L.spt_vad_push.restype = C.c_int
    L.spt_vad_result_free.argtypes = [C.POINTER(VadResult)]
    L.spt_vad_result_free.restype = None
    L.spt_vad_reset.argtypes = [vp, C.c_int32]
    L.spt_vad_reset.restype = C.c_int
    L.spt_vad_last_error.argtypes = [vp]
    L.spt_vad_last_error.restype = C.c_char_p
    L.spt_vad_destroy.argtypes = [vp]
    L.spt_vad_destroy.restype = None
    for fn in EXPORTS:
        if fn.startswith("spt_parakeet_") and fn not in ("spt_parakeet_default_model_params",
                                                          "spt_parakeet_default_infer_params", "spt_parakeet_destroy",
                                                          "spt_parakeet_last_error", "spt_parakeet_result_free",
                                                          "spt_parakeet_onnx_tensor", "spt_parakeet_onnx_piece",
                                                          "spt_parakeet_onnx_close"):
            getattr(L, fn).restype = C.c_int
    for fn in ("spt_weights_arena", "spt_weights_commit", "spt_ctx_create_replicas", "spt_transcribe_batch_replicas",
               "spt_weights_export", "spt_weights_import", "spt_ctx_info", "spt_transcribe", "spt_transcribe_batch", "spt_transcribe_batch_device",
               "spt_get_timings", "spt_get_call_stats", "spt_debug_mel", "spt_debug_mel_at", "spt_debug_encode", "spt_debug_weight_checksum",
               "spt_probe_kernel", "spt_tokenize", "spt_debug_ggml_tokenize", "spt_debug_ggml_dequant"):
        getattr(L, fn).restype = C.c_int
    _lib = L
    return L
