"""GPU box, developer A/B: encoder output of one large-v3 bf16 window (debug_encode) saved to
gpurun_out/enc_<tag>.npy, plus the encoder probe times, for bitwise comparison between builds /
environment switches."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

torch.cuda.init()
from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams
from spittle_amd.synth import synth_audio

tag = sys.argv[1]
e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=8))
e.load_model("synthetic:large-v3")
mel = e.debug_mel(synth_audio(0))
enc = e.debug_encode(mel)
np.save(f"gpurun_out/enc_{tag}.npy", enc)
p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True, max_new_tokens=4)
e.transcribe_batch([synth_audio(i) for i in range(8)], p)
print(json.dumps({"tag": tag, "enc_sum": float(np.abs(enc).sum()), "enc_fc1_gemm": e.probe("enc_fc1_gemm", 20),
                  "enc_attn": e.probe("enc_attn", 20)}))
