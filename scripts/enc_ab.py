"""GPU box, A/B of the encoder between builds on one box: imports spittle_amd from PKG_DIR (argv[1];
'.' = this tree), runs the C3 shape (large-v3 bf16, 8 x 30 s) with a short decode, and prints the
median encoder_ms of 7 calls after 2 warm-ups (HIP events, engine stream)."""
import json
import os
import sys

pkg = os.path.abspath(sys.argv[1])
sys.path.insert(0, pkg)
sys.path.insert(1, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
import spittle_amd  # noqa: E402
from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams  # noqa: E402
from spittle_amd.synth import synth_audio  # noqa: E402

nb = int(os.environ.get("ENC_AB_B", "8"))  # windows per call (1: the app's single-window call)
e = WhisperEngine(WhisperModelParams(dtype=os.environ.get("ENC_AB_DTYPE", "bf16"), max_batch=nb))
e.load_model(os.environ.get("ENC_AB_MODEL", "synthetic:large-v3"))
xs = [synth_audio(i) for i in range(nb)]
p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True, max_new_tokens=4)
for _ in range(2):
    e.transcribe_batch(xs, p)
enc = []
for _ in range(7):
    e.transcribe_batch(xs, p)
    enc.append(e.timings()["encoder_ms"])
print(json.dumps({"pkg": spittle_amd.__file__, "env": {k: v for k, v in os.environ.items() if k.startswith("SPT_")},
                  "encoder_ms_median": float(np.median(enc)), "encoder_ms": [round(v, 3) for v in enc]}))
e.unload_model()
