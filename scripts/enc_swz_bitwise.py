"""GPU box: the large-v3 2+2 bf16 encoder output with the encoder attention's V-tile swizzle on
(SPT_ATTN_SWZ=3) and off (1): a swizzle moves LDS addresses only, so the outputs must be bitwise equal."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
from oracle import oracle as O  # noqa: E402  (synthetic audio and the reference mel only)
from spittle_amd import WhisperEngine, WhisperModelParams  # noqa: E402

e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=2, seed=1234))
e.load_model("synthetic:large-v3:enc=2:dec=2")
mel = O.mel(O.synth_audio(1), 128)
out = {}
for s in ("1", "3"):
    os.environ["SPT_ATTN_SWZ"] = s
    out[s] = e.debug_encode(mel)
print("bitwise equal:", np.array_equal(out["1"], out["3"]), "max |diff|:", float(np.abs(out["1"] - out["3"]).max()))
e.unload_model()
