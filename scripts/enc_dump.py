"""GPU box: the encoder output of one seeded window (debug_encode) saved to an .npz, for bitwise
comparisons across switches read at engine creation.  usage: enc_dump.py MODEL DTYPE OUT.npz"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from spittle_amd import WhisperEngine, WhisperModelParams  # noqa: E402
from spittle_amd.synth import synth_audio  # noqa: E402

model, dtype, out = sys.argv[1], sys.argv[2], sys.argv[3]
e = WhisperEngine(WhisperModelParams(dtype=dtype, max_batch=1))
e.load_model(model)
mel = e.debug_mel(synth_audio(5))
enc = e.debug_encode(mel)
np.savez(out, enc=enc)
print(out, enc.shape, float(np.abs(enc).max()))
e.unload_model()
