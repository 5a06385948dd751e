"""GPU box, developer check: the encoder (large-v3 dims, 2 layers, bf16) run four times on the same
mel must be bitwise repeatable; prints the spread and saves run 0 (OUT) for cross-variant diffs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

torch.cuda.init()
from oracle import oracle as O
from spittle_amd import WhisperEngine, WhisperModelParams

e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=2, seed=1234))
e.load_model("synthetic:large-v3:enc=2:dec=2")
mel = O.mel(O.synth_audio(3), 128)
outs = [e.debug_encode(mel) for _ in range(4)]
print("repeatable:", all(bool((x == outs[0]).all()) for x in outs[1:]),
      "max spread:", max(float(np.abs(x - outs[0]).max()) for x in outs[1:]))
np.save(os.environ.get("OUT", "gpurun_out/enc.npy"), outs[0])
