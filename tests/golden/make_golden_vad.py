"""Golden vectors for the voice-activity gate (run in the build container; TEST INFRASTRUCTURE).

The model is the reference's own file, resources/models/silero_vad_v4.onnx (committed beside this
script as tests/golden/silero_vad_v4.onnx, sha256 a35ebf52fd3ce5f1469b2a36158dba761bc47b973ea3382b
3186ca15b1f5af28, so the GPU box has it).  oracle/silero.py interprets its ONNX graph in numpy
(and tests/test_vad_oracle.py checks that interpreter against an independent torch restatement);
this script records, for seeded speech-like streams (spittle_amd.synth.synth_speech), each 30 ms
frame's speech probability with the LSTM state carried from frame to frame (vad-rs), the app's
SmoothedVad(0.3; 15, 15, 2) decisions (audio.rs:132-134) and the kept audio's length and checksum.

Usage:  python tests/golden/make_golden_vad.py   (writes tests/golden/silero_vad.npz)
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from oracle import silero as S  # noqa: E402
from spittle_amd.synth import synth_speech  # noqa: E402

STREAMS = [(0, 6.0), (1, 4.0), (2, 3.0)]


def main():
    model = os.path.join(HERE, "silero_vad_v4.onnx")
    out = {}
    for k, (seed, sec) in enumerate(STREAMS):
        x = synth_speech(seed, sec)
        v = S.SileroVad(model, 0.3)
        n = x.size // S.FRAME
        frames = [x[i * S.FRAME:(i + 1) * S.FRAME] for i in range(n)]
        probs = np.array([v.prob(f) for f in frames], np.float32)
        voice = probs > np.float32(0.3)
        kept = S.gate_stream(list(voice), frames)
        kinds, sv = [], S.SmoothedVad(lambda f, it=iter(voice): next(it))
        for f in frames:
            r = sv.push_frame(f)
            kinds.append(0 if r.size == 0 else (1 if r.size == S.FRAME else 2))
        out[f"seed_{k}"] = np.int64(seed)
        out[f"seconds_{k}"] = np.float64(sec)
        out[f"prob_{k}"] = probs
        out[f"kind_{k}"] = np.array(kinds, np.uint8)
        out[f"kept_len_{k}"] = np.int64(kept.size)
        out[f"kept_sum_{k}"] = np.float64(kept.astype(np.float64).sum())
        out[f"hn_{k}"], out[f"cn_{k}"] = v.h.copy(), v.c.copy()
        print(f"stream {k}: {n} frames, speech frames {int(voice.sum())}, onsets {kinds.count(2)}, kept {kept.size}")
    np.savez_compressed(os.path.join(HERE, "silero_vad.npz"), **out)


if __name__ == "__main__":
    main()
