"""CPU oracle of Spittle's voice-activity gate (TEST INFRASTRUCTURE: imported by tests/ and the
golden-fixture script only; spittle_amd/ never imports it).

Reference path: the recorder's consumer thread pushes every 30 ms frame (480
samples at 16 kHz) through ``SmoothedVad::new(Box::new(SileroVad::new(vad_path, 0.3)), 15, 15, 2)``
(/root/reference/src-tauri/src/managers/audio.rs:132-134), whose model is the ONNX file that ships
with the app (resources/models/silero_vad_v4.onnx, audio.rs:295-307), run by vad-rs through ONNX
Runtime with its LSTM state (h, c) carried from frame to frame [vad-rs, recalled].

* ``Graph``: an interpreter of the model's own ONNX graph (oracle/onnx_graph.py reads it; numpy
  implementations of the ~30 standard ops it uses, ONNX operator semantics restated).  The file
  defines the network; nothing in it is executed as code.
* ``SileroVad``: ``prob > threshold`` per frame (vad/silero.rs:32-51), state carried.
* ``SmoothedVad``: the prefill / hangover / onset state machine, restated line by line from
  vad/smoothed.rs:43-104 (bit-exact given the same per-frame decisions).
"""
from __future__ import annotations

from collections import deque

import numpy as np

from . import onnx_graph as G

FRAME = 480  # 30 ms at 16 kHz (silero.rs:8-10)


# ------------------------------------------------------------------ ONNX op semantics (numpy)
def _conv(x, w, b, a):
    """Conv over the last axis (1-D: x [N][C][L], w [M][C/g][k])."""
    g = int(a.get("group", 1))
    s = int(a.get("strides", [1])[0])
    d = int(a.get("dilations", [1])[0])
    p = a.get("pads", [0, 0])
    x = np.pad(x, ((0, 0), (0, 0), (int(p[0]), int(p[1]))))
    N, C, L = x.shape
    M, Cg, k = w.shape
    Lo = (L - d * (k - 1) - 1) // s + 1
    out = np.zeros((N, M, Lo), np.float64)
    mg = M // g
    for gi in range(g):
        xs = x[:, gi * Cg:(gi + 1) * Cg].astype(np.float64)
        ws = w[gi * mg:(gi + 1) * mg].astype(np.float64)
        for t in range(k):
            seg = xs[:, :, t * d: t * d + s * (Lo - 1) + 1: s]          # [N][Cg][Lo]
            out[:, gi * mg:(gi + 1) * mg] += np.einsum("nct,mc->nmt", seg, ws[:, :, t])
    if b is not None:
        out += b.astype(np.float64)[None, :, None]
    return out.astype(np.float32)


def _slice(x, starts, ends, axes=None, steps=None):
    axes = list(range(len(starts))) if axes is None else [int(a) % x.ndim for a in axes]
    steps = [1] * len(starts) if steps is None else steps
    sl = [slice(None)] * x.ndim
    for st, en, ax, sp in zip(starts, ends, axes, steps):
        n = x.shape[ax]
        st, en, sp = int(st), int(en), int(sp)
        if sp > 0:
            st = max(0, min(n, st + n if st < 0 else st))
            en = max(0, min(n, en + n if en < 0 else en))
        else:
            st = max(-1, min(n - 1, st + n if st < 0 else st))
            en = max(-1, min(n - 1, en + n if en < 0 else en))
            en = None if en < 0 else en
        sl[ax] = slice(st, en, sp)
    return x[tuple(sl)]


def _sig(x):
    return (1.0 / (1.0 + np.exp(-x.astype(np.float64)))).astype(np.float32)


def _lstm(X, W, R, B, h0, c0, a):
    """ONNX LSTM, forward, gates i, o, f, c; X [T][N][I], W [1][4H][I], R [1][4H][H], B [1][8H]."""
    H = int(a["hidden_size"])
    W, R = W[0].astype(np.float64), R[0].astype(np.float64)
    Bw, Br = (B[0, :4 * H].astype(np.float64), B[0, 4 * H:].astype(np.float64)) if B is not None else (0.0, 0.0)
    h = h0[0].astype(np.float64)
    c = c0[0].astype(np.float64)
    Y = []
    for t in range(X.shape[0]):
        z = X[t].astype(np.float64) @ W.T + h @ R.T + Bw + Br
        i, o, f, g = z[:, :H], z[:, H:2 * H], z[:, 2 * H:3 * H], z[:, 3 * H:]
        i, o, f = 1 / (1 + np.exp(-i)), 1 / (1 + np.exp(-o)), 1 / (1 + np.exp(-f))
        c = f * c + i * np.tanh(g)
        h = o * np.tanh(c)
        Y.append(h.copy())
    Y = np.stack(Y)[:, None].astype(np.float32)           # [T][1][N][H]
    return Y, h[None].astype(np.float32), c[None].astype(np.float32)


class Graph:
    """Runs an onnx_graph.Graph (the silero_vad_v4 ops) on numpy values."""

    def __init__(self, g: G.Graph):
        self.g = g

    def run(self, feeds: dict) -> dict:
        return self._run(self.g, dict(feeds), dict(self.g.inits))

    def _run(self, g, env, consts):
        env = {**consts, **g.inits, **env}
        for n in g.nodes:
            x = [env[i] if i else None for i in n.inputs]
            a = n.attrs
            op = n.op
            if op == "If":
                br = a["then_branch"] if bool(np.asarray(x[0]).ravel()[0]) else a["else_branch"]
                sub = self._run(br, {}, env)
                outs = [sub[o] for o in br.outputs]
            elif op == "Identity":
                outs = [x[0]]
            elif op == "Shape":
                outs = [np.array(x[0].shape, np.int64)[int(a.get("start", 0)):]]
            elif op == "Gather":
                outs = [np.take(x[0], x[1], axis=int(a.get("axis", 0)))]
            elif op == "Unsqueeze":
                y = x[0]
                for ax in sorted(int(v) % (y.ndim + 1) for v in np.asarray(x[1]).ravel()):
                    y = np.expand_dims(y, ax)
                outs = [y]
            elif op == "Squeeze":
                axes = tuple(int(v) % x[0].ndim for v in np.asarray(x[1]).ravel()) if len(x) > 1 and x[1] is not None else None
                outs = [np.squeeze(x[0], axis=axes)]
            elif op == "Concat":
                outs = [np.concatenate([np.atleast_1d(v) for v in x], axis=int(a["axis"]))]
            elif op == "Reshape":
                shp = [int(s) for s in x[1]]
                shp = [x[0].shape[i] if s == 0 else s for i, s in enumerate(shp)]
                outs = [x[0].reshape(shp)]
            elif op == "Pad":
                p = [int(v) for v in x[1]]
                k = len(p) // 2
                mode = a.get("mode", b"constant")
                mode = mode.decode() if isinstance(mode, bytes) else mode
                outs = [np.pad(x[0], [(p[i], p[i + k]) for i in range(k)], mode="reflect" if mode == "reflect" else "constant")]
            elif op == "Equal":
                outs = [np.equal(x[0], x[1])]
            elif op == "Conv":
                outs = [_conv(x[0], x[1], x[2] if len(x) > 2 else None, a)]
            elif op == "Slice":
                outs = [_slice(x[0], x[1], x[2], x[3] if len(x) > 3 else None, x[4] if len(x) > 4 else None)]
            elif op == "Pow":
                outs = [np.power(x[0], x[1]).astype(np.float32)]
            elif op == "Add":
                outs = [(x[0] + x[1]).astype(np.result_type(x[0], x[1]))]
            elif op == "Mul":
                outs = [(x[0] * x[1]).astype(np.result_type(x[0], x[1]))]
            elif op == "Neg":
                outs = [-x[0]]
            elif op == "Sqrt":
                outs = [np.sqrt(x[0])]
            elif op == "Log":
                outs = [np.log(x[0])]
            elif op == "Relu":
                outs = [np.maximum(x[0], 0).astype(x[0].dtype)]
            elif op == "Sigmoid":
                outs = [_sig(x[0])]
            elif op == "ReduceMean":
                outs = [np.mean(x[0].astype(np.float64), axis=tuple(int(v) for v in a["axes"]),
                                keepdims=bool(a.get("keepdims", 1))).astype(np.float32)]
            elif op == "Transpose":
                outs = [np.transpose(x[0], [int(v) for v in a["perm"]])]
            elif op == "Cast":
                outs = [x[0].astype({9: np.bool_, 1: np.float32, 7: np.int64, 6: np.int32}[int(a["to"])])]
            elif op == "ConstantOfShape":
                v = a.get("value", np.zeros(1, np.float32))
                outs = [np.full([int(s) for s in x[0]], np.asarray(v).ravel()[0], dtype=np.asarray(v).dtype)]
            elif op == "Constant":
                outs = [np.asarray(a["value"])]
            elif op == "LSTM":
                outs = list(_lstm(x[0], x[1], x[2], x[3], x[5], x[6], a))
            else:
                raise NotImplementedError(op)
            for name, v in zip(n.outputs, outs):
                if name:
                    env[name] = v
        return env


class SileroVad:
    """vad/silero.rs SileroVad over vad-rs: one 480-sample frame -> prob, the LSTM state carried."""

    def __init__(self, model_path: str, threshold: float = 0.3):
        if not 0.0 <= threshold <= 1.0:
            raise ValueError("threshold must be between 0.0 and 1.0")
        self.graph = Graph(G.load(model_path))
        self.threshold = np.float32(threshold)
        self.reset()

    def reset(self):
        self.h = np.zeros((2, 1, 64), np.float32)
        self.c = np.zeros((2, 1, 64), np.float32)

    def prob(self, frame: np.ndarray) -> float:
        frame = np.asarray(frame, np.float32)
        if frame.size != FRAME:
            raise ValueError(f"expected {FRAME} samples, got {frame.size}")
        env = self.graph.run({"input": frame[None], "sr": np.array(16000, np.int64), "h": self.h, "c": self.c})
        self.h, self.c = env["hn"], env["cn"]
        return float(np.asarray(env["output"]).ravel()[0])

    def is_voice(self, frame) -> bool:
        return np.float32(self.prob(frame)) > self.threshold


class SmoothedVad:
    """vad/smoothed.rs:43-104: returns the samples a frame contributes (empty = Noise)."""

    def __init__(self, is_voice, prefill_frames=15, hangover_frames=15, onset_frames=2):
        self.is_voice, self.prefill, self.hangover, self.onset = is_voice, prefill_frames, hangover_frames, onset_frames
        self.reset()

    def reset(self):
        self.buf = deque()
        self.hang = 0
        self.ons = 0
        self.in_speech = False

    def push_frame(self, frame: np.ndarray) -> np.ndarray:
        self.buf.append(np.asarray(frame, np.float32).copy())
        while len(self.buf) > self.prefill + 1:
            self.buf.popleft()
        v = self.is_voice(frame)
        if not self.in_speech and v:
            self.ons += 1
            if self.ons >= self.onset:
                self.in_speech = True
                self.hang = self.hangover
                self.ons = 0
                return np.concatenate(list(self.buf))
            return np.zeros(0, np.float32)
        if self.in_speech and v:
            self.hang = self.hangover
            return np.asarray(frame, np.float32)
        if self.in_speech and not v:
            if self.hang > 0:
                self.hang -= 1
                return np.asarray(frame, np.float32)
            self.in_speech = False
            return np.zeros(0, np.float32)
        self.ons = 0
        return np.zeros(0, np.float32)


def gate_stream(frames_voice, frames, prefill=15, hangover=15, onset=2) -> np.ndarray:
    """The recorder's kept audio (recorder.rs:296-300: Speech frames appended, Noise dropped) for a
    stream of frames whose per-frame decisions are given."""
    it = iter(frames_voice)
    sv = SmoothedVad(lambda _f: next(it), prefill, hangover, onset)
    out = [sv.push_frame(f) for f in frames]
    return np.concatenate(out) if out else np.zeros(0, np.float32)
