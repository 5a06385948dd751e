"""Independent PyTorch restatement of the Parakeet-V3 forward pass (TEST INFRASTRUCTURE).

It pins the C oracle (oracle/po_model.c) with the building blocks PyTorch ships: torch.stft
(centre padding, the 400-sample window padded to n_fft), F.conv2d (stride / padding
semantics of the dw_striding subsampling), NeMo's rel_shift formulation of the relative-
position scores (pad + view, not the oracle's direct index), F.batch_norm, torch.nn.LSTM
(its gate order) and F.glu.  The model definition is NVIDIA NeMo's FastConformer-TDT
[upstream, recalled]; see oracle/parakeet_oracle.h.  Weights come from the oracle's tensor
table, so the two restatements share nothing but the weights.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def slaney_mel(n_mels: int, n_fft: int = 512, sr: int = 16000) -> np.ndarray:
    """librosa.filters.mel(norm='slaney', htk=False), restated in numpy (f64)."""
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0

    def hz2mel(f):
        f = np.asarray(f, np.float64)
        return np.where(f < min_log_hz, f / f_sp, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep)

    def mel2hz(m):
        return np.where(m < min_log_mel, f_sp * m, min_log_hz * np.exp(logstep * (m - min_log_mel)))

    pts = mel2hz(np.linspace(hz2mel(0.0), hz2mel(sr / 2), n_mels + 2))
    fft = np.linspace(0, sr / 2, n_fft // 2 + 1)
    lower = (fft[None, :] - pts[:-2, None]) / (pts[1:-1] - pts[:-2])[:, None]
    upper = (pts[2:, None] - fft[None, :]) / (pts[2:] - pts[1:-1])[:, None]
    w = np.maximum(0, np.minimum(lower, upper))
    return w * (2.0 / (pts[2:] - pts[:-2]))[:, None]


def mel(pcm: np.ndarray, n_mels: int = 128) -> torch.Tensor:
    x = torch.from_numpy(pcm.astype(np.float64))
    x = torch.cat([x[:1], x[1:] - 0.97 * x[:-1]])
    win = torch.hann_window(400, periodic=False, dtype=torch.float64)
    X = torch.stft(x, n_fft=512, hop_length=160, win_length=400, window=win, center=True, pad_mode="constant",
                   return_complex=True)
    p = X.abs() ** 2
    m = torch.from_numpy(slaney_mel(n_mels)) @ p
    m = torch.log(m + 2.0 ** -24)
    T = pcm.size // 160          # valid frames (NeMo get_seq_len; HF feature_extraction_parakeet.py:263)
    m = m[:, :T]
    mean = m.mean(1, keepdim=True)
    std = torch.sqrt(((m - mean) ** 2).sum(1, keepdim=True) / (T - 1)) + 1e-5
    return ((m - mean) / std).float()


class Weights:
    def __init__(self, model):
        self.m = model

    def __call__(self, tid: int, *shape) -> torch.Tensor:
        return torch.from_numpy(self.m.tensor(tid)).reshape(*shape)


def rel_shift(x: torch.Tensor) -> torch.Tensor:
    """NeMo RelPositionMultiHeadAttention.rel_shift: (h, t, 2t-1) -> aligned scores."""
    h, t1, t2 = x.shape
    x = F.pad(x, (1, 0))
    x = x.view(h, t2 + 1, t1)
    return x[:, 1:].reshape(h, t1, t2)


def encode(model, dims, mel_: torch.Tensor) -> torch.Tensor:
    W = Weights(model)
    C, d, H = dims.sub_ch, dims.d, dims.n_heads
    dk = d // H
    x = mel_.T[None, None]                                              # (1, 1, T, F)
    x = F.relu(F.conv2d(x, W(1, C, 1, 3, 3), W(2, C), stride=2, padding=1))
    x = F.conv2d(x, W(3, C, 1, 3, 3), W(4, C), stride=2, padding=1, groups=C)
    x = F.relu(F.conv2d(x, W(5, C, C, 1, 1), W(6, C)))
    x = F.conv2d(x, W(7, C, 1, 3, 3), W(8, C), stride=2, padding=1, groups=C)
    x = F.relu(F.conv2d(x, W(9, C, C, 1, 1), W(10, C)))
    _, _, T3, F3 = x.shape
    x = x.transpose(1, 2).reshape(T3, C * F3)
    x = F.linear(x, W(11, d, C * F3), W(12, d)) * math.sqrt(d)
    pos = torch.arange(T3 - 1, -T3, -1, dtype=torch.float64)[:, None]
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.float64) * -(math.log(10000.0) / d))
    pe = torch.zeros(2 * T3 - 1, d, dtype=torch.float64)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    pe = pe.float()
    ln = lambda y, b: F.layer_norm(y, (d,), W(b, d), W(b + 1, d), 1e-5)
    for l in range(dims.n_layers):
        b = 1000 + 64 * l
        ffn = lambda y, o: F.linear(F.silu(F.linear(y, W(o, dims.ff, d), W(o + 1, dims.ff))), W(o + 2, d, dims.ff), W(o + 3, d))
        x = x + 0.5 * ffn(ln(x, b + 0), b + 2)
        y = ln(x, b + 6)
        q = F.linear(y, W(b + 8, d, d), W(b + 9, d)).view(T3, H, dk).transpose(0, 1)
        k = F.linear(y, W(b + 10, d, d), W(b + 11, d)).view(T3, H, dk).transpose(0, 1)
        v = F.linear(y, W(b + 12, d, d), W(b + 13, d)).view(T3, H, dk).transpose(0, 1)
        p = F.linear(pe, W(b + 16, d, d)).view(-1, H, dk).transpose(0, 1)
        u_, v_ = W(b + 17, H, 1, dk), W(b + 18, H, 1, dk)
        ac = (q + u_) @ k.transpose(1, 2)
        bd = rel_shift((q + v_) @ p.transpose(1, 2))[:, :, :T3]
        att = torch.softmax((ac + bd) / math.sqrt(dk), -1)
        ctx = (att @ v).transpose(0, 1).reshape(T3, d)
        x = x + F.linear(ctx, W(b + 14, d, d), W(b + 15, d))
        y = ln(x, b + 19)
        y = F.glu(F.linear(y, W(b + 21, 2 * d, d), W(b + 22, 2 * d)), dim=-1)
        y = F.conv1d(y.T[None], W(b + 23, d, 1, dims.conv_k), W(b + 24, d), padding=dims.conv_k // 2, groups=d)
        y = F.batch_norm(y, W(b + 27, d), W(b + 28, d), W(b + 25, d), W(b + 26, d), False, 0.0, 1e-5)
        y = F.silu(y)[0].T
        x = x + F.linear(y, W(b + 29, d, d), W(b + 30, d))
        x = x + 0.5 * ffn(ln(x, b + 31), b + 33)
        x = ln(x, b + 37)
    return x


def tdt_greedy(model, dims, enc: torch.Tensor, max_symbols: int = 10):
    W = Weights(model)
    P, V = dims.pred, dims.n_vocab
    NO = V + 1 + dims.n_dur
    lstm = torch.nn.LSTM(P, P, num_layers=2)
    with torch.no_grad():
        for j in range(2):
            getattr(lstm, f"weight_ih_l{j}").copy_(W(90001 + 4 * j, 4 * P, P))
            getattr(lstm, f"weight_hh_l{j}").copy_(W(90002 + 4 * j, 4 * P, P))
            getattr(lstm, f"bias_ih_l{j}").copy_(W(90003 + 4 * j, 4 * P))
            getattr(lstm, f"bias_hh_l{j}").copy_(W(90004 + 4 * j, 4 * P))
    emb = W(90000, V + 1, P)
    fe = F.linear(enc, W(90009, P, dims.d), W(90010, P))
    wp, bp, wo, bo = W(90011, P, P), W(90012, P), W(90013, NO, P), W(90014, NO)

    def predict(tok, state):
        with torch.no_grad():
            out, state = lstm(emb[tok][None, None], state)
        return F.linear(out[0, 0], wp, bp), state

    gp, state = predict(V, None)
    toks, frames = [], []
    t, at_t, T3 = 0, 0, enc.shape[0]
    while t < T3:
        lg = F.linear(F.relu(fe[t] + gp), wo, bo)
        tk = int(torch.argmax(lg[:V + 1]))
        skip = int(torch.argmax(lg[V + 1:]))
        if tk != V:
            toks.append(tk)
            frames.append(t)
            gp, state = predict(tk, state)
            at_t += 1
        if skip == 0 and (tk == V or at_t >= max_symbols):
            skip = 1
        if skip > 0:
            at_t = 0
        t += skip
    return toks, frames
