"""Independent PyTorch restatement of Silero VAD v4's 16 kHz network (TEST INFRASTRUCTURE).

Pins oracle/silero.py's ONNX interpreter: it shares only the weights (read by name from the
model file), and uses torch's own conv1d / F.pad(reflect) / LSTM cell algebra, written from the
module structure of the silero-vad v4 model (feature_extractor STFT basis, adaptive_normalization,
first_layer + encoder.{3,7,11} depthwise-separable blocks, a 2-layer LSTM, decoder 1x1 conv)."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from oracle import onnx_graph as G


class TorchSilero:
    def __init__(self, path: str):
        g = G.load(path)
        br = g.nodes[1].attrs["then_branch"]                     # sr == 16000
        lstm_br = next(n for n in br.nodes if n.op == "If" and any(x.op == "LSTM" for x in n.attrs["then_branch"].nodes))
        st = lstm_br.attrs["then_branch"]
        t = lambda k: torch.from_numpy(np.asarray({**g.inits, **br.inits, **st.inits}[k], np.float32).copy())
        self.t = t
        lstms = [n for n in st.nodes if n.op == "LSTM"]
        self.lstm = [(t(n.inputs[1])[0], t(n.inputs[2])[0], t(n.inputs[3])[0]) for n in lstms]
        convs = [n for n in br.nodes if n.op == "Conv"]
        self.c = [(t(n.inputs[1]), t(n.inputs[2]) if len(n.inputs) > 2 else None) for n in convs]
        self.h = torch.zeros(2, 64)
        self.cs = torch.zeros(2, 64)

    def prob(self, frame: np.ndarray) -> float:
        c = self.c
        x = torch.from_numpy(np.asarray(frame, np.float32))[None, None]          # [1][1][480]
        x = F.pad(x, (96, 96), mode="reflect")
        ft = F.conv1d(x, c[0][0], stride=64)                                      # [1][258][7]
        mag = torch.sqrt(ft[:, :129] ** 2 + ft[:, 129:] ** 2)
        spect = torch.log(mag * 1048576.0 + 1.0)
        mean = spect.mean(dim=1, keepdim=True)
        mean = F.pad(mean, (3, 3), mode="reflect")
        mean = F.conv1d(mean, c[1][0]).mean(dim=-1, keepdim=True)
        x1 = torch.cat([mag, spect - mean], dim=1)                                # [1][258][7]

        def block(x, dw, pw, proj):
            y = F.relu(F.conv1d(x, dw[0], dw[1], padding=2, groups=x.shape[1]))
            y = F.conv1d(y, pw[0], pw[1])
            r = F.conv1d(x, proj[0], proj[1]) if proj is not None else x
            return F.relu(y + r)

        h = block(x1, c[2], c[3], c[4])
        h = F.relu(F.conv1d(h, c[5][0], c[5][1], stride=2))
        h = block(h, c[6], c[7], c[8])
        h = F.relu(F.conv1d(h, c[9][0], c[9][1], stride=2))
        h = block(h, c[10], c[11], None)
        h = F.relu(F.conv1d(h, c[12][0], c[12][1], stride=2))
        h = block(h, c[13], c[14], c[15])
        h = F.relu(F.conv1d(h, c[16][0], c[16][1]))                              # [1][64][1]
        inp = h[0, :, 0]
        for L, (W, R, B) in enumerate(self.lstm):                                 # ONNX gates i, o, f, c
            z = W @ inp + R @ self.h[L] + B[:256] + B[256:]
            i, o, f, g = torch.sigmoid(z[:64]), torch.sigmoid(z[64:128]), torch.sigmoid(z[128:192]), torch.tanh(z[192:])
            self.cs[L] = f * self.cs[L] + i * g
            self.h[L] = o * torch.tanh(self.cs[L])
            inp = self.h[L]
        y = F.conv1d(F.relu(self.h[1])[None, :, None], c[17][0], c[17][1])
        return float(torch.sigmoid(y).mean())
