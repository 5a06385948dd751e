"""Writes a Parakeet-V3 model directory shaped like the one the app downloads (TEST INFRASTRUCTURE).

The catalog's parakeet-tdt-0.6b-v3-int8 (/root/reference/src-tauri/resources/model_catalog.json:
229-241) is the onnx-asr export of NeMo's model that transcribe-rs 0.2.3 loads [upstream,
recalled]: encoder-model.int8.onnx, decoder_joint-model.int8.onnx, nemo128.onnx, vocab.txt.  No
such file exists offline, so this writer produces the same structure from the oracle's tensors, as
torch.onnx + ONNX Runtime's quantize_dynamic lay it out:

* node names carry module paths ("/layers.0/feed_forward1/linear1/MatMul_quant");
* Linear weights are transposed [K][N] constants with anonymous names ("onnx::MatMul_<n>"),
  quantised: "<w>_quantized" (int8 symmetric, or uint8 with a zero point) + "<w>_scale" +
  "<w>_zero_point", consumed by DynamicQuantizeLinear -> MatMulInteger, the bias added by an Add;
* parameters used as they are keep their state-dict names (biases, LayerNorm, pos_bias_u / v,
  BatchNorm statistics, the depthwise and strided convolutions);
* the prediction network's LSTM is two ONNX LSTM nodes (gates i, o, f, c; W [1][4H][in]) or, in
  the int8 export, DynamicQuantizeLSTM (W [1][in][4H] quantised);
* vocab.txt holds "<piece> <id>" lines, the blank last.

Variants exercise the loader's other paths: per-channel uint8 scales, BatchNorm folded into the
depthwise convolution, anonymous pos_bias initializers (matched by order), the QDQ form
(DequantizeLinear nodes) and external data.

The protobuf wire format is written by hand (onnx is not installed); field numbers follow
onnx/onnx.proto.  `expected` returns what a loader must recover: every tensor id's f32 values in
NeMo's layout (dequantised exactly as (q - zero_point) * scale in f32)."""
from __future__ import annotations

import os
import struct

import numpy as np

FLOAT, UINT8, INT8 = 1, 2, 3


# ------------------------------------------------------------------ protobuf wire format
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _ld(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _str(field: int, s: str) -> bytes:
    return _ld(field, s.encode())


def _int(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(v)


def tensor_proto(name: str, arr: np.ndarray, dtype: int, external=None) -> bytes:
    b = b"".join(_int(1, int(d)) for d in arr.shape)      # dims (unpacked, proto2 style)
    b += _int(2, dtype)
    b += _str(8, name)
    raw = np.ascontiguousarray(arr).tobytes()
    if external is None:
        b += _ld(9, raw)
    else:
        fname, fh = external
        off = fh.tell()
        fh.write(raw)
        for k, v in (("location", fname), ("offset", str(off)), ("length", str(len(raw)))):
            b += _ld(13, _str(1, k) + _str(2, v))
        b += _int(14, 1)
    return b


def attr_int(name: str, v: int) -> bytes:
    return _str(1, name) + _int(3, v) + _int(20, 2)


def node_proto(op: str, name: str, inputs, outputs, attrs=(), domain="") -> bytes:
    b = b"".join(_str(1, i) for i in inputs) + b"".join(_str(2, o) for o in outputs)
    b += _str(3, name) + _str(4, op)
    b += b"".join(_ld(5, a) for a in attrs)
    if domain:
        b += _str(7, domain)
    return b


def model_proto(nodes, inits) -> bytes:
    g = b"".join(_ld(1, n) for n in nodes) + _str(2, "main_graph") + b"".join(_ld(5, t) for t in inits)
    return _int(1, 8) + _str(2, "pytorch") + _ld(8, _str(1, "") + _int(2, 17)) + _ld(7, g)


# ------------------------------------------------------------------ quantisation (ORT dynamic)
def quantize(w: np.ndarray, mode: str, axis: int):
    """-> (q, scale, zero_point, dequantised f32) for mode 'int8' (symmetric, per tensor) or
    'uint8pc' (asymmetric, per channel along axis)."""
    w = w.astype(np.float32)
    if mode == "int8":
        s = np.float32(max(float(np.abs(w).max()), 1e-12) / 127.0)
        q = np.clip(np.rint(w / s), -127, 127).astype(np.int8)
        zp = np.zeros((), np.int8)
        deq = (q.astype(np.float32) - np.float32(0)) * s
        return q, np.array(s, np.float32), zp, deq
    red = tuple(i for i in range(w.ndim) if i != axis)
    lo = np.minimum(w.min(axis=red), 0).astype(np.float32)
    hi = np.maximum(w.max(axis=red), 0).astype(np.float32)
    s = np.maximum((hi - lo) / np.float32(255), np.float32(1e-12)).astype(np.float32)
    zp = np.clip(np.rint(-lo / s), 0, 255).astype(np.uint8)
    shape = [1] * w.ndim
    shape[axis] = -1
    q = np.clip(np.rint(w / s.reshape(shape)) + zp.reshape(shape), 0, 255).astype(np.uint8)
    deq = (q.astype(np.float32) - zp.astype(np.float32).reshape(shape)) * s.reshape(shape)
    return q, s, zp, deq


class _Graph:
    def __init__(self, quant: str, qdq: bool = False, external=None):
        self.nodes, self.inits, self.quant, self.qdq, self.ext = [], [], quant, qdq, external
        self.n = 100

    def anon(self, op: str) -> str:
        self.n += 1
        return f"onnx::{op}_{self.n}"

    def init(self, name, arr, dtype=FLOAT):
        ext = self.ext if (self.ext is not None and arr.size >= 1024) else None
        self.inits.append(tensor_proto(name, arr, dtype, ext))

    def qinit(self, name, w, axis):
        """a quantised weight (initializer triple, or QDQ: DequantizeLinear node); -> (input name
        for the consuming node, dequantised f32)"""
        q, s, zp, deq = quantize(w, self.quant, axis)
        dt = INT8 if q.dtype == np.int8 else UINT8
        self.init(name + "_quantized", q, dt)
        self.init(name + "_scale", s)
        self.init(name + "_zero_point", zp, dt)
        if self.qdq:
            out = name + "_dequantized"
            self.nodes.append(node_proto("DequantizeLinear", name + "_DequantizeLinear",
                                         [name + "_quantized", name + "_scale", name + "_zero_point"], [out]))
            return out, deq
        return name + "_quantized", deq

    def linear(self, path, W, b, x):
        """torch Linear (W [N][K]) as MatMul(Integer) on W^T [K][N] (+ Add); -> dequantised W [N][K]"""
        wt = np.ascontiguousarray(W.T)
        nm = self.anon("MatMul")
        if self.quant:
            inp, deq = self.qinit(nm, wt, axis=1)
            if self.qdq:
                self.nodes.append(node_proto("MatMul", f"/{path}/MatMul", [x, inp], [f"/{path}/MatMul_output_0"]))
            else:
                self.nodes.append(node_proto("DynamicQuantizeLinear", f"/{path}/MatMul_quant_dq", [x],
                                             [x + "_q", x + "_s", x + "_z"]))
                self.nodes.append(node_proto("MatMulInteger", f"/{path}/MatMul_quant",
                                             [x + "_q", inp, x + "_z", nm + "_zero_point"],
                                             [f"/{path}/MatMul_output_0"]))
            Wd = np.ascontiguousarray(deq.T)
        else:
            self.init(nm, wt)
            self.nodes.append(node_proto("MatMul", f"/{path}/MatMul", [x, nm], [f"/{path}/MatMul_output_0"]))
            Wd = W.astype(np.float32)
        y = f"/{path}/MatMul_output_0"
        if b is not None:
            bn = path.replace("/", ".") + ".bias"
            self.init(bn, b.astype(np.float32))
            self.nodes.append(node_proto("Add", f"/{path}/Add", [bn, y], [f"/{path}/Add_output_0"]))
            y = f"/{path}/Add_output_0"
        return Wd, y

    def conv(self, path, W, b, x, group=1, quant=False):
        pname = path.replace("/", ".")
        if quant and self.quant:
            inp, deq = self.qinit(pname + ".weight", W, axis=0)
            op = "Conv" if self.qdq else "ConvInteger"
            self.nodes.append(node_proto(op, f"/{path}/Conv_quant", [x, inp], [f"/{path}/Conv_output_0"],
                                         [attr_int("group", group)]))
            self.init(pname + ".bias", b.astype(np.float32))
            self.nodes.append(node_proto("Add", f"/{path}/Add", [f"/{path}/Conv_output_0", pname + ".bias"],
                                         [f"/{path}/Add_output_0"]))
            return deq.astype(np.float32)
        self.init(pname + ".weight", W.astype(np.float32))
        self.init(pname + ".bias", b.astype(np.float32))
        self.nodes.append(node_proto("Conv", f"/{path}/Conv", [x, pname + ".weight", pname + ".bias"],
                                     [f"/{path}/Conv_output_0"], [attr_int("group", group)]))
        return W.astype(np.float32)

    def layernorm(self, path, w, b, x):
        pname = path.replace("/", ".")
        self.init(pname + ".weight", w.astype(np.float32))
        self.init(pname + ".bias", b.astype(np.float32))
        self.nodes.append(node_proto("LayerNormalization", f"/{path}/LayerNormalization",
                                     [x, pname + ".weight", pname + ".bias"], [f"/{path}/LN_output_0"],
                                     [attr_int("axis", -1)]))

    def write(self, path):
        with open(path, "wb") as f:
            f.write(model_proto(self.nodes, self.inits))


def _w(model, tid, *shape):
    return model.tensor(tid).reshape(*shape)


LSTM_PERM = [0, 3, 1, 2]  # ONNX gate block g <- torch block LSTM_PERM[g]: (i, o, f, c) from (i, f, g, o)


def write_dir(path: str, model, dims, quant: str = "int8", fold_bn: bool = False, anon_pos_bias: bool = False,
              qdq: bool = False, external: bool = False, lstm_quant: bool = True, faults=()) -> dict:
    """Write the model directory; return {tensor id: f32 values (NeMo layout)} a loader must recover.
    faults (negative tests of the loader): "transposed_ff1" writes layer 0's feed_forward1.linear1
    MatMul operand as W instead of W^T; "third_pos_bias" adds a third unnamed [H][dk] Add in layer
    0's self_attn; "conflicting_q" adds a second linear_q MatMul with a different weight."""
    os.makedirs(path, exist_ok=True)
    d, C, H, L, ff, K, P, V = dims.d, dims.sub_ch, dims.n_heads, dims.n_layers, dims.ff, dims.conv_k, dims.pred, dims.n_vocab
    F3 = dims.n_mels
    for _ in range(3):
        F3 = (F3 - 1) // 2 + 1
    exp = {}
    suffix = ".int8.onnx" if quant else ".onnx"
    ext_name = "encoder-model" + suffix.replace(".onnx", ".onnx.data") if external else None
    fh = open(os.path.join(path, ext_name), "wb") if external else None
    g = _Graph(quant, qdq, (ext_name, fh) if external else None)
    x = "audio_signal"
    for tid, nm, shape, grp, q in ((1, "pre_encode/conv/conv.0", (C, 1, 3, 3), 1, False),
                                    (3, "pre_encode/conv/conv.2", (C, 1, 3, 3), C, False),
                                    (5, "pre_encode/conv/conv.3", (C, C, 1, 1), 1, True),
                                    (7, "pre_encode/conv/conv.5", (C, 1, 3, 3), C, False),
                                    (9, "pre_encode/conv/conv.6", (C, C, 1, 1), 1, True)):
        exp[tid] = g.conv(nm, _w(model, tid, *shape), model.tensor(tid + 1), x, grp, q)
        exp[tid + 1] = model.tensor(tid + 1)
    W, x = g.linear("pre_encode/out", _w(model, 11, d, C * F3), model.tensor(12), x)
    exp[11], exp[12] = W, model.tensor(12)
    for l in range(L):
        b = 1000 + 64 * l
        p = f"layers.{l}"
        for off, nm in ((0, "norm_feed_forward1"), (6, "norm_self_att"), (19, "norm_conv"), (31, "norm_feed_forward2"),
                        (37, "norm_out")):
            g.layernorm(f"{p}/{nm}", model.tensor(b + off), model.tensor(b + off + 1), x)
            exp[b + off], exp[b + off + 1] = model.tensor(b + off), model.tensor(b + off + 1)
        for off, nm, n_, k_ in ((2, "feed_forward1/linear1", ff, d), (4, "feed_forward1/linear2", d, ff),
                                (8, "self_attn/linear_q", d, d), (10, "self_attn/linear_k", d, d),
                                (12, "self_attn/linear_v", d, d), (14, "self_attn/linear_out", d, d),
                                (33, "feed_forward2/linear1", ff, d), (35, "feed_forward2/linear2", d, ff)):
            Wm = _w(model, b + off, n_, k_)
            if l == 0 and off == 2 and "transposed_ff1" in faults:
                Wm = np.ascontiguousarray(Wm.T)
            W, _ = g.linear(f"{p}/{nm}", Wm, model.tensor(b + off + 1), x)
            exp[b + off], exp[b + off + 1] = W, model.tensor(b + off + 1)
            if l == 0 and off == 8 and "conflicting_q" in faults:
                g.linear(f"{p}/{nm}", Wm * 2, model.tensor(b + off + 1), x)
        W, _ = g.linear(f"{p}/self_attn/linear_pos", _w(model, b + 16, d, d), None, "pos_emb")
        exp[b + 16] = W
        for k, (off, suf) in enumerate(((17, "u"), (18, "v"))):
            nm = g.anon("Add") if anon_pos_bias else f"{p}.self_attn.pos_bias_{suf}"
            g.init(nm, _w(model, b + off, H, d // H))
            g.nodes.append(node_proto("Add", f"/{p}/self_attn/Add" + ("" if k == 0 else "_1"), ["q", nm], [f"qb{k}"]))
            exp[b + off] = model.tensor(b + off)
        if l == 0 and "third_pos_bias" in faults:
            nm = g.anon("Add")
            g.init(nm, _w(model, b + 17, H, d // H))
            g.nodes.append(node_proto("Add", f"/{p}/self_attn/Add_2", ["q", nm], ["qb2"]))
        W = g.conv(f"{p}/conv/pointwise_conv1", _w(model, b + 21, 2 * d, d, 1), model.tensor(b + 22), x, 1, True)
        exp[b + 21], exp[b + 22] = W.reshape(-1), model.tensor(b + 22)
        dw, dwb = _w(model, b + 23, d, 1, K), model.tensor(b + 24)
        gam, bet, mu, var = (model.tensor(b + o) for o in (25, 26, 27, 28))
        if fold_bn:  # BatchNorm folded into the depthwise convolution (eval mode)
            sc = (gam / np.sqrt(var + np.float32(1e-5))).astype(np.float32)
            dw = (dw * sc[:, None, None]).astype(np.float32)
            dwb = ((dwb - mu) * sc + bet).astype(np.float32)
            g.conv(f"{p}/conv/depthwise_conv", dw, dwb, x, d)
            exp[b + 23], exp[b + 24] = dw.reshape(-1), dwb
            exp[b + 25], exp[b + 26] = np.ones(d, np.float32), np.zeros(d, np.float32)
            exp[b + 27], exp[b + 28] = np.zeros(d, np.float32), np.full(d, 1 - 1e-5, np.float32)
        else:
            g.conv(f"{p}/conv/depthwise_conv", dw, dwb, x, d)
            exp[b + 23], exp[b + 24] = dw.reshape(-1), dwb
            names = []
            for off, nm in ((25, "weight"), (26, "bias"), (27, "running_mean"), (28, "running_var")):
                names.append(f"{p}.conv.batch_norm.{nm}")
                g.init(names[-1], model.tensor(b + off))
                exp[b + off] = model.tensor(b + off)
            g.nodes.append(node_proto("BatchNormalization", f"/{p}/conv/batch_norm/BatchNormalization", [x] + names, ["bn"]))
        W = g.conv(f"{p}/conv/pointwise_conv2", _w(model, b + 29, d, d, 1), model.tensor(b + 30), x, 1, True)
        exp[b + 29], exp[b + 30] = W.reshape(-1), model.tensor(b + 30)
    g.write(os.path.join(path, "encoder-model" + suffix))
    if fh:
        fh.close()

    # decoder + joint
    g = _Graph(quant, qdq)
    emb = _w(model, 90000, V + 1, P)
    g.init("decoder.prediction.embed.weight", emb)
    g.nodes.append(node_proto("Gather", "/decoder/prediction/embed/Gather", ["decoder.prediction.embed.weight", "targets"], ["e"]))
    exp[90000] = model.tensor(90000)
    for j in range(2):
        wih, whh = _w(model, 90001 + 4 * j, 4 * P, P), _w(model, 90002 + 4 * j, 4 * P, P)
        bih, bhh = model.tensor(90003 + 4 * j), model.tensor(90004 + 4 * j)
        onx = lambda a: np.concatenate([a.reshape(4, P, -1)[LSTM_PERM[k]] for k in range(4)]).reshape(4 * P, -1)
        Wn, Rn = onx(wih)[None], onx(whh)[None]
        Bn = np.concatenate([onx(bih[:, None]).ravel(), onx(bhh[:, None]).ravel()])[None].astype(np.float32)
        nm = f"/decoder/prediction/dec_rnn/lstm/LSTM" + ("" if j == 0 else f"_{j}")
        bname = g.anon("LSTM")
        g.init(bname, Bn)
        if quant and lstm_quant:  # ORT DynamicQuantizeLSTM: W [1][in][4H], R [1][H][4H]
            wq, wd = g.qinit(g.anon("LSTM"), np.ascontiguousarray(Wn[0].T)[None], axis=2)
            rq, rd = g.qinit(g.anon("LSTM"), np.ascontiguousarray(Rn[0].T)[None], axis=2)
            ws, wz = wq.replace("_quantized", "_scale"), wq.replace("_quantized", "_zero_point")
            rs, rz = rq.replace("_quantized", "_scale"), rq.replace("_quantized", "_zero_point")
            g.nodes.append(node_proto("DynamicQuantizeLSTM", nm, ["e", wq, rq, bname, "", "", "", "", ws, wz, rs, rz],
                                      ["y", "yh", "yc"], [attr_int("hidden_size", P)], domain="com.microsoft"))
            Wd, Rd = wd[0].T, rd[0].T
        else:
            wname, rname = g.anon("LSTM"), g.anon("LSTM")
            g.init(wname, Wn.astype(np.float32))
            g.init(rname, Rn.astype(np.float32))
            g.nodes.append(node_proto("LSTM", nm, ["e", wname, rname, bname], ["y", "yh", "yc"],
                                      [attr_int("hidden_size", P)]))
            Wd, Rd = Wn[0], Rn[0]
        back = lambda a: np.concatenate([a.reshape(4, P, -1)[LSTM_PERM.index(k)] for k in range(4)]).reshape(4 * P, -1)
        exp[90001 + 4 * j] = back(np.asarray(Wd, np.float32)).ravel()
        exp[90002 + 4 * j] = back(np.asarray(Rd, np.float32)).ravel()
        exp[90003 + 4 * j], exp[90004 + 4 * j] = bih, bhh
    for tid, nm, shape in ((90009, "joint/enc", (P, d)), (90011, "joint/pred", (P, P)),
                           (90013, "joint/joint_net/joint_net.2", (V + 1 + dims.n_dur, P))):
        W, _ = g.linear(nm, _w(model, tid, *shape), model.tensor(tid + 1), "h")
        exp[tid], exp[tid + 1] = W, model.tensor(tid + 1)
    g.write(os.path.join(path, "decoder_joint-model" + suffix))
    with open(os.path.join(path, "nemo128.onnx"), "wb") as f:  # present in the export; not read
        f.write(model_proto([], []))
    with open(os.path.join(path, "vocab.txt"), "w", encoding="utf-8") as f:
        for i in range(V):
            f.write(("▁w%d" % i if i % 3 == 0 else "p%d" % i) + f" {i}\n")
        f.write(f"<blk> {V}\n")
    return {k: np.asarray(v, np.float32).ravel() for k, v in exp.items()}


def vocab_piece(i: int) -> str:
    return "▁w%d" % i if i % 3 == 0 else "p%d" % i
