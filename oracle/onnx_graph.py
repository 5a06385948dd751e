"""A minimal ONNX model reader in pure Python (TEST INFRASTRUCTURE, oracle side).

Decodes the protobuf wire format of onnx/onnx.proto's ModelProto -> GraphProto -> NodeProto /
TensorProto / AttributeProto by hand (the onnx package is not installed).  It is independent of
the product's C++ reader (spittle_amd/csrc/onnx_pb.cpp).  Nothing in a file is executed: tensors
become numpy arrays, nodes become (op_type, inputs, outputs, attributes) records, subgraphs (If
branches) are parsed the same way.  Used on the Silero VAD model that ships in the reference
(/root/reference/src-tauri/resources/models/silero_vad_v4.onnx) to generate golden fixtures.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

import numpy as np

_NP = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64, 9: np.bool_, 10: np.float16,
       11: np.float64, 12: np.uint32, 13: np.uint64}


def _varint(b: bytes, i: int):
    v, s = 0, 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        if not x & 0x80:
            return v, i
        s += 7


def _fields(b: bytes):
    i, n = 0, len(b)
    while i < n:
        tag, i = _varint(b, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        elif wt == 2:
            ln, i = _varint(b, i)
            v = b[i:i + ln]
            i += ln
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield f, wt, v


def _packed_varints(wt, v):
    if wt == 0:
        return [v]
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x)
    return out


def _signed(x: int) -> int:
    return x - (1 << 64) if x >= 1 << 63 else x


@dataclass
class Node:
    op: str
    name: str
    inputs: list
    outputs: list
    attrs: dict = field(default_factory=dict)


@dataclass
class Graph:
    nodes: list
    inits: dict
    inputs: list
    outputs: list


def tensor(b: bytes) -> tuple[str, np.ndarray]:
    dims, dt, name, raw, f32, i64, f64 = [], 1, "", None, [], [], []
    for f, wt, v in _fields(b):
        if f == 1:
            dims += [_signed(x) for x in _packed_varints(wt, v)]
        elif f == 2:
            dt = v
        elif f == 4:
            f32 += list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2 else [struct.unpack("<f", v)[0]]
        elif f in (5, 7):
            i64 += [_signed(x) for x in _packed_varints(wt, v)]
        elif f == 8:
            name = v.decode()
        elif f == 9:
            raw = v
        elif f == 10:
            f64 += list(struct.unpack(f"<{len(v) // 8}d", v)) if wt == 2 else [struct.unpack("<d", v)[0]]
    npdt = _NP[dt]
    if raw is not None:
        a = np.frombuffer(raw, dtype=npdt).copy()
    elif dt == 1:
        a = np.array(f32, np.float32)
    elif dt == 11:
        a = np.array(f64, np.float64)
    else:
        a = np.array(i64).astype(npdt)
    return name, a.reshape(dims) if dims else a.reshape(())


def _attr(b: bytes):
    name, val, ints, floats, typ = "", None, [], [], 0
    for f, wt, v in _fields(b):
        if f == 1:
            name = v.decode()
        elif f == 2:
            val = struct.unpack("<f", v)[0]
        elif f == 3:
            val = _signed(v)
        elif f == 4:
            val = v
        elif f == 5:
            val = tensor(v)[1]
        elif f == 6:
            val = graph(v)
        elif f == 7:
            floats += list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2 else [struct.unpack("<f", v)[0]]
        elif f == 8:
            ints += [_signed(x) for x in _packed_varints(wt, v)]
        elif f == 20:
            typ = v
    if typ == 7 or (val is None and ints):
        val = ints
    elif typ == 6 or (val is None and floats):
        val = floats
    return name, val


def _value_info_name(b: bytes) -> str:
    for f, _, v in _fields(b):
        if f == 1:
            return v.decode()
    return ""


def graph(b: bytes) -> Graph:
    nodes, inits, ins, outs = [], {}, [], []
    for f, _, v in _fields(b):
        if f == 1:
            ni, no, nm, op, at = [], [], "", "", {}
            for g, _, w in _fields(v):
                if g == 1:
                    ni.append(w.decode())
                elif g == 2:
                    no.append(w.decode())
                elif g == 3:
                    nm = w.decode()
                elif g == 4:
                    op = w.decode()
                elif g == 5:
                    k, x = _attr(w)
                    at[k] = x
            nodes.append(Node(op, nm, ni, no, at))
        elif f == 5:
            k, a = tensor(v)
            inits[k] = a
        elif f == 11:
            ins.append(_value_info_name(v))
        elif f == 12:
            outs.append(_value_info_name(v))
    return Graph(nodes, inits, ins, outs)


def load(path: str) -> Graph:
    with open(path, "rb") as fh:
        b = fh.read()
    for f, _, v in _fields(b):
        if f == 7:
            return graph(v)
    raise ValueError(f"{path}: no graph")
