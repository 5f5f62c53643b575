"""Minimal ONNX (protobuf wire format) reader/writer for the model files the reference loads.

The reference resolves ``scrfd_10g_bnkps.onnx`` / ``scrfd_2.5g_bnkps.onnx`` and
``arcface_r100.onnx`` (glintr100, or the w600k_r50 fallback) at
face_embedder.py:55-83, 598-606, 729-734 and runs them with onnxruntime/TensorRT.
This build needs only their weights: the graph is decoded here without the `onnx`
package (absent offline) and mapped onto the device programs by onnx_models.py.

Decoded subset of onnx.proto3: ModelProto.graph; GraphProto.{node, initializer, input,
output}; NodeProto.{input, output, name, op_type, attribute}; AttributeProto.{name, f, i,
s, t, floats, ints}; TensorProto.{dims, data_type, float_data, int32_data, int64_data,
double_data, raw_data, name, external_data}. Constant nodes become initializers.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple, Union

import numpy as np

# TensorProto.DataType -> numpy
_DTYPES = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64, 9: np.bool_,
           10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64}
_NP2ONNX = {np.dtype(v): k for k, v in _DTYPES.items()}


@dataclass
class Node:
    op: str
    inputs: List[str]
    outputs: List[str]
    name: str = ""
    attrs: Dict[str, object] = field(default_factory=dict)


@dataclass
class Graph:
    nodes: List[Node]
    inits: Dict[str, np.ndarray]
    inputs: List[str]
    outputs: List[str]
    name: str = ""


# ---------------------------------------------------------------------------
# wire format
# ---------------------------------------------------------------------------
def _varint(buf: memoryview, pos: int) -> Tuple[int, int]:
    shift = 0
    val = 0
    while True:
        b = buf[pos]
        pos += 1
        val |= (b & 0x7F) << shift
        if b < 0x80:
            return val, pos
        shift += 7
        if shift > 70:
            raise ValueError("malformed varint")


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _fields(buf: memoryview):
    """Yield (field_number, wire_type, value) over one message; value is an int for
    varint/fixed fields and a memoryview for length-delimited ones."""
    pos, end = 0, len(buf)
    while pos < end:
        key, pos = _varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = buf[pos:pos + n]
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fno, wt, v


def _packed_varints(v, wt) -> List[int]:
    if wt == 0:
        return [_signed64(v)]
    out, pos = [], 0
    while pos < len(v):
        x, pos = _varint(v, pos)
        out.append(_signed64(x))
    return out


def _str(v) -> str:
    return bytes(v).decode("utf-8")


def _tensor(buf: memoryview, base_dir: Optional[str]) -> Tuple[str, np.ndarray]:
    dims: List[int] = []
    dtype = 1
    name = ""
    raw = None
    floats: List[float] = []
    ints: List[int] = []
    doubles: List[float] = []
    ext: Dict[str, str] = {}
    for fno, wt, v in _fields(buf):
        if fno == 1:
            dims.extend(_packed_varints(v, wt))
        elif fno == 2:
            dtype = v
        elif fno == 4:
            floats.extend(np.frombuffer(bytes(v), "<f4").tolist() if wt == 2 else [struct.unpack("<f", struct.pack("<I", v))[0]])
        elif fno in (5, 7):
            ints.extend(_packed_varints(v, wt))
        elif fno == 8:
            name = _str(v)
        elif fno == 9:
            raw = bytes(v)
        elif fno == 10:
            doubles.extend(np.frombuffer(bytes(v), "<f8").tolist() if wt == 2 else [struct.unpack("<d", struct.pack("<Q", v))[0]])
        elif fno == 13:
            k = val = ""
            for f2, _, v2 in _fields(v):
                if f2 == 1:
                    k = _str(v2)
                elif f2 == 2:
                    val = _str(v2)
            ext[k] = val
    if dtype not in _DTYPES:
        raise ValueError(f"tensor {name!r}: unsupported data type {dtype}")
    dt = np.dtype(_DTYPES[dtype]).newbyteorder("<")
    if ext:
        if base_dir is None:
            raise ValueError(f"tensor {name!r} has external data but the model was not read from a file")
        loc = ext.get("location", "")
        # external data must stay inside the model's directory (the onnx package's own
        # checks, CVE-2022-25882 / CVE-2024-27318): no absolute paths, no escape via '..'
        # or symlinks
        if not loc or os.path.isabs(loc):
            raise ValueError(f"tensor {name!r}: external data location {loc!r} is not a relative path")
        root = os.path.realpath(base_dir)
        path = os.path.realpath(os.path.join(root, loc))
        if os.path.commonpath([root, path]) != root:
            raise ValueError(f"tensor {name!r}: external data location {loc!r} leaves the model directory")
        off = int(ext.get("offset", 0))
        n = int(ext["length"]) if "length" in ext else int(np.prod(dims)) * dt.itemsize
        if off < 0 or n < 0:
            raise ValueError(f"tensor {name!r}: negative external data offset/length")
        with open(path, "rb") as fh:
            fh.seek(off)
            raw = fh.read(n)
        if len(raw) != n:
            raise ValueError(f"tensor {name!r}: external data truncated ({len(raw)} of {n} bytes)")
    if raw is not None:
        arr = np.frombuffer(raw, dt).copy()
    elif dtype in (1,):
        arr = np.asarray(floats, np.float32)
    elif dtype == 11:
        arr = np.asarray(doubles, np.float64)
    elif dtype == 10:   # float16 lives in int32_data as bit patterns
        arr = np.asarray(ints, np.uint16).view(np.float16)
    else:
        arr = np.asarray(ints, dt)
    return name, arr.astype(dt.newbyteorder("="), copy=False).reshape(dims)


def _attr(buf: memoryview, base_dir) -> Tuple[str, object]:
    name = ""
    val: object = None
    floats: List[float] = []
    ints: List[int] = []
    for fno, wt, v in _fields(buf):
        if fno == 1:
            name = _str(v)
        elif fno == 2:
            val = struct.unpack("<f", struct.pack("<I", v))[0]
        elif fno == 3:
            val = _signed64(v)
        elif fno == 4:
            val = bytes(v)
        elif fno == 5:
            val = _tensor(v, base_dir)[1]
        elif fno == 7:
            floats.extend(np.frombuffer(bytes(v), "<f4").tolist() if wt == 2 else [struct.unpack("<f", struct.pack("<I", v))[0]])
        elif fno == 8:
            ints.extend(_packed_varints(v, wt))
    if val is None:
        val = floats if floats else ints
    return name, val


def _node(buf: memoryview, base_dir) -> Node:
    n = Node(op="", inputs=[], outputs=[])
    for fno, _, v in _fields(buf):
        if fno == 1:
            n.inputs.append(_str(v))
        elif fno == 2:
            n.outputs.append(_str(v))
        elif fno == 3:
            n.name = _str(v)
        elif fno == 4:
            n.op = _str(v)
        elif fno == 5:
            k, a = _attr(v, base_dir)
            n.attrs[k] = a
    return n


def _value_info_name(buf: memoryview) -> str:
    for fno, _, v in _fields(buf):
        if fno == 1:
            return _str(v)
    return ""


def read_model(src: Union[str, bytes]) -> Graph:
    """Decode an ONNX model file (or its bytes) into a Graph."""
    base_dir = None
    if isinstance(src, (bytes, bytearray)):
        data = bytes(src)
    else:
        base_dir = os.path.dirname(os.path.abspath(src))
        with open(src, "rb") as fh:
            data = fh.read()
    mv = memoryview(data)
    gbuf = None
    for fno, wt, v in _fields(mv):
        if fno == 7 and wt == 2:
            gbuf = v
    if gbuf is None:
        raise ValueError("not an ONNX model (no graph)")
    g = Graph(nodes=[], inits={}, inputs=[], outputs=[])
    for fno, _, v in _fields(gbuf):
        if fno == 1:
            g.nodes.append(_node(v, base_dir))
        elif fno == 2:
            g.name = _str(v)
        elif fno == 5:
            k, a = _tensor(v, base_dir)
            g.inits[k] = a
        elif fno == 11:
            g.inputs.append(_value_info_name(v))
        elif fno == 12:
            g.outputs.append(_value_info_name(v))
    keep = []
    for n in g.nodes:
        if n.op == "Constant" and "value" in n.attrs:
            g.inits[n.outputs[0]] = n.attrs["value"]
        else:
            keep.append(n)
    g.nodes = keep
    g.inputs = [i for i in g.inputs if i not in g.inits]
    return g


# ---------------------------------------------------------------------------
# writer (used to produce ONNX files in the exporters' layout for the loader's tests)
# ---------------------------------------------------------------------------
def _enc_varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fno: int, wt: int) -> bytes:
    return _enc_varint((fno << 3) | wt)


def _ld(fno: int, payload: bytes) -> bytes:
    return _key(fno, 2) + _enc_varint(len(payload)) + payload


def _enc_tensor(name: str, arr: np.ndarray) -> bytes:
    arr = np.ascontiguousarray(arr)
    if arr.dtype not in _NP2ONNX:
        raise ValueError(f"dtype {arr.dtype} not encodable")
    out = b"".join(_key(1, 0) + _enc_varint(int(d)) for d in arr.shape)
    out += _key(2, 0) + _enc_varint(_NP2ONNX[arr.dtype])
    out += _ld(8, name.encode())
    out += _ld(9, arr.astype(arr.dtype.newbyteorder("<"), copy=False).tobytes())
    return out


def _enc_attr(name: str, v) -> bytes:
    out = _ld(1, name.encode())
    if isinstance(v, float):
        return out + _key(2, 5) + struct.pack("<f", v) + _key(20, 0) + _enc_varint(1)
    if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
        return out + _key(3, 0) + _enc_varint(int(v)) + _key(20, 0) + _enc_varint(2)
    if isinstance(v, (bytes, str)):
        return out + _ld(4, v.encode() if isinstance(v, str) else v) + _key(20, 0) + _enc_varint(3)
    if isinstance(v, np.ndarray):
        return out + _ld(5, _enc_tensor("", v)) + _key(20, 0) + _enc_varint(4)
    v = list(v)
    if v and isinstance(v[0], float):
        return out + _ld(7, np.asarray(v, "<f4").tobytes()) + _key(20, 0) + _enc_varint(6)
    return out + _ld(8, b"".join(_enc_varint(int(x)) for x in v)) + _key(20, 0) + _enc_varint(7)


def write_model(path: Optional[str], g: Graph, opset: int = 11, producer: str = "pytorch") -> bytes:
    """Encode `g` as an ONNX ModelProto (ir_version 6); writes it to `path` when given."""
    gb = b""
    for n in g.nodes:
        nb = b"".join(_ld(1, s.encode()) for s in n.inputs) + b"".join(_ld(2, s.encode()) for s in n.outputs)
        nb += _ld(3, (n.name or n.outputs[0]).encode()) + _ld(4, n.op.encode())
        nb += b"".join(_ld(5, _enc_attr(k, v)) for k, v in n.attrs.items())
        gb += _ld(1, nb)
    gb += _ld(2, (g.name or "graph").encode())
    gb += b"".join(_ld(5, _enc_tensor(k, v)) for k, v in g.inits.items())
    gb += b"".join(_ld(11, _ld(1, s.encode())) for s in g.inputs)
    gb += b"".join(_ld(12, _ld(1, s.encode())) for s in g.outputs)
    mb = _key(1, 0) + _enc_varint(6) + _ld(2, producer.encode())
    mb += _ld(8, _ld(1, b"") + _key(2, 0) + _enc_varint(opset))
    mb += _ld(7, gb)
    if path:
        with open(path, "wb") as fh:
            fh.write(mb)
    return mb
