"""Minimal protobuf wire-format codec for the ONNX schema.

Neither ``onnx`` nor ``onnxruntime`` exist in this environment, so ONNX
``ModelProto`` files are read (and written, for our own synthetic models)
with a small schema-driven codec. The schema tables below list the ONNX IR
field numbers; unknown fields are skipped on decode. Messages decode into
plain ``Message`` objects (attribute access, repeated fields are lists).

Reference: the reference parses models with the ``onnx-protobuf`` Java
bindings (deep-learning/.../onnx/ONNXUtils.scala:267-370) and hands the bytes
to ONNX Runtime (ONNXRuntime.scala:25-44).
"""
from __future__ import annotations

import struct
from typing import Any, Dict, List, Tuple

import numpy as np

# field kinds
VARINT, SINT, FLOAT, DOUBLE, STRING, BYTES, MSG, PFLOAT, PDOUBLE, PINT, FIXED64 = range(11)

# name -> {field_number: (attr, kind, repeated, message_name|None)}
SCHEMA: Dict[str, Dict[int, Tuple[str, int, bool, Any]]] = {
    "ModelProto": {
        1: ("ir_version", VARINT, False, None),
        8: ("opset_import", MSG, True, "OperatorSetIdProto"),
        2: ("producer_name", STRING, False, None),
        3: ("producer_version", STRING, False, None),
        4: ("domain", STRING, False, None),
        5: ("model_version", VARINT, False, None),
        6: ("doc_string", STRING, False, None),
        7: ("graph", MSG, False, "GraphProto"),
        14: ("metadata_props", MSG, True, "StringStringEntryProto"),
        25: ("functions", MSG, True, "FunctionProto"),
    },
    "OperatorSetIdProto": {1: ("domain", STRING, False, None), 2: ("version", VARINT, False, None)},
    "StringStringEntryProto": {1: ("key", STRING, False, None), 2: ("value", STRING, False, None)},
    "GraphProto": {
        1: ("node", MSG, True, "NodeProto"),
        2: ("name", STRING, False, None),
        5: ("initializer", MSG, True, "TensorProto"),
        10: ("doc_string", STRING, False, None),
        11: ("input", MSG, True, "ValueInfoProto"),
        12: ("output", MSG, True, "ValueInfoProto"),
        13: ("value_info", MSG, True, "ValueInfoProto"),
    },
    "FunctionProto": {
        1: ("name", STRING, False, None),
        4: ("input", STRING, True, None),
        5: ("output", STRING, True, None),
        6: ("attribute", STRING, True, None),
        7: ("node", MSG, True, "NodeProto"),
        8: ("doc_string", STRING, False, None),
        9: ("opset_import", MSG, True, "OperatorSetIdProto"),
        10: ("domain", STRING, False, None),
    },
    "NodeProto": {
        1: ("input", STRING, True, None),
        2: ("output", STRING, True, None),
        3: ("name", STRING, False, None),
        4: ("op_type", STRING, False, None),
        7: ("domain", STRING, False, None),
        5: ("attribute", MSG, True, "AttributeProto"),
        6: ("doc_string", STRING, False, None),
    },
    "AttributeProto": {
        1: ("name", STRING, False, None),
        21: ("ref_attr_name", STRING, False, None),
        13: ("doc_string", STRING, False, None),
        20: ("type", VARINT, False, None),
        2: ("f", FLOAT, False, None),
        3: ("i", SINT, False, None),
        4: ("s", BYTES, False, None),
        5: ("t", MSG, False, "TensorProto"),
        6: ("g", MSG, False, "GraphProto"),
        7: ("floats", PFLOAT, True, None),
        8: ("ints", PINT, True, None),
        9: ("strings", BYTES, True, None),
        10: ("tensors", MSG, True, "TensorProto"),
        11: ("graphs", MSG, True, "GraphProto"),
    },
    "TensorProto": {
        1: ("dims", PINT, True, None),
        2: ("data_type", VARINT, False, None),
        4: ("float_data", PFLOAT, True, None),
        5: ("int32_data", PINT, True, None),
        6: ("string_data", BYTES, True, None),
        7: ("int64_data", PINT, True, None),
        8: ("name", STRING, False, None),
        12: ("doc_string", STRING, False, None),
        9: ("raw_data", BYTES, False, None),
        10: ("double_data", PDOUBLE, True, None),
        11: ("uint64_data", PINT, True, None),
        14: ("data_location", VARINT, False, None),
    },
    "ValueInfoProto": {
        1: ("name", STRING, False, None),
        2: ("type", MSG, False, "TypeProto"),
        3: ("doc_string", STRING, False, None),
    },
    "TypeProto": {
        1: ("tensor_type", MSG, False, "TypeProto.Tensor"),
        4: ("sequence_type", MSG, False, "TypeProto.Sequence"),
        5: ("map_type", MSG, False, "TypeProto.Map"),
        6: ("denotation", STRING, False, None),
    },
    "TypeProto.Tensor": {1: ("elem_type", VARINT, False, None), 2: ("shape", MSG, False, "TensorShapeProto")},
    "TypeProto.Sequence": {1: ("elem_type", MSG, False, "TypeProto")},
    "TypeProto.Map": {1: ("key_type", VARINT, False, None), 2: ("value_type", MSG, False, "TypeProto")},
    "TensorShapeProto": {1: ("dim", MSG, True, "TensorShapeProto.Dimension")},
    "TensorShapeProto.Dimension": {
        1: ("dim_value", SINT, False, None),
        2: ("dim_param", STRING, False, None),
        3: ("denotation", STRING, False, None),
    },
}

# TensorProto.DataType
UNDEFINED, FLOAT32, UINT8, INT8, UINT16, INT16, INT32, INT64, STRING_T, BOOL, FLOAT16, DOUBLE_T, UINT32, UINT64 = \
    range(14)
BFLOAT16 = 16
NP_OF = {FLOAT32: np.float32, UINT8: np.uint8, INT8: np.int8, UINT16: np.uint16, INT16: np.int16, INT32: np.int32,
         INT64: np.int64, BOOL: np.bool_, FLOAT16: np.float16, DOUBLE_T: np.float64, UINT32: np.uint32,
         UINT64: np.uint64, STRING_T: object}
ONNX_OF = {np.dtype(v): k for k, v in NP_OF.items() if v is not object}

# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_GRAPH, A_FLOATS, A_INTS, A_STRINGS, A_TENSORS, A_GRAPHS = range(1, 11)


class Message:
    """Decoded protobuf message: unset scalars read as their proto3 defaults."""

    __slots__ = ("_type", "__dict__")

    def __init__(self, type_name: str, **fields):
        self._type = type_name
        for num, (attr, kind, rep, sub) in SCHEMA[type_name].items():
            if rep:
                setattr(self, attr, [])
            elif kind == MSG:
                setattr(self, attr, None)
            elif kind in (STRING,):
                setattr(self, attr, "")
            elif kind == BYTES:
                setattr(self, attr, b"")
            elif kind in (FLOAT, DOUBLE):
                setattr(self, attr, 0.0)
            else:
                setattr(self, attr, 0)
        for k, v in fields.items():
            setattr(self, k, v)

    def HasField(self, name: str) -> bool:  # noqa: N802
        v = getattr(self, name)
        return v is not None and v != "" and v != b"" and v != [] and v != 0

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        keys = [a for a, *_ in SCHEMA[self._type].values() if self.HasField(a)]
        return f"{self._type}({', '.join(keys)})"


# ------------------------------------------------------------------ decode
def _varint(buf: memoryview, pos: int) -> Tuple[int, int]:
    result = 0
    shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if b < 0x80:
            return result, pos
        shift += 7


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _packed_varints(data: memoryview) -> List[int]:
    out = []
    pos, n = 0, len(data)
    while pos < n:
        v, pos = _varint(data, pos)
        out.append(_signed64(v))
    return out


def decode(type_name: str, data) -> Message:
    buf = memoryview(data)
    schema = SCHEMA[type_name]
    msg = Message(type_name)
    pos, n = 0, len(buf)
    while pos < n:
        key, pos = _varint(buf, pos)
        fnum, wt = key >> 3, key & 7
        if wt == 0:
            val, pos = _varint(buf, pos)
            payload = None
        elif wt == 1:
            val = bytes(buf[pos:pos + 8])
            pos += 8
            payload = None
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            payload = buf[pos:pos + ln]
            pos += ln
            val = None
        elif wt == 5:
            val = bytes(buf[pos:pos + 4])
            pos += 4
            payload = None
        else:
            raise ValueError(f"unsupported wire type {wt} in {type_name}")
        spec = schema.get(fnum)
        if spec is None:
            continue
        attr, kind, rep, sub = spec
        if kind == MSG:
            v = decode(sub, payload)
        elif kind == STRING:
            v = bytes(payload).decode("utf-8")
        elif kind == BYTES:
            v = bytes(payload)
        elif kind in (VARINT, SINT):
            v = _signed64(val) if kind == SINT else val
        elif kind == FLOAT:
            v = struct.unpack("<f", val)[0]
        elif kind == DOUBLE:
            v = struct.unpack("<d", val)[0]
        elif kind == PFLOAT:
            if payload is not None:
                getattr(msg, attr).extend(np.frombuffer(bytes(payload), dtype="<f4").tolist())
                continue
            v = struct.unpack("<f", val)[0]
        elif kind == PDOUBLE:
            if payload is not None:
                getattr(msg, attr).extend(np.frombuffer(bytes(payload), dtype="<f8").tolist())
                continue
            v = struct.unpack("<d", val)[0]
        elif kind == PINT:
            if payload is not None:
                getattr(msg, attr).extend(_packed_varints(payload))
                continue
            v = _signed64(val)
        else:  # pragma: no cover
            raise ValueError(kind)
        if rep:
            getattr(msg, attr).append(v)
        else:
            setattr(msg, attr, v)
    return msg


def load_model(data: bytes) -> Message:
    return decode("ModelProto", data)


# ------------------------------------------------------------------ encode
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


def _key(fnum: int, wt: int) -> bytes:
    return _enc_varint((fnum << 3) | wt)


def encode(msg: Message) -> bytes:
    out = bytearray()
    for fnum, (attr, kind, rep, sub) in sorted(SCHEMA[msg._type].items()):
        v = getattr(msg, attr)
        vals = v if rep else [v]
        if rep and not v:
            continue
        if kind in (PFLOAT, PDOUBLE, PINT):
            if kind == PFLOAT:
                payload = np.asarray(vals, dtype="<f4").tobytes()
            elif kind == PDOUBLE:
                payload = np.asarray(vals, dtype="<f8").tobytes()
            else:
                payload = b"".join(_enc_varint(int(x)) for x in vals)
            out += _key(fnum, 2) + _enc_varint(len(payload)) + payload
            continue
        for x in vals:
            # unset / default-valued optional scalars are omitted (decode restores the default)
            if not rep and (x is None or (kind != MSG and not x)):
                continue
            if kind == MSG:
                payload = encode(x)
                out += _key(fnum, 2) + _enc_varint(len(payload)) + payload
            elif kind in (STRING, BYTES):
                payload = x.encode("utf-8") if isinstance(x, str) else bytes(x)
                out += _key(fnum, 2) + _enc_varint(len(payload)) + payload
            elif kind in (VARINT, SINT):
                out += _key(fnum, 0) + _enc_varint(int(x))
            elif kind == FLOAT:
                out += _key(fnum, 5) + struct.pack("<f", float(x))
            elif kind == DOUBLE:
                out += _key(fnum, 1) + struct.pack("<d", float(x))
    return bytes(out)


# ------------------------------------------------------------------ tensors
def tensor_to_numpy(t: Message) -> np.ndarray:
    dims = [int(d) for d in t.dims]
    dt = t.data_type
    if dt == STRING_T:
        arr = np.array([s.decode("utf-8") for s in t.string_data], dtype=object)
        return arr.reshape(dims)
    if dt == BFLOAT16:
        if t.raw_data:
            u = np.frombuffer(t.raw_data, dtype="<u2").astype(np.uint32) << 16
        else:
            u = np.asarray(t.int32_data, dtype=np.uint32) << 16
        return u.view(np.float32).reshape(dims)
    np_dt = np.dtype(NP_OF[dt])
    if t.raw_data:
        return np.frombuffer(t.raw_data, dtype=np_dt.newbyteorder("<")).astype(np_dt).reshape(dims)
    if dt == FLOAT32:
        src = t.float_data
    elif dt == DOUBLE_T:
        src = t.double_data
    elif dt in (INT64,):
        src = t.int64_data
    elif dt in (UINT32, UINT64):
        src = t.uint64_data
    elif dt == FLOAT16:
        return np.asarray(t.int32_data, dtype=np.uint16).view(np.float16).reshape(dims)
    else:
        src = t.int32_data
    return np.asarray(src, dtype=np_dt).reshape(dims)


def numpy_to_tensor(arr, name: str = "") -> Message:
    a = np.asarray(arr)
    t = Message("TensorProto", name=name, dims=list(a.shape))
    if a.dtype == object or a.dtype.kind in "US":
        t.data_type = STRING_T
        t.string_data = [str(x).encode("utf-8") for x in a.ravel()]
        return t
    t.data_type = ONNX_OF[a.dtype]
    t.raw_data = np.ascontiguousarray(a).astype(a.dtype.newbyteorder("<")).tobytes()
    return t
