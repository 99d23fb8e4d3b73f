"""Pure-Python GraphDef codec (protobuf wire format) for the TF-1.x subset.

There is no protoc here; TensorFrames only needs GraphDef / NodeDef /
AttrValue / TensorProto / TensorShapeProto
(reference: src/main/protobuf/tensorflow/core/framework/graph.proto:14-112,
attr_value.proto:16-60, tensor.proto:13-60, tensor_shape.proto:12-45).
The native runtime has its own C++ decoder (csrc/proto/graphdef.cpp); this
module is what the Python DSL serialises with, plus a reader and a TF-style
text formatter used by the golden tests.
"""
from __future__ import annotations

import struct
import sys
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..utils import dtypes as D

_LITTLE = sys.byteorder == "little"

_DT_ENUM_NAMES = {
    0: "DT_INVALID", 1: "DT_FLOAT", 2: "DT_DOUBLE", 3: "DT_INT32", 4: "DT_UINT8", 5: "DT_INT16",
    6: "DT_INT8", 7: "DT_STRING", 8: "DT_COMPLEX64", 9: "DT_INT64", 10: "DT_BOOL", 14: "DT_BFLOAT16",
    19: "DT_HALF",
}


# ------------------------------------------------------------------ messages
class TensorShapeProto:
    def __init__(self, dims: Optional[List[int]] = None, unknown_rank: bool = False):
        self.dims = list(dims or [])
        self.unknown_rank = unknown_rank

    def __eq__(self, o):
        return isinstance(o, TensorShapeProto) and (self.dims, self.unknown_rank) == (o.dims, o.unknown_rank)

    def __repr__(self):
        return "<unknown>" if self.unknown_rank else f"TensorShapeProto({self.dims})"


class TensorProto:
    def __init__(self, dtype: int, shape: List[int], content: bytes = b"",
                 strings: Optional[List[bytes]] = None):
        self.dtype = dtype
        self.shape = list(shape)
        self.content = content
        self.strings = strings

    @staticmethod
    def from_numpy(arr: np.ndarray, dtype: Optional[int] = None) -> "TensorProto":
        if dtype is None:
            dtype = D.as_dtype(arr.dtype).enum
        if dtype == D.DT_STRING:
            vals = [v if isinstance(v, bytes) else str(v).encode() for v in np.asarray(arr).reshape(-1)]
            return TensorProto(dtype, list(np.shape(arr)), strings=vals)
        a = np.asarray(arr, dtype=D.numpy_dtype(dtype), order="C")
        if a.dtype.byteorder in ("<", "|") or (a.dtype.byteorder == "=" and _LITTLE):
            return TensorProto(dtype, list(a.shape), a.tobytes())  # already little-endian: one copy
        return TensorProto(dtype, list(a.shape), a.astype(a.dtype.newbyteorder("<")).tobytes())

    def to_numpy(self) -> np.ndarray:
        if self.dtype == D.DT_STRING:
            return np.array(self.strings or [], dtype=object).reshape(self.shape)
        npdt = np.dtype(D.numpy_dtype(self.dtype)).newbyteorder("<")
        n = int(np.prod(self.shape)) if self.shape else 1
        return np.frombuffer(self.content, dtype=npdt, count=n).reshape(self.shape).copy()

    def __eq__(self, o):
        return isinstance(o, TensorProto) and (self.dtype, self.shape, self.content, self.strings) == \
            (o.dtype, o.shape, o.content, o.strings)


class AttrValue:
    """kind in {list, s, i, f, b, type, shape, tensor, placeholder, func}."""

    __slots__ = ("kind", "value")

    def __init__(self, kind: str, value):
        self.kind = kind
        self.value = value

    # constructors
    @staticmethod
    def s(v) -> "AttrValue":
        return AttrValue("s", v if isinstance(v, bytes) else str(v).encode())

    @staticmethod
    def i(v) -> "AttrValue":
        return AttrValue("i", int(v))

    @staticmethod
    def f(v) -> "AttrValue":
        return AttrValue("f", float(v))

    @staticmethod
    def b(v) -> "AttrValue":
        return _B_ATTRS[bool(v)]

    @staticmethod
    def type(v) -> "AttrValue":
        # shared immutable instances: graphs rebuilt per iteration create
        # thousands of these (attr values are never mutated in place)
        e = v.enum if isinstance(v, D.DType) else D.as_dtype(v).enum
        a = _TYPE_ATTRS.get(e)
        if a is None:
            a = _TYPE_ATTRS[e] = AttrValue("type", e)
        return a

    @staticmethod
    def shape(dims: Optional[List[int]]) -> "AttrValue":
        if dims is None:
            return AttrValue("shape", TensorShapeProto(unknown_rank=True))
        return AttrValue("shape", TensorShapeProto([-1 if d is None else int(d) for d in dims]))

    @staticmethod
    def tensor(t: TensorProto) -> "AttrValue":
        return AttrValue("tensor", t)

    @staticmethod
    def ilist(vals) -> "AttrValue":
        return AttrValue("list", {"i": [int(v) for v in vals]})

    @staticmethod
    def slist(vals) -> "AttrValue":
        return AttrValue("list", {"s": [v if isinstance(v, bytes) else str(v).encode() for v in vals]})

    @staticmethod
    def tlist(vals) -> "AttrValue":
        return AttrValue("list", {"type": [D.as_dtype(v).enum for v in vals]})

    @staticmethod
    def shapelist(vals) -> "AttrValue":
        return AttrValue("list", {"shape": [TensorShapeProto(unknown_rank=True) if v is None else
                                            TensorShapeProto([-1 if d is None else d for d in v])
                                            for v in vals]})

    def __eq__(self, o):
        return isinstance(o, AttrValue) and self.kind == o.kind and self.value == o.value

    def __repr__(self):
        return f"AttrValue({self.kind}={self.value!r})"


_TYPE_ATTRS: Dict[int, AttrValue] = {}
_B_ATTRS = {False: AttrValue("b", False), True: AttrValue("b", True)}


class NodeDef:
    __slots__ = ("name", "op", "input", "attr", "device")

    def __init__(self, name: str, op: str, input: Optional[List[str]] = None,  # noqa: A002
                 attr: Optional[Dict[str, AttrValue]] = None, device: str = ""):
        self.name = name
        self.op = op
        self.input = list(input or [])
        self.attr = dict(attr or {})
        self.device = device

    @classmethod
    def _make(cls, name: str, op: str, input: List[str], attr: Dict[str, AttrValue]) -> "NodeDef":  # noqa: A002
        """Internal constructor: takes ownership of `input` / `attr` (no copies)."""
        n = cls.__new__(cls)
        n.name, n.op, n.input, n.attr, n.device = name, op, input, attr, ""
        return n

    def __repr__(self):
        return f"NodeDef({self.name!r}, {self.op!r}, inputs={self.input})"


class GraphDef:
    def __init__(self, node: Optional[List[NodeDef]] = None, producer: int = 0):
        self.node = list(node or [])
        self.producer = producer

    def SerializeToString(self) -> bytes:  # noqa: N802 (protobuf naming)
        return serialize_graphdef(self)

    def node_by_name(self, name: str) -> Optional[NodeDef]:
        for n in self.node:
            if n.name == name:
                return n
        return None


# ------------------------------------------------------------------ writer
_SMALL_VARINTS = tuple(bytes([i]) for i in range(128))


def _varint(v: int) -> bytes:
    if 0 <= v < 0x80:
        return _SMALL_VARINTS[v]
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


_KEYS = {}


def _key(field: int, wt: int) -> bytes:
    k = _KEYS.get((field, wt))
    if k is None:
        k = _KEYS[(field, wt)] = _varint((field << 3) | wt)
    return k


class _Rope:
    """Concatenation without copying: big payloads (tensor_content of model
    weights) are referenced, not re-copied at every nesting level, and
    joined once by `serialize_graphdef`."""

    __slots__ = ("parts", "n")

    def __init__(self, parts):
        self.parts = parts
        self.n = sum(len(p) for p in parts)

    def __len__(self):
        return self.n

    def __add__(self, o):
        return _Rope(self.parts + (o.parts if isinstance(o, _Rope) else [o]))

    def __radd__(self, o):
        return _Rope((list(o.parts) if isinstance(o, _Rope) else [o]) + self.parts)


def _ld(field: int, payload) -> bytes:
    head = _key(field, 2) + _varint(len(payload))
    if isinstance(payload, _Rope):
        return _Rope([head] + payload.parts)
    if len(payload) > 65536:
        return _Rope([head, payload])
    return head + payload


def _enc_shape(s: TensorShapeProto) -> bytes:
    if s.unknown_rank:
        return _key(3, 0) + _varint(1)
    out = b""
    for d in s.dims:
        out += _ld(2, _key(1, 0) + _varint(int(d)) if d != 0 else b"")
    return out


def _typed_val_field(dtype: int, arr: np.ndarray) -> bytes:
    """One element as a typed `*_val` field (what TF emits for single-element
    tensors; larger ones use `tensor_content`)."""
    v = arr.reshape(-1)[0]
    if dtype == D.DT_FLOAT:
        return _ld(5, struct.pack("<f", float(v)))
    if dtype == D.DT_DOUBLE:
        return _ld(6, struct.pack("<d", float(v)))
    if dtype == D.DT_INT64:
        return _ld(10, _varint(int(v)))
    if dtype == D.DT_BOOL:
        return _ld(11, _varint(1 if v else 0))
    if dtype == D.DT_HALF:
        return _ld(13, _varint(int(np.asarray(v, np.float16).view(np.uint16))))
    return _ld(7, _varint(int(v)))


def _enc_tensor(t: TensorProto) -> bytes:
    out = _key(1, 0) + _varint(t.dtype) + _ld(2, _enc_shape(TensorShapeProto(t.shape)))
    if t.dtype == D.DT_STRING:
        for s in t.strings or []:
            out += _ld(8, s)
    else:
        n = int(np.prod(t.shape)) if t.shape else 1
        if n == 1 and t.dtype != D.DT_BFLOAT16:
            out += _typed_val_field(t.dtype, t.to_numpy())
        elif n > 1:
            out += _ld(4, t.content)
    return out


def _enc_list(l: dict) -> bytes:
    out = b""
    for s in l.get("s", []):
        out += _ld(2, s)
    if l.get("i"):
        out += _ld(3, b"".join(_varint(v) for v in l["i"]))
    if l.get("f"):
        out += _ld(4, b"".join(struct.pack("<f", v) for v in l["f"]))
    if l.get("b"):
        out += _ld(5, b"".join(_varint(1 if v else 0) for v in l["b"]))
    if l.get("type"):
        out += _ld(6, b"".join(_varint(v) for v in l["type"]))
    for s in l.get("shape", []):
        out += _ld(7, _enc_shape(s))
    for t in l.get("tensor", []):
        out += _ld(8, _enc_tensor(t))
    return out


def _enc_attr(a: AttrValue) -> bytes:
    k, v = a.kind, a.value
    if k == "list":
        return _ld(1, _enc_list(v))
    if k == "s":
        return _ld(2, v)
    if k == "i":
        return _key(3, 0) + _varint(v)
    if k == "f":
        return _key(4, 5) + struct.pack("<f", v)
    if k == "b":
        return _key(5, 0) + _varint(1 if v else 0)
    if k == "type":
        return _key(6, 0) + _varint(v)
    if k == "shape":
        return _ld(7, _enc_shape(v))
    if k == "tensor":
        return _ld(8, _enc_tensor(v))
    if k == "placeholder":
        return _ld(9, v.encode() if isinstance(v, str) else v)
    if k == "func":
        return _ld(10, _ld(1, v.encode() if isinstance(v, str) else v))
    raise ValueError(f"unknown attr kind {k}")


# encoded `attr` map entries of small hashable values (dtype, int, bool,
# string attrs repeat across nodes and graphs): built once
_ATTR_ENTRIES: Dict[tuple, bytes] = {}


def _attr_entry(k: str, a: AttrValue) -> bytes:
    v = a.value
    # (floats stay out: -0.0 == 0.0 would share one encoding)
    if a.kind in ("type", "i", "b", "s") and isinstance(v, (int, bool, bytes, str)):
        key = (k, a.kind, v)
        e = _ATTR_ENTRIES.get(key)
        if e is None:
            e = _ld(5, _ld(1, k.encode()) + _ld(2, _enc_attr(a)))
            if len(_ATTR_ENTRIES) < 65536:
                _ATTR_ENTRIES[key] = e
        return e
    return _ld(5, _ld(1, k.encode()) + _ld(2, _enc_attr(a)))


def serialize_node(n: NodeDef) -> bytes:
    out = _ld(1, n.name.encode()) + _ld(2, n.op.encode())
    for i in n.input:
        out += _ld(3, i.encode())
    if n.device:
        out += _ld(4, n.device.encode())
    for k in sorted(n.attr):
        out += _attr_entry(k, n.attr[k])
    return out


def serialize_graphdef(g: GraphDef) -> bytes:
    parts = []
    for n in g.node:
        e = _ld(1, serialize_node(n))
        if isinstance(e, _Rope):
            parts.extend(e.parts)
        else:
            parts.append(e)
    if g.producer:
        parts.append(_ld(4, _key(1, 0) + _varint(g.producer)))
    return b"".join(parts)


# ------------------------------------------------------------------ reader
class _R:
    def __init__(self, b: bytes):
        self.b = memoryview(b)
        self.p = 0

    def done(self):
        return self.p >= len(self.b)

    def varint(self) -> int:
        v, shift = 0, 0
        while True:
            c = self.b[self.p]
            self.p += 1
            v |= (c & 0x7F) << shift
            if not c & 0x80:
                return v
            shift += 7

    def bytes_(self) -> bytes:
        n = self.varint()
        v = bytes(self.b[self.p:self.p + n])
        self.p += n
        return v

    def fixed32(self) -> bytes:
        v = bytes(self.b[self.p:self.p + 4])
        self.p += 4
        return v

    def fixed64(self) -> bytes:
        v = bytes(self.b[self.p:self.p + 8])
        self.p += 8
        return v

    def skip(self, wt):
        if wt == 0:
            self.varint()
        elif wt == 1:
            self.p += 8
        elif wt == 2:
            self.bytes_()
        elif wt == 5:
            self.p += 4
        else:
            raise ValueError(f"bad wire type {wt}")

    def fields(self):
        while not self.done():
            k = self.varint()
            yield k >> 3, k & 7


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _rep_varints(r: _R, wt: int) -> List[int]:
    if wt == 2:
        sub = _R(r.bytes_())
        out = []
        while not sub.done():
            out.append(sub.varint())
        return out
    return [r.varint()]


def _dec_shape(b: bytes) -> TensorShapeProto:
    r = _R(b)
    s = TensorShapeProto()
    for f, wt in r.fields():
        if f == 2:
            d = _R(r.bytes_())
            size = 0
            for f2, wt2 in d.fields():
                if f2 == 1:
                    size = _signed64(d.varint())
                else:
                    d.skip(wt2)
            s.dims.append(size)
        elif f == 3:
            s.unknown_rank = bool(r.varint())
        else:
            r.skip(wt)
    return s


def _dec_tensor(b: bytes) -> TensorProto:
    r = _R(b)
    dtype, shape, content, vals, strings = 0, [], None, [], []
    for f, wt in r.fields():
        if f == 1:
            dtype = r.varint()
        elif f == 2:
            shape = _dec_shape(r.bytes_()).dims
        elif f == 4:
            content = r.bytes_()
        elif f == 5:
            raw = r.bytes_() if wt == 2 else r.fixed32()
            vals += list(struct.unpack(f"<{len(raw) // 4}f", raw))
        elif f == 6:
            raw = r.bytes_() if wt == 2 else r.fixed64()
            vals += list(struct.unpack(f"<{len(raw) // 8}d", raw))
        elif f in (7, 10, 11, 13):
            vals += [_signed64(v) for v in _rep_varints(r, wt)]
        elif f == 8:
            strings.append(r.bytes_())
        else:
            r.skip(wt)
    n = int(np.prod(shape)) if shape else 1
    if dtype == D.DT_STRING:
        full = [strings[min(i, len(strings) - 1)] if strings else b"" for i in range(n)]
        return TensorProto(dtype, shape, strings=full)
    npdt = D.numpy_dtype(dtype)
    if content is not None:
        return TensorProto(dtype, shape, content)
    if not vals:
        arr = np.zeros(n, dtype=npdt)
    else:  # repeat-last-value fill rule
        arr = np.array([vals[min(i, len(vals) - 1)] for i in range(n)]).astype(npdt)
    return TensorProto(dtype, shape, arr.astype(np.dtype(npdt).newbyteorder("<")).tobytes())


def _dec_list(b: bytes) -> dict:
    r = _R(b)
    out: dict = {}
    for f, wt in r.fields():
        if f == 2:
            out.setdefault("s", []).append(r.bytes_())
        elif f == 3:
            out.setdefault("i", []).extend(_signed64(v) for v in _rep_varints(r, wt))
        elif f == 4:
            raw = r.bytes_() if wt == 2 else r.fixed32()
            out.setdefault("f", []).extend(struct.unpack(f"<{len(raw) // 4}f", raw))
        elif f == 5:
            out.setdefault("b", []).extend(bool(v) for v in _rep_varints(r, wt))
        elif f == 6:
            out.setdefault("type", []).extend(_rep_varints(r, wt))
        elif f == 7:
            out.setdefault("shape", []).append(_dec_shape(r.bytes_()))
        elif f == 8:
            out.setdefault("tensor", []).append(_dec_tensor(r.bytes_()))
        else:
            r.skip(wt)
    return out


def _dec_attr(b: bytes) -> AttrValue:
    r = _R(b)
    a = AttrValue("list", {})
    for f, wt in r.fields():
        if f == 1:
            a = AttrValue("list", _dec_list(r.bytes_()))
        elif f == 2:
            a = AttrValue("s", r.bytes_())
        elif f == 3:
            a = AttrValue("i", _signed64(r.varint()))
        elif f == 4:
            a = AttrValue("f", struct.unpack("<f", r.fixed32())[0])
        elif f == 5:
            a = AttrValue("b", bool(r.varint()))
        elif f == 6:
            a = AttrValue("type", r.varint())
        elif f == 7:
            a = AttrValue("shape", _dec_shape(r.bytes_()))
        elif f == 8:
            a = AttrValue("tensor", _dec_tensor(r.bytes_()))
        elif f == 9:
            a = AttrValue("placeholder", r.bytes_().decode())
        elif f == 10:
            fr = _R(r.bytes_())
            name = ""
            for f2, wt2 in fr.fields():
                if f2 == 1:
                    name = fr.bytes_().decode()
                else:
                    fr.skip(wt2)
            a = AttrValue("func", name)
        else:
            r.skip(wt)
    return a


def _dec_node(b: bytes) -> NodeDef:
    r = _R(b)
    n = NodeDef("", "")
    for f, wt in r.fields():
        if f == 1:
            n.name = r.bytes_().decode()
        elif f == 2:
            n.op = r.bytes_().decode()
        elif f == 3:
            n.input.append(r.bytes_().decode())
        elif f == 4:
            n.device = r.bytes_().decode()
        elif f == 5:
            e = _R(r.bytes_())
            k, v = "", None
            for f2, wt2 in e.fields():
                if f2 == 1:
                    k = e.bytes_().decode()
                elif f2 == 2:
                    v = _dec_attr(e.bytes_())
                else:
                    e.skip(wt2)
            n.attr[k] = v
        else:
            r.skip(wt)
    return n


class MalformedProtoError(ValueError):
    """Bytes that do not decode as the expected protobuf message."""


def parse_graphdef(b: bytes) -> GraphDef:
    """Decode GraphDef bytes; malformed input raises MalformedProtoError."""
    try:
        return _parse_graphdef(b)
    except MalformedProtoError:
        raise
    except (struct.error, IndexError, KeyError, UnicodeDecodeError, OverflowError, ValueError, TypeError) as e:
        raise MalformedProtoError(f"malformed GraphDef ({type(e).__name__}: {e})") from None


def _parse_graphdef(b: bytes) -> GraphDef:
    r = _R(b)
    g = GraphDef()
    for f, wt in r.fields():
        if f == 1:
            g.node.append(_dec_node(r.bytes_()))
        elif f == 4:
            v = _R(r.bytes_())
            for f2, wt2 in v.fields():
                if f2 == 1:
                    g.producer = v.varint()
                else:
                    v.skip(wt2)
        else:
            r.skip(wt)
    return g


# ------------------------------------------------------------------ text format
def _txt_shape(s: TensorShapeProto, ind: str) -> List[str]:
    if s.unknown_rank:
        return [f"{ind}unknown_rank: true"]
    out = []
    for d in s.dims:
        out += [f"{ind}dim {{", f"{ind}  size: {d}", f"{ind}}}"]
    return out


def _txt_tensor(t: TensorProto, ind: str) -> List[str]:
    out = [f"{ind}dtype: {_DT_ENUM_NAMES.get(t.dtype, t.dtype)}", f"{ind}tensor_shape {{"]
    out += _txt_shape(TensorShapeProto(t.shape), ind + "  ")
    out.append(f"{ind}}}")
    if t.dtype == D.DT_STRING:
        out += [f'{ind}string_val: "{s.decode(errors="replace")}"' for s in t.strings or []]
    else:
        arr = t.to_numpy().reshape(-1)
        if arr.size > 1:
            out.append(f'{ind}tensor_content: "{_c_escape(t.content)}"')
        else:
            key = {D.DT_FLOAT: "float_val", D.DT_DOUBLE: "double_val", D.DT_INT64: "int64_val",
                   D.DT_BOOL: "bool_val"}.get(t.dtype, "int_val")
            out += [f"{ind}{key}: {_num(v)}" for v in arr]
    return out


def _c_escape(b: bytes) -> str:
    """protobuf text-format byte escaping (octal for non-printables)."""
    out = []
    for c in b:
        ch = chr(c)
        if ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif ch == '"':
            out.append('\\"')
        elif ch == "'":
            out.append("\\'")
        elif ch == "\\":
            out.append("\\\\")
        elif 32 <= c < 127:
            out.append(ch)
        else:
            out.append(f"\\{c:03o}")
    return "".join(out)


def _num(v) -> str:
    if isinstance(v, (float, np.floating)):
        return repr(float(v)).replace("inf", "inf")
    if isinstance(v, (bool, np.bool_)):
        return "true" if v else "false"
    return str(int(v))


def _txt_attr(a: AttrValue, ind: str) -> List[str]:
    k, v = a.kind, a.value
    if k == "type":
        return [f"{ind}type: {_DT_ENUM_NAMES.get(v, v)}"]
    if k == "i":
        return [f"{ind}i: {v}"]
    if k == "f":
        return [f"{ind}f: {_num(v)}"]
    if k == "b":
        return [f"{ind}b: {'true' if v else 'false'}"]
    if k == "s":
        return [f'{ind}s: "{v.decode(errors="replace")}"']
    if k == "shape":
        return [f"{ind}shape {{"] + _txt_shape(v, ind + "  ") + [f"{ind}}}"]
    if k == "tensor":
        return [f"{ind}tensor {{"] + _txt_tensor(v, ind + "  ") + [f"{ind}}}"]
    if k == "list":
        out = [f"{ind}list {{"]
        for i in v.get("i", []):
            out.append(f"{ind}  i: {i}")
        for s in v.get("s", []):
            out.append(f'{ind}  s: "{s.decode(errors="replace")}"')
        for t in v.get("type", []):
            out.append(f"{ind}  type: {_DT_ENUM_NAMES.get(t, t)}")
        for s in v.get("shape", []):
            out += [f"{ind}  shape {{"] + _txt_shape(s, ind + "    ") + [f"{ind}  }}"]
        out.append(f"{ind}}}")
        return out
    return [f"{ind}{k}: {v}"]


def node_to_text(n: NodeDef) -> str:
    """TF text-proto rendering of a NodeDef (attrs sorted by key, like TF)."""
    out = [f'name: "{n.name}"', f'op: "{n.op}"']
    out += [f'input: "{i}"' for i in n.input]
    if n.device:
        out.append(f'device: "{n.device}"')
    for k in sorted(n.attr):
        out += ["attr {", f'  key: "{k}"', "  value {"] + _txt_attr(n.attr[k], "    ") + ["  }", "}"]
    return "\n".join(out) + "\n"
