"""TF-1.x-compatible graph builder (no TensorFlow needed).

Emits GraphDefs with the same op names, attributes and node-naming rules as
TF 1.x Python, so code written against ``tf.placeholder`` / ``tf.add`` /
``tf.reduce_sum`` ... for the reference works by swapping the import:

    from tensorframes_amd import tf
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        z = tf.add(x, 3, name="z")

Naming follows TF: a name is made unique per graph with ``_1``, ``_2`` ...
suffixes, and non-tensor op arguments become ``Const`` nodes named
``<op>/<arg>`` (e.g. ``Fill/dims``, ``z/y``), matching the golden NodeDefs the
reference's DSL is tested against (reference: src/test/scala/org/tensorframes/dsl/BasicSuite.scala:12-33,
src/main/scala/org/tensorframes/dsl/Paths.scala:13-56). Graph contexts are per
thread (the reference's DSL path state was a global, reference: Paths.scala:10).

Static shapes come from the native runtime's shape inference
(csrc/ir/*: one implementation shared with the executor).
"""
from __future__ import annotations

import builtins as _builtins
import contextlib
import struct
import threading
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from ..utils import dtypes as D
from ..utils.dtypes import (DType, as_dtype, bfloat16, bool_, double, float16, float32, float64,  # noqa: F401
                            int8, int16, int32, int64, string, uint8)
from . import proto as P

bool = bool_  # noqa: A001  (tf.bool)


# ------------------------------------------------------------------ shapes
class Dimension:
    def __init__(self, v: Optional[int]):
        self.value = v

    def __eq__(self, o):
        ov = o.value if isinstance(o, Dimension) else o
        return self.value == ov

    def __int__(self):
        return self.value

    def __index__(self):
        return self.value

    def __repr__(self):
        return f"Dimension({self.value})"


class TensorShape:
    def __init__(self, dims: Optional[Sequence[Optional[int]]]):
        self._dims = None if dims is None else [None if (d is None or d < 0) else int(d) for d in dims]

    @property
    def ndims(self) -> Optional[int]:
        return None if self._dims is None else len(self._dims)

    @property
    def dims(self):
        return None if self._dims is None else [Dimension(d) for d in self._dims]

    def as_list(self) -> List[Optional[int]]:
        if self._dims is None:
            raise ValueError("as_list() is not defined on an unknown TensorShape.")
        return list(self._dims)

    def is_fully_defined(self) -> bool:
        return self._dims is not None and all(d is not None for d in self._dims)

    def __len__(self):
        return len(self._dims or [])

    def __getitem__(self, i):
        return self._dims[i]

    def __iter__(self):
        return iter(self._dims or [])

    def __eq__(self, o):
        if isinstance(o, TensorShape):
            return self._dims == o._dims
        if isinstance(o, (list, tuple)):
            return self._dims == list(o)
        return NotImplemented

    def __repr__(self):
        if self._dims is None:
            return "TensorShape(None)"
        return "TensorShape([" + ", ".join("Dimension(None)" if d is None else f"Dimension({d})"
                                           for d in self._dims) + "])"


# ------------------------------------------------------------------ graph
class Graph:
    def __init__(self):
        self._nodes: List[P.NodeDef] = []
        self._ops: Dict[str, "Operation"] = {}
        self._names_in_use: Dict[str, int] = {}
        self._scope: List[str] = []
        self._infer_cache: Tuple[int, Dict[str, Any]] = (-1, {})
        self._lock = threading.Lock()
        # per-node wire encodings (nodes are append-only and never mutated once
        # added), so re-serializing a growing graph costs O(new nodes): shape
        # inference after every op otherwise re-encoded the whole graph
        self._enc_full: List[List[bytes]] = []
        self._enc_view: List[List[bytes]] = []

    # -- context
    @contextlib.contextmanager
    def as_default(self):
        _stack().append(self)
        try:
            yield self
        finally:
            _stack().pop()

    @contextlib.contextmanager
    def name_scope(self, name: str):
        if name is None or name == "":
            yield ""
            return
        if name.endswith("/"):
            scope = name[:-1]
        else:
            scope = self.unique_name(name)
        old = self._scope
        self._scope = scope.split("/") if scope else []
        try:
            yield scope + "/"
        finally:
            self._scope = old

    def unique_name(self, name: str, mark_as_used: bool = True) -> str:
        full = "/".join(self._scope + [name]) if self._scope else name
        key = full.lower()
        i = self._names_in_use.get(key, 0)
        if mark_as_used:
            self._names_in_use[key] = i + 1
        if i > 0:
            base = full
            while True:
                cand = f"{base}_{i}"
                if cand.lower() not in self._names_in_use:
                    full = cand
                    if mark_as_used:
                        self._names_in_use[cand.lower()] = 1
                    break
                i += 1
        return full

    # -- nodes
    def _add(self, node: P.NodeDef, n_out: int, out_dtypes: List[DType],
             inputs: Optional[List["Tensor"]] = None) -> "Operation":
        with self._lock:
            if node.name in self._ops:
                raise ValueError(f"Duplicate node name in graph: '{node.name}'")
            self._nodes.append(node)
            op = Operation(self, node, n_out, out_dtypes)
            if inputs is not None:
                op._inputs = inputs
            self._ops[node.name] = op
            return op

    def get_operations(self) -> List["Operation"]:
        return [self._ops[n.name] for n in self._nodes]

    def get_operation_by_name(self, name: str) -> "Operation":
        if name not in self._ops:
            raise KeyError(f"The name '{name}' refers to an Operation not in the graph.")
        return self._ops[name]

    def get_tensor_by_name(self, name: str) -> "Tensor":
        base, _, idx = name.partition(":")
        op = self.get_operation_by_name(base)
        return op.outputs[int(idx or 0)]

    def as_graph_element(self, obj, allow_tensor=True, allow_operation=True):
        if isinstance(obj, Tensor):
            if obj.graph is not self:
                raise ValueError(f"Tensor {obj} is not an element of this graph.")
            return obj
        if isinstance(obj, Operation):
            return obj
        if isinstance(obj, str):
            if ":" in obj:
                return self.get_tensor_by_name(obj)
            return self.get_operation_by_name(obj)
        raise TypeError(f"Can not convert a {type(obj).__name__} into a graph element.")

    def as_graph_def(self, add_shapes: bool = False) -> P.GraphDef:
        g = P.GraphDef(list(self._nodes), producer=24)
        if add_shapes:
            shapes = self._inferred()
            nodes = []
            for n in self._nodes:
                m = P.NodeDef(n.name, n.op, n.input, dict(n.attr), n.device)
                outs = shapes.get(n.name)
                if outs:
                    m.attr["_output_shapes"] = P.AttrValue.shapelist([o["shape"] for o in outs])
                nodes.append(m)
            g = P.GraphDef(nodes, producer=24)
        return g

    def serialize(self, upto: Optional[int] = None) -> bytes:
        """GraphDef bytes (of the first `upto` nodes); cached while the graph is
        unchanged (nodes are only ever appended, so the node count identifies
        the version)."""
        n = len(self._nodes) if upto is None else upto
        cached = getattr(self, "_ser_cache", None)
        if cached is not None and cached[0] == n:
            return cached[1]
        parts = [p for e in self._node_parts(False)[:n] for p in e]
        parts.append(P._ld(4, P._key(1, 0) + P._varint(24)))  # versions { producer: 24 }
        b = b"".join(parts)
        self._ser_cache = (n, b)
        return b

    def fast_key(self, upto: int):
        """(key, params) of the first `upto` nodes without serialising them:
        `key` is every node, input and attribute except the payloads of the
        candidate parameter constants (floating Consts of >= 2 elements, the
        candidates of the native Graph::structure_key), `params` maps those
        constants' names to their TensorProtos. A graph rebuilt with new
        parameter values (K-Means centres) has the same key, so its program
        is the known one with the payloads swapped (engine.program_for_spec)."""
        cached = getattr(self, "_fk_cache", None)
        if cached is not None and cached[0] == upto:
            return cached[1]
        parts = []
        params = {}
        # the per-node wire encodings (native encoder, cached: a later
        # serialize() reuses them); a parameter candidate contributes its name,
        # dtype and shape instead
        for nd, e in zip(self._nodes[:upto], self._node_parts(False)[:upto]):
            if nd.op == "Const":
                v = nd.attr.get("value")
                tp = v.value if v is not None and v.kind == "tensor" else None
                if tp is not None and tp.dtype in _PARAM_DTYPES and tp.strings is None:
                    n = 1
                    for d in tp.shape:
                        n *= d
                    if n >= 2:
                        params[nd.name] = tp
                        parts.append((nd.name, tp.dtype, tuple(tp.shape)))
                        continue
            parts.append(e[0] if len(e) == 1 else b"".join(e))
        r = (tuple(parts), params)
        self._fk_cache = (upto, r)
        return r

    @staticmethod
    def _view_node(n: P.NodeDef) -> P.NodeDef:
        if n.op == "Const" and "value" in n.attr:
            t = n.attr["value"].value
            numel = int(np.prod(t.shape)) if t.shape else 1
            if numel > 1024:
                return P.NodeDef(n.name, "Placeholder", [], {"dtype": P.AttrValue.type(t.dtype),
                                                          "shape": P.AttrValue.shape(t.shape)})
        return n

    def _node_parts(self, view: bool) -> List[List[bytes]]:
        """Encoded `node` fields (GraphDef field 1) of every node, extended with
        the nodes added since the last call."""
        with self._lock:
            cache = self._enc_view if view else self._enc_full
            other = self._enc_full if view else self._enc_view
            i = len(cache)  # (no range(): this module defines the tf.range op)
            enc = _native_encoder()
            if enc is not None and i < len(self._nodes):
                # one C++ pass (csrc/proto/pyencode.cpp); None marks a node it
                # does not cover, encoded below by graph/proto.py
                for n, e in zip(self._nodes[i:], enc(self._nodes[i:], 1024 if view else -1)):
                    if e is None:
                        vn = self._view_node(n) if view else n
                        e = P._ld(1, P.serialize_node(vn))
                        cache.append(list(e.parts) if isinstance(e, P._Rope) else [e])
                    else:
                        cache.append([e])
                return cache[:len(self._nodes)]
            for n in self._nodes[i:]:
                vn = self._view_node(n)
                if vn is n and i < len(other):  # same node in both views: encode once
                    cache.append(other[i])
                else:
                    e = P._ld(1, P.serialize_node(vn if view else n))
                    cache.append(list(e.parts) if isinstance(e, P._Rope) else [e])
                i += 1
            return cache[:len(self._nodes)]

    def _shape_view(self) -> bytes:
        """The graph for shape inference only: large constants are replaced by
        placeholders of the same dtype/shape (their values never decide a
        shape), so inference does not re-serialize megabytes of weights."""
        return b"".join(p for e in self._node_parts(True) for p in e)

    def _inferred(self) -> Dict[str, Any]:
        n = len(self._nodes)
        if self._infer_cache[0] != n:
            from .._native import _C
            res = _C.infer_all(self._shape_view())
            self._infer_cache = (n, res)
        return self._infer_cache[1]

    def finalize(self):
        pass

    def __enter__(self):
        self._ctx = self.as_default()
        return self._ctx.__enter__()

    def __exit__(self, *a):
        return self._ctx.__exit__(*a)


_ENCODER: List[Any] = []


def _native_encoder():
    """`_C.encode_nodes` when the extension is built (the DSL itself stays
    importable without it: graph/proto.py is the reference encoder)."""
    if not _ENCODER:
        try:
            from .._native import _C
            _ENCODER.append(getattr(_C, "encode_nodes", None))
        except Exception:  # noqa: BLE001
            _ENCODER.append(None)
    return _ENCODER[0]


_tls = threading.local()
_global_default = [Graph()]


def _stack() -> List[Graph]:
    if not hasattr(_tls, "stack"):
        _tls.stack = []
    return _tls.stack


def get_default_graph() -> Graph:
    st = _stack()
    return st[-1] if st else _global_default[0]


def reset_default_graph():
    _global_default[0] = Graph()


@contextlib.contextmanager
def name_scope(name: str):
    with get_default_graph().name_scope(name) as s:
        yield s


# reference-DSL spellings (reference: src/main/scala/org/tensorframes/dsl/package.scala:31-35)
scope = name_scope


@contextlib.contextmanager
def variable_scope(name_or_scope, default_name=None, reuse=None):
    """Graphs here are frozen (no variables), so a variable scope is a name scope."""
    with name_scope(name_or_scope or default_name) as s:
        yield s


@contextlib.contextmanager
def with_graph():
    with Graph().as_default() as g:
        yield g


_PARAM_DTYPES = frozenset((D.DT_FLOAT, D.DT_DOUBLE, D.DT_HALF, D.DT_BFLOAT16))


class Operation:
    # graphs rebuilt per iteration (K-Means) create thousands of these
    __slots__ = ("graph", "node_def", "_inputs", "outputs", "__weakref__")

    def __init__(self, graph: Graph, node: P.NodeDef, n_out: int, out_dtypes: List[DType]):
        self.graph = graph
        self.node_def = node
        self._inputs: Optional[List["Tensor"]] = None  # data inputs, when known at creation
        nd = len(out_dtypes)
        if n_out == 1:
            self.outputs = [Tensor(self, 0, out_dtypes[0] if nd else None)]
        else:
            self.outputs = [Tensor(self, i, out_dtypes[i] if i < nd else None) for i in _builtins.range(n_out)]

    @property
    def name(self) -> str:
        return self.node_def.name

    @property
    def type(self) -> str:
        return self.node_def.op

    @property
    def inputs(self) -> List["Tensor"]:
        if self._inputs is not None:
            return list(self._inputs)
        out = []
        for i in self.node_def.input:
            if not i.startswith("^"):
                out.append(self.graph.get_tensor_by_name(i if ":" in i else i + ":0"))
        return out

    def get_attr(self, name):
        a = self.node_def.attr[name]
        if a.kind == "type":
            return DType(a.value)
        if a.kind == "shape":
            return None if a.value.unknown_rank else a.value.dims
        return a.value

    def __repr__(self):
        return f"<tf.Operation '{self.name}' type={self.type}>"


class Tensor:
    __slots__ = ("op", "value_index", "_dtype", "_rank", "__weakref__")

    def __init__(self, op: Operation, value_index: int, dtype: Optional[DType]):
        self.op = op
        self.value_index = value_index
        self._dtype = dtype

    @property
    def graph(self) -> Graph:
        return self.op.graph

    @property
    def name(self) -> str:
        return f"{self.op.name}:{self.value_index}"

    @property
    def dtype(self) -> DType:
        if self._dtype is None:
            info = self.graph._inferred()[self.op.name][self.value_index]
            self._dtype = DType(info["dtype"])
        return self._dtype

    def get_shape(self) -> TensorShape:
        nd = self.op.node_def
        # placeholders and constants carry their shape: no graph inference
        # (rebuilding a graph per iteration, e.g. K-Means, asks for these often)
        if nd.op in ("Placeholder", "PlaceholderV2") and "shape" in nd.attr:
            shp = nd.attr["shape"].value
            return TensorShape(None if shp.unknown_rank else [None if d < 0 else d for d in shp.dims])
        if nd.op == "Const" and "value" in nd.attr:
            return TensorShape(list(nd.attr["value"].value.shape))
        info = self.graph._inferred()[self.op.name][self.value_index]
        return TensorShape(info["shape"])

    @property
    def shape(self) -> TensorShape:
        return self.get_shape()

    # -- operators (implicit constant lifting; reference: src/main/scala/org/tensorframes/dsl/Implicits.scala:121-123)
    def __add__(self, o):
        return add(self, o, name="add")

    def __radd__(self, o):
        return add(o, self, name="add")

    def __sub__(self, o):
        return subtract(self, o, name="sub")

    def __rsub__(self, o):
        return subtract(o, self, name="sub")

    def __mul__(self, o):
        return multiply(self, o, name="mul")

    def __rmul__(self, o):
        return multiply(o, self, name="mul")

    def __truediv__(self, o):
        return truediv(self, o, name="truediv")

    def __rtruediv__(self, o):
        return truediv(o, self, name="truediv")

    def __div__(self, o):
        return div(self, o)

    def __floordiv__(self, o):
        return floordiv(self, o, name="floordiv")

    def __mod__(self, o):
        return mod(self, o, name="mod")

    def __pow__(self, o):
        return pow(self, o, name="pow")

    def __neg__(self):
        return negative(self)

    def __abs__(self):
        return abs(self)

    def __matmul__(self, o):
        return matmul(self, o)

    def __lt__(self, o):
        return less(self, o)

    def __le__(self, o):
        return less_equal(self, o)

    def __gt__(self, o):
        return greater(self, o)

    def __ge__(self, o):
        return greater_equal(self, o)

    def __and__(self, o):
        return logical_and(self, o)

    def __or__(self, o):
        return logical_or(self, o)

    def __invert__(self):
        return logical_not(self)

    def __getitem__(self, item):
        return _slice_helper(self, item)

    def __hash__(self):
        return id(self)

    def __eq__(self, o):  # TF-1.x semantics: identity
        return self is o

    def eval(self, feed_dict=None, session=None):
        s = session or Session(self.graph)
        return s.run(self, feed_dict)

    def __repr__(self):
        try:
            shp = self.get_shape()
        except Exception:  # noqa: BLE001 (repr must not fail)
            shp = "?"
        return f"<tf.Tensor '{self.name}' shape={shp} dtype={self.dtype.name}>"


# ------------------------------------------------------------------ core builders
# value attrs of small constants, shared between graphs (TensorProto / AttrValue
# are never mutated once built): graphs rebuilt per iteration lift the same
# axes, multiples and scalars every time (K-Means: ~24 of its 53 nodes)
_CONST_ATTRS: Dict[tuple, Tuple["P.AttrValue", "P.AttrValue", DType]] = {}


def _small_const_key(value, dtype) -> Optional[tuple]:
    tv = type(value)
    de = None if dtype is None else as_dtype(dtype).enum
    if tv is int or tv is bool:
        return (tv, value, de)
    if tv is float:
        return (tv, struct.pack("<d", value), de)  # keeps -0.0 and NaN payloads apart
    if tv is np.ndarray and value.size <= 16 and value.dtype.kind in "iufb":
        return (tv, value.dtype.str, value.shape, value.tobytes(), de)
    if isinstance(value, np.generic) and value.dtype.kind in "iufb":
        return (np.ndarray, value.dtype.str, (), value.tobytes(), de)
    return None


def _const_node(graph: Graph, value, dtype: Optional[DType], name: str, shape=None) -> Tensor:
    key = _small_const_key(value, dtype) if shape is None else None
    ent = _CONST_ATTRS.get(key) if key is not None else None
    if ent is not None:
        node = P.NodeDef._make(name, "Const", [], {"dtype": ent[0], "value": ent[1]})
        return graph._add(node, 1, [ent[2]]).outputs[0]
    arr, dt = _to_numpy(value, dtype)
    if shape is not None:
        shape = [int(s) for s in shape]
        if arr.size == 1:
            arr = np.full(shape, arr.reshape(-1)[0], dtype=arr.dtype)
        else:
            arr = arr.reshape(shape)
    tp = P.TensorProto.from_numpy(arr, dt.enum)
    ta, va = P.AttrValue.type(dt), P.AttrValue.tensor(tp)
    if key is not None:
        if len(_CONST_ATTRS) > 4096:
            _CONST_ATTRS.clear()
        _CONST_ATTRS[key] = (ta, va, dt)
    node = P.NodeDef._make(name, "Const", [], {"dtype": ta, "value": va})
    return graph._add(node, 1, [dt]).outputs[0]


def _to_numpy(value, dtype: Optional[DType]) -> Tuple[np.ndarray, DType]:
    if isinstance(value, Tensor):
        raise TypeError("expected a python / numpy value")
    if dtype is not None:
        dtype = as_dtype(dtype)
        if dtype.enum == D.DT_STRING:
            return np.array(value, dtype=object), dtype
        return np.asarray(value, dtype=dtype.as_numpy_dtype), dtype
    arr = np.asarray(value)
    if arr.dtype.kind in ("U", "S", "O"):
        return np.array(value, dtype=object), string
    if arr.dtype == np.float64 and not isinstance(value, np.ndarray):
        return arr.astype(np.float32), float32  # TF default for python floats
    if arr.dtype == np.int64 and not isinstance(value, np.ndarray):
        return arr.astype(np.int32), int32  # TF default for python ints
    return arr, as_dtype(arr.dtype)


def convert_to_tensor(value, dtype=None, name=None) -> Tensor:
    if isinstance(value, Tensor):
        if dtype is not None and as_dtype(dtype) != value.dtype:
            raise TypeError(f"Tensor conversion requested dtype {as_dtype(dtype).name} for Tensor "
                            f"with dtype {value.dtype.name}: {value!r}")
        return value
    g = get_default_graph()
    return _const_node(g, value, dtype, g.unique_name(name or "Const"))


def _graph_of(values) -> Graph:
    for v in values:
        if isinstance(v, Tensor):
            return v.graph
        if isinstance(v, (list, tuple)):
            for w in v:
                if isinstance(w, Tensor):
                    return w.graph
    return get_default_graph()


def _op(op_type: str, inputs: List[Tuple[str, Any]], attrs: Dict[str, P.AttrValue],
        name: Optional[str], n_out: int = 1, out_dtypes: Optional[List[DType]] = None,
        dtype_hint: Optional[DType] = None, list_inputs: Sequence[str] = ()) -> Operation:
    """Create an op: open its name scope, lift python values to `<op>/<arg>` Consts.

    Hot for graphs rebuilt per iteration (K-Means): no default-graph context
    switch, and the op's name scope is only entered when a value is lifted."""
    g = _graph_of([v for _, v in inputs])
    op_name = g.unique_name(name or op_type)
    names: List[str] = []
    tensors: List[Tensor] = []
    g_scope = None
    try:
        for arg, v in inputs:
            if arg in list_inputs:
                vals = v
            elif isinstance(v, Tensor):
                names.append(v.op.node_def.name if v.value_index == 0 else v.name)
                tensors.append(v)
                continue
            else:
                vals = (v,)
            for j, item in enumerate(vals):
                if isinstance(item, Tensor):
                    t = item
                else:
                    if g_scope is None:
                        g_scope = g._scope
                        g._scope = op_name.split("/")
                    nm = arg if arg not in list_inputs else (f"{arg}_{j}" if j else arg)
                    t = _const_node(g, item, dtype_hint if dtype_hint is not None and
                                    not isinstance(item, np.ndarray) else None,
                                    g.unique_name(nm))
                names.append(t.op.node_def.name if t.value_index == 0 else t.name)
                tensors.append(t)
    finally:
        if g_scope is not None:
            g._scope = g_scope
    node = P.NodeDef._make(op_name, op_type, names, dict(attrs))
    return g._add(node, n_out, out_dtypes or [], tensors)


def _first_dtype(*vals) -> Optional[DType]:
    for v in vals:
        if isinstance(v, Tensor):
            return v.dtype
    return None


def _binary(op_type: str, x, y, name, out_dtype: Optional[DType] = None) -> Tensor:
    dt = _first_dtype(x, y)
    if dt is None:
        x = convert_to_tensor(x)
        dt = x.dtype
    op = _op(op_type, [("x", x), ("y", y)], {"T": P.AttrValue.type(dt)}, name,
             out_dtypes=[out_dtype or dt], dtype_hint=dt)
    return op.outputs[0]


def _unary(op_type: str, x, name) -> Tensor:
    x = convert_to_tensor(x)
    return _op(op_type, [("x", x)], {"T": P.AttrValue.type(x.dtype)}, name, out_dtypes=[x.dtype]).outputs[0]


# ------------------------------------------------------------------ public ops
def placeholder(dtype, shape=None, name=None) -> Tensor:
    dt = as_dtype(dtype)
    g = get_default_graph()
    nm = g.unique_name(name or "Placeholder")
    shp = None if shape is None else [None if (d is None or (isinstance(d, int) and d < 0)) else int(d)
                                      for d in (shape.as_list() if isinstance(shape, TensorShape) else shape)]
    node = P.NodeDef(nm, "Placeholder", [], {"dtype": P.AttrValue.type(dt), "shape": P.AttrValue.shape(shp)})
    return g._add(node, 1, [dt]).outputs[0]


def placeholder_with_default(input, shape, name=None) -> Tensor:  # noqa: A002
    input = convert_to_tensor(input)
    return _op("PlaceholderWithDefault", [("input", input)],
               {"dtype": P.AttrValue.type(input.dtype), "shape": P.AttrValue.shape(shape)}, name,
               out_dtypes=[input.dtype]).outputs[0]


def constant(value, dtype=None, shape=None, name="Const") -> Tensor:
    g = get_default_graph()
    return _const_node(g, value, as_dtype(dtype) if dtype is not None else None, g.unique_name(name), shape)


def identity(input, name=None) -> Tensor:  # noqa: A002
    return _unary("Identity", input, name)


def stop_gradient(input, name=None) -> Tensor:  # noqa: A002
    return _unary("StopGradient", input, name)


def add(x, y, name=None):
    return _binary("Add", x, y, name)


def subtract(x, y, name=None):
    return _binary("Sub", x, y, name)


sub = subtract


def multiply(x, y, name=None):
    return _binary("Mul", x, y, name)


mul = multiply


def div(x, y, name=None):
    return _binary("Div", x, y, name)


def truediv(x, y, name=None):
    dt = _first_dtype(x, y)
    if dt is not None and dt.is_integer:
        x = cast(x, float64)
        y = cast(y, float64)
    return _binary("RealDiv", x, y, name)


divide = truediv
realdiv = truediv


def floordiv(x, y, name=None):
    return _binary("FloorDiv", x, y, name)


def mod(x, y, name=None):
    return _binary("FloorMod", x, y, name)


floormod = mod


def maximum(x, y, name=None):
    return _binary("Maximum", x, y, name)


def minimum(x, y, name=None):
    return _binary("Minimum", x, y, name)


def pow(x, y, name=None):  # noqa: A001
    return _binary("Pow", x, y, name)


def squared_difference(x, y, name=None):
    return _binary("SquaredDifference", x, y, name)


def atan2(y, x, name=None):
    return _binary("Atan2", y, x, name)


def equal(x, y, name=None):
    return _binary("Equal", x, y, name, out_dtype=bool_)


def not_equal(x, y, name=None):
    return _binary("NotEqual", x, y, name, out_dtype=bool_)


def less(x, y, name=None):
    return _binary("Less", x, y, name, out_dtype=bool_)


def less_equal(x, y, name=None):
    return _binary("LessEqual", x, y, name, out_dtype=bool_)


def greater(x, y, name=None):
    return _binary("Greater", x, y, name, out_dtype=bool_)


def greater_equal(x, y, name=None):
    return _binary("GreaterEqual", x, y, name, out_dtype=bool_)


def logical_and(x, y, name=None):
    return _op("LogicalAnd", [("x", x), ("y", y)], {}, name, out_dtypes=[bool_], dtype_hint=bool_).outputs[0]


def logical_or(x, y, name=None):
    return _op("LogicalOr", [("x", x), ("y", y)], {}, name, out_dtypes=[bool_], dtype_hint=bool_).outputs[0]


def logical_not(x, name=None):
    return _op("LogicalNot", [("x", x)], {}, name, out_dtypes=[bool_]).outputs[0]


def add_n(inputs, name=None):
    inputs = [convert_to_tensor(i) for i in inputs]
    dt = inputs[0].dtype
    return _op("AddN", [("inputs", inputs)], {"T": P.AttrValue.type(dt), "N": P.AttrValue.i(len(inputs))},
               name, out_dtypes=[dt], list_inputs=("inputs",)).outputs[0]


def _mk_unary(op_type):
    def f(x, name=None):
        return _unary(op_type, x, name)
    f.__name__ = op_type.lower()
    return f


negative = _mk_unary("Neg")
neg = negative
abs = _mk_unary("Abs")  # noqa: A001
square = _mk_unary("Square")
sqrt = _mk_unary("Sqrt")
rsqrt = _mk_unary("Rsqrt")
exp = _mk_unary("Exp")
log = _mk_unary("Log")
log1p = _mk_unary("Log1p")
expm1 = _mk_unary("Expm1")
reciprocal = _mk_unary("Reciprocal")
inv = _mk_unary("Inv")
floor = _mk_unary("Floor")
ceil = _mk_unary("Ceil")
round = _mk_unary("Round")  # noqa: A001
sign = _mk_unary("Sign")
sin = _mk_unary("Sin")
cos = _mk_unary("Cos")
tan = _mk_unary("Tan")
tanh = _mk_unary("Tanh")
sigmoid = _mk_unary("Sigmoid")
erf = _mk_unary("Erf")
is_nan = _mk_unary("IsNan")
is_inf = _mk_unary("IsInf")
is_finite = _mk_unary("IsFinite")


_SAME_RANK_OPS = frozenset((
    "Identity", "Neg", "Abs", "Square", "Sqrt", "Rsqrt", "Exp", "Log", "Log1p", "Expm1", "Reciprocal", "Inv",
    "Floor", "Ceil", "Round", "Sign", "Sin", "Cos", "Tan", "Tanh", "Sigmoid", "Erf", "IsNan", "IsInf", "IsFinite",
    "LogicalNot", "Cast", "Relu", "Relu6", "Elu", "Selu", "Softplus", "Softsign", "Softmax", "LogSoftmax", "Tile",
    "BiasAdd", "ZerosLike", "OnesLike", "StopGradient", "CheckNumerics"))
_BROADCAST_OPS = frozenset((
    "Add", "AddV2", "Sub", "Mul", "RealDiv", "Div", "DivNoNan", "Maximum", "Minimum", "Pow", "SquaredDifference",
    "FloorDiv", "FloorMod", "Mod", "Less", "LessEqual", "Greater", "GreaterEqual", "Equal", "NotEqual",
    "LogicalAnd", "LogicalOr", "Atan2", "Select", "SelectV2"))
_REDUCE_OPS = frozenset(("Sum", "Min", "Max", "Prod", "Mean", "All", "Any"))


def _const_value(t: Tensor) -> Optional[np.ndarray]:
    nd = t.op.node_def
    if nd.op == "Const" and "value" in nd.attr:
        return nd.attr["value"].value.to_numpy()
    return None


def _static_rank(t: Tensor, depth: int = 0) -> Optional[int]:
    """Rank of `t` from the local op structure, without whole-graph shape
    inference (None when a rule does not apply). Reductions over all axes need
    only the rank, and graphs rebuilt per iteration (K-Means) would otherwise
    re-serialise and re-infer the whole graph for every `reduce_sum(x)`."""
    r = getattr(t, "_rank", False)
    if r is not False:
        return r
    nd = t.op.node_def
    r = None
    if nd.op in ("Placeholder", "PlaceholderV2", "Const"):
        s = t.get_shape()
        r = s.ndims
    elif depth < 64 and t.value_index == 0:
        ins = t.op.inputs
        if nd.op in _SAME_RANK_OPS and ins:
            r = _static_rank(ins[0], depth + 1)
        elif nd.op in _BROADCAST_OPS and ins:
            rs = [_static_rank(i, depth + 1) for i in ins]
            r = None if any(x is None for x in rs) else max(rs)
        elif nd.op == "MatMul":
            r = 2
        elif nd.op in ("Shape",):
            r = 1
        elif nd.op in ("Size", "Rank"):
            r = 0
        elif nd.op == "ExpandDims" and ins:
            r0 = _static_rank(ins[0], depth + 1)
            r = None if r0 is None else r0 + 1
        elif nd.op in ("ArgMin", "ArgMax") and ins:
            r0 = _static_rank(ins[0], depth + 1)
            r = None if r0 is None or r0 == 0 else r0 - 1
        elif nd.op == "Reshape" and len(ins) == 2:
            sv = _const_value(ins[1])
            r = None if sv is None else int(sv.size)
        elif nd.op in _REDUCE_OPS and len(ins) == 2:
            r0 = _static_rank(ins[0], depth + 1)
            ax = _const_value(ins[1])
            kd = nd.attr.get("keep_dims")
            if r0 is not None and ax is not None and kd is not None:
                axes = {int(a) % r0 for a in ax.reshape(-1)} if r0 else set()
                r = r0 if kd.value else r0 - len(axes)
    t._rank = r
    return r


def _axis_input(input_tensor: Tensor, axis) -> Any:
    if axis is None:
        rk = _static_rank(input_tensor)
        if rk is None:
            rk = input_tensor.get_shape().ndims
        if rk is not None:
            return constant(np.arange(rk, dtype=np.int32), dtype=int32)
        r = rank(input_tensor)
        return range(0, r, 1)
    if isinstance(axis, Tensor):
        return axis
    return np.asarray(axis, dtype=np.int32)


def _reduction(op_type: str, input_tensor, axis, keep_dims, name, reduction_indices, out_bool=False):
    if axis is None:
        axis = reduction_indices
    x = convert_to_tensor(input_tensor)
    ax = _axis_input(x, axis)
    dt = bool_ if out_bool else x.dtype
    attrs = {"T": P.AttrValue.type(x.dtype), "Tidx": P.AttrValue.type(int32),
             "keep_dims": P.AttrValue.b(keep_dims)}
    if out_bool:
        attrs.pop("T")
    return _op(op_type, [("input", x), ("reduction_indices", ax)], attrs, name, out_dtypes=[dt]).outputs[0]


def reduce_sum(input_tensor, axis=None, keep_dims=False, name=None, reduction_indices=None, keepdims=None):
    return _reduction("Sum", input_tensor, axis, bool_or(keepdims, keep_dims), name, reduction_indices)


def reduce_min(input_tensor, axis=None, keep_dims=False, name=None, reduction_indices=None, keepdims=None):
    return _reduction("Min", input_tensor, axis, bool_or(keepdims, keep_dims), name, reduction_indices)


def reduce_max(input_tensor, axis=None, keep_dims=False, name=None, reduction_indices=None, keepdims=None):
    return _reduction("Max", input_tensor, axis, bool_or(keepdims, keep_dims), name, reduction_indices)


def reduce_prod(input_tensor, axis=None, keep_dims=False, name=None, reduction_indices=None, keepdims=None):
    return _reduction("Prod", input_tensor, axis, bool_or(keepdims, keep_dims), name, reduction_indices)


def reduce_mean(input_tensor, axis=None, keep_dims=False, name=None, reduction_indices=None, keepdims=None):
    return _reduction("Mean", input_tensor, axis, bool_or(keepdims, keep_dims), name, reduction_indices)


def reduce_all(input_tensor, axis=None, keep_dims=False, name=None, reduction_indices=None, keepdims=None):
    return _reduction("All", input_tensor, axis, bool_or(keepdims, keep_dims), name, reduction_indices, True)


def reduce_any(input_tensor, axis=None, keep_dims=False, name=None, reduction_indices=None, keepdims=None):
    return _reduction("Any", input_tensor, axis, bool_or(keepdims, keep_dims), name, reduction_indices, True)


def bool_or(a, b):
    return b if a is None else a


def _argreduce(op_type, input, axis, name, output_type):  # noqa: A002
    x = convert_to_tensor(input)
    ax = 0 if axis is None else axis
    return _op(op_type, [("input", x), ("dimension", ax if isinstance(ax, Tensor) else np.int32(ax))],
               {"T": P.AttrValue.type(x.dtype), "Tidx": P.AttrValue.type(int32),
                "output_type": P.AttrValue.type(output_type)}, name,
               out_dtypes=[as_dtype(output_type)]).outputs[0]


def argmin(input, axis=None, name=None, dimension=None, output_type=int64):  # noqa: A002
    return _argreduce("ArgMin", input, axis if axis is not None else dimension, name, output_type)


def argmax(input, axis=None, name=None, dimension=None, output_type=int64):  # noqa: A002
    return _argreduce("ArgMax", input, axis if axis is not None else dimension, name, output_type)


def matmul(a, b, transpose_a=False, transpose_b=False, adjoint_a=False, adjoint_b=False, name=None):
    a = convert_to_tensor(a)
    b = convert_to_tensor(b, dtype=a.dtype)
    ta, tb = transpose_a or adjoint_a, transpose_b or adjoint_b
    ra, rb = a.get_shape().ndims, b.get_shape().ndims
    if (ra is not None and ra > 2) or (rb is not None and rb > 2):
        return _op("BatchMatMulV2", [("x", a), ("y", b)],
                   {"T": P.AttrValue.type(a.dtype), "adj_x": P.AttrValue.b(ta), "adj_y": P.AttrValue.b(tb)},
                   name, out_dtypes=[a.dtype]).outputs[0]
    return _op("MatMul", [("a", a), ("b", b)],
               {"T": P.AttrValue.type(a.dtype), "transpose_a": P.AttrValue.b(ta),
                "transpose_b": P.AttrValue.b(tb)}, name, out_dtypes=[a.dtype]).outputs[0]


def cast(x, dtype, name=None):
    x = convert_to_tensor(x)
    dt = as_dtype(dtype)
    if dt == x.dtype:
        return x
    return _op("Cast", [("x", x)], {"SrcT": P.AttrValue.type(x.dtype), "DstT": P.AttrValue.type(dt)},
               name, out_dtypes=[dt]).outputs[0]


to_float = lambda x, name="ToFloat": cast(x, float32, name)  # noqa: E731
to_double = lambda x, name="ToDouble": cast(x, float64, name)  # noqa: E731
to_int32 = lambda x, name="ToInt32": cast(x, int32, name)  # noqa: E731
to_int64 = lambda x, name="ToInt64": cast(x, int64, name)  # noqa: E731


def reshape(tensor, shape, name=None):
    t = convert_to_tensor(tensor)
    shp = shape if isinstance(shape, Tensor) else np.asarray(shape, dtype=np.int32)
    return _op("Reshape", [("tensor", t), ("shape", shp)],
               {"T": P.AttrValue.type(t.dtype), "Tshape": P.AttrValue.type(int32)}, name,
               out_dtypes=[t.dtype]).outputs[0]


def squeeze(input, axis=None, name=None, squeeze_dims=None):  # noqa: A002
    x = convert_to_tensor(input)
    ax = axis if axis is not None else squeeze_dims
    if isinstance(ax, int):
        ax = [ax]
    return _op("Squeeze", [("input", x)], {"T": P.AttrValue.type(x.dtype),
                                           "squeeze_dims": P.AttrValue.ilist(ax or [])}, name,
               out_dtypes=[x.dtype]).outputs[0]


def expand_dims(input, axis=None, name=None, dim=None):  # noqa: A002
    x = convert_to_tensor(input)
    ax = axis if axis is not None else dim
    return _op("ExpandDims", [("input", x), ("dim", ax if isinstance(ax, Tensor) else np.int32(ax))],
               {"T": P.AttrValue.type(x.dtype), "Tdim": P.AttrValue.type(int32)}, name,
               out_dtypes=[x.dtype]).outputs[0]


def shape(input, name=None, out_type=int32):  # noqa: A002
    x = convert_to_tensor(input)
    return _op("Shape", [("input", x)], {"T": P.AttrValue.type(x.dtype), "out_type": P.AttrValue.type(out_type)},
               name, out_dtypes=[as_dtype(out_type)]).outputs[0]


def size(input, name=None, out_type=int32):  # noqa: A002
    x = convert_to_tensor(input)
    return _op("Size", [("input", x)], {"T": P.AttrValue.type(x.dtype), "out_type": P.AttrValue.type(out_type)},
               name, out_dtypes=[as_dtype(out_type)]).outputs[0]


def rank(input, name=None):  # noqa: A002
    x = convert_to_tensor(input)
    return _op("Rank", [("input", x)], {"T": P.AttrValue.type(x.dtype)}, name, out_dtypes=[int32]).outputs[0]


def fill(dims, value, name=None):
    """`Fill` with `<name>/dims` and `<name>/value` constants
    (reference: src/main/scala/org/tensorframes/dsl/package.scala:66-85)."""
    vdt = value.dtype if isinstance(value, Tensor) else _to_numpy(value, None)[1]
    d = dims if isinstance(dims, Tensor) else np.asarray(dims, dtype=np.int32)
    return _op("Fill", [("dims", d), ("value", value)], {"T": P.AttrValue.type(vdt)}, name,
               out_dtypes=[vdt], dtype_hint=vdt).outputs[0]


def zeros(shape, dtype=float32, name=None):
    dt = as_dtype(dtype)
    return fill(shape, np.zeros((), dtype=dt.as_numpy_dtype), name=name or "zeros")


def ones(shape, dtype=float32, name=None):
    dt = as_dtype(dtype)
    return fill(shape, np.ones((), dtype=dt.as_numpy_dtype), name=name or "ones")


def zeros_like(tensor, dtype=None, name=None):
    return _unary("ZerosLike", tensor, name)


def ones_like(tensor, dtype=None, name=None):
    return _unary("OnesLike", tensor, name)


def range(start, limit=None, delta=1, dtype=None, name="range"):  # noqa: A001
    if limit is None:
        start, limit = 0, start
    dt = as_dtype(dtype) if dtype is not None else (_first_dtype(start, limit, delta) or int32)
    return _op("Range", [("start", start), ("limit", limit), ("delta", delta)],
               {"Tidx": P.AttrValue.type(dt)}, name, out_dtypes=[dt], dtype_hint=dt).outputs[0]


def tile(input, multiples, name=None):  # noqa: A002
    x = convert_to_tensor(input)
    m = multiples if isinstance(multiples, Tensor) else np.asarray(multiples, dtype=np.int32)
    return _op("Tile", [("input", x), ("multiples", m)],
               {"T": P.AttrValue.type(x.dtype), "Tmultiples": P.AttrValue.type(int32)}, name,
               out_dtypes=[x.dtype]).outputs[0]


def stack(values, axis=0, name="stack"):
    dt = _first_dtype(*values) or _to_numpy(values[0], None)[1]
    return _op("Pack", [("values", list(values))],
               {"T": P.AttrValue.type(dt), "N": P.AttrValue.i(len(values)), "axis": P.AttrValue.i(axis)},
               name, out_dtypes=[dt], dtype_hint=dt, list_inputs=("values",)).outputs[0]


pack = stack


def unstack(value, num=None, axis=0, name="unstack"):
    x = convert_to_tensor(value)
    if num is None:
        num = x.get_shape().as_list()[axis]
    op = _op("Unpack", [("value", x)], {"T": P.AttrValue.type(x.dtype), "num": P.AttrValue.i(num),
                                        "axis": P.AttrValue.i(axis)}, name, n_out=num,
             out_dtypes=[x.dtype] * num)
    return op.outputs


def pad(tensor, paddings, mode="CONSTANT", constant_values=0, name=None):
    x = convert_to_tensor(tensor)
    pads = np.asarray(paddings, dtype=np.int32) if not isinstance(paddings, Tensor) else paddings
    mode = mode.upper()
    if mode == "CONSTANT":
        if constant_values == 0:
            return _op("Pad", [("input", x), ("paddings", pads)],
                       {"T": P.AttrValue.type(x.dtype), "Tpaddings": P.AttrValue.type(int32)}, name or "Pad",
                       out_dtypes=[x.dtype]).outputs[0]
        return _op("PadV2", [("input", x), ("paddings", pads),
                             ("constant_values", np.asarray(constant_values, dtype=x.dtype.as_numpy_dtype))],
                   {"T": P.AttrValue.type(x.dtype), "Tpaddings": P.AttrValue.type(int32)}, name or "PadV2",
                   out_dtypes=[x.dtype]).outputs[0]
    if mode not in ("REFLECT", "SYMMETRIC"):
        raise ValueError(f"Unknown padding mode: {mode}")
    return _op("MirrorPad", [("input", x), ("paddings", pads)],
               {"T": P.AttrValue.type(x.dtype), "Tpaddings": P.AttrValue.type(int32),
                "mode": P.AttrValue.s(mode)}, name or "MirrorPad", out_dtypes=[x.dtype]).outputs[0]


def split(value, num_or_size_splits, axis=0, num=None, name="split"):
    x = convert_to_tensor(value)
    if isinstance(num_or_size_splits, int):
        n = num_or_size_splits
        op = _op("Split", [("split_dim", np.int32(axis)), ("value", x)],
                 {"T": P.AttrValue.type(x.dtype), "num_split": P.AttrValue.i(n)}, name, n_out=n,
                 out_dtypes=[x.dtype] * n)
        return op.outputs
    sizes = np.asarray(num_or_size_splits, dtype=np.int32).reshape(-1)
    n = int(num if num is not None else sizes.size)
    op = _op("SplitV", [("value", x), ("size_splits", sizes), ("split_dim", np.int32(axis))],
             {"T": P.AttrValue.type(x.dtype), "Tlen": P.AttrValue.type(int32), "num_split": P.AttrValue.i(n)},
             name, n_out=n, out_dtypes=[x.dtype] * n)
    return op.outputs


def _scan(op_type, x, axis, exclusive, reverse, name):
    x = convert_to_tensor(x)
    return _op(op_type, [("x", x), ("axis", np.int32(axis))],
               {"T": P.AttrValue.type(x.dtype), "Tidx": P.AttrValue.type(int32),
                "exclusive": P.AttrValue.b(exclusive), "reverse": P.AttrValue.b(reverse)}, name,
               out_dtypes=[x.dtype]).outputs[0]


def cumsum(x, axis=0, exclusive=False, reverse=False, name=None):
    return _scan("Cumsum", x, axis, exclusive, reverse, name)


def cumprod(x, axis=0, exclusive=False, reverse=False, name=None):
    return _scan("Cumprod", x, axis, exclusive, reverse, name)


def clip_by_value(t, clip_value_min, clip_value_max, name=None):
    x = convert_to_tensor(t)
    return _op("ClipByValue", [("t", x), ("clip_value_min", clip_value_min), ("clip_value_max", clip_value_max)],
               {"T": P.AttrValue.type(x.dtype)}, name, out_dtypes=[x.dtype], dtype_hint=x.dtype).outputs[0]


def reverse(tensor, axis, name=None):
    x = convert_to_tensor(tensor)
    return _op("ReverseV2", [("tensor", x), ("axis", np.asarray(axis, dtype=np.int32).reshape(-1))],
               {"T": P.AttrValue.type(x.dtype), "Tidx": P.AttrValue.type(int32)}, name,
               out_dtypes=[x.dtype]).outputs[0]


reverse_v2 = reverse


def gather_nd(params, indices, name=None):
    p = convert_to_tensor(params)
    i = convert_to_tensor(indices) if isinstance(indices, Tensor) else convert_to_tensor(
        np.asarray(indices, dtype=np.int32))
    return _op("GatherNd", [("params", p), ("indices", i)],
               {"Tparams": P.AttrValue.type(p.dtype), "Tindices": P.AttrValue.type(i.dtype)}, name,
               out_dtypes=[p.dtype]).outputs[0]


def concat(values, axis, name="concat"):
    dt = _first_dtype(*values) or _to_numpy(values[0], None)[1]
    return _op("ConcatV2", [("values", list(values)), ("axis", np.int32(axis) if not isinstance(axis, Tensor) else axis)],
               {"T": P.AttrValue.type(dt), "N": P.AttrValue.i(len(values)), "Tidx": P.AttrValue.type(int32)},
               name, out_dtypes=[dt], dtype_hint=dt, list_inputs=("values",)).outputs[0]


def transpose(a, perm=None, name="transpose"):
    x = convert_to_tensor(a)
    if perm is None:
        rk = x.get_shape().ndims
        perm = list(reversed(builtin_range(rk)))
    p = perm if isinstance(perm, Tensor) else np.asarray(perm, dtype=np.int32)
    return _op("Transpose", [("x", x), ("perm", p)],
               {"T": P.AttrValue.type(x.dtype), "Tperm": P.AttrValue.type(int32)}, name,
               out_dtypes=[x.dtype]).outputs[0]


builtin_range = _builtins.range


def _int_vector(v):
    """An int32 vector operand given as numbers, a Tensor, or a list mixing
    both (packed, as TF does for a computed crop offset)."""
    if isinstance(v, Tensor):
        return v
    if isinstance(v, (list, tuple)) and any(isinstance(e, Tensor) for e in v):
        return stack([e if isinstance(e, Tensor) else np.int32(e) for e in v])
    return np.asarray(v, dtype=np.int32)


def slice(input_, begin, size, name=None):  # noqa: A001
    x = convert_to_tensor(input_)
    return _op("Slice", [("input", x), ("begin", _int_vector(begin)), ("size", _int_vector(size))],
               {"T": P.AttrValue.type(x.dtype), "Index": P.AttrValue.type(int32)}, name,
               out_dtypes=[x.dtype]).outputs[0]


def strided_slice(input_, begin, end, strides=None, begin_mask=0, end_mask=0, ellipsis_mask=0,
                  new_axis_mask=0, shrink_axis_mask=0, name=None):
    x = convert_to_tensor(input_)
    if strides is None:
        strides = [1] * len(begin)
    return _op("StridedSlice", [("input", x), ("begin", np.asarray(begin, dtype=np.int32)),
                                ("end", np.asarray(end, dtype=np.int32)),
                                ("strides", np.asarray(strides, dtype=np.int32))],
               {"T": P.AttrValue.type(x.dtype), "Index": P.AttrValue.type(int32),
                "begin_mask": P.AttrValue.i(begin_mask), "end_mask": P.AttrValue.i(end_mask),
                "ellipsis_mask": P.AttrValue.i(ellipsis_mask), "new_axis_mask": P.AttrValue.i(new_axis_mask),
                "shrink_axis_mask": P.AttrValue.i(shrink_axis_mask)}, name or "strided_slice",
               out_dtypes=[x.dtype]).outputs[0]


def _slice_helper(t: Tensor, item) -> Tensor:
    if not isinstance(item, tuple):
        item = (item,)
    begin, end, strides = [], [], []
    bm = em = elm = nam = sam = 0
    for i, s in enumerate(item):
        if s is Ellipsis:
            begin.append(0); end.append(0); strides.append(1)
            elm |= 1 << i
        elif s is None:
            begin.append(0); end.append(0); strides.append(1)
            nam |= 1 << i
        elif isinstance(s, builtins_slice):
            begin.append(s.start or 0)
            end.append(s.stop or 0)
            strides.append(s.step or 1)
            if s.start is None:
                bm |= 1 << i
            if s.stop is None:
                em |= 1 << i
        else:
            begin.append(int(s)); end.append(int(s) + 1); strides.append(1)
            sam |= 1 << i
    return strided_slice(t, begin, end, strides, bm, em, elm, nam, sam)


builtins_slice = _builtins.slice


def gather(params, indices, axis=0, name=None):
    p = convert_to_tensor(params)
    ix = convert_to_tensor(indices) if isinstance(indices, Tensor) else np.asarray(indices, dtype=np.int32)
    idt = ix.dtype if isinstance(ix, Tensor) else as_dtype(ix.dtype)
    return _op("GatherV2", [("params", p), ("indices", ix), ("axis", np.int32(axis))],
               {"Tparams": P.AttrValue.type(p.dtype), "Tindices": P.AttrValue.type(idt),
                "Taxis": P.AttrValue.type(int32)}, name, out_dtypes=[p.dtype]).outputs[0]


def one_hot(indices, depth, on_value=1.0, off_value=0.0, axis=-1, dtype=float32, name=None):
    ix = convert_to_tensor(indices)
    dt = as_dtype(dtype)
    return _op("OneHot", [("indices", ix), ("depth", np.int32(depth)),
                          ("on_value", np.asarray(on_value, dtype=dt.as_numpy_dtype)),
                          ("off_value", np.asarray(off_value, dtype=dt.as_numpy_dtype))],
               {"T": P.AttrValue.type(dt), "TI": P.AttrValue.type(ix.dtype), "axis": P.AttrValue.i(axis)},
               name, out_dtypes=[dt]).outputs[0]


def where(condition, x=None, y=None, name=None):
    if x is None or y is None:
        raise NotImplementedError("where(condition) (index form) is data-dependent and not supported")
    dt = _first_dtype(x, y)
    return _op("Select", [("condition", condition), ("t", x), ("e", y)], {"T": P.AttrValue.type(dt)},
               name, out_dtypes=[dt], dtype_hint=dt).outputs[0]


def unsorted_segment_sum(data, segment_ids, num_segments, name=None):
    return _useg("UnsortedSegmentSum", data, segment_ids, num_segments, name)


def unsorted_segment_max(data, segment_ids, num_segments, name=None):
    return _useg("UnsortedSegmentMax", data, segment_ids, num_segments, name)


def unsorted_segment_min(data, segment_ids, num_segments, name=None):
    return _useg("UnsortedSegmentMin", data, segment_ids, num_segments, name)


def unsorted_segment_prod(data, segment_ids, num_segments, name=None):
    return _useg("UnsortedSegmentProd", data, segment_ids, num_segments, name)


def _useg(op_type, data, segment_ids, num_segments, name):
    x = convert_to_tensor(data)
    ids = convert_to_tensor(segment_ids)
    ns = num_segments if isinstance(num_segments, Tensor) else np.int32(num_segments)
    return _op(op_type, [("data", x), ("segment_ids", ids), ("num_segments", ns)],
               {"T": P.AttrValue.type(x.dtype), "Tindices": P.AttrValue.type(ids.dtype),
                "Tnumsegments": P.AttrValue.type(int32)}, name, out_dtypes=[x.dtype]).outputs[0]


# ------------------------------------------------------------------ tf.nn
def broadcast_to(input, shape, name=None):  # noqa: A002
    x = convert_to_tensor(input)
    return _op("BroadcastTo", [("input", x), ("shape", np.asarray(shape, dtype=np.int32))],
               {"T": P.AttrValue.type(x.dtype), "Tidx": P.AttrValue.type(int32)}, name, out_dtypes=[x.dtype]).outputs[0]


def depth_to_space(input, block_size, name=None, data_format="NHWC"):  # noqa: A002
    x = convert_to_tensor(input)
    return _op("DepthToSpace", [("input", x)],
               {"T": P.AttrValue.type(x.dtype), "block_size": P.AttrValue.i(block_size),
                "data_format": P.AttrValue.s(data_format)}, name, out_dtypes=[x.dtype]).outputs[0]


def space_to_depth(input, block_size, name=None, data_format="NHWC"):  # noqa: A002
    x = convert_to_tensor(input)
    return _op("SpaceToDepth", [("input", x)],
               {"T": P.AttrValue.type(x.dtype), "block_size": P.AttrValue.i(block_size),
                "data_format": P.AttrValue.s(data_format)}, name, out_dtypes=[x.dtype]).outputs[0]


def space_to_batch_nd(input, block_shape, paddings, name=None):  # noqa: A002
    x = convert_to_tensor(input)
    return _op("SpaceToBatchND", [("input", x), ("block_shape", np.asarray(block_shape, dtype=np.int32)),
                                  ("paddings", np.asarray(paddings, dtype=np.int32))],
               {"T": P.AttrValue.type(x.dtype), "Tblock_shape": P.AttrValue.type(int32),
                "Tpaddings": P.AttrValue.type(int32)}, name, out_dtypes=[x.dtype]).outputs[0]


def batch_to_space_nd(input, block_shape, crops, name=None):  # noqa: A002
    x = convert_to_tensor(input)
    return _op("BatchToSpaceND", [("input", x), ("block_shape", np.asarray(block_shape, dtype=np.int32)),
                                  ("crops", np.asarray(crops, dtype=np.int32))],
               {"T": P.AttrValue.type(x.dtype), "Tblock_shape": P.AttrValue.type(int32),
                "Tcrops": P.AttrValue.type(int32)}, name, out_dtypes=[x.dtype]).outputs[0]


class _NN:
    @staticmethod
    def relu(features, name=None):
        return _unary("Relu", features, name)

    @staticmethod
    def relu6(features, name=None):
        return _unary("Relu6", features, name)

    @staticmethod
    def elu(features, name=None):
        return _unary("Elu", features, name)

    @staticmethod
    def selu(features, name=None):
        return _unary("Selu", features, name)

    @staticmethod
    def sigmoid(x, name=None):
        return _unary("Sigmoid", x, name)

    @staticmethod
    def tanh(x, name=None):
        return _unary("Tanh", x, name)

    @staticmethod
    def softplus(features, name=None):
        return _unary("Softplus", features, name)

    @staticmethod
    def softmax(logits, name=None):
        return _op("Softmax", [("logits", logits)], {"T": P.AttrValue.type(logits.dtype)}, name,
                   out_dtypes=[logits.dtype]).outputs[0]

    @staticmethod
    def log_softmax(logits, name=None):
        return _op("LogSoftmax", [("logits", logits)], {"T": P.AttrValue.type(logits.dtype)}, name,
                   out_dtypes=[logits.dtype]).outputs[0]

    @staticmethod
    def conv2d_transpose(value, filter, output_shape, strides, padding="SAME",  # noqa: A002
                         data_format="NHWC", name=None, dilations=(1, 1, 1, 1)):
        """tf.nn.conv2d_transpose: a Conv2DBackpropInput node; `filter` is
        [height, width, output_channels, in_channels] as in TF."""
        x = convert_to_tensor(value)
        return _op("Conv2DBackpropInput",
                   [("input_sizes", np.asarray(output_shape, dtype=np.int32)), ("filter", filter),
                    ("out_backprop", x)],
                   {"T": P.AttrValue.type(x.dtype), "strides": P.AttrValue.ilist(strides),
                    "padding": P.AttrValue.s(padding), "data_format": P.AttrValue.s(data_format),
                    "dilations": P.AttrValue.ilist(dilations), "use_cudnn_on_gpu": P.AttrValue.b(True)},
                   name or "conv2d_transpose", out_dtypes=[x.dtype], dtype_hint=x.dtype).outputs[0]

    @staticmethod
    def l2_loss(t, name=None):
        return _op("L2Loss", [("t", t)], {"T": P.AttrValue.type(t.dtype)}, name, out_dtypes=[t.dtype]).outputs[0]

    @staticmethod
    def softmax_cross_entropy_with_logits(_sentinel=None, labels=None, logits=None, dim=-1, name=None):
        """Per-row loss (the op's first output; reference TF-1.x semantics)."""
        op = _op("SoftmaxCrossEntropyWithLogits", [("features", logits), ("labels", labels)],
                 {"T": P.AttrValue.type(logits.dtype)}, name, n_out=2, out_dtypes=[logits.dtype, logits.dtype])
        return op.outputs[0]

    softmax_cross_entropy_with_logits_v2 = softmax_cross_entropy_with_logits

    @staticmethod
    def sparse_softmax_cross_entropy_with_logits(_sentinel=None, labels=None, logits=None, name=None):
        lab = convert_to_tensor(labels)
        op = _op("SparseSoftmaxCrossEntropyWithLogits", [("features", logits), ("labels", lab)],
                 {"T": P.AttrValue.type(logits.dtype), "Tlabels": P.AttrValue.type(lab.dtype)}, name, n_out=2,
                 out_dtypes=[logits.dtype, logits.dtype])
        return op.outputs[0]

    @staticmethod
    def depth_to_space(input, block_size, name=None, data_format="NHWC"):  # noqa: A002
        return depth_to_space(input, block_size, name, data_format)

    @staticmethod
    def space_to_depth(input, block_size, name=None, data_format="NHWC"):  # noqa: A002
        return space_to_depth(input, block_size, name, data_format)

    @staticmethod
    def atrous_conv2d(value, filters, rate, padding, name=None):
        """TF-1.x emission: SpaceToBatchND -> VALID Conv2D -> BatchToSpaceND
        (paddings/crops computed for the static spatial size; SAME or VALID)."""
        x = convert_to_tensor(value)
        h, w = x.get_shape().as_list()[1:3]
        fh, fw = (filters.get_shape().as_list()[:2] if isinstance(filters, Tensor) else np.shape(filters)[:2])
        if h is None or w is None:
            raise ValueError("atrous_conv2d needs a static spatial size")
        ekh, ekw = (fh - 1) * rate + 1, (fw - 1) * rate + 1
        if padding == "SAME":
            ph, pw = ekh - 1, ekw - 1
            pads = [[ph // 2, ph - ph // 2], [pw // 2, pw - pw // 2]]
        else:
            pads = [[0, 0], [0, 0]]
        # extra bottom/right padding so that the padded size divides by rate
        base = [[pads[0][0], pads[0][1]], [pads[1][0], pads[1][1]]]
        crops = [[0, 0], [0, 0]]
        for i, s in enumerate((h, w)):
            tot = s + base[i][0] + base[i][1]
            extra = (-tot) % rate
            base[i][1] += extra
            crops[i][1] = extra
        with name_scope(name or "atrous_conv2d"):
            stb = space_to_batch_nd(x, [rate, rate], base)
            y = _NN.conv2d(stb, filters, [1, 1, 1, 1], "VALID")
            return batch_to_space_nd(y, [rate, rate], crops)

    @staticmethod
    def bias_add(value, bias, data_format=None, name=None):
        v = convert_to_tensor(value)
        return _op("BiasAdd", [("value", v), ("bias", bias)],
                   {"T": P.AttrValue.type(v.dtype), "data_format": P.AttrValue.s(data_format or "NHWC")},
                   name, out_dtypes=[v.dtype], dtype_hint=v.dtype).outputs[0]

    @staticmethod
    def conv2d(input, filter=None, strides=None, padding=None, use_cudnn_on_gpu=True,  # noqa: A002
               data_format="NHWC", dilations=(1, 1, 1, 1), name=None, filters=None):
        x = convert_to_tensor(input)
        w = filter if filter is not None else filters
        return _op("Conv2D", [("input", x), ("filter", w)],
                   {"T": P.AttrValue.type(x.dtype), "strides": P.AttrValue.ilist(strides),
                    "padding": P.AttrValue.s(padding), "data_format": P.AttrValue.s(data_format),
                    "use_cudnn_on_gpu": P.AttrValue.b(use_cudnn_on_gpu),
                    "dilations": P.AttrValue.ilist(dilations)}, name, out_dtypes=[x.dtype],
                   dtype_hint=x.dtype).outputs[0]

    @staticmethod
    def depthwise_conv2d_native(input, filter, strides, padding, data_format="NHWC",  # noqa: A002
                                dilations=(1, 1, 1, 1), name=None):
        x = convert_to_tensor(input)
        return _op("DepthwiseConv2dNative", [("input", x), ("filter", filter)],
                   {"T": P.AttrValue.type(x.dtype), "strides": P.AttrValue.ilist(strides),
                    "padding": P.AttrValue.s(padding), "data_format": P.AttrValue.s(data_format),
                    "dilations": P.AttrValue.ilist(dilations)}, name, out_dtypes=[x.dtype],
                   dtype_hint=x.dtype).outputs[0]

    @staticmethod
    def depthwise_conv2d(input, filter, strides, padding, rate=None, name=None, data_format="NHWC"):  # noqa: A002
        r = [1, 1] if rate is None else list(rate)
        return _NN.depthwise_conv2d_native(input, filter, strides, padding, data_format,
                                           [1, r[0], r[1], 1], name or "depthwise")

    @staticmethod
    def leaky_relu(features, alpha=0.2, name=None):
        x = convert_to_tensor(features)
        return _op("LeakyRelu", [("features", x)], {"T": P.AttrValue.type(x.dtype), "alpha": P.AttrValue.f(alpha)},
                   name, out_dtypes=[x.dtype]).outputs[0]

    @staticmethod
    def local_response_normalization(input, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5, name=None):  # noqa: A002
        x = convert_to_tensor(input)
        return _op("LRN", [("input", x)], {"T": P.AttrValue.type(x.dtype), "depth_radius": P.AttrValue.i(depth_radius),
                                           "bias": P.AttrValue.f(bias), "alpha": P.AttrValue.f(alpha),
                                           "beta": P.AttrValue.f(beta)}, name, out_dtypes=[x.dtype]).outputs[0]

    lrn = local_response_normalization

    @staticmethod
    def max_pool(value, ksize, strides, padding, data_format="NHWC", name=None):
        x = convert_to_tensor(value)
        return _op("MaxPool", [("input", x)],
                   {"T": P.AttrValue.type(x.dtype), "ksize": P.AttrValue.ilist(ksize),
                    "strides": P.AttrValue.ilist(strides), "padding": P.AttrValue.s(padding),
                    "data_format": P.AttrValue.s(data_format)}, name, out_dtypes=[x.dtype]).outputs[0]

    @staticmethod
    def avg_pool(value, ksize, strides, padding, data_format="NHWC", name=None):
        x = convert_to_tensor(value)
        return _op("AvgPool", [("value", x)],
                   {"T": P.AttrValue.type(x.dtype), "ksize": P.AttrValue.ilist(ksize),
                    "strides": P.AttrValue.ilist(strides), "padding": P.AttrValue.s(padding),
                    "data_format": P.AttrValue.s(data_format)}, name, out_dtypes=[x.dtype]).outputs[0]

    @staticmethod
    def fused_batch_norm(x, scale, offset, mean, variance, epsilon=0.001, data_format="NHWC",
                         is_training=False, name=None):
        x = convert_to_tensor(x)
        op = _op("FusedBatchNorm", [("x", x), ("scale", scale), ("offset", offset), ("mean", mean),
                                    ("variance", variance)],
                 {"T": P.AttrValue.type(x.dtype), "epsilon": P.AttrValue.f(epsilon),
                  "data_format": P.AttrValue.s(data_format), "is_training": P.AttrValue.b(is_training)},
                 name, n_out=5, out_dtypes=[x.dtype] * 5, dtype_hint=x.dtype)
        return op.outputs[0], op.outputs[1], op.outputs[2]

    @staticmethod
    def l2_normalize(x, axis=None, epsilon=1e-12, name=None, dim=None):
        ax = axis if axis is not None else dim
        with name_scope(name or "l2_normalize"):
            x = convert_to_tensor(x)
            sq = reduce_sum(square(x), ax, keep_dims=True)
            inv = rsqrt(maximum(sq, np.asarray(epsilon, dtype=x.dtype.as_numpy_dtype)))
            return multiply(x, inv, name=None)

    @staticmethod
    def top_k(input, k=1, sorted=True, name=None):  # noqa: A002
        x = convert_to_tensor(input)
        op = _op("TopKV2", [("input", x), ("k", np.int32(k))],
                 {"T": P.AttrValue.type(x.dtype), "sorted": P.AttrValue.b(sorted)}, name, n_out=2,
                 out_dtypes=[x.dtype, int32])
        return op.outputs[0], op.outputs[1]


nn = _NN()


class _Image:
    """``tf.image``: decoders (host ops, run by the map_rows host stage) and
    resize / crop / dtype conversion (GPU kernels)."""

    @staticmethod
    def decode_jpeg(contents, channels=0, name=None):
        return _op("DecodeJpeg", [("contents", contents)], {"channels": P.AttrValue.i(channels)}, name,
                   out_dtypes=[uint8], dtype_hint=string).outputs[0]

    @staticmethod
    def decode_png(contents, channels=0, dtype=uint8, name=None):
        dt = as_dtype(dtype)
        return _op("DecodePng", [("contents", contents)], {"channels": P.AttrValue.i(channels),
                                                    "dtype": P.AttrValue.type(dt)}, name,
                   out_dtypes=[dt], dtype_hint=string).outputs[0]

    @staticmethod
    def decode_image(contents, channels=0, dtype=uint8, name=None):
        dt = as_dtype(dtype)
        return _op("DecodeImage", [("contents", contents)], {"channels": P.AttrValue.i(channels),
                                                      "dtype": P.AttrValue.type(dt)}, name,
                   out_dtypes=[dt], dtype_hint=string).outputs[0]

    @staticmethod
    def resize_bilinear(images, size, align_corners=False, half_pixel_centers=False, name=None):
        x = convert_to_tensor(images)
        return _op("ResizeBilinear", [("images", x), ("size", _int_vector(size))],
                   {"T": P.AttrValue.type(x.dtype), "align_corners": P.AttrValue.b(align_corners),
                    "half_pixel_centers": P.AttrValue.b(half_pixel_centers)}, name,
                   out_dtypes=[float32]).outputs[0]

    @staticmethod
    def resize_nearest_neighbor(images, size, align_corners=False, half_pixel_centers=False, name=None):
        x = convert_to_tensor(images)
        return _op("ResizeNearestNeighbor", [("images", x), ("size", _int_vector(size))],
                   {"T": P.AttrValue.type(x.dtype), "align_corners": P.AttrValue.b(align_corners),
                    "half_pixel_centers": P.AttrValue.b(half_pixel_centers)}, name,
                   out_dtypes=[x.dtype]).outputs[0]

    @staticmethod
    def resize_images(images, size, method=0, align_corners=False, name=None):
        """TF-1.x ``resize_images``: 3-D images get a batch dim for the op (method
        0 = bilinear, 1 = nearest)."""
        x = convert_to_tensor(images)
        rank = x.get_shape().ndims
        with name_scope(name or "resize_images"):
            if rank == 3:
                x = expand_dims(x, 0)
            fn = _Image.resize_bilinear if method == 0 else _Image.resize_nearest_neighbor
            y = fn(x, size, align_corners=align_corners)
            if rank == 3:
                y = squeeze(y, [0])
            return y

    @staticmethod
    def central_crop_to(image, height, width, name=None):
        """Central crop of a [H, W, C] (or [N, H, W, C]) image with static H, W."""
        x = convert_to_tensor(image)
        dims = x.get_shape().as_list()
        h, w = dims[-3], dims[-2]
        if h is None or w is None:
            raise ValueError("central_crop_to needs static image height/width (resize first)")
        oy, ox = (h - height) // 2, (w - width) // 2
        if len(dims) == 3:
            return slice(x, [oy, ox, 0], [height, width, -1], name=name)
        return slice(x, [0, oy, ox, 0], [-1, height, width, -1], name=name)

    @staticmethod
    def convert_image_dtype(image, dtype, name=None):
        """uint8 [0,255] -> float [0,1) (and float -> float cast)."""
        x = convert_to_tensor(image)
        dt = as_dtype(dtype)
        if x.dtype == dt:
            return x
        with name_scope(name or "convert_image"):
            y = cast(x, dt)
            if x.dtype == uint8 and dt.is_floating:
                y = multiply(y, np.asarray(1.0 / 255.0, dtype=dt.as_numpy_dtype))
            return y


image = _Image()
math = __import__("types").SimpleNamespace(
    add=add, subtract=subtract, multiply=multiply, divide=truediv, square=square, sqrt=sqrt,
    reduce_sum=reduce_sum, reduce_min=reduce_min, reduce_max=reduce_max, reduce_mean=reduce_mean,
    argmin=argmin, argmax=argmax, reciprocal=reciprocal, exp=exp, log=log, abs=abs,
    unsorted_segment_sum=unsorted_segment_sum, maximum=maximum, minimum=minimum,
)


# ------------------------------------------------------------------ local evaluation
class Session:
    """Runs a DSL graph on local tensors through the native executor (CPU or
    the current GPU). Mirrors ``tf.Session().run(fetches, feed_dict)``."""

    def __init__(self, graph: Optional[Graph] = None, device=None):
        self.graph = graph or get_default_graph()
        self.device = device

    def run(self, fetches, feed_dict=None):
        from ..engine import run_graph
        single = not isinstance(fetches, (list, tuple))
        fl = [fetches] if single else list(fetches)
        feeds = {}
        for k, v in (feed_dict or {}).items():
            name = k.op.name if isinstance(k, Tensor) else str(k).split(":")[0]
            feeds[name] = v
        names = [f.name if isinstance(f, Tensor) else str(f) for f in fl]
        outs = run_graph(self.graph.serialize(), names, feeds, device=self.device)
        return outs[0] if single else outs

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
