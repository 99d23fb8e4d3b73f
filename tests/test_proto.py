"""GraphDef codec tests: byte-level decode of the reference's fixtures
(reference: src/test/resources/graph.pb, graph2.pb — copied to tests/fixtures),
TensorProto encodings (tensor_content, typed *_val, repeat-last fill rule),
round trips through the Python and C++ codecs
(reference: src/test/scala/org/tensorframes/DenseTensorSuite.scala:8-18)."""
import os
import struct

import numpy as np
import pytest

from tensorframes_amd._native import _C
from tensorframes_amd.graph import proto as P
from tensorframes_amd.utils import dtypes as D

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def _read(name):
    with open(os.path.join(FIX, name), "rb") as f:
        return f.read()


def test_reference_graph_pb_decodes():
    g = P.parse_graphdef(_read("ref_graph.pb"))
    names = {n.name: n for n in g.node}
    assert set(names) == {"matrix1", "x"}
    m = names["matrix1"]
    assert m.op == "Const"
    t = m.attr["value"].value
    assert t.dtype == D.DT_FLOAT and t.shape == [1, 2]
    np.testing.assert_array_equal(t.to_numpy(), np.array([[3.0, 3.0]], dtype=np.float32))
    x = names["x"]
    assert x.op == "Placeholder"
    assert x.attr["dtype"].value == D.DT_FLOAT


def test_reference_graph2_pb_runs_natively():
    b = _read("ref_graph2.pb")
    g = P.parse_graphdef(b)
    assert [n.op for n in g.node].count("Placeholder") == 2
    import torch
    from tensorframes_amd import engine
    out = engine.run_graph(b, ["out"], {"z_1": np.ones((2, 2), np.float32),
                                        "z_2": np.full((2, 2), 2, np.float32)}, device="cpu")
    np.testing.assert_array_equal(out[0], np.full((2, 2), 3, np.float32))


def test_cpp_roundtrip_is_stable():
    for name in ("ref_graph.pb", "ref_graph2.pb"):
        b = _read(name)
        once = _C.roundtrip_graphdef(b)
        assert _C.roundtrip_graphdef(once) == once
        g1, g2 = P.parse_graphdef(b), P.parse_graphdef(once)
        assert [(n.name, n.op, n.input) for n in g1.node] == [(n.name, n.op, n.input) for n in g2.node]


def test_python_serializer_matches_cpp_decoder():
    arr = np.arange(12, dtype=np.float64).reshape(3, 4)
    g = P.GraphDef([P.NodeDef("c", "Const", [], {"dtype": P.AttrValue.type(D.DT_DOUBLE),
                                                 "value": P.AttrValue.tensor(P.TensorProto.from_numpy(arr))})])
    b = P.serialize_graphdef(g)
    from tensorframes_amd import engine
    out = engine.run_graph(b, ["c"], {}, device="cpu")
    np.testing.assert_array_equal(out[0], arr)


def _tensor_bytes(dtype, dims, field, payload):
    shape = b"".join(P._ld(2, P._key(1, 0) + P._varint(d)) for d in dims)
    return P._key(1, 0) + P._varint(dtype) + P._ld(2, shape) + payload


def test_typed_vals_and_fill_rule():
    # double_val packed, fewer values than elements -> repeat last
    payload = P._ld(6, struct.pack("<2d", 1.5, 2.5))
    t = _C.decode_tensor_proto(_tensor_bytes(D.DT_DOUBLE, [4], 6, payload))
    assert t.tolist() == [1.5, 2.5, 2.5, 2.5]
    # int_val unpacked, int32
    payload = P._key(7, 0) + P._varint(7) + P._key(7, 0) + P._varint((1 << 64) - 3)
    t = _C.decode_tensor_proto(_tensor_bytes(D.DT_INT32, [3], 7, payload))
    assert t.tolist() == [7, -3, -3]
    # no values: zeros
    t = _C.decode_tensor_proto(_tensor_bytes(D.DT_INT64, [2, 2], 10, b""))
    assert t.tolist() == [[0, 0], [0, 0]]
    # python decoder agrees
    pt = P._dec_tensor(_tensor_bytes(D.DT_DOUBLE, [3], 6, P._ld(6, struct.pack("<d", 9.0))))
    assert pt.to_numpy().tolist() == [9.0, 9.0, 9.0]


@pytest.mark.parametrize("value,dtype", [(3.0, D.DT_DOUBLE), (7, D.DT_INT32), (2.5, D.DT_FLOAT),
                                         (1 << 40, D.DT_INT64)])
def test_scalar_tensor_little_endian(value, dtype):
    t = P.TensorProto.from_numpy(np.asarray(value, dtype=D.numpy_dtype(dtype)), dtype)
    fmt = {D.DT_DOUBLE: "<d", D.DT_INT32: "<i", D.DT_FLOAT: "<f", D.DT_INT64: "<q"}[dtype]
    assert t.content == struct.pack(fmt, value)
    assert t.shape == []
    back = _C.decode_tensor_proto(P._enc_tensor(t))
    assert back.item() == value


def test_attr_kinds_roundtrip():
    n = P.NodeDef("n", "Foo", ["a", "b:1", "^c"], {
        "s": P.AttrValue.s("SAME"), "i": P.AttrValue.i(-5), "f": P.AttrValue.f(0.25),
        "b": P.AttrValue.b(True), "t": P.AttrValue.type(D.DT_FLOAT),
        "shape": P.AttrValue.shape([None, 3]), "ul": P.AttrValue.ilist([1, 2, -1]),
        "tl": P.AttrValue.tlist([D.DT_FLOAT, D.DT_INT32]),
    })
    g2 = P.parse_graphdef(P.serialize_graphdef(P.GraphDef([n])))
    m = g2.node[0]
    assert m.input == ["a", "b:1", "^c"]
    assert m.attr["s"].value == b"SAME" and m.attr["i"].value == -5 and m.attr["f"].value == 0.25
    assert m.attr["b"].value is True and m.attr["t"].value == D.DT_FLOAT
    assert m.attr["shape"].value.dims == [-1, 3]
    assert m.attr["ul"].value["i"] == [1, 2, -1]
    assert m.attr["tl"].value["type"] == [D.DT_FLOAT, D.DT_INT32]


def _py_enc(n, view):
    from tensorframes_amd.graph.dsl import Graph
    vn = Graph._view_node(n) if view else n
    e = P._ld(1, P.serialize_node(vn))
    return b"".join(e.parts) if isinstance(e, P._Rope) else e


def _zoo_nodes():
    """Nodes covering every attr kind, typed-val dtype and view rule."""
    T = P.TensorProto.from_numpy
    nodes = []
    for i, (arr, dt) in enumerate([
            (np.float32(1.5), None), (np.float64(-2.25), None), (np.int32(-7), None), (np.int64(-(1 << 40)), None),
            (np.bool_(True), None), (np.float16(3.0), None), (np.uint8(200), None), (np.int16(-300), None),
            (np.int8(-5), None), (np.zeros((0, 3), np.float32), None), (np.arange(6, dtype=np.int32).reshape(2, 3), None),
            (np.ones((40, 40), np.float64), None),
            (np.array([b"ab", b"c"], dtype=object), D.DT_STRING)]):
        tp = T(arr, dt)
        nodes.append(P.NodeDef(f"c{i}", "Const", [], {"dtype": P.AttrValue.type(tp.dtype), "value": P.AttrValue.tensor(tp)}))
    bf = P.TensorProto(D.DT_BFLOAT16, [1], b"\x80\x3f")  # one bf16 element: tensor_content, not a typed val
    nodes.append(P.NodeDef("bf", "Const", [], {"dtype": P.AttrValue.type(D.DT_BFLOAT16), "value": P.AttrValue.tensor(bf)}))
    nodes.append(P.NodeDef("p", "Placeholder", [], {"dtype": P.AttrValue.type(D.DT_FLOAT),
                                                    "shape": P.AttrValue.shape([None, 3, 0])}))
    nodes.append(P.NodeDef("q", "Placeholder", [], {"dtype": P.AttrValue.type(D.DT_FLOAT), "shape": P.AttrValue.shape(None)},
                           device="/device:GPU:0"))
    nodes.append(P.NodeDef("conv", "Conv2D", ["p", "c1:0", "^q"], {
        "T": P.AttrValue.type(D.DT_FLOAT), "strides": P.AttrValue.ilist([1, 2, 2, 1]), "padding": P.AttrValue.s("SAME"),
        "data_format": P.AttrValue.s(b"NHWC"), "use_cudnn_on_gpu": P.AttrValue.b(False), "axis": P.AttrValue.i(-1),
        "alpha": P.AttrValue.f(0.1), "names": P.AttrValue.slist(["a", "b"]), "Ts": P.AttrValue.tlist([D.DT_FLOAT, D.DT_INT32]),
        "_output_shapes": P.AttrValue.shapelist([[None, 4], None, []]), "empty": P.AttrValue.ilist([]),
        "fl": P.AttrValue("list", {"f": [0.5, -1.0], "b": [True, False]}),
        "tl": P.AttrValue("list", {"tensor": [T(np.arange(3, dtype=np.int64))]}),
        "ph": P.AttrValue("placeholder", "x"), "fn": P.AttrValue("func", "my_fn")}))
    return nodes


@pytest.mark.parametrize("view", [False, True])
def test_native_node_encoder_is_byte_identical(view):
    """csrc/proto/pyencode.cpp must write exactly what graph/proto.py writes."""
    nodes = _zoo_nodes()
    enc = _C.encode_nodes(nodes, 1024 if view else -1)
    assert len(enc) == len(nodes)
    for n, e in zip(nodes, enc):
        assert e is not None, n.name
        assert e == _py_enc(n, view), n.name


def test_native_encoder_falls_back_and_dsl_graphs_match():
    # a value the native encoder does not take (numpy int in an int attr) -> None, Python encodes it
    odd = P.NodeDef("odd", "Foo", [], {"n": P.AttrValue("i", np.int64(3))})
    assert _C.encode_nodes([odd], -1) == [None]
    from tensorframes_amd import tf
    from tensorframes_amd.models import kmeans
    g = tf.Graph()
    with g.as_default():
        pts = tf.placeholder(tf.double, [None, 5], name="features")
        d = kmeans.tf_compute_distances(pts, np.random.default_rng(0).standard_normal((3, 5)))
        tf.reduce_sum(tf.reduce_min(d, 1), name="total")
        tf.constant(np.ones((64, 64), np.float32), name="big")
    g._nodes.append(odd)
    ref = b"".join(_py_enc(n, False) for n in g._nodes)
    assert g.serialize().startswith(ref)
    assert g._shape_view() == b"".join(_py_enc(n, True) for n in g._nodes)
