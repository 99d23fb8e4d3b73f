"""Algebraic GraphDef rewrites applied before a graph is planned.

pool-then-pointwise-conv reorder: `Conv2D_1x1(AvgPool(x))` ==
`AvgPool(Conv2D_1x1(x))`. A 1x1 stride-1 convolution acts on every pixel
independently and an average pool is a fixed weighted sum of pixels (per
output pixel, SAME padding included), so both are linear maps on different
axes and commute exactly in real arithmetic (the f32 result differs only by
summation order). The reordered form pools the conv's OUTPUT channels instead
of its input channels, and the 1x1 conv then reads the same tensor as its
sibling 1x1 convs: the pool branch of every Inception mixed block (reference
workload: src/main/python/tensorframes_snippets/read_image.py, BASELINE
config 5) pools 32-192 channels instead of 192-2048, and its conv joins the
block's horizontally fused sibling GEMM (runtime/executor.cpp).

Every fetchable tensor keeps its value: the rewritten Conv2D keeps its name
(now produced by the moved AvgPool), the original AvgPool node is untouched
(pruned from plans that no longer need it).
"""
from __future__ import annotations

from typing import Dict, List, Optional

from . import proto as P


def _node_of(ref: str) -> str:
    ref = ref[1:] if ref.startswith("^") else ref
    name, _, idx = ref.partition(":")
    return name if idx in ("", "0") else ref


def _ints(nd: P.NodeDef, key: str, default: List[int]) -> List[int]:
    a = nd.attr.get(key)
    if a is None or a.kind != "list":
        return default
    return list(a.value.get("i", default))


def _fmt(nd: P.NodeDef) -> str:
    a = nd.attr.get("data_format")
    v = a.value if a is not None else b"NHWC"
    return v.decode() if isinstance(v, bytes) else str(v)


def _weight_shape(nd: Optional[P.NodeDef]) -> Optional[List[int]]:
    if nd is None:
        return None
    if nd.op == "Const" and "value" in nd.attr:
        return list(nd.attr["value"].value.shape)
    if nd.op in ("Placeholder", "PlaceholderV2") and "shape" in nd.attr:  # a big Const in a light view
        shp = nd.attr["shape"].value
        return None if shp.unknown_rank else list(shp.dims)
    return None


def reorder_pool_conv(gdef: P.GraphDef) -> Optional[P.GraphDef]:
    """Patch (changed + new nodes) moving AvgPool after 1x1 stride-1 Conv2Ds
    that consume it; None when nothing matches."""
    nodes: Dict[str, P.NodeDef] = {n.name: n for n in gdef.node}
    uses: Dict[str, int] = {}
    for n in gdef.node:
        for i in n.input:
            if not i.startswith("^"):
                uses[_node_of(i)] = uses.get(_node_of(i), 0) + 1
    patch: List[P.NodeDef] = []
    for conv in gdef.node:
        if conv.op != "Conv2D" or len(conv.input) < 2 or _fmt(conv) != "NHWC":
            continue
        if _ints(conv, "strides", [1, 1, 1, 1]) != [1, 1, 1, 1] or _ints(conv, "dilations", [1, 1, 1, 1]) != [1, 1, 1, 1]:
            continue
        w = _weight_shape(nodes.get(_node_of(conv.input[1])))
        if w is None or len(w) != 4 or w[0] != 1 or w[1] != 1:
            continue
        pool = nodes.get(_node_of(conv.input[0]))
        if pool is None or pool.op != "AvgPool" or _fmt(pool) != "NHWC" or uses.get(pool.name, 0) != 1:
            continue
        pre = P.NodeDef(conv.name + "/_tfa_prepool", "Conv2D", [pool.input[0], conv.input[1]], dict(conv.attr),
                        conv.device)
        moved = P.NodeDef(conv.name, "AvgPool", [pre.name], dict(pool.attr), pool.device)
        patch += [pre, moved]
    return P.GraphDef(patch, gdef.producer) if patch else None


def optimize(graph_bytes: bytes) -> Optional[bytes]:
    """Rewritten GraphDef bytes, or None when no rewrite applies."""
    if b"AvgPool" not in graph_bytes or b"Conv2D" not in graph_bytes:
        return None
    from .._native import _C
    light = P.parse_graphdef(_C.light_graphdef(graph_bytes, 4096))
    patch = reorder_pool_conv(light)
    if patch is None:
        return None
    return _C.patch_graphdef(graph_bytes, P.serialize_graphdef(patch))


__all__ = ["optimize", "reorder_pool_conv"]
