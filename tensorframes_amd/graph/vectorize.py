"""Row-graph vectorisation for map_rows: rewrite a graph written against ONE
cell into the equivalent graph over a block of B cells (a new leading dim).

The reference runs map_rows one session.run per row (reference:
src/main/scala/org/tensorframes/impl/DebugRowOps.scala:832-856). Per-row
execution costs one program launch sequence per row; for row graphs built
from elementwise ops, reductions, reshapes and friends the block form gives
the same per-row results with one launch sequence per group of same-shaped
rows.

The rewrite is exact or refused: every op in the fetch closure that depends
on a fed cell must have a lifting rule below; anything else (Shape/Size, ops
with row-crossing semantics we cannot shift, mismatched broadcasting ranks)
makes `lift` return None and map_rows keeps its per-row loop. Tensors that
do not depend on the feeds are left untouched (constants broadcast against
the batched tensors, right-aligned, exactly as they did against one cell).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from ..utils import dtypes as D
from . import proto as P

# ops applied independently per element (any operand broadcasting checked below)
_UNARY = {
    "Abs", "Neg", "Square", "Sqrt", "Rsqrt", "Exp", "Expm1", "Log", "Log1p", "Reciprocal", "Inv", "Relu",
    "Relu6", "Elu", "Selu", "Sigmoid", "Tanh", "Softplus", "Softsign", "Floor", "Ceil", "Round", "Rint",
    "Sign", "Sin", "Cos", "Tan", "Erf", "LogicalNot", "IsNan", "IsInf", "IsFinite", "Cast", "Identity",
    "StopGradient", "Snapshot", "PreventGradient", "CheckNumerics", "ZerosLike", "OnesLike", "LeakyRelu",
}
_BINARY = {
    "Add", "AddV2", "Sub", "Mul", "Div", "RealDiv", "FloorDiv", "FloorMod", "TruncateDiv", "TruncateMod",
    "Mod", "Maximum", "Minimum", "Pow", "SquaredDifference", "Atan2", "DivNoNan", "Equal", "NotEqual",
    "Less", "LessEqual", "Greater", "GreaterEqual", "LogicalAnd", "LogicalOr", "BiasAdd",
}
_REDUCE = {"Sum", "Mean", "Max", "Min", "Prod", "All", "Any"}
_ARGRED = {"ArgMax", "ArgMin"}
_LAST_AXIS = {"Softmax", "LogSoftmax"}


class _Refuse(Exception):
    pass


def _const_node(name: str, arr: np.ndarray) -> P.NodeDef:
    tp = P.TensorProto.from_numpy(np.asarray(arr))
    return P.NodeDef(name, "Const", [], {"dtype": P.AttrValue.type(tp.dtype), "value": P.AttrValue.tensor(tp)})


def _split(inp: str) -> Tuple[str, int]:
    if inp.startswith("^"):
        return inp[1:], -1
    base, _, idx = inp.partition(":")
    return base, int(idx or 0)


def lift(gdef: P.GraphDef, fetches: List[str], feeds: List[str],
         infos: Dict[str, list], patch_only: bool = False) -> Optional[P.GraphDef]:
    """The block form of `gdef`, or None when the graph cannot be lifted
    exactly. `infos`: per-node inferred infos of the closure under the
    concrete cell shapes of one row group (`_C.infer_fed`). With
    `patch_only`, only the rewritten and new nodes are returned (to be
    applied with `_C.patch_graphdef` onto the full graph)."""
    try:
        return _lift(gdef, fetches, feeds, infos, patch_only)
    except _Refuse:
        return None


def _lift(gdef, fetches, feeds, infos, patch_only=False):
    nodes = {n.name: n for n in gdef.node}
    feed_set = set(feeds)
    # closure of the fetches, cut at feeds
    order, seen = [], set()

    def visit(name):
        stack = [(name, False)]
        while stack:
            n, done = stack.pop()
            if done:
                order.append(n)
                continue
            if n in seen:
                continue
            seen.add(n)
            stack.append((n, True))
            if n in feed_set:
                continue
            for i in nodes[n].input:
                stack.append((_split(i)[0], False))
    for f in fetches:
        visit(_split(f)[0])

    def rank(name, idx=0):
        info = infos.get(name)
        if not info or idx >= len(info) or info[idx]["shape"] is None:
            raise _Refuse(f"unknown rank of {name}:{idx}")
        return len(info[idx]["shape"])

    batched: Dict[str, bool] = {}
    out_nodes: Dict[str, P.NodeDef] = {}
    extra: List[P.NodeDef] = []

    def const_value(name) -> np.ndarray:
        nd = nodes.get(name)
        if nd is None or nd.op != "Const" or batched.get(name):
            raise _Refuse(f"{name} is not a constant")
        return np.asarray(nd.attr["value"].value.to_numpy())

    def shifted_const(node, arg_idx, fn):
        src = _split(node.input[arg_idx])[0]
        vals = fn(const_value(src))
        cname = f"{node.name}/_tfa_vec_{arg_idx}"
        extra.append(_const_node(cname, vals))
        new_inputs = list(node.input)
        new_inputs[arg_idx] = cname
        return new_inputs

    def shift_axes(a, r):
        a = np.asarray(a)
        return np.where(a >= 0, a + 1, a).astype(a.dtype)

    for name in order:
        nd = nodes[name]
        if name in feed_set:
            batched[name] = True
            if nd.op in ("Placeholder", "PlaceholderV2"):
                m = P.NodeDef(nd.name, nd.op, nd.input, dict(nd.attr), nd.device)
                shp = nd.attr.get("shape")
                if shp is not None and not shp.value.unknown_rank:
                    m.attr["shape"] = P.AttrValue.shape([None] + [None if d < 0 else d for d in shp.value.dims])
                out_nodes[name] = m
            else:
                out_nodes[name] = nd
            continue
        ins = [_split(i) for i in nd.input]
        data_ins = [(n, i) for n, i in ins if i >= 0]
        bflags = [batched.get(n, False) for n, _ in data_ins]
        if not any(bflags):
            batched[name] = False
            out_nodes[name] = nd
            continue
        batched[name] = True
        op = nd.op
        m = P.NodeDef(nd.name, op, list(nd.input), dict(nd.attr), nd.device)
        if op in _UNARY:
            pass
        elif op in _BINARY or op in ("Select", "SelectV2", "AddN", "ClipByValue"):
            if op == "BiasAdd" and nd.attr.get("data_format") and nd.attr["data_format"].value == b"NCHW":
                raise _Refuse("BiasAdd NCHW")
            ranks = [rank(n, i) for n, i in data_ins]
            br = max(r for r, b in zip(ranks, bflags) if b)
            if any(r > br for r, b in zip(ranks, bflags) if not b):
                raise _Refuse(f"{op}: constant operand outranks the cell")
            if op in ("Select", "BiasAdd") and len(set(r for r, b in zip(ranks, bflags) if b)) != 1:
                raise _Refuse(f"{op} with batched operands of different ranks")
            # a lower-rank batched operand [B, *c] gets unit dims after the batch
            # dim ([B, 1.., *c]) so it broadcasts against [B, *cell] as its cell did
            new_inputs = list(m.input)
            k = 0
            for pos, inp in enumerate(nd.input):
                n_, i_ = _split(inp)
                if i_ < 0:
                    continue
                r_, b_ = ranks[k], bflags[k]
                k += 1
                if b_ and r_ < br:
                    cur = inp
                    for e in range(br - r_):
                        en = f"{nd.name}/_tfa_vec_expand{pos}_{e}"
                        extra.append(_const_node(en + "/dim", np.asarray(1, np.int32)))
                        extra.append(P.NodeDef(en, "ExpandDims", [cur, en + "/dim"],
                                               {"T": P.AttrValue.type(infos[n_][i_]["dtype"]),
                                                "Tdim": P.AttrValue.type(D.DT_INT32)}))
                        cur = en
                    new_inputs[pos] = cur
            m.input = new_inputs
        elif op in _REDUCE:
            if bflags[1]:
                raise _Refuse("data-dependent reduction axes")
            r = rank(*data_ins[0])
            ax = const_value(_split(nd.input[1])[0])
            if ax.size == 0:
                pass  # reduce over nothing
            m.input = shifted_const(nd, 1, lambda a: shift_axes(a, r))
        elif op in _ARGRED:
            if bflags[1]:
                raise _Refuse("data-dependent arg axis")
            m.input = shifted_const(nd, 1, lambda a: shift_axes(a, 0))
        elif op in _LAST_AXIS:
            if rank(*data_ins[0]) < 1:
                raise _Refuse("softmax of a scalar")
        elif op == "Reshape":
            if bflags[1]:
                raise _Refuse("data-dependent reshape")
            shp = const_value(_split(nd.input[1])[0]).reshape(-1)
            if (shp == -1).any():
                # the cell's own -1 stays; the batch dim comes from the input's
                # leading dim, made explicit by an extra -1 only if unambiguous
                raise _Refuse("reshape with -1 inside the cell")
            m.input = shifted_const(nd, 1, lambda s: np.concatenate([[-1], np.asarray(s).reshape(-1)]).astype(s.dtype))
        elif op == "ExpandDims":
            if bflags[1]:
                raise _Refuse("data-dependent expand axis")
            m.input = shifted_const(nd, 1, lambda a: shift_axes(a, 0))
        elif op == "Squeeze":
            dims = list(nd.attr["squeeze_dims"].value.get("i", [])) if "squeeze_dims" in nd.attr else []
            if not dims:
                raise _Refuse("Squeeze without explicit dims")  # would squeeze a batch of one
            m.attr["squeeze_dims"] = P.AttrValue.ilist([d + 1 if d >= 0 else d for d in dims])
        elif op == "Transpose":
            if bflags[1]:
                raise _Refuse("data-dependent perm")
            m.input = shifted_const(nd, 1, lambda p: np.concatenate([[0], np.asarray(p).reshape(-1) + 1]).astype(p.dtype))
        elif op == "ConcatV2":
            if not all(bflags[:-1]) or bflags[-1]:
                raise _Refuse("concat of batched and constant parts")
            m.input = shifted_const(nd, len(nd.input) - 1, lambda a: shift_axes(a, 0))
        elif op == "Pack":
            if not all(bflags):
                raise _Refuse("pack of batched and constant parts")
            ax = nd.attr["axis"].value if "axis" in nd.attr else 0
            m.attr["axis"] = P.AttrValue.i(ax + 1 if ax >= 0 else ax)
        elif op in ("Cumsum", "Cumprod", "ReverseV2"):
            if bflags[1]:
                raise _Refuse(f"data-dependent {op} axis")
            m.input = shifted_const(nd, 1, lambda a: shift_axes(a, 0))
        elif op in ("Pad", "PadV2", "MirrorPad"):
            if any(bflags[1:]):
                raise _Refuse("data-dependent padding")
            m.input = shifted_const(nd, 1, lambda p: np.concatenate(
                [np.zeros((1, 2), np.asarray(p).dtype), np.asarray(p).reshape(-1, 2)]).astype(np.asarray(p).dtype))
        elif op in ("Split", "SplitV"):
            ax_i = 0 if op == "Split" else 2
            if any(b for k, b in enumerate(bflags) if k != (1 if op == "Split" else 0)):
                raise _Refuse("data-dependent split")
            m.input = shifted_const(nd, ax_i, lambda a: shift_axes(a, 0))
        elif op == "MatMul":
            # cell [m,k] x const [k,n]: the batch [B,m,k] is flattened to ONE
            # [B*m,k] x [k,n] GEMM (the MFMA kernel, fusable epilogue) and the
            # result viewed back as [B,m,n]
            if bflags[1] or rank(*data_ins[0]) != 2 or nd.attr.get("transpose_a") and nd.attr["transpose_a"].value:
                raise _Refuse("MatMul form not liftable")
            a_shape = infos[data_ins[0][0]][data_ins[0][1]]["shape"]
            o_shape = infos[name][0]["shape"]
            if any(d is None or d < 0 for d in list(a_shape) + list(o_shape)):
                raise _Refuse("MatMul with unknown cell dims")
            flat, mm = f"{name}/_tfa_vec_flat", f"{name}/_tfa_vec_mm"
            tattr = {"T": nd.attr["T"], "Tshape": P.AttrValue.type(D.DT_INT32)}
            extra.append(_const_node(flat + "/shape", np.asarray([-1, a_shape[1]], np.int32)))
            extra.append(P.NodeDef(flat, "Reshape", [nd.input[0], flat + "/shape"], dict(tattr)))
            extra.append(P.NodeDef(mm, "MatMul", [flat, nd.input[1]], dict(nd.attr), nd.device))
            extra.append(_const_node(name + "/_tfa_vec_shape", np.asarray([-1] + list(o_shape), np.int32)))
            m = P.NodeDef(nd.name, "Reshape", [mm, name + "/_tfa_vec_shape"], dict(tattr), nd.device)
        else:
            raise _Refuse(f"no lifting rule for {op}")
        out_nodes[name] = m

    for f in fetches:
        n, i = _split(f)
        if not batched.get(n, False):
            raise _Refuse("fetch does not depend on the row")  # per-row loop handles constants
    # feeds outside the fetch closure are still fed a batch
    for name in feeds:
        if name not in out_nodes and name in nodes and nodes[name].op in ("Placeholder", "PlaceholderV2"):
            nd = nodes[name]
            m = P.NodeDef(nd.name, nd.op, nd.input, dict(nd.attr), nd.device)
            shp = nd.attr.get("shape")
            if shp is not None and not shp.value.unknown_rank:
                m.attr["shape"] = P.AttrValue.shape([None] + [None if d < 0 else d for d in shp.value.dims])
            out_nodes[name] = m
    if patch_only:
        changed = [m for name, m in out_nodes.items() if m is not nodes[name]]
        return P.GraphDef(changed + extra, gdef.producer)
    new = [out_nodes.get(n.name, n) for n in gdef.node] + extra
    return P.GraphDef(new, gdef.producer)


def bakes_cell_sizes(gdef: "P.GraphDef") -> bool:
    """True when the lifted graph hard-codes cell dims (a lifted MatMul's
    [-1, m, n] reshape), so it is valid only for the cell shapes it was
    lifted for."""
    return any(n.name.endswith("/_tfa_vec_shape") for n in gdef.node)


__all__ = ["lift", "bakes_cell_sizes"]
