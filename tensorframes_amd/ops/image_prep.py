"""The batched image pre-stage of map_rows image scoring: the per-row part of
an image-scoring graph (decoded uint8 image -> the batch-of-one tensor the CNN
reads), recognised from the graph and run for a whole chunk of rows as ONE
ragged kernel (kernels/image.hip ragged_prep_kernel) instead of a short
program per row.

What it takes (reference: src/main/python/tensorframes_snippets/read_image.py:
35-75, the slim-style eval preprocessing the reference's users feed it, and
TFDataOps.scala:86-103 / DebugRowOps.scala:819-857 for the per-row contract):

* the pixel chain: Cast to float, ExpandDims(0) / Squeeze / Identity,
  ONE ResizeBilinear (uint8 or float input; any mode), ONE Slice (a crop),
  up to 4 elementwise steps with a constant (Add / Sub / Mul / RealDiv; a
  scalar or one value per channel), and a per-channel split -> elementwise ->
  concat (a mean subtraction written channel by channel), in graph order;
* the resize size and the crop offsets either as constants or computed from
  the image's own shape (Shape -> StridedSlice / Cast / arithmetic / Round /
  Minimum / Select / Pack ...: an aspect-preserving resize to a smallest side
  and its central crop). That shape-only part is evaluated here, on the host,
  once per chunk, for all its rows at once (numpy, the engine's own rounding
  rules: Round half to even, integer Div truncating, float ops in the tensor's
  dtype), and each row's (OH, OW, oy, ox) goes to the kernel.

Anything else keeps the per-row program. The batched result equals the
per-row program bit for bit (the kernel rounds like the CPU executor's ops:
no fused multiply-add), which tests/test_gpu_image_prep.py checks against the
CPU executor."""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import engine
from .._native import _C
from ..graph import proto as P
from ..utils import dtypes as D

_KIND = {"Add": 0, "AddV2": 0, "Sub": 1, "Mul": 2, "RealDiv": 3, "Div": 3}


class Unsupported(Exception):
    """the graph (or this chunk) is outside what the batched pre-stage models"""


class ImagePrep:
    """A recognised pre-stage: C channels (None: the decoder's), resize to
    (OH, OW) with `mode` (0 default, 1 align_corners, 2 half_pixel_centers),
    crop h x w at (oy, ox), elementwise `ops` [(kind, values)]. `dyn`, when
    set, gives each row's (OH, OW, oy, ox) from the chunk's image sizes."""

    def __init__(self, C, OH, OW, mode, oy, ox, h, w, ops, dyn: Optional[Callable] = None):
        self.C, self.OH, self.OW, self.mode = C, OH, OW, mode
        self.oy, self.ox, self.h, self.w, self.ops = oy, ox, h, w, ops
        self.dyn = dyn
        self._inflight: List[tuple] = []  # (event, pinned buffer) of copies not yet known done

    def channels(self, hf=None) -> Optional[int]:
        """The channel count the chain fixes (the cut's shape, a Slice size or
        a per-channel constant), else the decoder's (`channels` 1 / 3 / 4)."""
        if self.C is not None:
            return self.C
        return hf.channels if hf is not None and hf.channels in (1, 3, 4) else None

    def row_params(self, hw: np.ndarray) -> Optional[np.ndarray]:
        """int32 [R, 4] = each row's (OH, OW, oy, ox), or None when they are
        the constants; raises Unsupported when a row's values are outside what
        the kernel does (the chunk then runs per row)."""
        if self.dyn is None:
            return None
        p = self.dyn(hw)
        OH, OW, oy, ox = p[:, 0], p[:, 1], p[:, 2], p[:, 3]
        if not (np.all(OH > 0) and np.all(OW > 0) and np.all(oy >= 0) and np.all(ox >= 0) and
                np.all(oy + self.h <= OH) and np.all(ox + self.w <= OW)):
            raise Unsupported("a row's crop falls outside its resized image")
        return np.ascontiguousarray(p, dtype=np.int32)

    def run(self, imgs, dev) -> Optional[torch.Tensor]:
        """None when the chunk's images do not share one uint8 [H, W, C]
        layout the chain accepts (e.g. gray and RGB files under
        `channels=0`): the caller then runs those rows one by one."""
        arrs = [np.asarray(t) for t in imgs]
        C = self.C if self.C is not None else (arrs[0].shape[2] if arrs and arrs[0].ndim == 3 else None)
        if C is None or any(a.ndim != 3 or a.shape[2] != C or a.dtype != np.uint8 for a in arrs) or \
                any(len(v) not in (1, C) for _, v in self.ops):
            return None
        sizes = np.array([a.size for a in arrs], dtype=np.int64)
        offs = np.zeros(len(arrs), dtype=np.int64)
        np.cumsum(sizes[:-1], out=offs[1:])
        hw = np.array([[a.shape[0], a.shape[1]] for a in arrs], dtype=np.int32).reshape(-1, 2)
        total = int(sizes.sum())
        # meta (offsets, sizes) and pixels in one page-locked buffer, one DMA
        mbytes = offs.nbytes + hw.nbytes
        buf = _C.empty_pinned([mbytes + total], torch.uint8)
        hb = buf.numpy()
        hb[:offs.nbytes] = offs.view(np.uint8)
        hb[offs.nbytes:mbytes] = hw.reshape(-1).view(np.uint8)
        np.concatenate([a.reshape(-1) for a in arrs], out=hb[mbytes:])
        return self.run_packed(buf, offs.nbytes, mbytes, dev, C)

    def run_packed(self, buf: torch.Tensor, offs_nbytes: int, mbytes: int, dev, C: int) -> Optional[torch.Tensor]:
        """`buf` = [int64 offsets | int32 hw pairs | pixels] in pinned memory
        (the layout _C.JpegBatch decodes into), C channels per pixel. None:
        a row's computed sizes are outside the kernel's (run per row)."""
        rp = None
        if self.dyn is not None:
            hw = buf.numpy()[offs_nbytes:mbytes].view(np.int32).reshape(-1, 2)
            try:
                rp = torch.from_numpy(self.row_params(hw)).pin_memory()
            except Unsupported:
                return None
        d = engine.device_empty(buf.numel(), torch.uint8, dev)
        d.copy_(buf, non_blocking=True)
        # the pinned buffer returns to its pool only once its DMA has run
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        self._inflight = [(e, b) for e, b in self._inflight if not e.query()] + [(ev, buf)]
        doffs = d[:offs_nbytes].view(torch.int64)
        dhw = d[offs_nbytes:mbytes].view(torch.int32)
        return _C.ragged_image_prep(d[mbytes:], doffs, dhw, C, self.OH, self.OW, self.mode, self.oy, self.ox,
                                    self.h, self.w, self.ops, rp)


# ---------------------------------------------------------------- shape-only part

class _ShapeEval:
    """Evaluates the shape-only subgraph feeding a resize size / crop offset,
    for all rows of a chunk at once: every value is a numpy array with a
    leading row axis. Leaves are Const nodes and Shape of a pixel-chain tensor
    (whose per-row shape the chain walk recorded); anything else reading the
    pixels, or an op not listed, is Unsupported."""

    def __init__(self, by_name, shape_of: Dict[str, Callable]):
        self.by_name, self.shape_of = by_name, shape_of

    def __call__(self, ref: str, dims: Dict[int, Tuple[np.ndarray, np.ndarray]], R: int) -> np.ndarray:
        self.dims, self.R, self.memo = dims, R, {}
        return self.value(ref)

    def value(self, ref: str) -> np.ndarray:
        name, _, idx = ref.lstrip("^").partition(":")
        if idx not in ("", "0"):
            raise Unsupported(f"output {idx} of {name}")
        if name in self.memo:
            return self.memo[name]
        nd = self.by_name.get(name)
        if nd is None:
            raise Unsupported(f"no node {name}")
        v = self._eval(nd)
        self.memo[name] = v
        return v

    def _ins(self, nd):
        return [i for i in nd.input if not i.startswith("^")]

    def _eval(self, nd) -> np.ndarray:
        op, R = nd.op, self.R
        ins = self._ins(nd)
        if op == "Const":
            if "value" not in nd.attr:
                raise Unsupported("Const without value")
            v = np.asarray(nd.attr["value"].value.to_numpy())
            return np.broadcast_to(v[None], (R,) + v.shape)
        if op == "Shape":
            src = ins[0].split(":")[0]
            if src not in self.shape_of:
                raise Unsupported(f"Shape of {src}, not a pixel-chain tensor")
            dt = nd.attr["out_type"].value if "out_type" in nd.attr else D.DT_INT32
            try:
                return self.shape_of[src](self.dims, R).astype(D.numpy_dtype(dt))
            except KeyError:
                raise Unsupported(f"Shape of {src} before its size is known") from None
        if op in ("Identity", "StopGradient"):
            return self.value(ins[0])
        if op == "Cast":
            x = self.value(ins[0])
            dt = D.numpy_dtype(nd.attr["DstT"].value)
            if np.dtype(dt).kind == "b" or x.dtype.kind == "b":
                raise Unsupported("Cast to/from bool")
            if np.dtype(dt).kind in "iu" and x.dtype.kind == "f":
                x = np.trunc(x)  # C conversion: toward zero
            return x.astype(dt)
        if op in ("Round", "Rint"):
            return np.rint(self.value(ins[0]))  # half to even (TF Round)
        if op in ("Floor", "Ceil"):
            x = self.value(ins[0])
            return np.floor(x) if op == "Floor" else np.ceil(x)
        if op in ("Add", "AddV2", "Sub", "Mul", "RealDiv", "Div", "TruncateDiv", "FloorDiv", "Maximum", "Minimum",
                  "Greater", "Less", "GreaterEqual", "LessEqual", "Equal", "NotEqual"):
            a, b = self.value(ins[0]), self.value(ins[1])
            if a.dtype != b.dtype:
                raise Unsupported(f"{op}: {a.dtype} vs {b.dtype}")
            a, b = _align(a, b)
            isint = a.dtype.kind in "iu"
            with np.errstate(all="ignore"):
                if op in ("Add", "AddV2"):
                    return a + b
                if op == "Sub":
                    return a - b
                if op == "Mul":
                    return a * b
                if op in ("RealDiv", "Div", "TruncateDiv"):
                    if isint:
                        if np.any(b == 0):
                            raise Unsupported("integer division by zero")
                        q = np.abs(a) // np.abs(b)
                        return np.where((a < 0) != (b < 0), -q, q).astype(a.dtype)
                    return a / b
                if op == "FloorDiv":
                    if isint:
                        if np.any(b == 0):
                            raise Unsupported("integer division by zero")
                        return np.floor_divide(a, b)
                    return np.floor(a / b)
                if op == "Maximum":
                    return np.maximum(a, b)
                if op == "Minimum":
                    return np.minimum(a, b)
                return {"Greater": np.greater, "Less": np.less, "GreaterEqual": np.greater_equal,
                        "LessEqual": np.less_equal, "Equal": np.equal, "NotEqual": np.not_equal}[op](a, b)
        if op in ("Select", "SelectV2"):
            c, t, e = (self.value(i) for i in ins[:3])
            if c.dtype.kind != "b" or t.dtype != e.dtype:
                raise Unsupported("Select operands")
            if c.ndim < t.ndim:
                c = c.reshape(c.shape + (1,) * (t.ndim - c.ndim))
            return np.where(c, t, e)
        if op == "Pack":
            if (nd.attr["axis"].value if "axis" in nd.attr else 0) != 0:
                raise Unsupported("Pack axis")
            vals = [self.value(i) for i in ins]
            if any(v.ndim != 1 for v in vals) or len({v.dtype for v in vals}) != 1:
                raise Unsupported("Pack of non-scalars")
            return np.stack(vals, axis=1)
        if op == "ConcatV2":
            vals = [self.value(i) for i in ins[:-1]]
            ax = self.value(ins[-1])
            if any(v.ndim != 2 for v in vals) or np.any(ax != 0) or len({v.dtype for v in vals}) != 1:
                raise Unsupported("ConcatV2 of non-vectors")
            return np.concatenate(vals, axis=1)
        if op == "StridedSlice":
            return self._strided_slice(nd, ins)
        raise Unsupported(f"op {op} in the shape part")

    def _strided_slice(self, nd, ins):
        x = self.value(ins[0])
        b, e, s = (self.value(i) for i in ins[1:4])
        if x.ndim != 2 or b.ndim != 2 or b.shape[1] != 1 or np.any(b != b[:1]) or np.any(e != e[:1]) or \
                np.any(s != s[:1]):
            raise Unsupported("StridedSlice of a per-row vector with constant bounds only")
        a = {k: (nd.attr[k].value if k in nd.attr else 0) for k in
             ("begin_mask", "end_mask", "ellipsis_mask", "new_axis_mask", "shrink_axis_mask")}
        if a["ellipsis_mask"] or a["new_axis_mask"]:
            raise Unsupported("StridedSlice masks")
        bi, ei, si = int(b[0, 0]), int(e[0, 0]), int(s[0, 0])
        n = x.shape[1]
        if a["shrink_axis_mask"] & 1:
            i = bi + n if bi < 0 else bi
            if not 0 <= i < n:
                raise Unsupported("StridedSlice index out of range")
            return x[:, i]
        sl = slice(None if a["begin_mask"] & 1 else bi, None if a["end_mask"] & 1 else ei, si)
        return x[:, sl]


def _align(a, b):
    """broadcast per-row operands of different per-row ranks (scalar vs vector)"""
    if a.ndim < b.ndim:
        a = a.reshape(a.shape + (1,) * (b.ndim - a.ndim))
    elif b.ndim < a.ndim:
        b = b.reshape(b.shape + (1,) * (a.ndim - b.ndim))
    return a, b


# ---------------------------------------------------------------- the pixel chain

def match(graph_bytes: bytes, row_feeds: List[str], cut: str, cut_shape=None) -> Optional[ImagePrep]:
    """The chain feed -> cut as an ImagePrep, or None when it is anything else."""
    if len(row_feeds) != 1:
        return None
    try:
        light = P.parse_graphdef(_C.light_graphdef(graph_bytes, 4096))
    except Exception:  # noqa: BLE001 - not recognisable: the per-row path stays
        return None
    try:
        return _match(light, row_feeds[0].split(":")[0], cut, cut_shape)
    except Unsupported:
        return None


def _match(light, feed: str, cut: str, cut_shape) -> ImagePrep:
    by_name = {nd.name: nd for nd in light.node}
    consumers: Dict[str, List[Tuple[str, int]]] = {}  # "name:k" -> [(consumer, input slot)]
    for nd in light.node:
        for slot, i in enumerate(nd.input):
            if i.startswith("^"):
                continue
            nm, _, k = i.partition(":")
            consumers.setdefault(f"{nm}:{k or 0}", []).append((nd.name, slot))

    def const(ref):
        nd = by_name.get(ref.split(":")[0])
        if nd is None or nd.op != "Const" or "value" not in nd.attr:
            return None
        try:
            return np.asarray(nd.attr["value"].value.to_numpy())
        except Exception:  # noqa: BLE001
            return None

    def attr_b(nd, k):
        a = nd.attr.get(k)
        return bool(a.value) if a is not None else False

    def ins_of(nd):
        return [i for i in nd.input if not i.startswith("^")]

    # cut: [1, h, w, C], static
    if cut_shape is None or len(cut_shape) != 4 or cut_shape[0] != 1 or any(d is None or d < 1 for d in cut_shape):
        raise Unsupported("cut shape")
    h, w, C = int(cut_shape[1]), int(cut_shape[2]), int(cut_shape[3])
    if C > 4:
        raise Unsupported("more than 4 channels")

    # per-row shape of each pixel-chain tensor, by stage: 0 decoded (H, W),
    # 1 resized (OH, OW), 2 cropped (h, w); rank 4 adds the batch-of-one dim
    shape_of: Dict[str, Callable] = {}

    def record(name, stage, rank):
        def shp(dims, R, stage=stage, rank=rank):
            hh, ww = dims[stage] if stage < 2 else (np.full(R, h), np.full(R, w))
            cols = ([np.ones(R, np.int64)] if rank == 4 else []) + [hh, ww, np.full(R, C)]
            return np.stack([np.asarray(c, np.int64) for c in cols], axis=1)
        shape_of[name] = shp

    def ev(ref, dims, R):  # a fresh evaluator per call (chunks may run on several threads)
        return _ShapeEval(by_name, shape_of)(ref, dims, R)

    stage, rank, is_float = 0, 3, False
    size_ref = size_c = None
    crop = None  # (begin const or ref, size const or ref, rank at the slice)
    mode, ops, squeeze_checks = 0, [], []
    cur = f"{feed}:0"
    record(feed, 0, 3)
    while cur.split(":")[0] != cut:
        nxt = consumers.get(cur, [])
        if len(nxt) != 1:
            # a Shape read of the pixels besides the one chain consumer is fine
            chain = [(n, s) for n, s in nxt if by_name[n].op != "Shape"]
            if len(chain) != 1:
                raise Unsupported("the pixel chain branches")
            nxt = chain
        name, slot = nxt[0]
        nd = by_name[name]
        ins = ins_of(nd)
        op = nd.op
        if op in _KIND:
            if not is_float or len(ins) != 2 or (op in ("Sub", "RealDiv", "Div") and slot != 0):
                raise Unsupported(f"{op} placement")
            v = const(ins[1 - slot])
            if v is None or v.dtype != np.float32:
                raise Unsupported(f"{op}: not a float32 constant")
            v = _per_channel(v, C)
            ops.append((_KIND[op], v))
        elif op in ("Split", "SplitV"):
            if not is_float or slot != (1 if op == "Split" else 0):
                raise Unsupported(f"{op} placement")
            cur = _split_chain(nd, ins, rank, C, consumers, by_name, const, ops)
            record(cur.split(":")[0], stage, rank)
            continue
        elif slot != 0:
            raise Unsupported(f"pixels as input {slot} of {op}")
        elif op in ("Identity", "StopGradient"):
            pass
        elif op == "Cast":
            if nd.attr.get("DstT") is None or nd.attr["DstT"].value != D.DT_FLOAT:
                raise Unsupported("Cast to non-float")
            is_float = True
        elif op == "ExpandDims":
            dim = const(ins[1])
            if rank != 3 or dim is None or int(dim.reshape(-1)[0]) != 0:
                raise Unsupported("ExpandDims")
            rank = 4
        elif op == "Squeeze":
            a = nd.attr.get("squeeze_dims")
            dims = list(a.value.get("i", [])) if a is not None else []
            if rank != 4 or dims not in ([0], [-4], []):
                raise Unsupported("Squeeze")
            if not dims:  # every size-1 dim goes: fine while H, W, C > 1
                if C == 1:
                    raise Unsupported("Squeeze of a 1-channel image")
                squeeze_checks.append(stage)
            rank = 3
        elif op == "ResizeBilinear":
            if rank != 4 or stage != 0 or ops:
                raise Unsupported("ResizeBilinear placement")
            sz = const(ins[1])
            if sz is not None:
                if sz.size != 2:
                    raise Unsupported("resize size")
                size_c = [int(v) for v in sz.reshape(-1)]
            else:
                size_ref = ins[1]
            align, half = attr_b(nd, "align_corners"), attr_b(nd, "half_pixel_centers")
            mode = 1 if align else (2 if half else 0)
            stage, is_float = 1, True
        elif op == "Slice":
            if crop is not None:  # (elementwise steps before it commute with a crop)
                raise Unsupported("Slice placement")
            if stage == 0:  # a crop of the decoded image itself: an identity resize
                stage = 1
            b, s = const(ins[1]), const(ins[2])
            if s is not None:
                s = [int(v) for v in s.reshape(-1)]
                if len(s) != rank or s[-3:-1] != [h, w] or s[-1] not in (-1, C) or (rank == 4 and s[0] not in (1, -1)):
                    raise Unsupported("Slice size")
            crop = (b if b is not None else ins[1], s if s is not None else ins[2], rank)
            stage = 2
        else:
            raise Unsupported(f"op {op} in the pixel chain")
        cur = f"{name}:0"
        record(name, stage, rank)
    if not is_float or rank != 4 or len(ops) > 4:
        raise Unsupported("chain end")
    if stage == 0 and crop is None and size_c is None and size_ref is None:
        stage = 2  # neither resize nor crop: images of the cut's size only

    # ---- resize size and crop offset: constants, or per-row from the shapes
    dyn_size = size_ref is not None or (size_c is None)
    if size_c is not None and crop is None and size_c != [h, w]:
        raise Unsupported("resize without a crop to another size")
    b_ref = s_ref = None
    oy = ox = 0
    if crop is not None:
        b, s, crank = crop
        if isinstance(b, str):
            b_ref = b
        else:
            b = [int(v) for v in b.reshape(-1)]
            if len(b) != crank or b[-1] != 0 or (crank == 4 and b[0] != 0):
                raise Unsupported("Slice begin")
            oy, ox = b[-3], b[-2]
        if isinstance(s, str):
            s_ref = s
    OH, OW = size_c if size_c is not None else (0, 0)
    if not dyn_size and b_ref is None and s_ref is None and not squeeze_checks:
        if oy < 0 or ox < 0 or oy + h > OH or ox + w > OW:
            raise Unsupported("crop outside the resize")
        return ImagePrep(C, OH, OW, mode, oy, ox, h, w, ops)

    def dyn(hw: np.ndarray) -> np.ndarray:
        R = hw.shape[0]
        H, W = hw[:, 0].astype(np.int64), hw[:, 1].astype(np.int64)
        dims = {0: (H, W)}
        if size_ref is not None:
            sz = ev(size_ref, dims, R)
            if sz.shape != (R, 2):
                raise Unsupported("resize size shape")
            rh, rw = sz[:, 0].astype(np.int64), sz[:, 1].astype(np.int64)
        elif size_c is not None:
            rh, rw = np.full(R, OH, np.int64), np.full(R, OW, np.int64)
        else:  # no resize: the identity (scale 1, exact)
            rh, rw = H, W
        dims[1] = (rh, rw)
        if mode != 0 and size_ref is None and size_c is None:
            raise Unsupported("identity resize needs mode 0")
        for st in squeeze_checks:
            sh, sw = dims[st]
            if np.any(sh <= 1) or np.any(sw <= 1):
                raise Unsupported("a Squeeze would drop an image dim")
        if b_ref is not None:
            bb = ev(b_ref, dims, R)
            crank = crop[2]
            if bb.ndim != 2 or bb.shape[1] != crank or np.any(bb[:, -1] != 0) or (crank == 4 and np.any(bb[:, 0] != 0)):
                raise Unsupported("crop begin")
            py, px = bb[:, -3].astype(np.int64), bb[:, -2].astype(np.int64)
        else:
            py, px = np.full(R, oy, np.int64), np.full(R, ox, np.int64)
        if crop is None and (np.any(rh != h) or np.any(rw != w)):
            raise Unsupported("an image (or its resize) is not the cut's size")
        if s_ref is not None:
            ss = ev(s_ref, dims, R)
            if ss.ndim != 2 or np.any(ss[:, -3] != h) or np.any(ss[:, -2] != w) or \
                    np.any((ss[:, -1] != -1) & (ss[:, -1] != C)):
                raise Unsupported("crop size")
        return np.stack([rh, rw, py, px], axis=1)

    # the shape part must be evaluable at all (e.g. on one 300 x 400 image)
    try:
        dyn(np.array([[300, 400]], np.int32))
    except Unsupported as e:
        if not any(t in str(e) for t in ("outside", "drop", "cut's size")):
            raise
    return ImagePrep(C, OH, OW, mode, oy, ox, h, w, ops, dyn=dyn)


def _per_channel(v: np.ndarray, C: int) -> List[float]:
    """a scalar or per-channel constant ([C], [1, C], [1, 1, C], ...) as a list"""
    if v.size == 1:
        return [float(v.reshape(-1)[0])]
    if v.shape[-1] != C or v.size != C:
        raise Unsupported("constant is not per-channel")
    return [float(x) for x in v.reshape(-1)]


def _split_chain(nd, ins, rank, C, consumers, by_name, const, ops) -> str:
    """Split along the channel axis -> per-channel elementwise chains ->
    ConcatV2 in channel order, folded into per-channel steps. Returns the
    concat's output ref (the chain continues there)."""
    if nd.op == "Split":
        ax, val = const(ins[0]), ins[1]
        if val.split(":")[0] not in by_name:
            raise Unsupported("Split input")
    else:
        val, sizes, ax = ins[0], const(ins[1]), const(ins[2])
        if sizes is None or list(sizes.reshape(-1)) != [1] * C:
            raise Unsupported("SplitV sizes")
    n = int(nd.attr["num_split"].value) if "num_split" in nd.attr else -1
    if ax is None or int(ax.reshape(-1)[0]) not in (rank - 1, -1) or n != C:
        raise Unsupported("Split along channels only")
    chains, tails = [], []
    for j in range(C):
        ref, steps = f"{nd.name}:{j}", []
        while True:
            nxt = consumers.get(ref, [])
            if len(nxt) != 1:
                raise Unsupported("a split branch branches")
            cname, slot = nxt[0]
            c = by_name[cname]
            if c.op == "ConcatV2":
                tails.append((cname, slot))
                break
            cins = [i for i in c.input if not i.startswith("^")]
            if c.op not in _KIND or len(cins) != 2 or (c.op in ("Sub", "RealDiv", "Div") and slot != 0):
                raise Unsupported(f"{c.op} in a split branch")
            v = const(cins[1 - slot])
            if v is None or v.dtype != np.float32 or v.size != 1:
                raise Unsupported("split-branch constant")
            steps.append((_KIND[c.op], float(v.reshape(-1)[0])))
            ref = f"{cname}:0"
        chains.append(steps)
    cat = {t[0] for t in tails}
    if len(cat) != 1 or [t[1] for t in tails] != list(range(C)):
        raise Unsupported("the branches do not concat back in channel order")
    cname = tails[0][0]
    cnd = by_name[cname]
    cins = [i for i in cnd.input if not i.startswith("^")]
    cax = const(cins[-1])
    if len(cins) != C + 1 or cax is None or int(cax.reshape(-1)[0]) not in (rank - 1, -1):
        raise Unsupported("concat axis")
    kinds = [[k for k, _ in s] for s in chains]
    if any(k != kinds[0] for k in kinds):
        raise Unsupported("branches with different steps")
    for q, kind in enumerate(kinds[0]):
        ops.append((kind, [chains[j][q][1] for j in range(C)]))
    return f"{cname}:0"
