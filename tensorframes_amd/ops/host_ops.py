"""Host ops: graph nodes whose work runs on the CPU before the GPU program.

Image decoders (``DecodeJpeg``/``DecodePng``/``DecodeImage``/``DecodeBmp``)
turn a binary cell into a uint8 ``[H, W, C]`` tensor. The reference scored
JPEG bytes from a binary DataFrame column through a frozen VGG-16 graph with
``map_rows(..., feed_dict={'DecodeJpeg/contents': 'image_data'})``
(reference: src/main/python/tensorframes_snippets/read_image.py:42,147-167),
with libtensorflow decoding inside the session. Here the decode is a host
stage: `plan_host_stage` finds the decoder nodes in the fetch closure and the
binary column (or constant) feeding each one; the native program is then cut
at those nodes, and each row's decoded image is fed in place of the node's
output. Everything downstream (cast, resize, crop, the CNN) runs on the GPU.
The native runtime registers the same ops for shape inference only
(csrc/ir/ops_nn.cpp), so graphs containing them analyze normally.
"""
from __future__ import annotations

import io
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from ..utils import dtypes as D

DECODE_OPS = ("DecodeJpeg", "DecodePng", "DecodeImage", "DecodeBmp")


def _pil():
    try:
        from PIL import Image
    except ImportError as e:  # pragma: no cover - PIL is part of the image
        raise RuntimeError("image decode host ops need Pillow (PIL)") from e
    return Image


def decode_image(data: bytes, channels: int = 0, dtype: int = D.DT_UINT8) -> np.ndarray:
    """Decode JPEG/PNG/BMP/GIF bytes to ``[H, W, C]`` (TF decode_* semantics:
    channels 0 keeps the file's channels, 1 gray, 3 RGB, 4 RGBA)."""
    Image = _pil()
    if isinstance(data, str):
        data = data.encode("latin-1")
    with Image.open(io.BytesIO(bytes(data))) as im:
        if channels == 1:
            im = im.convert("L")
        elif channels == 3:
            im = im.convert("RGB")
        elif channels == 4:
            im = im.convert("RGBA")
        elif channels == 0:
            if im.mode not in ("L", "RGB", "RGBA"):
                im = im.convert("RGBA" if "A" in im.mode else "RGB")
        else:
            raise ValueError(f"decode: channels must be 0, 1, 3 or 4, got {channels}")
        arr = np.array(im, dtype=np.uint8)  # a writable copy
    if arr.ndim == 2:
        arr = arr[:, :, None]
    if dtype != D.DT_UINT8:
        raise ValueError(f"decode: unsupported output dtype {D.dtype_name(dtype)}")
    return np.ascontiguousarray(arr)


@dataclass
class HostFeed:
    node: str                  # decoder node; its output 0 is fed to the program
    op: str
    channels: int
    dtype: int
    column: Optional[str]      # binary column feeding `contents` (None: constant)
    const_value: Optional[np.ndarray] = None  # decoded constant contents

    def decode(self, cell) -> np.ndarray:
        return decode_image(cell, self.channels, self.dtype)


def _closure(inputs_of, fetch_nodes: List[str], stop: set) -> List[str]:
    seen, stack, order = set(), list(fetch_nodes), []
    while stack:
        n = stack.pop()
        if n in seen:
            continue
        seen.add(n)
        order.append(n)
        if n in stop:
            continue
        for i in inputs_of(n):
            stack.append(i.lstrip("^").split(":")[0])
    return order


def plan_host_stage(graph, fetch_refs: List[str], feed_dict: Dict[str, str],
                    columns: Dict[str, object]) -> List[HostFeed]:
    """The decoder nodes reachable from the fetches (`graph`: the native
    graph; nothing is parsed in Python, so big models stay cheap), each bound
    to the binary column (through `feed_dict` on its contents node, or a
    placeholder named like a column) or to its constant contents."""
    ops = dict(zip(graph.node_names(), graph.node_ops()))
    cache: Dict[str, List[str]] = {}

    def inputs_of(n):
        if n not in cache:
            cache[n] = list(graph.node_inputs(n)) if n in ops else []
        return cache[n]
    fetch_nodes = [r.split(":")[0] for r in fetch_refs]
    host = [n for n in _closure(inputs_of, fetch_nodes, set()) if ops.get(n) in DECODE_OPS]
    # only the decoders not hidden behind another decoder
    reachable = set(_closure(inputs_of, fetch_nodes, set(host)))
    feeds: List[HostFeed] = []
    for n in host:
        if n not in reachable:
            continue
        attr = graph.node_attr_scalars(n)
        src = inputs_of(n)[0].split(":")[0]
        src_op = ops.get(src)
        col = feed_dict.get(src)
        if col is None and src_op in ("Placeholder", "PlaceholderV2") and src in columns:
            col = src
        hf = HostFeed(n, ops[n], int(attr.get("channels", 0)), int(attr.get("dtype", D.DT_UINT8)), col)
        if col is None:
            if src_op != "Const":
                raise ValueError(f"{ops[n]} node '{n}': its contents '{src}' must be fed from a binary "
                                 f"column (feed_dict={{'{src}': <column>}})")
            vals = graph.const_strings(src)
            if not vals:
                raise ValueError(f"{ops[n]} node '{n}': constant contents '{src}' is empty")
            hf.const_value = hf.decode(vals[0])
        feeds.append(hf)
    return feeds
