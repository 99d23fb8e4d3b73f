"""DataFrame checkpoints: write a frame's partitions + schema to a directory
and read them back, so iterative jobs (K-Means, ...) can resume and computed
columns survive the process.

The reference kept no checkpoints (Spark lineage + `.cache()`; its `analyze`
metadata lives in the schema, reference:
src/main/scala/org/tensorframes/ExperimentalOperations.scala:35-47). Format,
chosen so that loading never executes anything from the files:

    <dir>/schema.json              fields (name, type tree, nullable, metadata),
                                   partition count, format version
    <dir>/part-00003.safetensors   dense columns of partition 3 (+ ragged cells)
    <dir>/part-00003.json          row count, ragged cell shapes, object columns
                                   (strings; bytes as base64)
    <dir>/_SUCCESS                 written last (after all ranks finished)

Every rank writes the partitions it owns (p % world == rank) and reads them
back the same way; device-resident columns are copied to the host first.
"""
from __future__ import annotations

import base64
import json
import os
from typing import Any, Dict, List

import numpy as np
import torch

from ..parallel import dist
from ..utils import dtypes as D
from .block import Block, ObjectColumn, RaggedColumn
from .types import (ArrayType, BinaryType, BooleanType, DataType, DoubleType, FloatType, IntegerType, LongType,
                    StringType, StructField, StructType)

FORMAT_VERSION = 1
_SCALARS = {t.type_name: t for t in (DoubleType(), FloatType(), IntegerType(), LongType(), BooleanType(),
                                     StringType(), BinaryType())}


def _type_to_json(t: DataType) -> Any:
    if isinstance(t, ArrayType):
        return {"array": _type_to_json(t.elementType), "containsNull": t.containsNull}
    if t.type_name not in _SCALARS:
        raise TypeError(f"checkpoint: unsupported column type {t}")
    return t.type_name


def _type_from_json(j: Any) -> DataType:
    if isinstance(j, dict):
        return ArrayType(_type_from_json(j["array"]), j.get("containsNull", False))
    return _SCALARS[j]


def _meta_to_json(m: Dict[str, Any]) -> Dict[str, Any]:
    out = {}
    for k, v in m.items():
        out[k] = list(v) if isinstance(v, (list, tuple)) else v
    return out


def schema_to_json(schema: StructType) -> List[Dict[str, Any]]:
    return [{"name": f.name, "type": _type_to_json(f.dataType), "nullable": f.nullable,
             "metadata": _meta_to_json(f.metadata)} for f in schema.fields]


def schema_from_json(j) -> StructType:
    return StructType([StructField(f["name"], _type_from_json(f["type"]), f["nullable"], f["metadata"])
                       for f in j])


def _part(path: str, pid: int, ext: str) -> str:
    return os.path.join(path, f"part-{pid:05d}.{ext}")


def _write_block(path: str, pid: int, b: Block):
    from safetensors.torch import save_file
    tensors: Dict[str, torch.Tensor] = {}
    info: Dict[str, Any] = {"nrows": b.nrows, "dense": [], "ragged": {}, "object": {}}
    for name, col in b.columns.items():
        if isinstance(col, torch.Tensor):
            tensors[f"d/{name}"] = col.detach().to("cpu").contiguous()
            info["dense"].append(name)
        elif isinstance(col, RaggedColumn):
            shapes = [list(np.shape(c)) for c in col.cells]
            flat = np.concatenate([np.asarray(c).reshape(-1) for c in col.cells]) if col.cells else \
                np.zeros(0, D.numpy_dtype(col.tf_dtype))
            tensors[f"r/{name}"] = torch.from_numpy(np.ascontiguousarray(flat))
            info["ragged"][name] = {"shapes": shapes, "tf_dtype": col.tf_dtype}
        elif isinstance(col, ObjectColumn):
            vals = []
            for v in col.values:
                if isinstance(v, (bytes, bytearray)):
                    vals.append({"b64": base64.b64encode(bytes(v)).decode("ascii")})
                else:
                    vals.append(v)
            info["object"][name] = vals
        else:
            raise TypeError(f"checkpoint: cannot store column '{name}' of type {type(col).__name__}")
    save_file(tensors, _part(path, pid, "safetensors"))
    with open(_part(path, pid, "json"), "w") as f:
        json.dump(info, f)


def _read_block(path: str, pid: int) -> Block:
    from safetensors.torch import load_file
    with open(_part(path, pid, "json")) as f:
        info = json.load(f)
    tensors = load_file(_part(path, pid, "safetensors"))
    cols: Dict[str, Any] = {}
    for name in info["dense"]:
        cols[name] = tensors[f"d/{name}"]
    for name, r in info["ragged"].items():
        flat = tensors[f"r/{name}"].numpy()
        cells, off = [], 0
        for shp in r["shapes"]:
            n = int(np.prod(shp)) if shp else 1
            cells.append(flat[off:off + n].reshape(shp).copy())
            off += n
        cols[name] = RaggedColumn(cells, r["tf_dtype"])
    for name, vals in info["object"].items():
        cols[name] = ObjectColumn([bytearray(base64.b64decode(v["b64"])) if isinstance(v, dict) and "b64" in v
                                   else v for v in vals])
    return Block(info["nrows"], cols)


def write_checkpoint(df, path: str) -> str:
    """Materialise `df` and write it under `path` (created; existing part
    files are overwritten). Returns `path`."""
    os.makedirs(path, exist_ok=True)
    ok = os.path.join(path, "_SUCCESS")
    if dist.rank() == 0 and os.path.exists(ok):
        os.remove(ok)
    dist.barrier()
    for pid, b in df._iter_blocks():
        _write_block(path, pid, b)
    dist.barrier()
    if dist.rank() == 0:
        with open(os.path.join(path, "schema.json"), "w") as f:
            json.dump({"version": FORMAT_VERSION, "num_partitions": df.num_partitions,
                       "fields": schema_to_json(df.schema)}, f, indent=1)
        with open(ok, "w") as f:
            f.write("ok\n")
    dist.barrier()
    return path


def read_checkpoint(path: str):
    """The DataFrame written by `write_checkpoint` (lazy: partitions load on
    first use, each rank reading its own)."""
    from .dataframe import DataFrame, _Generated
    if not os.path.exists(os.path.join(path, "_SUCCESS")):
        raise FileNotFoundError(f"no complete checkpoint at {path} (missing _SUCCESS)")
    with open(os.path.join(path, "schema.json")) as f:
        meta = json.load(f)
    if meta.get("version") != FORMAT_VERSION:
        raise ValueError(f"checkpoint format version {meta.get('version')} is not supported")
    schema = schema_from_json(meta["fields"])
    nparts = int(meta["num_partitions"])
    return DataFrame(schema, _Generated(nparts, lambda p: _read_block(path, p)), nparts)
