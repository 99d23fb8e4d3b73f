"""PySpark interop: TensorFrames programs written against Spark DataFrames run
unchanged on this engine.

The reference *is* a Spark package: every operator takes a
`pyspark.sql.DataFrame` (reference: src/main/python/tensorframes/core.py:175-336)
and tensor shapes live in the Spark field metadata under "org.spartf.shape" /
"org.sparktf.type" (src/main/scala/org/tensorframes/MetadataConstants.scala:19,27).
Here a Spark DataFrame is brought in through Arrow, column metadata included
(`from_spark`), the operators run on the GPU engine, and results can be handed
back to a SparkSession (`to_spark`). The operators in `core` accept Spark
DataFrames directly and convert them on entry.

pyspark is optional (it is not installed in every environment): everything is
duck-typed and pyspark is imported only inside `to_spark`.
"""
from __future__ import annotations

import json
from typing import Any, Optional, Sequence

from .column_info import SHAPE_KEY, TYPE_KEY


def is_spark_dataframe(obj: Any) -> bool:
    mod = type(obj).__module__ or ""
    return mod.startswith("pyspark.sql") and hasattr(obj, "schema") and (
        hasattr(obj, "toArrow") or hasattr(obj, "_collect_as_arrow") or hasattr(obj, "toPandas"))


def is_spark_grouped(obj: Any) -> bool:
    mod = type(obj).__module__ or ""
    return mod.startswith("pyspark.sql") and type(obj).__name__ == "GroupedData"


def _spark_field_meta(sdf) -> dict:
    out = {}
    for f in sdf.schema.fields:
        md = getattr(f, "metadata", None) or {}
        keep = {k: md[k] for k in (SHAPE_KEY, TYPE_KEY) if k in md}
        if keep:
            out[f.name] = keep
    return out


def spark_to_arrow(sdf):
    """Collect a Spark DataFrame as a `pyarrow.Table` (Spark 4 `toArrow`,
    Spark 3 `_collect_as_arrow`, else through pandas) with the tensor metadata
    of every field copied onto the Arrow fields."""
    import pyarrow as pa
    if hasattr(sdf, "toArrow"):
        table = sdf.toArrow()
    elif hasattr(sdf, "_collect_as_arrow"):
        batches = sdf._collect_as_arrow()
        table = pa.Table.from_batches(batches) if batches else pa.table({})
    else:
        table = pa.Table.from_pandas(sdf.toPandas(), preserve_index=False)
    meta = _spark_field_meta(sdf)
    if meta:
        fields = []
        for f in table.schema:
            m = meta.get(f.name)
            if m:
                md = dict(f.metadata or {})
                md.update({k.encode(): json.dumps(v).encode() for k, v in m.items()})
                f = f.with_metadata(md)
            fields.append(f)
        table = table.cast(pa.schema(fields))
    return table


def from_spark(sdf, num_partitions: Optional[int] = None):
    """Engine DataFrame with the rows, schema and tensor metadata of a Spark
    DataFrame. The partition count follows the Spark RDD unless given."""
    from .arrow_io import from_arrow
    if num_partitions is None:
        try:
            num_partitions = int(sdf.rdd.getNumPartitions())
        except Exception:  # noqa: BLE001  (no RDD access, e.g. Spark Connect)
            num_partitions = None
    return from_arrow(spark_to_arrow(sdf), num_partitions)


def from_spark_grouped(sgd, keys: Optional[Sequence[str]] = None):
    """Engine GroupedData for a Spark `df.groupBy(...)` result. The grouping
    columns are read from the JVM RelationalGroupedDataset (the reference reads
    them by reflection as well: DebugRowOps.scala:707-730) unless given."""
    sdf = getattr(sgd, "_df", None)
    if sdf is None:
        raise TypeError("aggregate: cannot reach the DataFrame behind this Spark GroupedData; "
                        "use tfs.from_spark(df).groupBy(...) instead")
    if keys is None:
        keys = _spark_group_keys(sgd)
    return from_spark(sdf).groupBy(*keys)


def _spark_group_keys(sgd):
    jgd = getattr(sgd, "_jgd", None)
    names = []
    try:
        exprs = jgd.groupingExprs()
        it = exprs.iterator()
        while it.hasNext():
            names.append(str(it.next().sql()).strip("`"))
    except Exception as e:  # noqa: BLE001
        raise TypeError("aggregate: the grouping columns of this Spark GroupedData are not readable; "
                        "use tfs.from_spark(df).groupBy(...) instead") from e
    return names


def _spark_type(dt):
    from pyspark.sql import types as T
    from .types import (ArrayType, BinaryType, BooleanType, DoubleType, FloatType, IntegerType, LongType,
                        StringType)
    if isinstance(dt, ArrayType):
        return T.ArrayType(_spark_type(dt.elementType), containsNull=False)
    table = {DoubleType: T.DoubleType, FloatType: T.FloatType, IntegerType: T.IntegerType, LongType: T.LongType,
             BooleanType: T.BooleanType, StringType: T.StringType, BinaryType: T.BinaryType}
    for ours, theirs in table.items():
        if isinstance(dt, ours):
            return theirs()
    raise TypeError(f"to_spark: no Spark type for {dt}")


def spark_schema(schema):
    """pyspark StructType for an engine schema, tensor metadata included."""
    from pyspark.sql import types as T
    return T.StructType([
        T.StructField(f.name, _spark_type(f.dataType), f.nullable,
                      {k: v for k, v in f.metadata.items() if k in (SHAPE_KEY, TYPE_KEY)})
        for f in schema.fields])


def to_spark(df, spark):
    """Spark DataFrame (created in `spark`, a SparkSession) with the rows of an
    engine DataFrame, its column types and tensor metadata."""
    from .arrow_io import to_arrow
    pdf = to_arrow(df).to_pandas()
    for f in df.schema.fields:  # Spark wants nested lists, not numpy cells
        if f.name in pdf and len(pdf) and hasattr(pdf[f.name].iloc[0], "tolist"):
            pdf[f.name] = pdf[f.name].map(lambda v: v.tolist() if hasattr(v, "tolist") else v)
    return spark.createDataFrame(pdf, schema=spark_schema(df.schema))
