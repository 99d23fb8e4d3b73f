"""tensorframes_amd — an MI355X-native DataFrame tensor engine with the
TensorFrames API (map_blocks, map_rows, reduce_blocks, reduce_rows,
aggregate, analyze, print_schema, block, row).

    import tensorframes_amd as tfs
    from tensorframes_amd import tf          # TF-1.x-compatible graph builder

    df = tfs.create_dataframe([tfs.Row(x=float(i)) for i in range(10)])
    with tf.Graph().as_default():
        x = tf.placeholder(tf.double, shape=[None], name="x")
        z = tf.add(x, 3, name="z")
        df2 = tfs.map_blocks(z, df)

Graphs are TF GraphDef protobufs (built with `tensorframes_amd.tf` or loaded
from bytes/files); they execute on a native C++ planner/executor whose
kernels are hand-written HIP for gfx950 (CDNA4), one process per GPU,
with RCCL collectives across GPUs.
"""
from . import _native  # noqa: F401  (loads / builds the native extension)
from .config import Config, config, set_config
from .core import (InputNotFoundException, InvalidDimensionException, InvalidTypeException,
                   TensorFramesError, aggregate, analyze, analyze_graph, block, explain, map_blocks,
                   map_rows, print_schema, reduce_blocks, reduce_rows, row)
from .frame.column_info import (SHAPE_KEY, TYPE_KEY, ColumnInformation, DataFrameInfo, HighDimException,
                                SparkTFColInfo)
from .frame.dataframe import (DataFrame, GroupedData, create_dataframe, createDataFrame, from_columns,
                              generate, tensor_field)
from .frame.arrow_io import from_arrow, read_parquet, to_arrow, write_parquet
from .frame.spark_io import from_spark, to_spark
from .frame.checkpoint import read_checkpoint, write_checkpoint
from .frame.dataframe import range_ as range  # noqa: A001
from .frame.types import (ArrayType, BinaryType, DoubleType, FloatType, IntegerType, LongType, Row,
                          StringType, StructField, StructType)
from .graph import dsl as tf  # noqa: F401
from .operations import Operations, Ops, ShapeDescription, convert_block_to_row, explain_detailed, ops
from .graph import dsl
from . import scala_dsl  # noqa: F401  (the Scala DSL vocabulary)
from .parallel import dist
from .utils.logging import initialize_logging, metrics
from .utils.shape import Shape

__version__ = "0.1.0"

__all__ = ["reduce_rows", "map_rows", "reduce_blocks", "map_blocks", "analyze", "print_schema",
           "aggregate", "block", "row"]
