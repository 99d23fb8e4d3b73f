"""Column tensor info and `analyze` (reference:
src/test/scala/org/tensorframes/ExtraOperationsSuite.scala:8-99,
src/main/scala/org/tensorframes/ColumnInformation.scala:124-138)."""
import pytest

import tensorframes_amd as tfs
from tensorframes_amd.frame.column_info import ColumnInformation, DataFrameInfo
from tensorframes_amd.frame.types import (ArrayType, DoubleType, IntegerType, StructField, StructType)
from tensorframes_amd.utils.shape import Shape

U = -1


def infos(df):
    return [c.stf for c in DataFrameInfo.get(df.schema).cols]


def test_default_info_double():
    s, = infos(tfs.create_dataframe([(0.0,)], ["a"]))
    assert s.dataType == DoubleType() and s.shape == Shape(U)


def test_default_info_int():
    df = tfs.create_dataframe([(0,)], StructType([StructField("a", IntegerType(), False)]))
    s, = infos(df)
    assert s.dataType == IntegerType() and s.shape == Shape(U)


def test_default_info_arrays():
    s1, s2, s3 = infos(tfs.create_dataframe([(0.0, [1.0], [[1.0]])], ["a", "b", "c"]))
    assert s1.shape == Shape(U) and s2.shape == Shape(U, U) and s3.shape == Shape(U, U, U)
    assert s1.dataType == s2.dataType == s3.dataType == DoubleType()


def test_simple_analysis():
    s, = infos(tfs.analyze(tfs.create_dataframe([(0.0,)], ["a"])))
    assert s.shape == Shape(1)


def test_analysis_multiple_partitions_of_different_sizes():
    df = tfs.create_dataframe([(0.0,)] * 10, ["a"]).repartition(3)
    s, = infos(tfs.analyze(df))
    assert s.shape == Shape(U)


def test_analysis_equal_partitions():
    df = tfs.create_dataframe([(0.0,)] * 10, ["a"], num_partitions=2)
    s, = infos(tfs.analyze(df))
    assert s.shape == Shape(5)


def test_analysis_variable_sizes():
    _, s2 = infos(tfs.analyze(tfs.create_dataframe([(0.0, [0.0]), (1.0, [1.0, 1.0])], ["a", "b"])))
    assert s2.shape == Shape(2, U)


def test_second_order_analysis():
    df = tfs.create_dataframe([(0.0, [0.0, 0.0]), (1.0, [1.0, 1.0]), (2.0, [2.0, 2.0])], ["a", "b"])
    _, s2 = infos(tfs.analyze(df))
    assert s2.shape == Shape(3, 2)


def test_analysis_skips_empty_partitions():
    df = tfs.create_dataframe([(0.0,), (1.0,)], ["a"], num_partitions=4)  # sizes 0,1,0,1
    s, = infos(tfs.analyze(df))
    assert s.shape == Shape(1)


def test_metadata_keys_and_print_schema(capsys):
    df = tfs.analyze(tfs.create_dataframe([([1.0, 2.0],)], ["y"]))
    f = df.schema["y"]
    assert f.metadata["org.spartf.shape"] == [1, 2]
    assert f.metadata["org.sparktf.type"] == "DoubleType"
    tfs.print_schema(df)
    out = capsys.readouterr().out
    assert out == "root\n |-- y: array (nullable = true) double[1,2]\n"
    assert df.explain_tensors() == "DataFrame[DoubleType[1,2]]"


def test_struct_field_builder():
    f = ColumnInformation.struct_field("z", 2, Shape(U, 3))
    assert f.dataType == ArrayType(DoubleType(), False) and f.nullable is False
    assert ColumnInformation(f).stf.shape == Shape(U, 3)


def test_shape_semantics():
    assert Shape(3, 2).check_more_precise_than(Shape(U, 2))
    assert not Shape(U, 2).check_more_precise_than(Shape(3, 2))
    assert not Shape(3).check_more_precise_than(Shape(3, 1))
    assert str(Shape(U, 2)) == "[?,2]"
    assert Shape(2, 3).num_elements() == 6 and Shape(U).num_elements() is None
    assert Shape(4).prepend(U) == Shape(U, 4) and Shape(1, 2).tail() == Shape(2)
    with pytest.raises(ValueError):
        Shape(-2)
