"""PySpark adapter driven through a minimal stand-in of the
pyspark API surface it uses (pyspark itself is not installed in this image):
``BarrierTaskContext`` (get / partitionId / getTaskInfos / allGather / barrier /
resources), ``DataFrame.rdd.barrier().mapPartitions(...).collect()`` and
``DataFrame.mapInArrow``. One barrier task (world 1) exercises the executor
code path without a second process."""
import sys
import types

import numpy as np
import pytest


class _TaskInfo:
    address = "127.0.0.1:7077"


class _Ctx:
    current = None

    def __init__(self, pid, n):
        self.pid, self.n = pid, n

    @classmethod
    def get(cls):
        return cls.current

    def partitionId(self):  # noqa: N802
        return self.pid

    def getTaskInfos(self):  # noqa: N802
        return [_TaskInfo() for _ in range(self.n)]

    def allGather(self, msg):  # noqa: N802
        return [msg]

    def barrier(self):
        pass

    def resources(self):
        return {}


class _Row(dict):
    def asDict(self):  # noqa: N802
        return dict(self)


class _Vec:
    def __init__(self, a):
        self.a = np.asarray(a)

    def toArray(self):  # noqa: N802
        return self.a


class _Barrier:
    def __init__(self, parts):
        self.parts = parts

    def mapPartitions(self, fn):  # noqa: N802
        parts = self.parts

        class _Res:
            def collect(self):
                out = []
                for i, p in enumerate(parts):
                    _Ctx.current = _Ctx(i, len(parts))
                    out.extend(fn(iter(p)))
                return out

        return _Res()


class _RDD:
    def __init__(self, parts):
        self.parts = parts

    def barrier(self):
        return _Barrier(self.parts)


class _Batches(list):
    """mapInArrow's result: the output batches; collect() gives their rows (a Spark DataFrame's collect)."""

    def collect(self):
        return [row for b in self for row in b.to_pylist()]


class _SparkDF:
    def __init__(self, rows, arrow_table, arrow_barrier=True):
        self.rdd = _RDD([rows])
        self.table = arrow_table
        self.arrow_barrier = arrow_barrier
        self.arrow_fit_calls = 0

    def mapInArrow(self, fn, schema, barrier=False):  # noqa: N802
        if barrier:
            if not self.arrow_barrier:  # Spark < 3.5
                raise TypeError("mapInArrow() got an unexpected keyword argument 'barrier'")
            self.arrow_fit_calls += 1
            _Ctx.current = _Ctx(0, 1)
        return _Batches(fn(iter(self.table.to_batches(max_chunksize=256))))


@pytest.fixture
def fake_pyspark(monkeypatch):
    mod = types.ModuleType("pyspark")
    mod.BarrierTaskContext = _Ctx
    monkeypatch.setitem(sys.modules, "pyspark", mod)
    return mod


def test_fit_and_transform_through_pyspark_surface(fake_pyspark):
    from synapseml_amd.core import DataFrame
    from synapseml_amd.lightgbm import LightGBMClassifier
    from synapseml_amd.parallel.spark import fit_on_spark, transform_on_spark

    rng = np.random.default_rng(0)
    X = rng.standard_normal((1000, 4))
    y = (X[:, 0] - X[:, 1] > 0).astype(float)
    rows = [_Row(features=_Vec(x), label=float(t)) for x, t in zip(X, y)]
    import pyarrow as pa

    # the training partition as Spark ships it after vector_to_array: array<double> features + a label column
    train_table = pa.table({"features": pa.array([list(x) for x in X], type=pa.list_(pa.float64())), "label": y})
    table = DataFrame({"features": X}).toArrow()
    local = LightGBMClassifier(deviceType="cpu", numIterations=10).fit(DataFrame({"features": X, "label": y}))
    # Spark >= 3.5: barrier mapInArrow, the partition arrives as Arrow (no Row objects)
    sdf_arrow = _SparkDF(None, train_table)
    model = fit_on_spark(LightGBMClassifier(deviceType="cpu", numIterations=10), sdf_arrow, use_gpu=False)
    assert sdf_arrow.arrow_fit_calls == 1
    assert model.getNativeModel().split("parameters:")[0] == local.getNativeModel().split("parameters:")[0]
    # Spark < 3.5: the Row path, same model
    sdf = _SparkDF(rows, table, arrow_barrier=False)
    model = fit_on_spark(LightGBMClassifier(deviceType="cpu", numIterations=10), sdf, use_gpu=False)
    assert model.getNativeModel().split("parameters:")[0] == local.getNativeModel().split("parameters:")[0]
    batches = transform_on_spark(model, sdf, schema=None)
    out = DataFrame.fromArrow(batches)
    assert out.count() == 1000
    np.testing.assert_allclose(np.stack(out["probability"].tolist()) if out["probability"].dtype == object
                               else out["probability"], local.transform(DataFrame({"features": X}))["probability"])
