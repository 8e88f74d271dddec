import json
import os

import numpy as np
import pytest

from synapseml_amd.core import DataFrame, DenseVector, Pipeline, SparseVector, Vectors, createDataFrame
from synapseml_amd.core.params import Param, Params, TypeConverters as T
from synapseml_amd.core.pipeline import Estimator, Model, PipelineStage, Transformer
from synapseml_amd.core.serialize import java_deserialize_bytes, java_serialize_bytes
from synapseml_amd.core.utils import ParamsStringBuilder, find_unused_column_name, retry_with_timeout


class AddConst(Transformer):
    inputCol = Param("in", "x", T.toString)
    outputCol = Param("out", "y", T.toString)
    value = Param("constant", 1.0, T.toFloat)

    def _transform(self, df):
        return df.withColumn(self.getOutputCol(), df[self.getInputCol()] + self.getValue())


class MeanModel(Model):
    mean = Param("mean", 0.0, T.toFloat)
    blob = Param("bytes", None, complex=True)

    def _transform(self, df):
        return df.withColumn("centered", df["x"] - self.getMean())


class MeanEstimator(Estimator):
    def _fit(self, df):
        return MeanModel(mean=float(np.mean(df["x"])), blob=b"\x00\x01abc")


def test_dataframe_basics():
    df = DataFrame({"x": np.arange(10.0), "s": [str(i) for i in range(10)]}, num_partitions=3)
    assert df.count() == 10 and df.getNumPartitions() == 3
    assert [b - a for a, b in df.partition_bounds()] == [3, 3, 4]
    f = df.filter(df["x"] > 4)
    assert f.count() == 5 and f.getNumPartitions() == 3
    w = df.withColumn("z", df["x"] * 2).select("x", "z")
    assert w.columns == ["x", "z"]
    r = w.collect()[3]
    assert r.z == 6.0 and r["x"] == 3.0
    a, b = df.randomSplit([0.5, 0.5], seed=1)
    assert a.count() + b.count() == 10
    m = df.mapPartitions(lambda p: p.withColumn("n", np.full(p.count(), p.count())))
    assert list(m["n"]) == [3, 3, 3, 3, 3, 3, 4, 4, 4, 4]
    u = df.union(df)
    assert u.count() == 20 and u.getNumPartitions() == 6
    assert df.coalesce(1).getNumPartitions() == 1
    g = df.withColumn("k", np.arange(10) % 2).groupBy("k").agg(total=("x", "sum"))
    assert dict(zip(g["k"], g["total"])) == {0: 20.0, 1: 25.0}
    j = df.join(DataFrame({"s": ["1", "2"], "t": [10, 20]}), "s")
    assert sorted(j["t"].tolist()) == [10, 20]
    pdf = df.toPandas()
    assert DataFrame.fromPandas(pdf).count() == 10


def test_vector_columns():
    df = createDataFrame([{"v": Vectors.dense([1.0, 2.0])}, {"v": Vectors.dense([3.0, 4.0])}])
    assert df["v"].shape == (2, 2)
    sp = createDataFrame([{"v": SparseVector(4, [1], [2.0])}, {"v": DenseVector([1, 0, 0, 1])}])
    assert sp["v"].dtype == object
    from synapseml_amd.core.linalg import as_csr, as_matrix

    m = as_matrix(sp["v"])
    assert m.shape == (2, 4) and m[0, 1] == 2.0
    indptr, idx, val, width = as_csr(sp["v"])
    assert width == 4 and list(indptr) == [0, 1, 3]


def test_params_and_copy():
    t = AddConst(value=3.0)
    assert t.getValue() == 3.0 and t.getInputCol() == "x"
    t2 = t.copy({"value": 5.0})
    assert t2.getValue() == 5.0 and t.getValue() == 3.0
    assert "value" in t.explainParams()
    with pytest.raises(AttributeError):
        t.set("nope", 1)


def test_pipeline_fit_transform_save_load(tmp_path):
    df = DataFrame({"x": np.arange(5.0)})
    pipe = Pipeline(stages=[AddConst(value=1.0), MeanEstimator()])
    model = pipe.fit(df)
    out = model.transform(df)
    np.testing.assert_allclose(out["centered"], out["x"] - 2.0)
    p = str(tmp_path / "pm")
    model.save(p)
    meta = json.loads(open(os.path.join(p, "metadata", "part-00000")).readline())
    assert set(meta) >= {"class", "timestamp", "sparkVersion", "uid", "paramMap", "defaultParamMap"}
    loaded = PipelineStage.load(p)
    np.testing.assert_allclose(loaded.transform(df)["centered"], out["centered"])
    mm = loaded.getStages()[1]
    assert mm.getBlob() == b"\x00\x01abc"
    blob_file = os.path.join(p, "complexParams", "stages", "stage_0001", "complexParams", "blob", "data.bin")
    raw = open(blob_file, "rb").read()
    assert raw[:4] == bytes.fromhex("aced0005")


def test_java_byte_array_roundtrip():
    for b in [b"", b"abc", bytes(range(256)) * 10]:
        assert java_deserialize_bytes(java_serialize_bytes(b)) == b


def test_params_string_builder_first_wins():
    sb = ParamsStringBuilder()
    sb.append("num_leaves=5 lambda_l1=0.1")
    sb.appendParamValueIfNotThere("num_leaves", 31).appendParamValueIfNotThere("max_bin", 255)
    sb.appendParamValueIfNotThere("flag", True).appendParamListIfNotThere("cats", [1, 2])
    assert sb.result == "num_leaves=5 lambda_l1=0.1 max_bin=255 flag=true cats=1,2"


def test_misc_utils():
    assert find_unused_column_name("a", ["a", "a_1"]) == "a_2"
    calls = []

    def flaky():
        calls.append(1)
        if len(calls) < 3:
            raise RuntimeError("x")
        return 7

    assert retry_with_timeout(flaky, backoffs_ms=(0, 1, 1, 1)) == 7


def test_dataframe_arrow_roundtrip():
    import pyarrow as pa

    from synapseml_amd.core import DataFrame

    X = np.arange(12, dtype=np.float64).reshape(4, 3)
    df = DataFrame({"features": X, "label": np.array([0.0, 1.0, 1.0, 0.0]), "name": np.array(["a", "b", "c", "d"],
                                                                                              dtype=object)})
    t = df.toArrow()
    assert isinstance(t, pa.Table) and pa.types.is_fixed_size_list(t.schema.field("features").type)
    back = DataFrame.fromArrow(t, num_partitions=2)
    np.testing.assert_array_equal(back["features"], X)
    assert back["name"].tolist() == ["a", "b", "c", "d"]
    assert back.getNumPartitions() == 2
    # record batches (Spark mapInArrow delivers an iterator of them)
    b2 = DataFrame.fromArrow(t.to_batches(max_chunksize=2))
    np.testing.assert_array_equal(b2["label"], df["label"])


def test_sas_scrubber():
    from synapseml_amd.core.logging import payload, scrub

    sig = "sig=" + "a1B2c3D4e5%2F" * 4 + "%3D"
    msg = f"GET https://acct.blob.core.windows.net/c/f?sv=2020&{sig}&se=x failed"
    out = scrub(msg)
    assert "sig=####" in out and sig not in out and out.startswith("GET https://acct")
    assert scrub("no token here") == "no token here"
    assert "sig=####" in payload(object(), "fit", error=RuntimeError(msg))["errorMessage"]


def test_certified_events_sink():
    """fit/transform payloads reach registered sinks; the Fabric client posts them to <endpoint>/telemetry."""
    import json
    import threading
    from http.server import BaseHTTPRequestHandler, HTTPServer

    import numpy as np

    from synapseml_amd.core import DataFrame
    from synapseml_amd.core.logging import add_event_sink, remove_event_sink
    from synapseml_amd.featurize import VectorAssembler
    from synapseml_amd.utils.fabric import CertifiedEventClient

    got = []

    class H(BaseHTTPRequestHandler):
        def do_POST(self):  # noqa: N802
            got.append((self.path, json.loads(self.rfile.read(int(self.headers["Content-Length"])))))
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    seen = []
    try:
        add_event_sink(seen.append)
        df = DataFrame({"a": np.arange(3.0), "b": np.ones(3)})
        VectorAssembler(inputCols=["a", "b"], outputCol="v").transform(df)
        assert any(p["method"] == "transform" and p["className"] == "VectorAssembler" for p in seen)
        st = CertifiedEventClient.log_to_certified_events(
            CertifiedEventClient.feature_name(seen[-1]), "VectorAssembler.transform", {"k": "v"},
            endpoint=f"http://127.0.0.1:{srv.server_port}")
        assert st == 200 and got[0][0] == "/telemetry"
        assert got[0][1]["feature_name"] == "Featurize" and got[0][1]["attributes"] == {"k": "v"}
    finally:
        remove_event_sink(seen.append)
        srv.shutdown()


def test_certified_event_sink_never_blocks(monkeypatch):
    """telemetry posts run on a background thread from a bounded queue, so a slow endpoint adds
    no latency to transform()."""
    import time

    from synapseml_amd.utils.fabric import CertifiedEventClient

    posted = []

    def slow_post(feature, activity, attrs, endpoint=None, timeout=5.0):
        time.sleep(0.5)
        posted.append(activity)
        return 200

    monkeypatch.setattr(CertifiedEventClient, "log_to_certified_events", staticmethod(slow_post))
    t0 = time.perf_counter()
    for _ in range(3):
        CertifiedEventClient.sink({"method": "transform", "className": "X", "module": "synapseml_amd.stages.x"})
    assert time.perf_counter() - t0 < 0.2
    CertifiedEventClient.flush(5.0)
    assert posted == ["X.transform"] * 3
