"""Stage tests (model: reference core/src/test/scala/.../stages/*Suite.scala)."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.core.linalg import DenseVector
from synapseml_amd.stages import (Cacher, ClassBalancer, DropColumns, DynamicMiniBatchTransformer, EnsembleByKey,
                                  Explode, FixedMiniBatchTransformer, FlattenBatch, Lambda, MultiColumnAdapter,
                                  PartitionConsolidator, RenameColumn, Repartition, SelectColumns,
                                  StratifiedRepartition, SummarizeData, TextPreprocessor, Timer, Trie, UDFTransformer,
                                  UnicodeNormalize)


def _df(n=10, parts=2):
    return DataFrame({"a": np.arange(n), "b": np.arange(n) * 2.0, "s": np.array([f"x{i}" for i in range(n)],
                                                                               dtype=object)}, num_partitions=parts)


def test_minibatch_and_flatten_roundtrip():
    df = _df(10, 2)
    b = FixedMiniBatchTransformer(batchSize=3).transform(df)
    assert b.count() == 4  # partitions of 5: [3,2] + [3,2]
    assert b["a"][0] == [0, 1, 2] and b["a"][1] == [3, 4]
    f = FlattenBatch().transform(b)
    assert f["a"].tolist() == list(range(10))
    assert f["s"].tolist() == [f"x{i}" for i in range(10)]
    d = DynamicMiniBatchTransformer(maxBatchSize=4).transform(df)
    assert [len(x) for x in d["a"]] == [4, 1, 4, 1]


def test_simple_column_stages():
    df = _df()
    assert DropColumns(cols=["a"]).transform(df).columns == ["b", "s"]
    assert SelectColumns(cols=["s", "a"]).transform(df).columns == ["s", "a"]
    assert "z" in RenameColumn(inputCol="a", outputCol="z").transform(df).columns
    with pytest.raises(ValueError):
        DropColumns(cols=["nope"]).transform(df)
    assert Repartition(n=3).transform(df).getNumPartitions() == 3
    assert PartitionConsolidator().transform(df).getNumPartitions() == 1
    assert Cacher().transform(df).count() == 10
    lam = Lambda().set("transformFunc", lambda d: d.withColumn("c", d["a"] + 1))
    assert lam.transform(df)["c"].tolist() == list(range(1, 11))
    u = UDFTransformer(inputCol="a", outputCol="sq").setUDF(lambda v: v * v).transform(df)
    assert u["sq"].tolist() == [i * i for i in range(10)]
    u2 = UDFTransformer(inputCols=["a", "b"], outputCol="sum").setUDF(lambda x, y: x + y).transform(df)
    assert u2["sum"].tolist() == [3.0 * i for i in range(10)]


def test_explode_unicode_text_preprocessor():
    col = np.empty(2, dtype=object)
    col[0] = [1, 2]
    col[1] = [3]
    e = Explode(inputCol="l", outputCol="x").transform(DataFrame({"l": col, "k": [7, 8]}))
    assert e["x"].tolist() == [1, 2, 3] and e["k"].tolist() == [7, 7, 8]
    un = UnicodeNormalize(inputCol="t", outputCol="n", form="NFKD").transform(
        DataFrame({"t": np.array(["Ｃafé"], dtype=object)}))
    assert un["n"][0] == "café"
    tp = TextPreprocessor(inputCol="t", outputCol="o", map={"happy": "sad", "hap": "smile", "o": "0"},
                          normFunc="lowerCase")
    out = tp.transform(DataFrame({"t": np.array(["I'm Happy today ok", "happyday hap ", "no"], dtype=object)}))
    assert out["o"][0] == "I'm sad t0 0"  # after a match the rest of the word is skipped
    assert out["o"][1] == "sad smile "  # rest of a matched word is skipped
    assert out["o"][2] == "no"  # a key ending exactly at the end of the text is not matched (reference quirk)
    t = Trie().putAll({"ab": "X"})
    assert t.mapText("abc ab!") == "X X!"


def test_class_balancer_and_stratified():
    df = DataFrame({"label": np.array([0, 0, 0, 1]), "v": np.arange(4)})
    m = ClassBalancer(inputCol="label").fit(df)
    assert m.transform(df)["weight"].tolist() == [1.0, 1.0, 1.0, 3.0]
    big = DataFrame({"label": np.array([0] * 90 + [1] * 10), "v": np.arange(100)}, num_partitions=4)
    eq = StratifiedRepartition(labelCol="label", mode="equal", seed=1).transform(big)
    for p in eq.partitions():
        assert set(p["label"].tolist()) == {0, 1}
    lab = eq["label"]
    assert abs((lab == 1).mean() - 0.5) < 0.05
    orig = StratifiedRepartition(labelCol="label", mode="original").transform(big)
    assert orig.count() == 100 and all(set(p["label"].tolist()) == {0, 1} for p in orig.partitions())


def test_ensemble_by_key():
    vec = np.empty(4, dtype=object)
    for i in range(4):
        vec[i] = DenseVector([i, 2 * i])
    df = DataFrame({"k": [1, 1, 2, 2], "score": [1.0, 3.0, 5.0, 7.0], "v": vec})
    out = EnsembleByKey(keys=["k"], cols=["score", "v"]).transform(df)
    assert dict(zip(out["k"].tolist(), out["mean(score)"].tolist())) == {1: 2.0, 2: 6.0}
    assert np.asarray(out["mean(v)"][1]).tolist() == [2.5, 5.0]
    nc = EnsembleByKey(keys=["k"], cols=["score"], colNames=["avg"], collapseGroup=False).transform(df)
    assert nc.count() == 4 and "avg" in nc.columns


def test_summarize_data():
    df = DataFrame({"x": np.array([1.0, 2.0, 3.0, 4.0, np.nan]), "s": np.array(["a", "b", "a", None, "c"],
                                                                                dtype=object)})
    s = SummarizeData().transform(df)
    r = {f: i for i, f in enumerate(s["Feature"].tolist())}
    assert s["Count"][r["x"]] == 4 and s["Missing_Value_Count"][r["x"]] == 1
    assert s["Unique_Value_Count"][r["s"]] == 3 and s["Missing_Value_Count"][r["s"]] == 1
    assert s["Min"][r["x"]] == 1.0 and s["Max"][r["x"]] == 4.0 and s["Median"][r["x"]] == 2.0
    assert abs(s["Sample_Variance"][r["x"]] - np.var([1, 2, 3, 4], ddof=1)) < 1e-12
    assert np.isnan(s["Min"][r["s"]])


def test_timer_and_multicolumn_adapter():
    from synapseml_amd.featurize import ValueIndexer

    df = DataFrame({"a": np.array(["x", "y", "x"], dtype=object), "b": np.array(["p", "p", "q"], dtype=object)})
    t = Timer(logToScala=False).set("stage", ValueIndexer(inputCol="a", outputCol="ai"))
    m = t.fit(df)
    assert m.transform(df)["ai"].tolist() == [0, 1, 0]
    mca = MultiColumnAdapter(inputCols=["a", "b"], outputCols=["ai", "bi"]).set("baseStage", ValueIndexer())
    out = mca.fit(df).transform(df)
    assert out["bi"].tolist() == [0, 0, 1]


def test_iterator_batchers():
    """Batchers.scala equivalents over lazy iterators (reference: core/.../stages/Batchers.scala)."""
    import threading
    import time as _t

    from synapseml_amd.stages import DynamicBufferedBatcher, FixedBatcher, FixedBufferedBatcher, TimeIntervalBatcher

    assert list(FixedBatcher(range(7), 3)) == [[0, 1, 2], [3, 4, 5], [6]]
    assert list(FixedBufferedBatcher(iter(range(7)), 3, max_buffer_size=1)) == [[0, 1, 2], [3, 4, 5], [6]]
    assert list(FixedBatcher([], 3)) == []

    def slow():
        for i in range(6):
            _t.sleep(0.01)
            yield i

    got = list(DynamicBufferedBatcher(slow()))
    assert sum(got, []) == list(range(6)) and all(len(b) >= 1 for b in got)
    # a slow consumer sees larger batches: everything buffered meanwhile
    b = DynamicBufferedBatcher(iter(range(100)))
    first = next(b)
    _t.sleep(0.05)
    rest = sum(list(b), [])
    assert first + rest == list(range(100)) and max(len(first), len(rest)) > 1
    tb = list(TimeIntervalBatcher(iter(range(10)), millis=1000, max_buffer_size=4))
    assert tb == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]

    def boom():
        yield 1
        raise RuntimeError("source failed")

    import pytest

    with pytest.raises(RuntimeError):
        list(FixedBufferedBatcher(boom(), 5))
    assert threading.active_count() < 50
