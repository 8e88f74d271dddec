"""Featurize / base learners / TrainClassifier / ComputeModelStatistics
(model: reference core/src/test/scala/.../featurize/*, train/Verify*.scala).
Reference numbers come from downloaded CSVs not present here; synthetic data
and sklearn comparators stand in (parity unpinned)."""
import datetime as dt

import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.core.linalg import SparseVector
from synapseml_amd.featurize import (CleanMissingData, CountSelector, DataConversion, Featurize, HashingTF, IDF,
                                     IndexToValue, MultiNGram, OneHotEncoder, PageSplitter, RegexTokenizer,
                                     StringIndexer, TextFeaturizer, ValueIndexer, VectorAssembler)
from synapseml_amd.featurize.ml import murmur3_spark
from synapseml_amd.models import (BinaryClassificationEvaluator, GBTClassifier, LinearRegression,
                                  LogisticRegression, MulticlassClassificationEvaluator, NaiveBayes,
                                  RandomForestClassifier, RegressionEvaluator)
from synapseml_amd.train import (ComputeModelStatistics, ComputePerInstanceStatistics, TrainClassifier,
                                 TrainRegressor)


def _obj(v):
    a = np.empty(len(v), dtype=object)
    for i, x in enumerate(v):
        a[i] = x
    return a


def test_value_indexer_roundtrip_with_nulls():
    df = DataFrame({"c": _obj(["b", None, "a", "b", "c"])})
    m = ValueIndexer(inputCol="c", outputCol="i").fit(df)
    out = m.transform(df)
    assert out["i"].tolist() == [1, 3, 0, 1, 2]  # nulls after the sorted non-null levels
    assert out.metadata("i")["ml_attr"]["type"] == "nominal"
    back = IndexToValue(inputCol="i", outputCol="v").transform(out)
    assert back["v"].tolist() == ["b", None, "a", "b", "c"]
    nums = DataFrame({"x": np.array([3.0, 1.0, 2.0, 1.0])})
    assert ValueIndexer(inputCol="x", outputCol="i").fit(nums).transform(nums)["i"].tolist() == [2, 0, 1, 0]


def test_clean_missing_and_conversion():
    df = DataFrame({"x": np.array([1.0, np.nan, 3.0, 5.0]), "y": np.array([1.0, 2.0, np.nan, 2.0])})
    mean = CleanMissingData(inputCols=["x", "y"], outputCols=["x2", "y2"]).fit(df).transform(df)
    assert mean["x2"].tolist() == [1.0, 3.0, 3.0, 5.0]
    med = CleanMissingData(inputCols=["y"], outputCols=["y"], cleaningMode="Median").fit(df).transform(df)
    assert med["y"].tolist() == [1.0, 2.0, 2.0, 2.0]
    cust = CleanMissingData(inputCols=["x"], outputCols=["x"], cleaningMode="Custom", customValue="-1").fit(df)
    assert cust.transform(df)["x"].tolist() == [1.0, -1.0, 3.0, 5.0]
    d = DataFrame({"a": np.array([1, 0, 2]), "s": _obj(["1.5", "2", "3"])})
    assert DataConversion(cols=["a"], convertTo="boolean").transform(d)["a"].tolist() == [True, False, True]
    assert DataConversion(cols=["s"], convertTo="double").transform(d)["s"].tolist() == [1.5, 2.0, 3.0]
    assert DataConversion(cols=["a"], convertTo="string").transform(d)["a"].tolist() == ["1", "0", "2"]
    cat = DataConversion(cols=["s"], convertTo="toCategorical").transform(d)
    assert cat["s"].tolist() == [0, 1, 2]
    assert DataConversion(cols=["s"], convertTo="clearCategorical").transform(cat)["s"].tolist() == ["1.5", "2", "3"]
    ts = DataFrame({"t": _obj(["2020-01-02 03:04:05"])})
    conv = DataConversion(cols=["t"], convertTo="date").transform(ts)
    assert conv["t"][0] == dt.datetime(2020, 1, 2, 3, 4, 5)


def test_text_pipeline_pieces():
    assert murmur3_spark("a") == murmur3_spark("a") and isinstance(murmur3_spark("hello"), int)
    df = DataFrame({"t": _obj(["the quick brown fox", "the lazy dog", None])})
    tok = RegexTokenizer(inputCol="t", outputCol="w").transform(df)
    assert tok["w"][0] == ["the", "quick", "brown", "fox"]
    tf = HashingTF(inputCol="w", outputCol="tf", numFeatures=64).transform(tok.filter(np.array([1, 1, 0], bool)))
    v = tf["tf"][0]
    assert isinstance(v, SparseVector) and v.values.sum() == 4
    idf = IDF(inputCol="tf", outputCol="idf").fit(tf).transform(tf)
    the_idx = murmur3_spark("the") % 64
    r0 = dict(zip(idf["idf"][0].indices.tolist(), idf["idf"][0].values.tolist()))
    assert r0[the_idx] == pytest.approx(np.log(3 / 3))  # term in every doc -> 0
    full = TextFeaturizer(inputCol="t", outputCol="f", numFeatures=128, useStopWordsRemover=True, useNGram=True,
                          nGramLength=2).fit(df.limit(2))
    out = full.transform(df.limit(2))
    assert out.columns == ["t", "f"] and out["f"][0].size == 128
    mg = MultiNGram(inputCol="w", outputCol="g", lengths=[1, 2]).transform(tok.limit(1))
    assert "quick brown" in mg["g"][0] and "fox" in mg["g"][0]
    ps = PageSplitter(inputCol="t", outputCol="p", maximumPageLength=10, minimumPageLength=5).transform(df.limit(1))
    pages = ps["p"][0]
    assert "".join(pages) == "the quick brown fox" and all(len(p) <= 10 for p in pages)


def test_count_selector_indexer_ohe_assembler():
    vecs = _obj([SparseVector(10, [1, 5], [1.0, 2.0]), SparseVector(10, [5, 7], [3.0, 1.0])])
    df = DataFrame({"v": vecs})
    cs = CountSelector(inputCol="v", outputCol="o").fit(df)
    assert cs.getIndices() == [1, 5, 7]
    assert cs.transform(df)["o"][1].toArray().tolist() == [0.0, 3.0, 1.0]
    s = DataFrame({"c": _obj(["a", "b", "a", "c"]), "x": np.arange(4.0)})
    si = StringIndexer(inputCol="c", outputCol="ci").fit(s).transform(s)
    assert si["ci"].tolist() == [0.0, 1.0, 0.0, 2.0]
    oh = OneHotEncoder(inputCols=["ci"], outputCols=["oh"]).fit(si).transform(si)
    assert oh["oh"][1].toArray().tolist() == [0.0, 1.0]  # dropLast
    va = VectorAssembler(inputCols=["x", "oh"], outputCol="f").transform(oh)
    assert va["f"][1].toArray().tolist() == [1.0, 0.0, 1.0]


def test_featurize_mixed_types():
    n = 50
    rng = np.random.default_rng(0)
    df = DataFrame({"num": rng.normal(size=n), "int": rng.integers(0, 4, n), "txt": _obj(
        [f"word{i % 5} other" if i % 7 else None for i in range(n)]), "nan": np.where(np.arange(n) % 5 == 0, np.nan,
                                                                                     1.0)})
    cat = ValueIndexer(inputCol="int", outputCol="cat").fit(df).transform(df)
    m = Featurize(inputCols=["num", "cat", "txt", "nan"], outputCol="features", numFeatures=64).fit(cat)
    out = m.transform(cat)
    assert set(out.columns) == set(cat.columns) | {"features"}
    f0 = out["features"][0]
    arr = f0.toArray() if hasattr(f0, "toArray") else np.asarray(f0)
    assert not np.isnan(arr).any()
    # numeric + one-hot(4 levels, dropLast -> 3) + selected text slots + imputed column
    assert len(arr) >= 1 + 3 + 1 + 1


def _binary_df(n=800, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 6))
    w = rng.normal(size=6)
    y = (X @ w + 0.2 * rng.normal(size=n) > 0).astype(np.float64)
    return DataFrame({"features": X, "label": y}), X, y


def test_base_learners_vs_sklearn():
    from sklearn.linear_model import LogisticRegression as SkLR
    from sklearn.metrics import roc_auc_score

    df, X, y = _binary_df()
    m = LogisticRegression(maxIter=200).fit(df)
    ours = roc_auc_score(y, m.transform(df)["probability"][:, 1])
    sk = roc_auc_score(y, SkLR(C=1e6, max_iter=1000).fit(X, y).predict_proba(X)[:, 1])
    assert abs(ours - sk) < 0.01
    for est in (GBTClassifier(maxIter=20), RandomForestClassifier(numTrees=10), NaiveBayes(modelType="gaussian")):
        o = est.fit(df).transform(df)
        assert BinaryClassificationEvaluator(rawPredictionCol="probability").evaluate(o) > 0.9
        assert MulticlassClassificationEvaluator(metricName="accuracy").evaluate(o) > 0.8
    Xr = X
    yr = X @ np.arange(6.0) + 3.0
    r = LinearRegression().fit(DataFrame({"features": Xr, "label": yr}))
    np.testing.assert_allclose(r.coefficients.toArray(), np.arange(6.0), atol=1e-6)
    assert r.intercept == pytest.approx(3.0, abs=1e-6)
    assert RegressionEvaluator().evaluate(r.transform(DataFrame({"features": Xr, "label": yr}))) < 1e-6


def test_train_classifier_and_statistics():
    rng = np.random.default_rng(1)
    n = 500
    a = rng.normal(size=n)
    b = rng.choice(["x", "y", "z"], size=n)
    y = np.where(a + (b == "x") * 1.5 + 0.3 * rng.normal(size=n) > 0.5, ">50K", "<=50K")
    df = DataFrame({"a": a, "b": _obj(list(b)), "income": _obj(list(y))})
    model = TrainClassifier(labelCol="income", numFeatures=32).fit(df)
    scored = model.transform(df)
    assert set(["scores", "scored_probabilities", "scored_labels"]) <= set(scored.columns)
    assert set(scored["scored_labels"].tolist()) <= {">50K", "<=50K"}
    stats = ComputeModelStatistics().transform(scored)
    assert stats["accuracy"][0] > 0.85 and stats["AUC"][0] > 0.9
    assert stats["confusion_matrix"][0].shape == (2, 2)
    # multiclass with a tree learner
    y3 = np.where(a > 0.7, "hi", np.where(a < -0.7, "lo", "mid"))
    df3 = DataFrame({"a": a, "b": _obj(list(b)), "lab": _obj(list(y3))})
    m3 = TrainClassifier(labelCol="lab", model=RandomForestClassifier(numTrees=8)).fit(df3)
    st3 = ComputeModelStatistics().transform(m3.transform(df3))
    assert st3["accuracy"][0] > 0.8 and "macro_averaged_recall" in st3.columns


def test_train_regressor_and_per_instance():
    rng = np.random.default_rng(2)
    x = rng.normal(size=300)
    df = DataFrame({"x": x, "c": _obj(list(rng.choice(["p", "q"], size=300))), "y": 2 * x + 1})
    m = TrainRegressor(labelCol="y").fit(df)
    out = m.transform(df)
    st = ComputeModelStatistics().transform(out)
    assert st["R^2"][0] > 0.99 and st["root_mean_squared_error"][0] < 0.05
    pi = ComputePerInstanceStatistics().transform(out)
    assert "L1_loss" in pi.columns and pi["L2_loss"].max() < 0.05
