"""SparkML-equivalent learners and text / image primitives that the framework's estimators build on
(TrainClassifier, causal, AutoML, TextFeaturizer, ImageTransformer) exercised directly: fit / transform on
small synthetic data with known structure."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame


def _cls_data(n=600, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, 4))
    y = ((X[:, 0] + 0.5 * X[:, 1] > 0)).astype(np.float64)
    return DataFrame({"features": X, "label": y}), X, y


@pytest.mark.parametrize("name", ["DecisionTreeClassifier", "RandomForestClassifier", "GBTClassifier",
                                  "LogisticRegression", "NaiveBayes", "MultilayerPerceptronClassifier"])
def test_classifiers_learn(name):
    import synapseml_amd.models as M

    df, X, y = _cls_data()
    kw = {"layers": [4, 8, 2], "maxIter": 60} if name == "MultilayerPerceptronClassifier" else {}
    if name == "NaiveBayes":  # multinomial NB: non-negative counts whose proportions differ by class
        C = np.abs(X)
        C[y == 1, 0] += 2.0
        C[y == 0, 1] += 2.0
        df = DataFrame({"features": C, "label": y})
    if name in ("DecisionTreeClassifier", "RandomForestClassifier", "GBTClassifier"):
        kw["deviceType"] = "cpu"
    m = getattr(M, name)(**kw).fit(df)
    out = m.transform(df)
    acc = float((np.asarray(out["prediction"], np.float64) == y).mean())
    assert acc > 0.85, (name, acc)
    if "probability" in out.columns:
        p = np.stack([np.asarray(v.toArray() if hasattr(v, "toArray") else v) for v in out["probability"]])
        np.testing.assert_allclose(p.sum(1), 1.0, rtol=1e-6)


@pytest.mark.parametrize("name", ["DecisionTreeRegressor", "RandomForestRegressor", "GBTRegressor", "LinearRegression"])
def test_regressors_learn(name):
    import synapseml_amd.models as M

    rng = np.random.default_rng(1)
    X = rng.uniform(-1, 1, (800, 3))
    y = 3 * X[:, 0] - 2 * X[:, 1] + 0.05 * rng.standard_normal(800)
    df = DataFrame({"features": X, "label": y})
    kw = {} if name == "LinearRegression" else {"deviceType": "cpu"}
    m = getattr(M, name)(**kw).fit(df)
    pred = np.asarray(m.transform(df)["prediction"], np.float64)
    r2 = 1 - ((pred - y) ** 2).sum() / ((y - y.mean()) ** 2).sum()
    assert r2 > 0.8, (name, r2)


def test_text_primitives():
    from synapseml_amd.featurize.ml import NGram, RegexTokenizer, StopWordsRemover, Tokenizer

    df = DataFrame({"text": np.array(["The quick brown fox", "a Lazy dog"], dtype=object)})
    t = Tokenizer(inputCol="text", outputCol="tok").transform(df)
    assert list(t["tok"][0]) == ["the", "quick", "brown", "fox"]
    r = RegexTokenizer(inputCol="text", outputCol="rt", pattern=r"\s+").transform(df)
    assert list(r["rt"][1]) == ["a", "lazy", "dog"]
    s = StopWordsRemover(inputCol="tok", outputCol="nostop", stopWords=["the", "a"]).transform(t)
    assert list(s["nostop"][0]) == ["quick", "brown", "fox"]
    g = NGram(inputCol="nostop", outputCol="ng", n=2).transform(s)
    assert list(g["ng"][0]) == ["quick brown", "brown fox"]


def test_image_stage_classes():
    """the ImageTransformer stage objects (reference ImageTransformer.scala stage maps) applied one by one"""
    from synapseml_amd.image import ImageTransformer, make_image_row

    rng = np.random.default_rng(2)
    img = rng.integers(0, 255, (20, 30, 3), dtype=np.uint8)
    df = DataFrame({"image": np.array([make_image_row(img)], dtype=object)})
    out = (ImageTransformer(inputCol="image", outputCol="o").crop(2, 3, 16, 10).colorFormat(6)
           .blur(3, 3).threshold(100, 255, 0).transform(df))
    o = out["o"][0]
    data = np.frombuffer(o["data"], np.uint8)
    assert (o["height"], o["width"], o["nChannels"]) == (16, 10, 1)
    assert data.size == 16 * 10  # cropped to 16 x 10, one gray channel
    assert set(np.unique(data)).issubset({0, 255})
