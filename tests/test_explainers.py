"""Explainer tests (model: reference core/src/test/scala/.../explainers/*Suite.scala): SHAP values of a
linear model equal w_j * (x_j - E[x_j]); LIME recovers linear coefficients; ICE/PDP shapes."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.core.pipeline import Transformer
from synapseml_amd.explainers import (ICETransformer, ImageLIME, ImageSHAP, TabularLIME, TabularSHAP, TextLIME,
                                      TextSHAP, VectorLIME, VectorSHAP, lasso, least_squares, shap_coalitions, slic)


class _Linear(Transformer):
    """probability[1] = w . x + b over named columns or a vector column."""

    def __init__(self, w=None, b=0.0, cols=None, vec=None, **kw):
        super().__init__(**kw)
        self.w, self.b, self.cols, self.vec = np.asarray(w, float), b, cols, vec

    def _transform(self, df):
        from synapseml_amd.core.linalg import as_matrix

        X = as_matrix(df[self.vec]) if self.vec else np.stack([np.asarray(df[c], float) for c in self.cols], 1)
        s = X @ self.w + self.b
        return df.withColumn("probability", np.stack([1 - s, s], 1))


def test_regression_helpers():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(200, 3))
    y = X @ np.array([1.0, -2.0, 0.0]) + 0.5
    r = least_squares(X, y, np.ones(200))
    np.testing.assert_allclose(r.coefficients, [1, -2, 0], atol=1e-10)
    assert r.intercept == pytest.approx(0.5) and r.rSquared == pytest.approx(1.0)
    l1 = lasso(X, y, np.ones(200), alpha=0.1)
    assert abs(l1.coefficients[2]) < 1e-9 and l1.coefficients[0] > 0.7
    Z, w = shap_coalitions(3, 100, rng, 1e8)
    assert Z.shape == (8, 3) and w[0] == 1e8 and w[1] == 1e8 and Z[1].sum() == 3 and Z[0].sum() == 0


def test_tabular_and_vector_shap_exact_for_linear_model():
    rng = np.random.default_rng(1)
    bg = DataFrame({"a": rng.normal(size=30), "b": rng.normal(size=30), "c": rng.normal(size=30)})
    w = np.array([0.5, -1.0, 2.0])
    model = _Linear(w, 0.1, cols=["a", "b", "c"])
    inst = DataFrame({"a": [1.0, -1.0], "b": [2.0, 0.5], "c": [0.0, 1.0]})
    out = TabularSHAP(inputCols=["a", "b", "c"], outputCol="shap", targetClasses=[1], model=model,
                      backgroundData=bg).transform(inst)
    mu = np.array([bg["a"].mean(), bg["b"].mean(), bg["c"].mean()])
    for i in range(2):
        x = np.array([inst["a"][i], inst["b"][i], inst["c"][i]])
        phi = out["shap"][i][0].toArray()
        np.testing.assert_allclose(phi[1:], w * (x - mu), atol=1e-6)
        assert phi[0] == pytest.approx(w @ mu + 0.1, abs=1e-6)
        assert out["r2"][i].toArray()[0] == pytest.approx(1.0, abs=1e-9)
    vbg = DataFrame({"v": np.stack([bg["a"], bg["b"], bg["c"]], 1)})
    vinst = DataFrame({"v": np.array([[1.0, 2.0, 0.0]])})
    vs = VectorSHAP(inputCol="v", outputCol="shap", targetClasses=[1], model=_Linear(w, 0.1, vec="v"),
                    backgroundData=vbg).transform(vinst)
    np.testing.assert_allclose(vs["shap"][0][0].toArray()[1:], w * (np.array([1.0, 2.0, 0.0]) - mu), atol=1e-6)


def test_lime_recovers_linear_coefficients():
    rng = np.random.default_rng(2)
    w = np.array([1.5, -0.5])
    bg = DataFrame({"v": rng.normal(size=(100, 2))})
    out = VectorLIME(inputCol="v", outputCol="lime", targetClasses=[1], model=_Linear(w, 0.0, vec="v"),
                     backgroundData=bg, numSamples=500).transform(DataFrame({"v": np.array([[0.3, 0.7]])}))
    np.testing.assert_allclose(out["lime"][0][0].toArray(), w, atol=1e-6)
    tb = DataFrame({"x": rng.normal(size=50), "y": rng.normal(size=50)})
    t = TabularLIME(inputCols=["x", "y"], outputCol="lime", targetClasses=[1], model=_Linear(w, 0.0, cols=["x", "y"]),
                    backgroundData=tb).transform(DataFrame({"x": [0.1], "y": [0.2]}))
    np.testing.assert_allclose(t["lime"][0][0].toArray(), w, atol=1e-6)


class _WordModel(Transformer):
    def _transform(self, df):
        s = np.asarray([1.0 if "good" in t.split() else 0.0 for t in df["text"].tolist()])
        return df.withColumn("probability", np.stack([1 - s, s], 1))


class _RedModel(Transformer):
    def _transform(self, df):
        from synapseml_amd.image import row_to_array

        s = np.asarray([row_to_array(r)[:8, :8, 2].mean() / 255.0 for r in df["image"].tolist()])
        return df.withColumn("probability", np.stack([1 - s, s], 1))


def test_text_and_image_explainers():
    df = DataFrame({"text": np.array(["this is good stuff"], dtype=object)})
    s = TextSHAP(inputCol="text", outputCol="shap", targetClasses=[1], model=_WordModel()).transform(df)
    phi = s["shap"][0][0].toArray()
    assert np.argmax(phi[1:]) == 2 and phi[3] == pytest.approx(1.0, abs=1e-6)
    assert s["tokens"][0] == ["this", "is", "good", "stuff"]
    l = TextLIME(inputCol="text", outputCol="lime", targetClasses=[1], model=_WordModel(), numSamples=300) \
        .transform(df)
    assert np.argmax(l["lime"][0][0].toArray()) == 2
    from synapseml_amd.image import make_image_row

    img = np.zeros((32, 32, 3), np.uint8)
    img[:8, :8, 2] = 255
    img[16:, 16:] = 90
    idf = DataFrame({"image": np.array([make_image_row(img)], dtype=object)})
    labels = slic(img, 8, 130)
    assert labels.max() >= 3
    sh = ImageSHAP(inputCol="image", outputCol="shap", targetClasses=[1], model=_RedModel(), cellSize=8,
                   numSamples=64).transform(idf)
    phi = sh["shap"][0][0].toArray()
    red_sp = labels[2, 2]
    assert np.argmax(phi[1:]) == red_sp
    li = ImageLIME(inputCol="image", outputCol="lime", targetClasses=[1], model=_RedModel(), cellSize=8,
                   numSamples=200).transform(idf)
    assert np.argmax(li["lime"][0][0].toArray()) == red_sp


def test_ice_pdp_and_feature_importance():
    rng = np.random.default_rng(3)
    df = DataFrame({"a": rng.normal(size=40), "b": rng.normal(size=40),
                    "c": np.array(["x", "y"] * 20, dtype=object)})

    class M(Transformer):
        def _transform(self, d):
            s = 2 * np.asarray(d["a"], float) + np.asarray([1.0 if v == "x" else 0.0 for v in d["c"].tolist()])
            return d.withColumn("probability", np.stack([1 - s, s], 1))

    ind = ICETransformer(model=M(), targetClasses=[1], numericFeatures=[{"name": "a", "numSplits": 4}],
                         categoricalFeatures=[{"name": "c"}]).transform(df)
    assert ind.count() == 40 and len(ind["a_dependence"][0]) == 5 and set(ind["c_dependence"][0]) == {"x", "y"}
    avg = ICETransformer(model=M(), targetClasses=[1], kind="average",
                         numericFeatures=[{"name": "a", "numSplits": 2, "rangeMin": 0.0, "rangeMax": 1.0}]) \
        .transform(df)
    pdp = avg["a_dependence"][0]
    keys = sorted(pdp)
    assert pdp[keys[2]].toArray()[0] - pdp[keys[0]].toArray()[0] == pytest.approx(2.0)
    feat = ICETransformer(model=M(), targetClasses=[1], kind="feature", numericFeatures=[{"name": "a"}],
                          categoricalFeatures=[{"name": "c"}]).transform(df)
    assert feat["featureNames"].tolist() == ["c_dependence", "a_dependence"]
    assert feat["pdpBasedDependence"][0].toArray()[0] == pytest.approx(0.25)


def test_kernel_shap_coalitions_follow_reference_allocation():
    """KernelSHAP coalitions (KernelSHAPSampler.scala generateSampleSizes / generateCoalitions, pinned by the
    reference's KernelSHAPSamplerSupportSuite): exact enumeration when the budget covers every size class,
    the paired size allocation with random fill otherwise."""
    import numpy as np

    from synapseml_amd.explainers.local import effective_num_samples, shap_coalitions, shap_sample_sizes

    rng = np.random.default_rng(0)
    Z, w = shap_coalitions(5, 32, rng, 1e8)
    s = Z.sum(1)
    assert len(Z) == 32 and w[0] == 1e8 and w[1] == 1e8
    assert [int((s == k).sum()) for k in range(6)] == [1, 5, 10, 10, 5, 1]
    assert len({tuple(r) for r in Z}) == 32  # every subset exactly once
    Z, w = shap_coalitions(500, 4, rng, 1e8)
    s = Z.sum(1)
    assert len(Z) == 4 and list(w) == [1e8, 1e8, 1.0, 1.0]
    assert [int((s == k).sum()) for k in (0, 500, 1, 2)] == [1, 1, 1, 1]
    Z, w = shap_coalitions(500, 1000, rng, 1e8)
    s = Z.sum(1)
    assert len(Z) == 1000 and (w[:2] == 1e8).all() and (w[2:] == 1.0).all()
    assert [int((s == k).sum()) for k in (0, 500, 1, 499, 2, 498)] == [1, 1, 74, 74, 37, 37]
    # budget clamp (KernelSHAPBase.getEffectiveNumSamples) and the kernel weights of enumerated sizes
    assert effective_num_samples(None, 3) == 8 and effective_num_samples(None, 20) == 2 * 20 + 2048
    assert effective_num_samples(1, 20) == 22
    sizes = shap_sample_sizes(6, 62, lambda k: float(k))
    assert [x for x, _ in sizes] == [6, 6, 15, 15, 20] and [wt for _, wt in sizes] == [1.0, 1.0, 2.0, 2.0, 3.0]
    for bad in ((5, 0), (5, 31)):
        with pytest.raises(ValueError):
            shap_sample_sizes(*bad, lambda k: 1.0)
