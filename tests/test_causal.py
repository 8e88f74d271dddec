"""Causal tests (model: reference core/src/test/scala/.../causal/*Suite.scala): effects recovered on
synthetic data with known ground truth."""
import numpy as np
import pytest

from synapseml_amd.causal import (DiffInDiffEstimator, DoubleMLEstimator, OrthoForestDMLEstimator,
                                  ResidualTransformer, SyntheticControlEstimator, SyntheticDiffInDiffEstimator,
                                  simplex_least_squares)
from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.models import LinearRegression, LogisticRegression


def test_double_ml_recovers_ate():
    rng = np.random.default_rng(0)
    n = 3000
    X = rng.normal(size=(n, 3))
    t = (X[:, 0] + rng.normal(size=n) > 0).astype(np.int32)  # 0/1 integer column for a classifier
    y = 2.0 * t + X @ np.array([1.0, -1.0, 0.5]) + rng.normal(size=n) * 0.5
    df = DataFrame({"features": X, "treatment": t, "outcome": y})
    est = DoubleMLEstimator(treatmentModel=LogisticRegression(), outcomeModel=LinearRegression(), maxIter=5)
    m = est.fit(df)
    assert m.getAvgTreatmentEffect() == pytest.approx(2.0, abs=0.2)
    lo, hi = m.getConfidenceInterval()
    assert lo <= m.getAvgTreatmentEffect() <= hi
    assert m.getPValue() < 0.01
    assert len(m.getRawTreatmentEffects()) == 5


def test_double_ml_reference_semantics():
    """Column/model type checks, weight support, commons-math percentiles, single-iteration p-value
    (reference DoubleMLEstimator.scala validateColTypeWithModel / DoubleMLModel)."""
    from synapseml_amd.causal import commons_percentile

    rng = np.random.default_rng(3)
    n = 1500
    X = rng.normal(size=(n, 2))
    t = (X[:, 0] + rng.normal(size=n) > 0).astype(np.int64)
    y = 1.5 * t + X[:, 1] + 0.3 * rng.normal(size=n)
    df = DataFrame({"features": X, "treatment": t, "outcome": y, "w": np.ones(n)})
    with pytest.raises(TypeError, match="classification"):  # double outcome with a classifier
        DoubleMLEstimator(treatmentModel=LogisticRegression(), outcomeModel=LogisticRegression()).fit(df)
    with pytest.raises(ValueError, match="0 or 1"):
        DoubleMLEstimator(treatmentModel=LogisticRegression(), outcomeModel=LinearRegression()).fit(
            df.withColumn("treatment", t * 2))
    with pytest.raises(ValueError, match="maxIter"):
        DoubleMLEstimator(treatmentModel=LogisticRegression(), outcomeModel=LinearRegression(), maxIter=0).fit(df)
    m = DoubleMLEstimator(treatmentModel=LogisticRegression(), outcomeModel=LinearRegression(), weightCol="w").fit(df)
    assert m.getAvgTreatmentEffect() == pytest.approx(1.5, abs=0.2)
    with pytest.raises(ValueError, match="maxIter >= 2"):
        m.getPValue()
    # commons-math Percentile (legacy estimation): position p(n+1)/100
    v = [1.0, 2.0, 3.0, 4.0]
    assert commons_percentile(v, 50) == pytest.approx(2.5)
    assert commons_percentile(v, 97.5) == 4.0 and commons_percentile(v, 2.5) == 1.0
    assert commons_percentile(v, 25) == pytest.approx(1.25)


def test_ortho_forest_heterogeneous_effect():
    rng = np.random.default_rng(1)
    n = 2000
    W = rng.normal(size=(n, 2))
    Xh = rng.uniform(0, 1, size=(n, 1))
    t = W[:, 0] + rng.normal(size=n)
    effect = 1.0 + 2.0 * (Xh[:, 0] > 0.5)
    y = effect * t + W[:, 1] + 0.1 * rng.normal(size=n)
    df = DataFrame({"XW": W, "X": Xh, "treatment": t, "outcome": y})
    m = OrthoForestDMLEstimator(treatmentModel=LinearRegression(), outcomeModel=LinearRegression(), numTrees=10,
                                maxDepth=3, minSamplesLeaf=20).fit(df)
    out = m.transform(DataFrame({"X": np.array([[0.2], [0.8]])}))
    lo_eff, hi_eff = out["EffectAverage"]
    assert len(m.getForest()) == 2 * 10  # one forest per cross-fitting half
    assert lo_eff == pytest.approx(1.0, abs=0.4) and hi_eff == pytest.approx(3.0, abs=0.5)
    assert (out["EffectLowerBound"] <= out["EffectUpperBound"]).all()


def test_residual_transformer_and_did():
    df = DataFrame({"label": [1.0, 0.0], "prediction": [0.25, 0.5]})
    assert ResidualTransformer().transform(df)["residual"].tolist() == [0.75, -0.5]
    rng = np.random.default_rng(2)
    rows = []
    for unit in range(40):
        tr = unit < 20
        for post in (0, 1):
            y = 1.0 + 0.5 * tr + 0.7 * post + 3.0 * tr * post + 0.01 * rng.normal()
            rows.append((float(tr), float(post), y))
    t, p, y = map(np.asarray, zip(*rows))
    m = DiffInDiffEstimator().fit(DataFrame({"treatment": t, "postTreatment": p, "outcome": y}))
    assert m.getSummary().treatmentEffect == pytest.approx(3.0, abs=0.02)


def test_simplex_ls_and_synthetic_estimators():
    A = np.array([[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]])
    w, c, _ = simplex_least_squares(A, A @ np.array([0.3, 0.7]), intercept=False, max_iter=2000, tol=1e-14)
    np.testing.assert_allclose(w, [0.3, 0.7], atol=1e-3)
    rng = np.random.default_rng(3)
    T_, U = 12, 8
    base = rng.normal(size=(U, 1)) + np.linspace(0, 2, T_)[None, :]
    treated = 0
    Y = base.copy()
    Y[treated] = 0.5 * base[1] + 0.5 * base[2]
    Y[treated, 8:] += 5.0
    rows = []
    for u in range(U):
        for t in range(T_):
            rows.append((u, t, Y[u, t], float(u == treated), float(t >= 8)))
    u, t, y, tr, p = map(np.asarray, zip(*rows))
    df = DataFrame({"unit": u, "time": t, "outcome": y, "treatment": tr, "postTreatment": p})
    sc = SyntheticControlEstimator(maxIter=3000, tol=1e-12).fit(df)
    assert sc.getSummary().treatmentEffect == pytest.approx(5.0, abs=0.3)
    assert sc.getUnitWeights().count() == U
    sdid = SyntheticDiffInDiffEstimator(maxIter=3000, tol=1e-12).fit(df)
    assert sdid.getSummary().treatmentEffect == pytest.approx(5.0, abs=0.5)
    assert sdid.getTimeWeights() is not None
    # index DataFrames map weight positions to time / unit values (BaseDiffInDiffEstimator.scala:105-119)
    ti, ui = sdid.getTimeIndex(), sdid.getUnitIndex()
    assert ti.count() == T_ and ui.count() == U
    assert list(ti[sdid.getTimeIndexCol()]) == list(range(T_)) and list(ti["time"]) == list(range(T_))
    assert list(ui["unit"]) == list(range(U))


def test_ortho_forest_variable_transformer():
    import numpy as np

    from synapseml_amd.causal import OrthoForestVariableTransformer
    from synapseml_amd.core.dataframe import DataFrame

    df = DataFrame({"TResid": np.array([2.0, -0.5]), "OResid": np.array([1.0, 1.0])})
    out = OrthoForestVariableTransformer().transform(df)
    np.testing.assert_allclose(out["_tmp_tsOutcome"], [0.5, -2.0])
    np.testing.assert_allclose(out["_tmp_twOutcome"], [4.0, 0.25])
    import pytest

    with pytest.raises(TypeError):
        OrthoForestVariableTransformer().transform(DataFrame({"TResid": np.array([1, 2]), "OResid": np.ones(2)}))
