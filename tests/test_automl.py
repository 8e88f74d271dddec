"""AutoML tests (model: reference core/src/test/scala/.../automl/VerifyTuneHyperparameters.scala,
VerifyFindBestModel.scala)."""
import numpy as np

from synapseml_amd.automl import (DiscreteHyperParam, FindBestModel, GridSpace, HyperparamBuilder, RandomSpace,
                                  RangeHyperParam, TuneHyperparameters)
from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.models import GBTClassifier, LogisticRegression
from synapseml_amd.train import TrainClassifier


def _df(n=400, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    y = (X[:, 0] - X[:, 1] + 0.3 * rng.normal(size=n) > 0).astype(float)
    return DataFrame({"features": X, "label": y})


def test_spaces():
    lr = LogisticRegression()
    hp = HyperparamBuilder().addHyperparam(lr, "regParam", DiscreteHyperParam([0.0, 0.1])) \
        .addHyperparam(lr, "maxIter", DiscreteHyperParam([10, 50])).build()
    grid = list(GridSpace(hp).paramMaps())
    assert len(grid) == 4 and {(lr.uid, "regParam"): 0.1, (lr.uid, "maxIter"): 50} in grid
    rnd = RandomSpace([(lr, "regParam", RangeHyperParam(0.0, 1.0))], seed=3).paramMaps()
    vals = [next(rnd)[(lr.uid, "regParam")] for _ in range(5)]
    assert all(0 <= v < 1 for v in vals) and len(set(vals)) == 5


def test_tune_hyperparameters_picks_best():
    df = _df()
    lr = LogisticRegression()
    gbt = GBTClassifier()
    hp = HyperparamBuilder().addHyperparam(lr, "regParam", DiscreteHyperParam([0.0, 10.0])) \
        .addHyperparam(gbt, "maxIter", DiscreteHyperParam([5, 10])).build()
    tuned = TuneHyperparameters(models=[lr, gbt], evaluationMetric="accuracy", numFolds=2, numRuns=4,
                                parallelism=2, paramSpace=GridSpace(hp)).fit(df)
    assert tuned.getBestMetric() > 0.85
    out = tuned.transform(df)
    assert "prediction" in out.columns
    auc_tuned = TuneHyperparameters(models=[lr], evaluationMetric="AUC", numFolds=2, numRuns=2,
                                    paramSpace=GridSpace(hp)).fit(df)
    assert auc_tuned.getBestMetric() > 0.9


def test_find_best_model():
    df = _df()
    good = TrainClassifier(labelCol="label", model=LogisticRegression()).fit(df.withColumn(
        "label", np.asarray(df["label"])))
    bad_df = df.withColumn("label", np.random.default_rng(9).integers(0, 2, df.count()).astype(float))
    bad = TrainClassifier(labelCol="label", model=LogisticRegression()).fit(bad_df)
    best = FindBestModel(models=[bad, good], evaluationMetric="AUC").fit(df)
    assert best.getBestModel() is good
    assert best.getAllModelMetrics().count() == 2
    assert best.getRocCurve() is not None and best.getBestModelMetrics()["AUC"][0] > 0.9
