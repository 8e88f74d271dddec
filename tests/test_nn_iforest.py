"""Nearest neighbours + isolation forest (model: reference core/src/test/scala/.../nn/BallTreeTest.scala,
KNNTest.scala, ConditionalKNNTest.scala, isolationforest/VerifyIsolationForest.scala)."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.isolationforest import IsolationForest
from synapseml_amd.nn import KNN, BallTree, ConditionalBallTree, ConditionalKNN


def test_ball_tree_matches_bruteforce():
    rng = np.random.default_rng(0)
    K = rng.normal(size=(500, 8))
    bt = BallTree(K, list(range(500)), leafSize=10)
    for _ in range(10):
        q = rng.normal(size=8)
        got = [m.index for m in bt.findMaximumInnerProducts(q, 5)]
        assert got == list(np.argsort(-(K @ q), kind="stable")[:5])
    labels = ["a" if i % 3 else "b" for i in range(500)]
    cbt = ConditionalBallTree(K, list(range(500)), labels, leafSize=10)
    q = rng.normal(size=8)
    got = [m.index for m in cbt.findMaximumInnerProducts(q, {"b"}, 3)]
    allowed = np.asarray([l == "b" for l in labels])
    sc = np.where(allowed, K @ q, -np.inf)
    assert got == list(np.argsort(-sc, kind="stable")[:3])


def test_knn_and_conditional_knn():
    rng = np.random.default_rng(1)
    K = rng.normal(size=(100, 4))
    df = DataFrame({"features": K, "values": np.arange(100), "label": np.array([i % 2 for i in range(100)])})
    m = KNN(k=3).fit(df)
    out = m.transform(df.limit(5))
    res = out[m.getOutputCol()][0]
    assert [r["value"] for r in res] == list(np.argsort(-(K @ K[0]))[:3])
    cond = np.empty(5, dtype=object)
    for i in range(5):
        cond[i] = [1]
    cq = df.limit(5).withColumn("conditioner", cond)
    cm = ConditionalKNN(k=2).fit(df)
    res = cm.transform(cq)[cm.getOutputCol()][0]
    assert all(r["label"] == 1 for r in res) and len(res) == 2


def test_isolation_forest_finds_outliers():
    rng = np.random.default_rng(2)
    X = np.concatenate([rng.normal(size=(500, 3)), rng.normal(size=(10, 3)) * 0.5 + 8.0])
    df = DataFrame({"features": X})
    m = IsolationForest(numEstimators=50, contamination=0.02, randomSeed=3).fit(df)
    out = m.transform(df)
    s = out["outlierScore"]
    assert s[500:].min() > np.quantile(s[:500], 0.95)
    assert out["predictedLabel"][500:].mean() >= 0.8 and out["predictedLabel"][:500].mean() < 0.05
