"""Recommendation tests (model: reference core/src/test/scala/.../recommendation/SARSpec.scala,
RankingAdapterSpec, RankingEvaluatorSpec, RecommendationIndexerSpec)."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.recommendation import (ALS, SAR, AdvancedRankingMetrics, RankingAdapter, RankingEvaluator,
                                          RankingTrainValidationSplit, RecommendationIndexer)


def _ratings(n_users=30, n_items=20, seed=0):
    rng = np.random.default_rng(seed)
    rows = []
    for u in range(n_users):
        group = u % 2
        items = rng.choice(np.arange(group * 10, group * 10 + 10), size=6, replace=False)
        for i in items:
            rows.append((float(u), float(i), float(rng.integers(3, 6))))
    u, i, r = zip(*rows)
    return DataFrame({"customerID": np.asarray(u), "itemID": np.asarray(i), "rating": np.asarray(r)})


def test_sar_similarity_and_recommendations():
    df = _ratings()
    sar = SAR(userCol="customerID", itemCol="itemID", ratingCol="rating", supportThreshold=1,
              similarityFunction="jaccard")
    m = sar.fit(df)
    recs = m.recommendForAllUsers(5)
    assert recs.count() == 30
    # users of group 0 only get items 0..9 recommended
    for u, r in zip(recs["customerID"].tolist(), recs["recommendations"].tolist()):
        items = [x["itemID"] for x in r]
        assert all((it < 10) == (int(u) % 2 == 0) for it in items)
    item_df = m.getItemDataFrame()
    row0 = dict(zip(item_df["itemID"].tolist(), item_df["itemAffinities"].tolist()))[0.0]
    assert row0[0] == pytest.approx(1.0)  # jaccard(i, i) == 1
    scored = m.transform(df.limit(5))
    assert not np.isnan(scored["prediction"]).any()
    for fn in ("lift", "cooccurrence"):
        SAR(userCol="customerID", itemCol="itemID", ratingCol="rating", similarityFunction=fn,
            supportThreshold=1).fit(df).recommendForAllUsers(3)


def test_sar_time_decay():
    df = DataFrame({"user": [0.0, 0.0, 1.0], "item": [0.0, 1.0, 1.0], "rating": [1.0, 1.0, 1.0],
                    "time": np.array(["2020/01/01T1:00:00", "2020/01/31T1:00:00", "2020/01/31T1:00:00"],
                                     dtype=object)})
    m = SAR(startTime="2020/01/31T1:00:00", startTimeFormat="yyyy/MM/dd'T'h:mm:ss", supportThreshold=1).fit(df)
    aff = np.stack(m.getUserDataFrame()["flatList"].tolist())
    assert aff[0, 0] == pytest.approx(0.5, rel=1e-3)  # 30 days = one half-life
    assert aff[0, 1] == pytest.approx(1.0)


def test_ranking_metrics():
    m = AdvancedRankingMetrics([([1, 2, 3], [1, 3]), ([4, 5], [6])], k=3, n_items=6)
    idcg = 1 + 1 / np.log2(3)
    assert m.ndcg() == pytest.approx(((1 + 1 / np.log2(4)) / idcg + 0) / 2)
    assert m.map() == pytest.approx(((1 + 2 / 3) / 2 + 0) / 2)
    assert m.precision_at_k() == pytest.approx((2 / 3 + 0) / 2)
    assert m.mrr() == pytest.approx(0.5)
    assert m.diversity_at_k() == pytest.approx(5 / 6)


def test_ranking_adapter_and_split_with_als():
    df = _ratings()
    als = ALS(userCol="customerID", itemCol="itemID", ratingCol="rating", rank=4, maxIter=5, regParam=0.1)
    adapter = RankingAdapter(userCol="customerID", itemCol="itemID", ratingCol="rating", k=5).set("recommender", als)
    out = adapter.fit(df).transform(df)
    assert out.count() == 30 and len(out["prediction"][0]) == 5
    ev = RankingEvaluator(k=5)
    assert 0 < ev.evaluate(out) <= 1.0
    assert set(ev.getMetricsMap(out)) >= {"map", "ndcgAt", "mrr"}
    sar = SAR(userCol="customerID", itemCol="itemID", ratingCol="rating", supportThreshold=1)
    tvs = RankingTrainValidationSplit(userCol="customerID", itemCol="itemID", ratingCol="rating",
                                      estimatorParamMaps=[{"similarityFunction": "jaccard"},
                                                          {"similarityFunction": "lift"}]) \
        .set("estimator", sar).set("evaluator", RankingEvaluator(k=3))
    m = tvs.fit(df)
    assert len(m.getValidationMetrics()) == 2
    assert m.recommendForAllUsers(3).count() == 30


def test_recommendation_indexer():
    df = DataFrame({"u": np.array(["a", "b", "a"], dtype=object), "i": np.array(["x", "x", "y"], dtype=object),
                    "r": [1.0, 2.0, 3.0]})
    m = RecommendationIndexer(userInputCol="u", userOutputCol="uid", itemInputCol="i", itemOutputCol="iid",
                              ratingCol="r").fit(df)
    out = m.transform(df)
    assert out["uid"].tolist() == [0.0, 1.0, 0.0] and out["iid"].tolist() == [0.0, 0.0, 1.0]
    assert m.recoverUser(1) == "b" and m.recoverItem(5) == "-1"
