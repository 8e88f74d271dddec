"""Data balance measures (model: reference core/src/test/scala/.../exploratory/*Suite.scala)."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.exploratory import AggregateBalanceMeasure, DistributionBalanceMeasure, FeatureBalanceMeasure


def _df():
    g = np.array(["M", "M", "M", "F"] * 10, dtype=object)
    lab = np.array([1, 0, 1, 1] * 10)
    return DataFrame({"gender": g, "label": lab})


def test_aggregate_measures():
    r = AggregateBalanceMeasure(sensitiveCols=["gender"]).transform(_df())["AggregateBalanceMeasure"][0]
    p = np.array([0.75, 0.25])
    norm = p / p.mean()
    assert r["theil_l_index"] == pytest.approx(-np.log(norm).mean())
    assert r["theil_t_index"] == pytest.approx((norm * np.log(norm)).mean())
    assert r["atkinson_index"] == pytest.approx(1 - np.exp(np.log(norm).sum()) ** 0.5)
    uniform = DataFrame({"gender": np.array(["M", "F"] * 5, dtype=object)})
    assert AggregateBalanceMeasure(sensitiveCols=["gender"]).transform(uniform)["AggregateBalanceMeasure"][0][
        "theil_t_index"] == pytest.approx(0.0)


def test_distribution_measures():
    out = DistributionBalanceMeasure(sensitiveCols=["gender"]).transform(_df())
    r = out["DistributionBalanceMeasure"][0]
    obs = np.array([0.75, 0.25])
    assert r["total_variation_dist"] == pytest.approx(0.25)
    assert r["inf_norm_dist"] == pytest.approx(0.25)
    assert r["kl_divergence"] == pytest.approx((obs * np.log(obs / 0.5)).sum())
    assert r["chi_sq_stat"] == pytest.approx(((30 - 20) ** 2 + (10 - 20) ** 2) / 20)
    assert 0 <= r["chi_sq_p_value"] <= 1
    custom = DistributionBalanceMeasure(sensitiveCols=["gender"], referenceDistribution=[{"M": 0.75, "F": 0.25}])
    assert custom.transform(_df())["DistributionBalanceMeasure"][0]["kl_divergence"] == pytest.approx(0.0)


def test_feature_balance_measures():
    out = FeatureBalanceMeasure(sensitiveCols=["gender"], labelCol="label").transform(_df())
    assert out.count() == 1 and out["ClassA"][0] == "M" and out["ClassB"][0] == "F"
    r = out["FeatureBalanceMeasure"][0]
    # P(y=1 | M) = 20/30, P(y=1 | F) = 1
    assert r["dp"] == pytest.approx(2 / 3 - 1.0)
