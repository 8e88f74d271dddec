"""Cyber package (reference tests: core/src/test/python/synapsemltest/cyber/**:
test_collaborative_filtering.py, test_complement_access.py, test_indexers.py,
test_scalers.py)."""
import numpy as np

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.cyber import (AccessAnomaly, ComplementAccessTransformer, ConnectedComponents, DataFactory,
                                 IdIndexer, LinearScalarScaler, MultiIndexer, StandardScalarScaler)


def _obj(v):
    a = np.empty(len(v), dtype=object)
    for i, x in enumerate(v):
        a[i] = x
    return a


def test_id_indexer_partitioned_and_undo():
    df = DataFrame({"tenant": _obj(["t1", "t1", "t2", "t2", "t1"]), "user": _obj(["b", "a", "a", "c", "b"])})
    m = IdIndexer("user", "tenant", "uid", reset_per_partition=True).fit(df)
    out = m.transform(df)
    assert out["uid"].tolist() == [2, 1, 1, 2, 2] and "user" not in out
    assert m.undo_transform(out)["user"].tolist() == ["b", "a", "a", "c", "b"]
    g = IdIndexer("user", "tenant", "uid", reset_per_partition=False).fit(df).transform(df)
    assert g["uid"].tolist() == [2, 1, 3, 4, 2]
    unseen = m.transform(DataFrame({"tenant": _obj(["t1"]), "user": _obj(["zzz"])}))
    assert unseen["uid"].tolist() == [0]
    mm = MultiIndexer([IdIndexer("user", "tenant", "uid", True)]).fit(df)
    assert mm.get_model_by_input_col("user") is not None and mm.get_model_by_output_col("uid") is not None


def test_scalers_per_partition():
    df = DataFrame({"t": _obj(["a"] * 3 + ["b"] * 3), "x": np.asarray([1.0, 2.0, 3.0, 10.0, 10.0, 10.0])})
    s = StandardScalarScaler("x", "t", "z", coefficient_factor=2.0).fit(df).transform(df)
    np.testing.assert_allclose(s["z"][:3], 2.0 * (np.array([1, 2, 3]) - 2) / np.std([1, 2, 3]))
    np.testing.assert_allclose(s["z"][3:], 0.0)
    lin = LinearScalarScaler("x", "t", "y", 5.0, 10.0).fit(df).transform(df)
    np.testing.assert_allclose(lin["y"], [5.0, 7.5, 10.0, 7.5, 7.5, 7.5])


def test_complement_access_excludes_seen():
    df = DataFrame({"t": _obj([0] * 4), "u": np.asarray([1, 1, 2, 3]), "r": np.asarray([1, 2, 2, 3])})
    comp = ComplementAccessTransformer("t", ["u", "r"], 10).transform(df)
    seen = {(1, 1), (1, 2), (2, 2), (3, 3)}
    pairs = set(zip(comp["u"].tolist(), comp["r"].tolist()))
    assert pairs and not (pairs & seen)
    assert all(1 <= u <= 3 and 1 <= r <= 3 for u, r in pairs)


def test_connected_components():
    df = DataFrame({"t": _obj([0, 0, 0]), "u": _obj(["a", "b", "c"]), "r": _obj(["x", "x", "y"])})
    users, res = ConnectedComponents("t", "u", "r").components(df)
    assert users[(0, "a")] == users[(0, "b")] != users[(0, "c")]
    assert res[(0, "y")] == users[(0, "c")]


def test_access_anomaly_separates_departments():
    f = DataFactory(num_hr_users=6, num_hr_resources=20, num_fin_users=5, num_fin_resources=18, num_eng_users=8,
                    num_eng_resources=30)
    train = f.create_clustered_training_data(0.3)
    train = train.withColumn("tenant", np.zeros(train.count(), dtype=np.int64))
    model = AccessAnomaly(rankParam=6, maxIter=15, seed=0).fit(train)
    scored = model.transform(train)["anomaly_score"]
    assert abs(np.mean(scored)) < 1e-6 and abs(np.std(scored) - 1.0) < 1e-6  # normalised on training data
    intra = f.create_clustered_intra_test_data(train)
    inter = f.create_clustered_inter_test_data()
    si = model.transform(intra.withColumn("tenant", np.zeros(intra.count(), dtype=np.int64)))["anomaly_score"]
    so = model.transform(inter.withColumn("tenant", np.zeros(inter.count(), dtype=np.int64)))["anomaly_score"]
    assert np.nanmean(so) > np.nanmean(si) + 0.5


def test_access_anomaly_explicit_mode_and_components():
    f = DataFactory(num_hr_users=4, num_hr_resources=10, num_fin_users=4, num_fin_resources=10, num_eng_users=4,
                    num_eng_resources=10, single_component=False)
    train = f.create_clustered_training_data(0.5)
    m = AccessAnomaly(tenantCol="tenant", rankParam=4, maxIter=8, applyImplicitCf=False, complementsetFactor=2,
                      seed=1).fit(train)
    inter = f.create_clustered_inter_test_data()
    s = m.transform(inter)["anomaly_score"]
    assert np.isinf(s).all()  # departments are disconnected components
