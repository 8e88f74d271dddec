"""Vowpal Wabbit-compatible learner tests (model: reference
vw/src/test/scala/.../VerifyVowpalWabbit*.scala and SURVEY §8.2)."""
import json

import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.core.linalg import SparseVector
from synapseml_amd.vw import (ContextualBanditMetrics, CressieRead, CressieReadInterval, Ips, KahanSum, Snips,
                              VectorZipper, VowpalWabbitClassifier, VowpalWabbitContextualBandit,
                              VowpalWabbitCSETransformer, VowpalWabbitDSJsonTransformer, VowpalWabbitFeaturizer,
                              VowpalWabbitGeneric, VowpalWabbitGenericProgressive, VowpalWabbitInteractions,
                              VowpalWabbitMurmurWithPrefix, VowpalWabbitRegressor, murmur_hash)
from synapseml_amd.ops import native


def _u(x):
    return x & 0xFFFFFFFF


# ------------------------------------------------------------------ hashing
def test_murmur_golden_values():
    ns = _u(murmur_hash("features", 0))
    assert ns == 2493003127
    assert _u(murmur_hash("marie", ns)) == 0xECACEC8A
    assert _u(murmur_hash("markus", ns)) == 0x07388F83
    assert _u(murmur_hash("fun", ns)) == 0xA23CC374
    assert _u(murmur_hash("in", ns)) == 0x30AC2EF4
    assert _u(murmur_hash("inmarkus", ns)) == 0x02233B72
    # standard MurmurHash3_x86_32 vectors
    assert _u(murmur_hash("", 0)) == 0
    assert _u(murmur_hash("", 1)) == 0x514E28B7
    assert _u(murmur_hash("test", 0)) == 0xBA6BD213
    assert _u(murmur_hash("Hello, world!", 0)) == 0xC0363E43
    assert _u(murmur_hash("The quick brown fox jumps over the lazy dog", 0)) == 0x2E4FF723


def test_murmur_with_prefix_matches_concat():
    m = VowpalWabbitMurmurWithPrefix("prefix")
    for s in ["", "a", "héllo", "x" * 100]:
        assert m.hash(s, 17) == murmur_hash("prefix" + s, 17)
    vw = native.load("_vw")
    batch = vw.murmur_batch(["a", "bb", "ccc"], 5, "pre")
    assert [int(b) for b in batch] == [_u(murmur_hash("pre" + s, 5)) for s in ["a", "bb", "ccc"]]


def test_murmur_static_hash_str_and_bytes():
    from synapseml_amd.vw import VowpalWabbitMurmur

    for s in ["", "features", "héllo"]:
        assert VowpalWabbitMurmur.hash(s, 0) == murmur_hash(s, 0)
        assert VowpalWabbitMurmur.hash(s.encode("utf-8"), 0) == murmur_hash(s, 0)
    assert _u(VowpalWabbitMurmur.hash(b"test", 0)) == 0xBA6BD213
    assert VowpalWabbitMurmur.hash("Hello, world!", 0) < 0  # signed like the JVM int (0xC0363E43)


# ------------------------------------------------------------------ featurizer
def test_featurizer_strings_numeric_and_collisions():
    df = DataFrame({"in": ["markus", "marie"], "num": [2.0, 0.0], "flag": [True, False]})
    out = VowpalWabbitFeaturizer(inputCols=["in", "num", "flag"], numBits=18).transform(df)
    ns = _u(murmur_hash("features", 0))
    mask = (1 << 18) - 1
    v0 = out["features"][0]
    assert isinstance(v0, SparseVector) and v0.size == 1 << 18
    exp = {(_u(murmur_hash("inmarkus", ns)) & mask): 1.0, (_u(murmur_hash("num", ns)) & mask): 2.0,
           (_u(murmur_hash("flag", ns)) & mask): 1.0}
    assert dict(zip(v0.indices.tolist(), v0.values.tolist())) == exp
    v1 = out["features"][1]  # zero numeric + false bool dropped
    assert len(v1.indices) == 1 and v1.indices[0] == (_u(murmur_hash("inmarie", ns)) & mask)
    assert 211826 in v0.indices.tolist()


def test_featurizer_string_split_and_no_prefix():
    df = DataFrame({"text": ["marie markus marie"]})
    out = VowpalWabbitFeaturizer(stringSplitInputCols=["text"], prefixStringsWithColumnName=False,
                                 numBits=18).transform(df)
    v = out["features"][0]
    m = dict(zip(v.indices.tolist(), v.values.tolist()))
    assert m[60554] == 2.0 and m[36739] == 1.0
    # collisions removed instead of summed
    out2 = VowpalWabbitFeaturizer(stringSplitInputCols=["text"], prefixStringsWithColumnName=False, numBits=18,
                                  sumCollisions=False).transform(df)
    m2 = dict(zip(out2["features"][0].indices.tolist(), out2["features"][0].values.tolist()))
    assert m2[60554] == 1.0


def test_featurizer_preserve_order_bits():
    df = DataFrame({"a": ["x"], "b": ["y"]})
    out = VowpalWabbitFeaturizer(inputCols=["a", "b"], numBits=10, preserveOrderNumBits=2).transform(df)
    v = out["features"][0]
    assert v.size == 1 << 30
    assert sorted((v.indices >> 28).tolist()) == [0, 1]
    with pytest.raises(ValueError):
        VowpalWabbitFeaturizer(inputCols=["a"], numBits=29, preserveOrderNumBits=2).transform(df)


def test_interactions():
    df = DataFrame({"a": np.empty(1, object), "b": np.empty(1, object)})
    df = df.withColumn("a", np.array([SparseVector(8, [1, 2], [1.0, 2.0])], dtype=object))
    df = df.withColumn("b", np.array([SparseVector(8, [3], [5.0])], dtype=object))
    out = VowpalWabbitInteractions(inputCols=["a", "b"], outputCol="ab", numBits=10).transform(df)
    v = out["ab"][0]
    fnv = 16777619
    exp = {((1 * fnv) ^ 3) & 1023: 5.0, ((2 * fnv) ^ 3) & 1023: 10.0}
    assert dict(zip(v.indices.tolist(), v.values.tolist())) == exp


# ------------------------------------------------------------------ learners
def _binary_df(n=4000, d=10, seed=0, parts=1):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    w = rng.normal(size=d)
    y = (X @ w + 0.3 * rng.normal(size=n) > 0).astype(np.float64)
    return DataFrame({"features": X, "label": y}, num_partitions=parts), X, y


def _auc(y, s):
    from sklearn.metrics import roc_auc_score

    return roc_auc_score(y, s)


def test_classifier_binary_learns():
    df, X, y = _binary_df()
    m = VowpalWabbitClassifier(labelConversion=True, passThroughArgs="--loss_function logistic").fit(df)
    out = m.transform(df)
    assert _auc(y, out["probability"][:, 1]) > 0.95
    acc = (out["prediction"] == y).mean()
    assert acc > 0.85
    stats = m.getPerformanceStatistics()
    assert stats["numberOfExamplesPerPass"][0] == len(y)


def test_classifier_logistic_link_equivalent():
    df, X, y = _binary_df(n=1000)
    a = VowpalWabbitClassifier(labelConversion=True, passThroughArgs="--loss_function logistic").fit(df)
    b = VowpalWabbitClassifier(labelConversion=True,
                               passThroughArgs="--loss_function logistic --link logistic").fit(df)
    pa = a.transform(df)["probability"][:, 1]
    pb = b.transform(df)["probability"][:, 1]
    np.testing.assert_allclose(pa, pb, rtol=1e-4, atol=1e-5)


def test_regressor_and_adaptive_rmse():
    rng = np.random.default_rng(1)
    X = rng.normal(size=(5000, 6))
    y = X @ np.array([1.0, -2.0, 0.5, 0.0, 3.0, 1.5]) + 0.1 * rng.normal(size=5000)
    df = DataFrame({"features": X, "label": y})
    for args in ["", "--adaptive"]:
        m = VowpalWabbitRegressor(passThroughArgs=args, numPasses=3).fit(df)
        p = m.transform(df)["prediction"]
        rmse = np.sqrt(np.mean((p - y) ** 2))
        assert rmse < 0.15, (args, rmse)


def test_multiclass_oaa_probabilities():
    rng = np.random.default_rng(2)
    n, k = 3000, 4
    centers = rng.normal(scale=3, size=(k, 5))
    lab = rng.integers(1, k + 1, size=n)
    X = centers[lab - 1] + rng.normal(size=(n, 5))
    df = DataFrame({"features": X, "label": lab.astype(np.float64)})
    m = VowpalWabbitClassifier(numClasses=k, passThroughArgs=f"--oaa {k} --probabilities --loss_function logistic",
                               numPasses=2).fit(df)
    out = m.transform(df)
    probs = out["probability"]
    assert probs.shape == (n, k)
    np.testing.assert_allclose(probs.sum(1), 1.0, atol=1e-4)
    assert (np.argmax(probs, 1) + 1 == lab).mean() > 0.8


def test_additional_features_and_interactions_param():
    rng = np.random.default_rng(3)
    a = rng.normal(size=(2000, 3))
    b = rng.normal(size=(2000, 3))
    y = (a[:, 0] * b[:, 1] > 0).astype(np.float64)  # needs the cross term
    df = DataFrame({"a": a, "b": b, "label": y})
    lin = VowpalWabbitClassifier(featuresCol="a", additionalFeatures=["b"], labelConversion=True,
                                 passThroughArgs="--loss_function logistic", numPasses=3).fit(df)
    quad = VowpalWabbitClassifier(featuresCol="a", additionalFeatures=["b"], labelConversion=True,
                                  passThroughArgs="--loss_function logistic", interactions=["ab"],
                                  numPasses=3).fit(df)
    auc_lin = _auc(y, lin.transform(df)["probability"][:, 1])
    auc_quad = _auc(y, quad.transform(df)["probability"][:, 1])
    assert auc_quad > 0.9 > auc_lin


def test_save_load_and_readable_model(tmp_path):
    from synapseml_amd.core.pipeline import PipelineStage

    df, X, y = _binary_df(n=500)
    m = VowpalWabbitClassifier(labelConversion=True, passThroughArgs="--loss_function logistic").fit(df)
    p = tmp_path / "vwm"
    m.save(str(p))
    m2 = PipelineStage.load(str(p))
    np.testing.assert_allclose(m.transform(df)["probability"], m2.transform(df)["probability"])
    txt = m.getReadableModel()
    assert "bits" in txt.lower() or ":" in txt
    m.saveNativeModel(str(tmp_path / "native.model"))
    assert (tmp_path / "native.model").stat().st_size > 0


def test_initial_model_continues():
    df, X, y = _binary_df(n=2000)
    a = VowpalWabbitClassifier(labelConversion=True, passThroughArgs="--loss_function logistic").fit(df)
    b = VowpalWabbitClassifier(labelConversion=True, passThroughArgs="--loss_function logistic",
                               initialModel=a.getModel()).fit(df)
    assert b.getPerformanceStatistics()["numberOfExamplesPerPass"][0] == 2000
    assert not np.allclose(a.transform(df)["rawPrediction"], b.transform(df)["rawPrediction"])


def test_split_col_training():
    df, X, y = _binary_df(n=2000, parts=2)
    df = df.withColumn("split", np.arange(2000) % 3)
    m = VowpalWabbitClassifier(labelConversion=True, passThroughArgs="--loss_function logistic",
                               splitCol="split").fit(df)
    assert _auc(y, m.transform(df)["probability"][:, 1]) > 0.9


def test_empty_partition_ok():
    df, X, y = _binary_df(n=300)
    empty = df.filter(np.zeros(300, bool))
    m = VowpalWabbitClassifier(labelConversion=True).fit(df)
    assert m.transform(empty).count() == 0


# ------------------------------------------------------------------ generic text format
def test_generic_text_format():
    rng = np.random.default_rng(4)
    lines = []
    ys = []
    for _ in range(2000):
        a, b = rng.normal(size=2)
        yv = 1 if a - b > 0 else -1
        ys.append(yv)
        lines.append(f"{yv} |f a:{a:.4f} b:{b:.4f}")
    df = DataFrame({"value": np.array(lines, dtype=object)})
    m = VowpalWabbitGeneric(passThroughArgs="--loss_function logistic --link logistic", numPasses=2).fit(df)
    p = m.transform(df)["prediction"]
    assert _auc(np.array(ys) > 0, p) > 0.97
    prog = VowpalWabbitGenericProgressive(passThroughArgs="--loss_function logistic").transform(df)
    assert prog["prediction"].shape == (2000,)


def test_generic_csoaa_text():
    lines = ["1:0.0 2:1.0 3:1.0 | a", "1:1.0 2:0.0 3:1.0 | b", "1:1.0 2:1.0 3:0.0 | c"] * 200
    df = DataFrame({"value": np.array(lines, dtype=object)})
    m = VowpalWabbitGeneric(passThroughArgs="--csoaa 3").fit(df)
    p = m.transform(DataFrame({"value": np.array(["| a", "| b", "| c"], dtype=object)}))["prediction"]
    assert p.tolist() == [1.0, 2.0, 3.0]


def test_unsupported_reduction_raises():
    with pytest.raises(Exception):
        native.load("_vw").VW("--cats 4")


# ------------------------------------------------------------------ contextual bandit
def _cb_df(n=3000, seed=5):
    rng = np.random.default_rng(seed)
    shared, actions, chosen, cost, prob = [], [], [], [], []
    for _ in range(n):
        s = rng.normal(size=3)
        acts = [np.eye(3)[j] for j in range(3)]
        best = int(np.argmax(s))
        c = int(rng.integers(0, 3))
        shared.append(s)
        actions.append(acts)
        chosen.append(c + 1)
        cost.append(-1.0 if c == best else 0.0)
        prob.append(1 / 3)
    sh = np.stack(shared)
    acol = np.empty(n, dtype=object)
    for i, a in enumerate(actions):
        acol[i] = a
    return DataFrame({"shared": sh, "features": acol, "chosenAction": np.array(chosen), "label": np.array(cost),
                      "probability": np.array(prob)}), sh


def test_contextual_bandit_learns_policy():
    df, sh = _cb_df()
    cb = VowpalWabbitContextualBandit(epsilon=0.1, passThroughArgs="--cb_explore_adf -q sf", numPasses=2)
    m = cb.fit(df)
    out = m.transform(df)
    pred = np.array([np.argmax(p) for p in out["prediction"]])
    assert (pred == np.argmax(sh, 1)).mean() > 0.7
    np.testing.assert_allclose([sum(p) for p in out["prediction"][:20]], 1.0, atol=1e-5)
    with pytest.raises(NotImplementedError):
        VowpalWabbitContextualBandit(passThroughArgs="--cb 3").fit(df)


def test_cb_parallel_fit():
    df, _ = _cb_df(n=500)
    cb = VowpalWabbitContextualBandit(passThroughArgs="--cb_explore_adf")
    models = cb.fit(df, [{cb.epsilon: 0.1}, {cb.epsilon: 0.3}])
    assert len(models) == 2


def test_cb_metrics():
    m = ContextualBanditMetrics()
    m.addExample(0.5, 1.0, 1.0)
    m.addExample(0.5, 0.0, 0.0)
    assert m.getIpsEstimate() == pytest.approx(1.0)
    assert m.getSnipsEstimate() == pytest.approx(1.0)


# ------------------------------------------------------------------ policy eval
def test_kahan_sum():
    k = KahanSum()
    for _ in range(10):
        k = k + 0.1
    assert k.toDouble() == pytest.approx(1.0, abs=1e-15)
    assert (KahanSum(1.0) + KahanSum(2.0)).toDouble() == 3.0


def test_policy_estimators():
    df = DataFrame({"probLog": [0.5, 0.25, 0.5], "reward": [1.0, 0.0, 1.0], "probPred": [1.0, 0.5, 0.0]})
    assert Ips().evaluate(df) == pytest.approx((2 * 1 + 2 * 0 + 0) / 3)
    assert Snips().evaluate(df) == pytest.approx(2.0 / 4.0)
    cr = CressieRead().evaluate(df, wMin=0, wMax=100)
    assert np.isfinite(cr)
    iv = CressieReadInterval(True).evaluate(df, wMin=0, wMax=100)
    assert iv.lower <= iv.upper


def test_dsjson_and_cse():
    rng = np.random.default_rng(6)
    lines = []
    for i in range(200):
        idx = int(rng.integers(0, 2))
        lines.append(json.dumps({"EventId": f"e{i}", "_label_cost": float(-(idx == 0)), "_label_probability": 0.5,
                                 "_labelIndex": idx, "a": [1, 2], "c": {"x": 1}, "other": float(i % 2)}))
    df = DataFrame({"value": np.array(lines, dtype=object)})
    t = VowpalWabbitDSJsonTransformer(rewards={"reward": "_label_cost", "r2": "other"}).transform(df)
    assert t["EventId"][0] == "e0" and t["probLog"][0] == pytest.approx(0.5)
    assert set(t["rewards"][0].keys()) == {"reward", "r2"}
    preds = np.empty(200, dtype=object)
    for i in range(200):
        preds[i] = [(0, 0.9), (1, 0.1)]
    t = t.withColumn("predictions", preds)
    cse = VowpalWabbitCSETransformer().transform(t)
    assert cse["exampleCount"][0] == 200
    r = cse["reward"][0]
    assert r["minReward"] == -1.0 and r["maxReward"] == 0.0
    # policy always picks action 0 (cost -1): ips ~ -1
    assert r["ips"] == pytest.approx(-1.0, abs=0.25)
    assert r["snips"] == pytest.approx(-1.0)
    strat = VowpalWabbitCSETransformer(metricsStratificationCols=["chosenActionIndex"]).transform(t)
    assert strat.count() == 2


def test_vector_zipper():
    df = DataFrame({"a": [1, 2], "b": [3, 4]})
    out = VectorZipper(inputCols=["a", "b"], outputCol="z").transform(df)
    assert [list(x) for x in out["z"]] == [[1, 3], [2, 4]]


# ------------------------------------------------------------------ distributed (gloo, 2 ranks)
def _vw_rank_fn(part, rank, world):
    from synapseml_amd.vw import VowpalWabbitClassifier as C

    m = C(labelConversion=True, passThroughArgs="--loss_function logistic", numPasses=2,
          numSyncsPerPass=1).fit(part)
    return m.getModel()


def test_distributed_allreduce_gloo():
    from synapseml_amd.parallel.runtime import run_partitions

    df, X, y = _binary_df(n=2000, parts=2)
    models = run_partitions(_vw_rank_fn, df, num_workers=2)
    assert len(models) == 2
    # after the final end-of-pass allreduce the weight tables are identical
    vw = native.load("_vw")
    w0 = np.asarray(vw.VW("--testonly", models[0]).weights())
    w1 = np.asarray(vw.VW("--testonly", models[1]).weights())
    np.testing.assert_allclose(w0, w1, rtol=1e-6, atol=1e-7)


def test_gpu_path_quadratic_expansion_matches_native_hashing():
    """The host expansion the GPU learner uses for -q (learners._interaction_block) produces the
    native core's interaction features: index (a * FNV) ^ b (32-bit), value a.x * b.x, j >= i within
    one namespace."""
    from synapseml_amd.vw.learners import _interaction_block

    rng = np.random.default_rng(0)
    n = 50

    def block(g):
        lens = rng.integers(0, 5, size=n)
        ip = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        return (g, ip, rng.integers(0, 2 ** 32, size=ip[-1], dtype=np.uint64).astype(np.uint32),
                rng.standard_normal(ip[-1]).astype(np.float32))

    A, B = block("a"), block("b")
    for pair, same in (("ab", False), ("aa", True)):
        _, ip, idx, val = _interaction_block([A, B], pair, n)
        for r in range(n):
            fa = list(zip(A[2][A[1][r]:A[1][r + 1]], A[3][A[1][r]:A[1][r + 1]]))
            fb = fa if same else list(zip(B[2][B[1][r]:B[1][r + 1]], B[3][B[1][r]:B[1][r + 1]]))
            exp = []
            for i, (ha, xa) in enumerate(fa):
                for j, (hb, xb) in enumerate(fb):
                    if same and j < i:
                        continue
                    exp.append((((int(ha) * 16777619) & 0xFFFFFFFF) ^ int(hb), np.float32(xa * xb)))
            got = list(zip(idx[ip[r]:ip[r + 1]].tolist(), val[ip[r]:ip[r + 1]].tolist()))
            assert [e[0] for e in exp] == [g[0] for g in got]
            np.testing.assert_allclose([e[1] for e in exp], [g[1] for g in got], rtol=1e-6)


def test_hash_strings_packed_matches_murmur():
    """Packed-UTF-8 batched murmur (one native call per column) == per-string murmur3 (SURVEY §8.2 goldens)."""
    import numpy as np

    from synapseml_amd.vw.featurizer import hash_strings, murmur_hash

    rng = np.random.default_rng(0)
    xs = ["", "a", "fun", "inmarkus", "héllo wörld ✓"] + ["".join(chr(97 + int(c)) for c in rng.integers(0, 26, n))
                                                        for n in rng.integers(0, 40, 500)]
    for seed in (0, 2493003127):
        got = hash_strings(xs, seed, device="cpu")
        assert got.tolist() == [murmur_hash(x, seed) & 0xFFFFFFFF for x in xs]
    assert hash_strings(["marie", "markus"], 2493003127, (1 << 18) - 1, device="cpu").tolist() == [60554, 36739]
    assert hash_strings([], 1, device="cpu").tolist() == []


def _cats_df():
    return DataFrame({"value": np.array(["ca 185.121:0.657567:6.20426e-05 | a b",
                                         "ca 772.592:0.458316:6.20426e-05 | b c",
                                         "ca 15140.6:0.31791:6.20426e-05 | d"], dtype=object)})


def test_generic_cats_pdf_matches_reference():
    """Mirror of VerifyVowpalWabbitGeneric.scala:107-132 ('Verify VowpalWabbitGeneric using CATS'): the pdf
    segments of the first example after training on three CATS-labelled examples."""
    from synapseml_amd.vw import VowpalWabbitGeneric

    m = VowpalWabbitGeneric(passThroughArgs="--cats_pdf 3 --bandwidth 5000 --min_value 0 --max_value 20000").fit(
        _cats_df())
    seg = m.transform(_cats_df().slice(0, 1))["segments"][0]
    got = [(s["left"], s["right"], s["pdfValue"]) for s in seg]
    want = [(0.0, 8333.333, 1.165e-4), (8333.333, 20000.0, 2.5e-6)]
    assert len(got) == len(want)
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-3)
    # the density integrates to one
    assert abs(sum((r - l) * v for l, r, v in got) - 1.0) < 1e-4


def test_generic_cats_action_pdf_value():
    from synapseml_amd.vw import VowpalWabbitGeneric

    m = VowpalWabbitGeneric(passThroughArgs="--cats 3 --bandwidth 5000 --min_value 0 --max_value 20000").fit(
        _cats_df())
    out = m.transform(_cats_df())
    a, p = out["action"], out["pdf"]
    assert ((a >= 0) & (a <= 20000)).all()
    assert np.all(p > 0)


def test_cats_learns_the_cheap_region():
    """Costs low near 15000 and high elsewhere: the learned policy's window moves there."""
    from synapseml_amd.vw import VowpalWabbitGeneric

    rng = np.random.default_rng(0)
    lines = []
    for _ in range(3000):
        a = rng.uniform(0, 20000)
        cost = 0.0 if 12000 < a < 18000 else 1.0
        lines.append(f"ca {a:.2f}:{cost}:{1 / 20000:.8f} | x")
    df = DataFrame({"value": np.array(lines, dtype=object)})
    m = VowpalWabbitGeneric(passThroughArgs="--cats_pdf 4 --bandwidth 2500 --min_value 0 --max_value 20000").fit(df)
    seg = m.transform(df.slice(0, 1))["segments"][0]
    best = max(seg, key=lambda s: s["pdfValue"])
    assert 12000 <= (best["left"] + best["right"]) / 2 <= 18000, seg


@pytest.mark.parametrize("args", ["--nn 10", "--boosting 3", "--cb_explore 4", "--bogus_flag", "--cats 1 --bandwidth 1 "
                                  "--min_value 0 --max_value 1", "--cats_pdf 3 --min_value 0 --max_value 10"])
def test_unknown_or_unsupported_options_are_rejected(args):
    """options the engine does not implement must raise, never train a different model."""
    from synapseml_amd.vw import VowpalWabbitGeneric

    df = DataFrame({"value": np.array(["1 | a b"], dtype=object)})
    with pytest.raises(RuntimeError):
        VowpalWabbitGeneric(passThroughArgs=args).fit(df)


def test_generic_prediction_schemas():
    """Prediction columns follow the learner's prediction type (VowpalWabbitSchema.scala)."""
    from synapseml_amd.vw import VowpalWabbitGeneric

    reg = DataFrame({"value": np.array(["1 | a:1 b:2", "0 | a:2 c:1"], dtype=object)})
    out = VowpalWabbitGeneric().fit(reg).transform(reg)
    assert "prediction" in out and "confidence" in out
    mc = DataFrame({"value": np.array(["1 | a", "2 | b", "3 | c"], dtype=object)})
    out = VowpalWabbitGeneric(passThroughArgs="--oaa 3").fit(mc).transform(mc)
    assert out["prediction"].dtype == np.int64


def test_set_initial_model_from_fitted_model():
    """VowpalWabbitPythonBase.setInitialModel takes a fitted model (reference VowpalWabbitPythonBase.py:22-26):
    warm-starting from it continues where it stopped (lower loss than a cold start on the same pass)."""
    import numpy as np

    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.vw import VowpalWabbitRegressor

    rng = np.random.default_rng(0)
    X = rng.normal(size=(3000, 5))
    y = X @ np.array([1.0, -2.0, 0.5, 0.0, 3.0])
    df = DataFrame({"features": X, "label": y})
    first = VowpalWabbitRegressor().fit(df)
    warm = VowpalWabbitRegressor().setInitialModel(first).fit(df)
    cold = VowpalWabbitRegressor().fit(df)
    err = lambda m: float(np.mean((m.transform(df)["prediction"] - y) ** 2))  # noqa: E731
    assert err(warm) < err(cold)
    assert VowpalWabbitRegressor().setInitialModel(first.getModel()).getInitialModel() == bytes(first.getModel())


def _touched(args, blocks):
    """weight-table slots an example's features touch in the native learner (one squared-loss update)"""
    from synapseml_amd.ops import native

    vw = native.load("_vw").VW(args + " --noconstant -b 24")
    vw.learn_batch(blocks, np.ones(1, np.float32), None, None, None, True)
    lines = vw.readable_model().split("Checksum: 0\n:0\n", 1)[1].strip().splitlines()
    return {int(l.split(":")[0]) for l in lines if l}


def _one_row(feats):
    return [(g, np.array([0, len(ix)], np.int64), np.array(ix, np.uint32), np.array(xs, np.float32))
            for g, ix, xs in feats]


def test_wildcard_and_cubic_interactions_vw_semantics():
    """`-q ::` expands to the combinations with repetition of the namespaces present (aa ab ac bb bc cc, each
    unordered pair once, first namespace = the smaller), `-q a:` to a crossed with every namespace, and
    `--cubic :::` / `--cubic aab` keep non-decreasing feature positions inside repeated namespaces (VW without
    --leave_duplicate_interactions). Hash (a * FNV) ^ b [* FNV ^ c], masked to the table."""
    P, M = 16777619, (1 << 24) - 1
    A, B, C = [1, 2], [10], [100, 101]
    blocks = _one_row([("c", C, [2.0, 1.0]), ("a", A, [1.0, 0.5]), ("b", B, [1.0])])  # unsorted on purpose
    base = set(A + B + C)

    def q(x, y, same):
        return {((i * P) ^ j) & M for k, i in enumerate(x) for l, j in enumerate(y) if not same or l >= k}

    def cub(x, y, z, s12, s23):
        out = set()
        for i1, a in enumerate(x):
            for i2, b in enumerate(y):
                if s12 and i2 < i1:
                    continue
                for i3, c in enumerate(z):
                    if s23 and i3 < i2:
                        continue
                    out.add(((((a * P) ^ b) * P) ^ c) & M)
        return out

    exp_qq = base | q(A, A, 1) | q(A, B, 0) | q(A, C, 0) | q(B, B, 1) | q(B, C, 0) | q(C, C, 1)
    assert _touched("-q ::", blocks) == {x & M for x in exp_qq}
    exp_qa = base | q(A, A, 1) | q(A, B, 0) | q(A, C, 0)
    assert _touched("-q a:", blocks) == {x & M for x in exp_qa}
    ns = {"a": A, "b": B, "c": C}
    exp_c = set(base)
    for t in ("aaa", "aab", "aac", "abb", "abc", "acc", "bbb", "bbc", "bcc", "ccc"):
        exp_c |= cub(ns[t[0]], ns[t[1]], ns[t[2]], t[0] == t[1], t[1] == t[2])
    assert _touched("--cubic :::", blocks) == {x & M for x in exp_c}
    assert _touched("--cubic aab", blocks) == {x & M for x in base | cub(A, A, B, True, False)}
    # an explicit pair is NOT canonicalised: -q ba hashes b first
    assert _touched("-q ba", blocks) == {x & M for x in base | q(B, A, 0)}


def test_fit_fans_out_over_executor_tasks(monkeypatch):
    """VowpalWabbitClassifier.fit runs min(executor tasks, partitions) tasks itself
    (VowpalWabbitBase.scala:124-137, VowpalWabbitBaseLearner.scala:180-211) and keeps the first partition's
    model - the model every rank holds after the end-of-pass average."""
    from synapseml_amd.parallel.runtime import run_partitions
    from synapseml_amd.vw import VowpalWabbitClassifier as C

    df, X, y = _binary_df(n=2000, parts=2)
    explicit = run_partitions(_vw_rank_fn, df, num_workers=2)[0]
    monkeypatch.setenv("SML_EXECUTOR_TASKS", "2")
    m = C(labelConversion=True, passThroughArgs="--loss_function logistic", numPasses=2, numSyncsPerPass=1).fit(df)
    vw = native.load("_vw")
    np.testing.assert_allclose(np.asarray(vw.VW("--testonly", m.getModel()).weights()),
                               np.asarray(vw.VW("--testonly", explicit).weights()), rtol=1e-6, atol=1e-7)
    assert m.transform(df)["prediction"].shape[0] == 2000


def test_stager_rejects_null_source():
    """The pinned host->HBM stager refuses a null source before any copy thread runs (the round-4 segfault)."""
    assert native.load("_vw")._stager_rejects_null()


def test_model_cache_is_keyed_on_the_model_object():
    """Replacing the model bytes always rebuilds the cached scorer, even if the new object reuses the old id."""
    from synapseml_amd.vw import VowpalWabbitRegressor

    rng = np.random.default_rng(0)
    X = rng.standard_normal((200, 4))
    df = DataFrame({"features": X, "label": X[:, 0] * 2.0})
    m = VowpalWabbitRegressor().fit(df)
    p1 = m.transform(df)["prediction"]
    m2 = VowpalWabbitRegressor(passThroughArgs="-l 0.01").fit(df)
    m.set("model", bytes(m2.getModel()))
    p2 = m.transform(df)["prediction"]
    np.testing.assert_allclose(p2, m2.transform(df)["prediction"])
    assert not np.allclose(p1, p2)


@pytest.mark.parametrize("loss,label", [("hinge", 1.0), ("quantile", 3.0)])
def test_invariant_update_does_not_overshoot(loss, label):
    """Importance-invariant updates for hinge / quantile (VW's getUpdate): one example with a huge importance
    weight moves the prediction up to the margin / the label, never past it (the plain gradient step of
    earlier builds overshot by orders of magnitude)."""
    from synapseml_amd.vw import VowpalWabbitRegressor

    X = np.array([[1.0, 0.5, -0.25]])
    df = DataFrame({"features": X, "label": np.array([label]), "w": np.array([1e4])})
    m = VowpalWabbitRegressor(passThroughArgs=f"--loss_function {loss}", weightCol="w").fit(df)
    p = float(m.transform(df)["prediction"][0])
    bound = 1.0 if loss == "hinge" else label
    assert 0.0 < p <= bound * (1 + 1e-4), p
