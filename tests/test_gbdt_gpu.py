"""HIP backend vs the CPU oracle (same binned data, same params)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(n=60000, f=12, seed=0, nan_frac=0.0, cat=False):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, f))
    if cat:
        X[:, 0] = rng.integers(0, 12, size=n)
    if nan_frac:
        m = rng.random((n, f)) < nan_frac
        m[:, 0] = False
        X[m] = np.nan
    s = X[:, 0] * (0.2 if cat else 1.0) + np.nan_to_num(X[:, 1]) * np.nan_to_num(X[:, 2]) + 0.5 * np.sin(np.nan_to_num(X[:, 3]))
    if cat:
        s += (X[:, 0] % 3 == 1) * 1.5
    y = (s + 0.5 * rng.standard_normal(n) > 0).astype(np.float32)
    return X, y


def _tree_blocks(model: str):
    return model.split("end of trees")[0].split("Tree=")[1:]


def _field(block: str, key: str):
    lines = [l for l in block.splitlines() if l.startswith(key + "=")]
    return lines[0].split("=", 1)[1] if lines else None


def _assert_same_trees(mc: str, mg: str, rtol=1e-6, atol=1e-8):
    """Every tree of the device model equals the fp64 host oracle's: identical structure (split features,
    bin thresholds, decision types, children, leaf and node row counts) and node / leaf values to the
    precision the int64 fixed-point histograms allow (plus ulp-level differences of device exp/log in the
    gradients of non-quadratic objectives)."""
    tc, tg = _tree_blocks(mc), _tree_blocks(mg)
    assert len(tc) == len(tg)
    for i, (a, b) in enumerate(zip(tc, tg)):
        for k in ("num_leaves", "split_feature", "threshold", "decision_type", "left_child", "right_child",
                  "leaf_count", "internal_count", "num_cat", "cat_boundaries", "cat_threshold"):
            assert _field(a, k) == _field(b, k), (i, k)
        for k in ("leaf_value", "internal_value", "internal_weight", "leaf_weight", "split_gain"):
            va, vb = _field(a, k), _field(b, k)
            if va is None:
                assert vb is None
                continue
            np.testing.assert_allclose(np.array(vb.split(), float), np.array(va.split(), float), rtol=rtol,
                                       atol=atol, err_msg=f"tree {i} {k}")


def _train(X, y, params, iters):
    from synapseml_amd.ops import native

    g = native.gbdt()
    ref = g.DatasetReference.from_sample(X[:50000], len(X), params, [f"f{i}" for i in range(X.shape[1])])
    ds = g.Dataset(ref, len(X))
    ds.push_dense(X, 0)
    ds.set_label(y)
    b = g.Booster(ds, params, None)
    for _ in range(iters):
        b.update()
    return b


@pytest.mark.parametrize("extra", ["", "lambda_l1=0.5 lambda_l2=1.0 min_data_in_leaf=50", "max_depth=4 num_leaves=15"])
def test_gpu_trees_match_cpu(extra):
    from sklearn.metrics import roc_auc_score

    X, y = _data()
    base = f"objective=binary num_leaves=31 learning_rate=0.1 {extra}"
    bc = _train(X, y, base + " device_type=cpu", 5)
    bg = _train(X, y, base + " device_type=gpu", 5)
    assert bg.backend == "hip"
    mc, mg = bc.save_model_string(), bg.save_model_string()
    # every tree identical to the host oracle (structure, counts; values to the histogram precision)
    _assert_same_trees(mc, mg)
    pc = bc.predict(X, 0, 0, -1)[:, 0]
    pg = bg.predict(X, 0, 0, -1)[:, 0]
    assert abs(roc_auc_score(y, pc) - roc_auc_score(y, pg)) < 2e-3
    # training scores kept on the device equal the model's own predictions
    np.testing.assert_allclose(bg.train_scores(), pg, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("f,fpg", [(5, "32"), (17, "32"), (28, "32"), (40, "32"), (70, "32"), (28, "16"), (40, "16")])
def test_gpu_histogram_feature_groups_match_cpu(f, fpg, monkeypatch):
    """The rotated bin-major LDS histogram over every feature-group shape: one partial 16-wide group (5),
    32-wide groups with padding slots (17, 28), a 32-wide group plus a 16-step tail (40), three groups (70),
    and the 16-feature-group kernel (SML_HIST_FPG=16, read at booster construction). The first two trees
    must equal the CPU oracle's split for split."""
    monkeypatch.setenv("SML_HIST_FPG", fpg)
    rng = np.random.default_rng(f)
    X = rng.standard_normal((40000, f))
    w = rng.standard_normal(f) * (rng.random(f) < 0.5)
    y = (X @ w + 0.7 * X[:, f - 1] * X[:, 0] + 0.5 * rng.standard_normal(len(X)) > 0).astype(np.float32)
    base = "objective=binary num_leaves=31 learning_rate=0.1"
    bc = _train(X, y, base + " device_type=cpu", 2)
    bg = _train(X, y, base + " device_type=gpu", 2)
    assert bg.backend == "hip"
    mc, mg = bc.save_model_string(), bg.save_model_string()
    line = lambda s, k: [l for l in s.splitlines() if l.startswith(k + "=")][0]
    for t in range(2):
        tc = mc.split(f"Tree={t}")[1].split(f"Tree={t + 1}")[0]
        tg = mg.split(f"Tree={t}")[1].split(f"Tree={t + 1}")[0]
        assert line(tc, "split_feature") == line(tg, "split_feature")
        assert line(tc, "threshold") == line(tg, "threshold")
        np.testing.assert_allclose(np.array(line(tc, "leaf_value").split("=")[1].split(), float),
                                   np.array(line(tg, "leaf_value").split("=")[1].split(), float), rtol=1e-6, atol=1e-9)


def test_gpu_missing_and_categorical():
    from sklearn.metrics import roc_auc_score

    X, y = _data(nan_frac=0.1, cat=True)
    p = "objective=binary num_leaves=31 categorical_feature=0"
    bc = _train(X, y, p + " device_type=cpu", 8)
    bg = _train(X, y, p + " device_type=gpu", 8)
    assert bg.backend == "hip"
    # NaN (missing-bin default directions) and categorical bitset splits: tree for tree the host's
    _assert_same_trees(bc.save_model_string(), bg.save_model_string())
    pc = bc.predict(X, 1, 0, -1)[:, 0]
    pg = bg.predict(X, 1, 0, -1)[:, 0]
    assert abs(roc_auc_score(y, pc) - roc_auc_score(y, pg)) < 1e-6
    np.testing.assert_allclose(bg.train_scores(), bg.predict(X, 0, 0, -1)[:, 0], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("obj", ["regression", "multiclass num_class=3", "poisson"])
def test_gpu_objectives(obj):
    X, y = _data(n=30000)
    if obj.startswith("multiclass"):
        y = (np.digitize(X[:, 0] + X[:, 1], [-0.5, 0.5])).astype(np.float32)
    elif obj == "poisson":
        y = np.random.default_rng(1).poisson(np.exp(0.3 * X[:, 0])).astype(np.float32)
    else:
        y = (X[:, 0] * 2 + X[:, 1] ** 2).astype(np.float32)
    bc = _train(X, y, f"objective={obj} device_type=cpu", 5)
    bg = _train(X, y, f"objective={obj} device_type=gpu", 5)
    _assert_same_trees(bc.save_model_string(), bg.save_model_string())
    pc = bc.predict(X, 1, 0, -1)
    pg = bg.predict(X, 1, 0, -1)
    np.testing.assert_allclose(pg, pc, rtol=1e-6, atol=1e-9)


def test_gpu_bagging_goss_rf():
    X, y = _data(n=40000)
    for extra in ["bagging_fraction=0.7 bagging_freq=1", "boosting=goss", "boosting=rf bagging_fraction=0.6 bagging_freq=1"]:
        bg = _train(X, y, f"objective=binary device_type=gpu {extra}", 12)
        s = bg.train_scores()
        p = bg.predict(X, 0, 0, -1)[:, 0]
        np.testing.assert_allclose(s, p, rtol=1e-5, atol=1e-5)


def test_gpu_predictor_matches_cpu_predict():
    from synapseml_amd.ops import native

    X, y = _data(n=50000, nan_frac=0.05)
    b = _train(X, y, "objective=binary device_type=gpu", 10)
    gp = native.gbdt().GpuPredictor(b, 0, -1, -1)
    np.testing.assert_allclose(gp.predict(X, False), b.predict(X, 0, 0, -1), rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(gp.predict(X, True), b.predict(X, 1, 0, -1), rtol=1e-10, atol=1e-10)
    np.testing.assert_array_equal(gp.predict_leaf(X), b.predict(X, 2, 0, -1).astype(np.int32))


def test_classifier_api_on_gpu():
    from synapseml_amd.core import DataFrame
    from synapseml_amd.lightgbm import LightGBMClassifier

    X, y = _data(n=30000)
    df = DataFrame({"features": X, "label": y.astype(float)})
    m = LightGBMClassifier(numIterations=10).fit(df)
    assert m.getLightGBMBooster().native.backend == "hip"
    out = m.transform(df)
    assert out["probability"].shape == (30000, 2)


def test_gpu_training_is_deterministic():
    """Single-pass partition writes rows in tile-claim order; the integer
    histograms make the trees bitwise independent of that order."""
    X, y = _data(n=200000, f=10, seed=3)
    p = "objective=binary num_leaves=63 learning_rate=0.1 device_type=gpu"
    m1 = _train(X, y, p, 8).save_model_string()
    m2 = _train(X, y, p, 8).save_model_string()
    assert m1 == m2


def test_gpu_device_stats_populated():
    """Device-side timings (hipEvent pairs) and memory in use are reported
    through Booster.stats()."""
    X, y = _data(n=100000, f=10, seed=5)
    b = _train(X, y, "objective=binary num_leaves=31 device_type=gpu", 6)
    s = b.stats()
    assert s["trees"] == 6
    assert s["device_tree_ms"] > 0.0
    assert s["device_score_ms"] > 0.0
    assert s["device_mem_mb"] > 1.0


def test_p2p_allreduce_two_ranks_one_gpu():
    """K21 one-shot P2P allreduce: two processes share the box's GPU through
    IPC; exact sums, and data-parallel GBDT over it equals the host comm."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29533", os.path.join(root, "tools", "p2p_check.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    import re

    # the two ranks print concurrently: their JSON records can share a line
    lines = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", p.stdout)]
    assert p.returncode == 0 and len(lines) == 2, p.stdout[-2000:] + p.stderr[-3000:]
    for o in lines:
        assert o["p2p_active"], o
        assert o["allreduce_exact"] and o["train_models_equal"] and o["ranks_agree"], o
        assert o["voting_gpu_eq_cpu"] and o["voting_ranks_agree"], o


@pytest.mark.parametrize("kind", ["binary_nan_cat", "multiclass", "rf"])
def test_gpu_treeshap_matches_cpu(kind):
    """K10: wave64 path-packed TreeSHAP vs the host recursion."""
    from synapseml_amd.ops import native

    g = native.gbdt()
    if kind == "binary_nan_cat":
        X, y = _data(n=30000, f=10, seed=11, nan_frac=0.05, cat=True)
        p = "objective=binary num_leaves=31 categorical_feature=0 device_type=gpu"
    elif kind == "multiclass":
        X, _ = _data(n=30000, f=10, seed=12)
        y = (np.digitize(X[:, 0] + X[:, 1], [-0.7, 0.7])).astype(np.float32)
        p = "objective=multiclass num_class=3 num_leaves=31 device_type=gpu"
    else:
        X, y = _data(n=30000, f=10, seed=13)
        p = "objective=binary boosting=rf bagging_fraction=0.7 bagging_freq=1 num_leaves=63 device_type=gpu"
    b = _train(X, y, p, 12)
    Xt = np.ascontiguousarray(X[:3000])
    cpu = b.predict(Xt, 3, 0, -1)
    gp = g.GpuPredictor(b, 0, -1, -1)
    gpu = gp.predict_contrib(b, Xt)
    assert gpu is not None and gpu.shape == cpu.shape
    np.testing.assert_allclose(gpu, cpu, rtol=1e-9, atol=1e-9)
    # local accuracy: contributions sum to the raw score
    raw = b.predict(Xt, 0, 0, -1)
    K = raw.shape[1]
    sums = gpu.reshape(len(Xt), K, -1).sum(-1)
    np.testing.assert_allclose(sums, raw, rtol=1e-8, atol=1e-8)


def _rank_data(seed=21, nq=300, long_queries=True):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(2, 60, size=nq)
    if long_queries:
        sizes[:3] = [300, 700, 257]  # > 256 docs: the global-scratch path of the kernel
    n = int(sizes.sum())
    X = rng.standard_normal((n, 8))
    rel = np.clip(np.round(X[:, 0] + 0.5 * X[:, 1] + 1.5 + 0.4 * rng.standard_normal(n)), 0, 4).astype(np.float32)
    return X, rel, sizes.astype(np.int32)


def _train_rank(X, y, sizes, params, iters):
    from synapseml_amd.ops import native

    g = native.gbdt()
    ref = g.DatasetReference.from_sample(X, len(X), params, [f"f{i}" for i in range(X.shape[1])])
    ds = g.Dataset(ref, len(X))
    ds.push_dense(X, 0)
    ds.set_label(y)
    ds.set_group(sizes)
    b = g.Booster(ds, params, None)
    for _ in range(iters):
        b.update()
    return b


@pytest.mark.parametrize("maxpos", [20, 80])
def test_gpu_lambdarank_gradients_match_host(maxpos):
    """K2 ranking: the wave-per-query lambdarank kernel vs the host pairwise loop (register, LDS and global paths)."""
    X, y, sizes = _rank_data()
    p = f"objective=lambdarank num_leaves=15 min_data_in_leaf=5 eval_at=5 max_position={maxpos}"
    bc = _train_rank(X, y, sizes, p + " device_type=cpu", 1)
    bg = _train_rank(X, y, sizes, p + " device_type=gpu", 1)
    assert bg.backend == "hip"
    gc, hc = bc.gradients()
    gg, hg = bg.gradients()
    np.testing.assert_allclose(gg, gc, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(hg, hc, rtol=1e-5, atol=1e-7)
    # later iterations (non-zero scores, ties broken by index) stay in step
    bc = _train_rank(X, y, sizes, p + " device_type=cpu", 6)
    bg = _train_rank(X, y, sizes, p + " device_type=gpu", 6)
    pc = bc.predict(X, 0, 0, -1)[:, 0]
    pg = bg.predict(X, 0, 0, -1)[:, 0]
    assert np.corrcoef(pc, pg)[0, 1] > 0.999
    np.testing.assert_allclose(bg.train_scores(), pg, rtol=1e-5, atol=1e-5)


def test_gpu_lambdarank_monotone_gain_form_is_bitwise(monkeypatch):
    """With strictly increasing label gains the register kernel takes the pair's orientation from the sign
    of the gain difference (no label compare); it must give bitwise the gradients and trees of the
    label-compare form, through the all-tied first iteration (exact tie-aware ranks) and the later ones
    (strict ranks, checked for ties by the rank -> document scatter)."""
    X, y, sizes = _rank_data(long_queries=False)
    p = "objective=lambdarank num_leaves=15 min_data_in_leaf=5 eval_at=5 max_position=20 device_type=gpu"
    out = {}
    for v in ("0", "1"):
        monkeypatch.setenv("SML_RANK_MONO", v)
        b = _train_rank(X, y, sizes, p, 4)
        out[v] = (b.gradients(), b.save_model_string())
    (g0, h0), m0 = out["0"]
    (g1, h1), m1 = out["1"]
    assert np.array_equal(g0, g1) and np.array_equal(h0, h1)
    assert m0 == m1


def _lambdarank_oracle(score, label, sizes, max_position=20, sigma=1.0, norm=True):
    """numpy LambdaRank gradients (LightGBM's rank_objective: stable-sort ranks with ties by index, pairs of
    different labels with min(rank) < max_position, |delta DCG| scaled by 1 / (0.01 + |ds|) when the query's
    scores differ, log2(1 + sum) / sum normalisation), fp64 throughout"""
    gain = 2.0 ** np.arange(31) - 1.0
    g = np.zeros(len(score))
    h = np.zeros(len(score))
    b = 0
    for c in sizes:
        sc, lb = score[b:b + c], label[b:b + c].astype(int)
        order = np.argsort(-sc, kind="stable")
        rk = np.empty(c, int)
        rk[order] = np.arange(c)
        disc = 1.0 / np.log2(2.0 + rk)
        ideal = np.sort(gain[np.minimum(lb, 30)])[::-1][:max_position]
        mdcg = (ideal / np.log2(2.0 + np.arange(len(ideal)))).sum()
        imd = 1.0 / mdcg if mdcg > 0 else 0.0
        use_norm = norm and sc.max() != sc.min()
        lam = np.zeros(c)
        hes = np.zeros(c)
        suml = 0.0
        for i in range(c):
            for j in range(i + 1, c):
                if lb[i] == lb[j] or min(rk[i], rk[j]) >= max_position:
                    continue
                hi, lo = (i, j) if lb[i] > lb[j] else (j, i)
                ds = sc[hi] - sc[lo]
                dn = (gain[min(lb[hi], 30)] - gain[min(lb[lo], 30)]) * abs(disc[hi] - disc[lo]) * imd
                if use_norm:
                    dn /= 0.01 + abs(ds)
                p = 1.0 / (1.0 + np.exp(sigma * ds))
                pl = -sigma * dn * p
                ph = sigma * sigma * dn * p * (1.0 - p)
                lam[hi] += pl
                lam[lo] -= pl
                hes[hi] += ph
                hes[lo] += ph
                suml -= 2.0 * pl
        nf = np.log2(1.0 + suml) / suml if (norm and suml > 0) else 1.0
        g[b:b + c] = lam * nf
        h[b:b + c] = hes * nf
        b += c
    return g, h


def test_gpu_lambdarank_ties_after_first_iteration():
    """Duplicate documents keep tied scores on every iteration: the strict-rank fast path must detect the
    ties (rank -> document scatter) and fall back to the index-ordered ranks. The kernel's gradients at
    iteration 3 against a numpy LambdaRank oracle evaluated on the same (tied) scores."""
    X, y, sizes = _rank_data(long_queries=False)
    X = X.copy()
    X[1::2] = X[0::2][: len(X[1::2])]  # every odd row duplicates its predecessor's features
    p = "objective=lambdarank num_leaves=15 min_data_in_leaf=5 eval_at=5 max_position=20 device_type=gpu"
    bg = _train_rank(X, y, sizes, p, 2)
    s2 = np.asarray(bg.train_scores(), np.float64).reshape(-1)
    assert len(np.unique(s2)) < len(s2) - len(s2) // 4  # ties survive training
    bg.update()
    gg, hg = bg.gradients()
    go, ho = _lambdarank_oracle(s2, y, sizes)
    scale = np.abs(go).max()
    np.testing.assert_allclose(gg, go, rtol=1e-4, atol=1e-5 * scale)
    np.testing.assert_allclose(hg, ho, rtol=1e-4, atol=1e-5 * np.abs(ho).max())


def test_gpu_lambdarank_transpose_reduce_is_bitwise(monkeypatch):
    """The lambdarank register kernel's transpose-reduced top-document sums (eight documents per round of
    shuffles) use WaveSumF's xor pairing: gradients bitwise equal to one wave sum per top document."""
    X, y, sizes = _rank_data()
    p = "objective=lambdarank num_leaves=15 min_data_in_leaf=5 eval_at=5 max_position=20 device_type=gpu"
    out = {}
    for v in ("0", "1"):
        monkeypatch.setenv("SML_RANK_TREDUCE", v)
        b = _train_rank(X, y, sizes, p, 3)
        out[v] = (b.gradients(), b.save_model_string())
    (g0, h0), m0 = out["0"]
    (g1, h1), m1 = out["1"]
    assert np.array_equal(g0, g1) and np.array_equal(h0, h1)
    assert m0 == m1


def test_gpu_bagging_draws_the_host_bag():
    """K8: device bagging draws the same rows as the host (counter-based RNG), so trees match the CPU oracle."""
    X, y = _data(n=50000)
    for extra in ["bagging_fraction=0.6 bagging_freq=1", "pos_bagging_fraction=0.5 neg_bagging_fraction=0.8 bagging_freq=2"]:
        base = f"objective=binary num_leaves=31 {extra}"
        bc = _train(X, y, base + " device_type=cpu", 3)
        bg = _train(X, y, base + " device_type=gpu", 3)
        mc, mg = bc.save_model_string(), bg.save_model_string()
        for t in ("Tree=0", "Tree=2"):
            tc = mc.split(t)[1].split("Tree=")[0]
            tg = mg.split(t)[1].split("Tree=")[0]
            line = lambda s, k: [l for l in s.splitlines() if l.startswith(k + "=")][0]
            assert line(tc, "split_feature") == line(tg, "split_feature"), (extra, t)
            assert line(tc, "leaf_count") == line(tg, "leaf_count"), (extra, t)


def test_gpu_goss_matches_host():
    """K8: device GOSS (radix top-k threshold + sampled rescaling) vs the host path."""
    from sklearn.metrics import roc_auc_score

    X, y = _data(n=60000)
    p = "objective=binary boosting=goss learning_rate=0.5 num_leaves=31 top_rate=0.2 other_rate=0.1"
    bc = _train(X, y, p + " device_type=cpu", 5)
    bg = _train(X, y, p + " device_type=gpu", 5)
    gc, _ = bc.gradients()
    gg, _ = bg.gradients()
    # same rows rescaled by the same factor (gradients may differ in the last ulp between host and device exp)
    mult = (len(X) - int(len(X) * 0.2)) / int(len(X) * 0.1)
    big_c = np.abs(gc) > 0
    assert abs(np.mean(np.isclose(np.abs(gg), np.abs(gc), rtol=1e-3)) - 1.0) < 0.01
    pc, pg = bc.predict(X, 0, 0, -1)[:, 0], bg.predict(X, 0, 0, -1)[:, 0]
    assert abs(roc_auc_score(y, pc) - roc_auc_score(y, pg)) < 3e-3
    np.testing.assert_allclose(bg.train_scores(), pg, rtol=1e-5, atol=1e-5)
    assert big_c.any() and mult > 1


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_gpu_bin_encode_bit_identical(dtype):
    """K1: device bin encoding == host ValueToBin (NaN / zero-as-missing / categorical / unknown categories)."""
    from synapseml_amd.ops import native

    g = native.gbdt()
    rng = np.random.default_rng(7)
    n = 70000
    X = rng.standard_normal((n, 9))
    X[:, 0] = rng.integers(0, 40, size=n)          # categorical
    X[:, 1] = np.where(rng.random(n) < 0.3, 0.0, X[:, 1])
    X[rng.random((n, 9)) < 0.05] = np.nan
    X[:, 2] = np.round(X[:, 2] * 3)                  # few distinct values
    X[:, 8] = 1.0                                    # trivial feature
    for params in ["categorical_feature=0", "categorical_feature=0 zero_as_missing=true", "use_missing=false"]:
        ref = g.DatasetReference.from_sample(X[:20000], n, params, [f"f{i}" for i in range(9)])
        Xt = X.copy()
        Xt[:100, 0] = 1000  # categories never seen in the sample
        Xt = Xt.astype(dtype)
        a = g.Dataset(ref, n)
        a.push_dense(Xt, 0)
        b = g.Dataset(ref, n)
        b.push_dense_gpu(Xt[:40000], 0)
        b.push_dense_gpu(Xt[40000:], 40000)
        np.testing.assert_array_equal(a.bins, b.bins, err_msg=params)


@pytest.mark.parametrize("extra", ["monotone_constraints=1,-1,0,0,0,0,0,0,0,0,0,0",
                                   "monotone_constraints=1,-1,0,0,0,0,0,0,0,0,0,0 monotone_penalty=1.5"])
def test_gpu_monotone_constraints_match_cpu(extra):
    """Monotone constraints (basic method) in the device split search / choose bookkeeping."""
    X, _ = _data(n=60000)
    y = (1.5 * X[:, 0] - np.sin(3 * X[:, 0]) - X[:, 1] + 0.8 * np.cos(3 * X[:, 1]) + X[:, 2] ** 2).astype(np.float32)
    base = f"objective=regression num_leaves=31 {extra}"
    bc = _train(X, y, base + " device_type=cpu", 4)
    bg = _train(X, y, base + " device_type=gpu", 4)
    mc, mg = bc.save_model_string(), bg.save_model_string()
    line = lambda s, k: [l for l in s.splitlines() if l.startswith(k + "=")][0]
    for t in ("Tree=0", "Tree=3"):
        tc = mc.split(t)[1].split("Tree=")[0]
        tg = mg.split(t)[1].split("Tree=")[0]
        assert line(tc, "split_feature") == line(tg, "split_feature")
        np.testing.assert_allclose(np.array(line(tc, "leaf_value").split("=")[1].split(), float),
                                   np.array(line(tg, "leaf_value").split("=")[1].split(), float), rtol=1e-4, atol=1e-6)
    grid = np.linspace(-2.5, 2.5, 51)
    rows = np.repeat(X[:20], len(grid), axis=0)
    rows[:, 0] = np.tile(grid, 20)
    p = bg.predict(rows, 0, 0, -1)[:, 0].reshape(20, len(grid))
    assert (np.diff(p, axis=1) >= -1e-12).all()


def test_gpu_feature_fraction_bynode_matches_cpu():
    """feature_fraction_bynode: per-node feature subsets drawn from a (seed, tree, node, feature) hash on both backends."""
    X, y = _data(n=50000)
    base = "objective=binary num_leaves=31 feature_fraction_bynode=0.5 feature_fraction=0.8"
    bc = _train(X, y, base + " device_type=cpu", 4)
    bg = _train(X, y, base + " device_type=gpu", 4)
    line = lambda s, k: [l for l in s.splitlines() if l.startswith(k + "=")][0]
    mc, mg = bc.save_model_string(), bg.save_model_string()
    for t in ("Tree=0", "Tree=3"):
        tc = mc.split(t)[1].split("Tree=")[0]
        tg = mg.split(t)[1].split("Tree=")[0]
        assert line(tc, "split_feature") == line(tg, "split_feature")


def test_gpu_training_metrics_on_device():
    """K11: auc / binary_logloss / binary_error / rmse of the device-resident training scores vs the host
    formulas (sorted trapezoid AUC with ties, clipped logloss)."""
    from sklearn.metrics import roc_auc_score

    X, y = _data(n=80000)
    X[:, 0] = np.round(X[:, 0], 1)  # coarse feature -> many tied scores
    b = _train(X, y, "objective=binary metric=auc,binary_logloss,binary_error device_type=gpu", 6)
    ev = dict(b.eval(0))
    s = b.train_scores()
    p = 1 / (1 + np.exp(-s))
    assert abs(ev["auc"] - roc_auc_score(y, s)) < 1e-9
    pc = np.clip(p, 1e-15, 1 - 1e-15)
    np.testing.assert_allclose(ev["binary_logloss"], -np.mean(y * np.log(pc) + (1 - y) * np.log(1 - pc)), rtol=1e-9)
    np.testing.assert_allclose(ev["binary_error"], np.mean((p > 0.5) != (y > 0)), rtol=1e-12)
    yr = (X[:, 0] * 2 + X[:, 1] ** 2).astype(np.float32)
    r = _train(X, yr, "objective=regression metric=rmse,l1 device_type=gpu", 4)
    er = dict(r.eval(0))
    sr = r.train_scores()
    np.testing.assert_allclose(er["rmse"], np.sqrt(np.mean((sr - yr) ** 2)), rtol=1e-9)
    np.testing.assert_allclose(er["l1"], np.mean(np.abs(sr - yr)), rtol=1e-9)


def test_gpu_histogram_quantisation_skewed_hessians():
    """Near-separable binary data driven to confident predictions: most rows end with hessians many orders
    of magnitude below the largest one. The HIP histogram accumulates (g, h) in 64-bit fixed point (per-row
    quantum <= count * max / 2^61, at least the precision of the reference's fp64 accumulation of fp32
    gradients): every tree must have the fp64 host oracle's structure, with node hessian sums and leaf
    values equal to ~1e-9."""
    rng = np.random.default_rng(17)
    n, f = 120000, 8
    X = rng.standard_normal((n, f))
    y = (X[:, 0] + 0.3 * X[:, 1] + 0.02 * rng.standard_normal(n) > 0).astype(np.float32)
    base = "objective=binary num_leaves=15 learning_rate=0.5 min_sum_hessian_in_leaf=1e-3"
    iters = 60  # by then ~45% of the rows have h < 1e-6 against max h ~0.25
    bc = _train(X, y, base + " device_type=cpu", iters)
    bg = _train(X, y, base + " device_type=gpu", iters)
    assert bg.backend == "hip"
    # the gradients of the last iteration really are skewed (h spans many decades)
    gc, hc = bc.gradients()
    hc = np.asarray(hc, dtype=np.float64)
    assert hc.max() / max(np.median(hc), 1e-300) > 1e4
    mc, mg = bc.save_model_string(), bg.save_model_string()
    blocks = lambda s: s.split("end of trees")[0].split("Tree=")[1:]
    tc, tg = blocks(mc), blocks(mg)
    assert len(tc) == len(tg) == iters
    field = lambda t, k: np.array([l for l in t.splitlines() if l.startswith(k + "=")][0].split("=")[1].split(), float)
    same_structure = 0
    for a, b in zip(tc, tg):
        if "split_feature" not in a or "split_feature" not in b:
            continue
        if np.array_equal(field(a, "split_feature"), field(b, "split_feature")) and \
                np.array_equal(field(a, "threshold"), field(b, "threshold")):
            same_structure += 1
            # per-node hessian sums and leaf values agree to the (64-bit) quantisation error
            np.testing.assert_allclose(field(a, "internal_weight"), field(b, "internal_weight"), rtol=1e-9, atol=1e-12)
            np.testing.assert_allclose(field(a, "leaf_value"), field(b, "leaf_value"), rtol=1e-7, atol=1e-12)
    assert same_structure == iters, same_structure
    pc = bc.predict(X, 0, 0, -1)[:, 0]
    pg = bg.predict(X, 0, 0, -1)[:, 0]
    ll = lambda p: float(-np.mean(y * np.log(np.clip(p, 1e-15, 1)) + (1 - y) * np.log(np.clip(1 - p, 1e-15, 1))))
    assert abs(ll(pc) - ll(pg)) <= 0.02 * ll(pc) + 1e-6, (ll(pc), ll(pg))


@pytest.mark.parametrize("obj", ["binary", "binary scale_pos_weight=3", "cross_entropy"])
def test_gpu_fused_score_grad_root_pass(obj, monkeypatch):
    """score_grad_hist_kernel (score update + next gradients + next root
    histogram in one pass, a-priori fixed-point scale) against the unfused
    launches (SML_PREP=0): same trees, scores equal the model's predictions and
    the gradients left on the device match the objective at those scores."""
    X, y = _data(n=80000, seed=11)
    w = np.random.default_rng(2).uniform(0.5, 2.0, len(X)).astype(np.float32)
    p = f"objective={obj} num_leaves=31 learning_rate=0.2 device_type=gpu"

    def fit(prep):
        monkeypatch.setenv("SML_PREP", prep)
        from synapseml_amd.ops import native

        g = native.gbdt()
        ref = g.DatasetReference.from_sample(X[:50000], len(X), p, [f"f{i}" for i in range(X.shape[1])])
        ds = g.Dataset(ref, len(X))
        ds.push_dense(X, 0)
        ds.set_label(y)
        ds.set_weight(w)
        b = g.Booster(ds, p, None)
        for _ in range(6):
            b.update()
        return b

    bf, bu = fit("1"), fit("0")
    line = lambda s, k: [l for l in s.splitlines() if l.startswith(k + "=")]
    mf, mu = bf.save_model_string(), bu.save_model_string()
    assert line(mf, "split_feature")[:3] == line(mu, "split_feature")[:3]
    s = bf.train_scores()
    np.testing.assert_allclose(s, bf.predict(X, 0, 0, -1)[:, 0], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(s, bu.train_scores(), rtol=1e-3, atol=1e-3)
    g, h = bf.gradients()
    z = 1.0 / (1.0 + np.exp(-s))
    if obj == "cross_entropy":
        ge, he = (z - y) * w, z * (1 - z) * w
    else:
        lw = np.where(y > 0, 3.0 if "scale_pos" in obj else 1.0, 1.0)
        ge, he = (z - y) * lw * w, z * (1 - z) * lw * w
    np.testing.assert_allclose(g, ge, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(h, he, rtol=1e-4, atol=1e-6)


def _with_valid(X, y, Xv, yv, params, iters, sizes=None, vsizes=None, wv=None):
    from synapseml_amd.ops import native

    g = native.gbdt()
    ref = g.DatasetReference.from_sample(X[:50000], len(X), params, [f"f{i}" for i in range(X.shape[1])])
    ds = g.Dataset(ref, len(X))
    ds.push_dense(X, 0)
    ds.set_label(y)
    dv = g.Dataset(ref, len(Xv))
    dv.push_dense(Xv, 0)
    dv.set_label(yv)
    if wv is not None:
        dv.set_weight(wv)
    if sizes is not None:
        ds.set_group(sizes)
        dv.set_group(vsizes)
    b = g.Booster(ds, params, None)
    b.add_valid(dv, "valid_0")
    for _ in range(iters):
        b.update()
    return b


def _assert_device_metrics_match_host(b, idx):
    dev, host = dict(b.eval(idx)), dict(b.eval(idx, device=False))
    assert dev.keys() == host.keys() and dev
    for k in dev:
        np.testing.assert_allclose(dev[k], host[k], rtol=1e-9, atol=1e-12, err_msg=k)
    return dev


@pytest.mark.parametrize("boosting", ["gbdt", "rf bagging_fraction=0.7 bagging_freq=1", "dart drop_rate=0.3"])
def test_gpu_validation_set_on_device_binary(boosting):
    """K11: the validation set's scores live in HBM - every tree is folded in by the device traversal
    (gbdt add, rf running mean, dart renormalisation) - and auc / logloss / error reduce there; both
    equal the host paths (model predict, host metric formulas) on weighted data with NaNs and ties."""
    X, y = _data(n=60000, nan_frac=0.05)
    Xv, yv = _data(n=20000, seed=5, nan_frac=0.05)
    Xv[:, 0] = np.round(Xv[:, 0], 1)
    wv = np.random.default_rng(3).uniform(0.5, 2.0, size=len(yv)).astype(np.float32)
    p = f"objective=binary num_leaves=31 metric=auc,binary_logloss,binary_error boosting={boosting} device_type=gpu"
    b = _with_valid(X, y, Xv, yv, p, 8, wv=wv)
    assert b.backend == "hip" and b.valid_on_device(0)
    np.testing.assert_allclose(b.valid_scores(0), b.predict(Xv, 0, 0, -1)[:, 0], rtol=1e-9, atol=1e-10)
    _assert_device_metrics_match_host(b, 1)


def test_gpu_validation_set_on_device_multiclass_categorical():
    X, _ = _data(n=40000, cat=True)
    y = (np.nan_to_num(X[:, 1]) > 0.3).astype(np.float32) + (X[:, 0] % 4 == 1)
    Xv, _ = _data(n=15000, seed=9, cat=True)
    yv = (np.nan_to_num(Xv[:, 1]) > 0.3).astype(np.float32) + (Xv[:, 0] % 4 == 1)
    p = "objective=multiclass num_class=3 num_leaves=15 categorical_feature=0 metric=multi_logloss,multi_error device_type=gpu"
    b = _with_valid(X, y.astype(np.float32), Xv, yv.astype(np.float32), p, 6)
    assert b.valid_on_device(0)
    raw = b.predict(Xv, 0, 0, -1)  # n x K
    np.testing.assert_allclose(b.valid_scores(0), raw.T.reshape(-1), rtol=1e-9, atol=1e-10)
    _assert_device_metrics_match_host(b, 1)


def test_gpu_ranking_metrics_on_device():
    """ndcg@k / map@k (one wave per query, top-k by repeated wave arg-max in the host's stable order)
    on the training set and a validation set, vs the host loops at 1e-9; queries up to 700 documents."""
    X, y, sizes = _rank_data()
    Xv, yv, vsizes = _rank_data(seed=33, nq=200)
    p = "objective=lambdarank num_leaves=15 min_data_in_leaf=5 metric=ndcg,map eval_at=1,3,5,10 device_type=gpu"
    b = _with_valid(X, y, Xv, yv, p, 5, sizes=sizes, vsizes=vsizes)
    assert b.valid_on_device(0)
    dev = _assert_device_metrics_match_host(b, 1)
    assert {"ndcg@1", "ndcg@10", "map@3"} <= dev.keys()
    _assert_device_metrics_match_host(b, 0)
    np.testing.assert_allclose(b.valid_scores(0), b.predict(Xv, 0, 0, -1)[:, 0], rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("extra", ["num_leaves=31", "num_leaves=255 min_data_in_leaf=5", "num_leaves=63 max_depth=5",
                                   "num_leaves=127 min_data_in_leaf=5",
                                   "num_leaves=31 categorical_feature=0 monotone_constraints=0,1,-1",
                                   "num_leaves=2", "num_leaves=31 min_gain_to_split=5.0",
                                   "num_leaves=31 objective=multiclass num_class=3"])
@pytest.mark.parametrize("spec", ["1", "3", "16"])
def test_gpu_batched_growth_equals_sequential(extra, spec, monkeypatch):
    """Batched speculative growth (bplan_kernel ..; SML_GBDT_SPEC=k expansions per round) builds exactly the
    trees of the one-split-at-a-time growth (SML_GBDT_SPEC=0): byte-identical model text, for small / deep /
    depth-capped / categorical + monotone / stump-like / gain-limited / multiclass trees (31 / 63 / 127 / 255
    leaves: the plan kernel's one, two and four frontier slots per lane)."""
    X, y = _data(n=80000, nan_frac=0.02, cat="categorical" in extra)
    if "multiclass" in extra:
        y = (np.digitize(np.nan_to_num(X[:, 0] + X[:, 1]), [-0.5, 0.5])).astype(np.float32)
    p = ("objective=binary " if "objective" not in extra else "") + f"learning_rate=0.2 {extra} device_type=gpu"

    def fit(k):
        monkeypatch.setenv("SML_GBDT_SPEC", k)
        return _train(X, y, p, 6).save_model_string()

    seq, bat = fit("0"), fit(spec)
    assert bat == seq


@pytest.mark.parametrize("extra", ["num_leaves=31", "num_leaves=255 min_data_in_leaf=5",
                                   "num_leaves=31 categorical_feature=0 monotone_constraints=0,1,-1",
                                   "num_leaves=31 objective=multiclass num_class=3"])
@pytest.mark.parametrize("wide,spec_max", [("16", "8"), ("1", "15"), ("4", "6")])
def test_gpu_adaptive_round_width_equals_sequential(extra, wide, spec_max, monkeypatch):
    """Adaptive round width (SML_GBDT_WIDE=d: a round whose expansions hold <= 1/d of the rows keeps
    speculating up to SML_GBDT_SPEC_MAX expansions; d = 1 widens every round): byte-identical models to
    one-split growth, through the plan's slow absorb path (more than 15 children) and the fast one."""
    X, y = _data(n=80000, nan_frac=0.02, cat="categorical" in extra)
    if "multiclass" in extra:
        y = (np.digitize(np.nan_to_num(X[:, 0] + X[:, 1]), [-0.5, 0.5])).astype(np.float32)
    p = ("objective=binary " if "objective" not in extra else "") + f"learning_rate=0.2 {extra} device_type=gpu"
    monkeypatch.setenv("SML_GBDT_SPEC", "0")
    seq = _train(X, y, p, 6).save_model_string()
    monkeypatch.setenv("SML_GBDT_SPEC", "4")
    monkeypatch.setenv("SML_GBDT_WIDE", wide)
    monkeypatch.setenv("SML_GBDT_SPEC_MAX", spec_max)
    assert _train(X, y, p, 6).save_model_string() == seq


@pytest.mark.parametrize("extra", ["num_leaves=31", "num_leaves=255 min_data_in_leaf=5",
                                   "num_leaves=31 categorical_feature=0 monotone_constraints=0,1,-1",
                                   "num_leaves=31 objective=cross_entropy", "num_leaves=31 objective=regression"])
def test_gpu_index_only_partition_equals_ordered_gradients(extra, monkeypatch):
    """SML_GBDT_IDX=1 (the default): the batched partition moves row ids only and bhist gathers (g, h) from the
    interleaved copy the fused score / gradient pass writes (or packed once per tree for objectives without the
    fused pass) - byte-identical models to the ordered-gradient partition (SML_GBDT_IDX=0) and to one-split
    growth; the host still reads the current gradients (unpacked on demand)."""
    X, y = _data(n=80000, nan_frac=0.02, cat="categorical" in extra)
    if "regression" in extra:
        y = (X[:, 0] + np.nan_to_num(X[:, 1]) * 0.5).astype(np.float32)
    p = ("objective=binary " if "objective" not in extra else "") + f"learning_rate=0.2 {extra} device_type=gpu"

    def fit(idx, spec="4"):
        monkeypatch.setenv("SML_GBDT_IDX", idx)
        monkeypatch.setenv("SML_GBDT_SPEC", spec)
        return _train(X, y, p, 6)

    b1, b0 = fit("1"), fit("0")
    assert b1.save_model_string() == b0.save_model_string() == fit("0", "0").save_model_string()
    (g1, h1), (g0, h0) = b1.gradients(), b0.gradients()
    np.testing.assert_array_equal(g1, g0)
    np.testing.assert_array_equal(h1, h0)


def test_gpu_single_pass_scoring_float32_rows():
    """K9 batch scoring: float32 rows are scored as they are (no float64 copy) in one chunked upload +
    traversal pass; raw and probability come from that single pass and equal the host predictor."""
    X, y = _data(n=70000, nan_frac=0.03)
    b = _train(X, y, "objective=binary num_leaves=31 device_type=gpu", 20)
    from synapseml_amd.lightgbm.booster import LightGBMBooster

    lb = LightGBMBooster(native_booster=b)
    X32 = X.astype(np.float32)
    host = b.predict(X32.astype(np.float64), 0, 0, -1)
    gp = lb._gpu("gpu")
    np.testing.assert_allclose(gp.predict_raw(X32), host, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(gp.predict_raw(X32.astype(np.float64)), host, rtol=1e-12, atol=1e-12)
    raw, prob = lb.score_both(X32, classification=True)
    np.testing.assert_allclose(raw[:, 1], host[:, 0], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(prob[:, 1], b.predict(X32.astype(np.float64), 1, 0, -1)[:, 0], rtol=1e-12, atol=1e-12)


def test_num_tasks_fit_fans_out_on_gpu():
    """LightGBMClassifier(numTasks=2).fit(df) on the device runs 2 partition tasks itself (LightGBMBase.scala:
    449-456, 608-628). On a one-GPU box the tasks share the device (gloo control plane, shared-device
    histogram allreduce); the model is byte-identical to the one-task model on the same data and bins."""
    from synapseml_amd.core import DataFrame
    from synapseml_amd.lightgbm import LightGBMClassifier

    X, y = _data(n=40000, f=10)
    df = DataFrame({"features": X, "label": y}, num_partitions=2)
    one = LightGBMClassifier(deviceType="gpu", numIterations=5, numTasks=1)
    m1 = one.fit(df)
    ref = one._last_reference
    est = LightGBMClassifier(deviceType="gpu", numIterations=5, numTasks=2, referenceDataset=ref)
    m2 = est.fit(df)
    assert len(est.getTaskMeasures()) == 2
    # int64 histograms under a global scale: the 2-task model is bitwise the 1-task model
    assert m2.getNativeModel().split("parameters:")[0] == m1.getNativeModel().split("parameters:")[0]


def test_gpu_small_hessian_leaves_match_fp64():
    """The device histograms' fixed-point scale on confident binary predictions: leaf values equal
    the fp64 sums over the routed rows (tests/test_lightgbm.py::_small_hessian_leaf_check)."""
    from tests.test_lightgbm import _small_hessian_leaf_check

    _small_hessian_leaf_check("gpu")


@pytest.mark.parametrize("extra", ["num_leaves=31", "num_leaves=255 min_data_in_leaf=5", "num_leaves=2",
                                   "num_leaves=31 objective=cross_entropy",
                                   "num_leaves=31 categorical_feature=0 monotone_constraints=0,1,-1",
                                   "num_leaves=31 bagging_fraction=0.7 bagging_freq=1",
                                   "num_leaves=31 objective=multiclass num_class=3", "num_leaves=63 objective=regression"])
def test_gpu_row_leaf_scatter_equals_tree_walk(extra, monkeypatch):
    """After batched growth the fused score pass reads every row's leaf from the final leaves' row segments
    (leaf_scatter_kernel) instead of walking the tree per row: bitwise the same scores, gradients and models
    (SML_GBDT_ROW_LEAF=0 walks); bagged trees keep the walk (out-of-bag rows are not partitioned)."""
    X, y = _data(n=80000, nan_frac=0.02, cat="categorical" in extra)
    p = ("objective=binary " if "objective" not in extra else "") + f"learning_rate=0.2 {extra} device_type=gpu"

    def fit(v):
        monkeypatch.setenv("SML_GBDT_ROW_LEAF", v)
        return _train(X, y, p, 8)

    a, b = fit("1"), fit("0")
    assert a.save_model_string() == b.save_model_string()
    np.testing.assert_array_equal(a.train_scores(), b.train_scores())
    (ga, ha), (gb, hb) = a.gradients(), b.gradients()
    np.testing.assert_array_equal(ga, gb)
    np.testing.assert_array_equal(ha, hb)


def test_gpu_row_leaf_map_ranker_equals_tree_walk(monkeypatch):
    """The plain score kernel (objectives without the fused pass: lambdarank here) reads the row -> leaf map
    too: bitwise the walk's scores and models."""
    X, y, sizes = _rank_data()
    p = "objective=lambdarank num_leaves=31 min_data_in_leaf=5 eval_at=5 device_type=gpu"
    out = {}
    for v in ("1", "0"):
        monkeypatch.setenv("SML_GBDT_ROW_LEAF", v)
        b = _train_rank(X, y, sizes, p, 5)
        out[v] = (b.save_model_string(), np.asarray(b.train_scores()))
    assert out["1"][0] == out["0"][0]
    np.testing.assert_array_equal(out["1"][1], out["0"][1])
