"""GPU hogwild VW learner (csrc/vw/vw_gpu.hip) vs the exact CPU learner."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.ops import native
from synapseml_amd.vw import VowpalWabbitClassifier, VowpalWabbitRegressor
from synapseml_amd.vw.learners import _merged_csr, namespace_blocks


def _binary(n=20000, d=20, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d))
    w = rng.normal(size=d)
    y = (X @ w + 0.3 * rng.normal(size=n) > 0).astype(np.float64)
    return DataFrame({"features": X, "label": y}), y


def test_merged_csr_matches_blocks():
    df = DataFrame({"a": np.array([[1.0, 0.0], [0.0, 2.0]]), "b": np.array([[3.0], [0.0]])})
    blocks = namespace_blocks(df, ["a", "b"], 0)
    ip, idx, val = _merged_csr(blocks, 2, True)
    assert ip.tolist() == [0, 3, 5]
    assert val.tolist() == [1.0, 3.0, 1.0, 2.0, 1.0]
    assert idx[2] == 11650396 and idx[4] == 11650396


@pytest.mark.parametrize("args", ["--cats 4 --bandwidth 1 --min_value 0 --max_value 1",
                                  "--cats_pdf 4 --bandwidth 1 --min_value 0 --max_value 1"])
def test_gpu_rejects_reductions_it_does_not_run(args):
    """Reductions a vector-column estimator cannot feed on the device (CATS labels are VW text: the device
    CATS learner runs through VowpalWabbitGeneric) are refused by name before any GPU work, never silently run
    on the host."""
    df, _ = _binary(n=50)
    with pytest.raises(ValueError, match="deviceType='gpu' does not run"):
        VowpalWabbitRegressor(deviceType="gpu", passThroughArgs=args).fit(df)


def test_gpu_request_without_gpu_fails_loudly():
    if native.load("_vw").gpu_available():
        pytest.skip("GPU present")
    df, _ = _binary(n=100)
    with pytest.raises(RuntimeError):
        VowpalWabbitClassifier(deviceType="gpu", labelConversion=True).fit(df)


@pytest.mark.gpu
def test_gpu_classifier_matches_cpu_quality():
    """Hogwild quality on DENSE features: every example of a batch updates the same 21 weights, the worst case
    for stale reads. At 256 examples in flight the progressive loss varied 0.42-0.74 run to run with rare
    divergent runs (loss 3.0, AUC 0.87-0.98; r5 pass 18 probe, both staging paths); 64 in flight is the batch
    this checks. Hashed sparse data (the bench) barely collides."""
    from sklearn.metrics import roc_auc_score

    df, y = _binary()
    args = "--loss_function logistic"
    gpu = VowpalWabbitClassifier(deviceType="gpu", labelConversion=True, passThroughArgs=args, numPasses=3,
                                 gpuBatchSize=64).fit(df)
    cpu = VowpalWabbitClassifier(labelConversion=True, passThroughArgs=args, numPasses=3).fit(df)
    ag = roc_auc_score(y, gpu.transform(df)["probability"][:, 1])
    ac = roc_auc_score(y, cpu.transform(df)["probability"][:, 1])
    assert ag > 0.97 and ag > ac - 0.01, (ag, ac)
    assert gpu.getPerformanceStatistics()["numberOfExamplesPerPass"][0] > 0


@pytest.mark.gpu
def test_gpu_regressor_rmse():
    rng = np.random.default_rng(1)
    X = rng.normal(size=(20000, 6))
    y = X @ np.array([1.0, -2.0, 0.5, 0.0, 3.0, 1.5]) + 0.1 * rng.normal(size=20000)
    df = DataFrame({"features": X, "label": y})
    m = VowpalWabbitRegressor(deviceType="gpu", numPasses=5, gpuBatchSize=256).fit(df)
    p = m.transform(df)["prediction"]
    assert np.sqrt(np.mean((p - y) ** 2)) < 0.3


@pytest.mark.gpu
def test_gpu_quadratic_interactions_syncs_and_initial_model():
    """-q on the GPU learner (host-expanded with the native hashing), numSyncsPerPass chunking and
    initialModel warm start; predictions go through the native model, which applies -q itself."""
    rng = np.random.default_rng(3)
    n = 20000
    A = rng.normal(size=(n, 3))
    B = rng.normal(size=(n, 3))
    y = A[:, 0] * B[:, 1] - 0.5 * A[:, 2] * B[:, 0] + 0.05 * rng.normal(size=n)  # pure cross terms
    df = DataFrame({"a": A, "b": B, "label": y})
    kw = dict(featuresCol="a", additionalFeatures=["b"], numPasses=4, gpuBatchSize=256)
    lin = VowpalWabbitRegressor(deviceType="gpu", **kw).fit(df)
    quad = VowpalWabbitRegressor(deviceType="gpu", passThroughArgs="-q ab", numSyncsPerPass=3, **kw).fit(df)
    rmse = lambda m: float(np.sqrt(np.mean((m.transform(df)["prediction"] - y) ** 2)))
    assert rmse(quad) < 0.5 * rmse(lin), (rmse(quad), rmse(lin))
    # warm start from the trained model: a single extra pass keeps the quality
    warm = VowpalWabbitRegressor(deviceType="gpu", passThroughArgs="-q ab", initialModel=quad.getModel(),
                                 **dict(kw, numPasses=1)).fit(df)
    assert rmse(warm) < 1.2 * rmse(quad) + 0.05


@pytest.mark.gpu
def test_murmur_batch_kernel_matches_host():
    """K13: the HIP batched murmur kernel equals the host hash on random UTF-8 strings."""
    import numpy as np

    from synapseml_amd.vw.featurizer import hash_strings

    rng = np.random.default_rng(1)
    xs = ["", "ü", "inmarkus"] + ["".join(chr(int(c)) for c in rng.integers(32, 0x2FF, n))
                                  for n in rng.integers(0, 70, 300_000)]
    for seed, mask in ((0, 0xFFFFFFFF), (2493003127, (1 << 18) - 1)):
        np.testing.assert_array_equal(hash_strings(xs, seed, mask, device="gpu"),
                                      hash_strings(xs, seed, mask, device="cpu"))


@pytest.mark.gpu
@pytest.mark.parametrize("args", ["", "--sgd", "--adaptive", "--normalized --invariant", "--loss_function logistic -l 0.3",
                                  "--loss_function quantile --quantile_tau 0.3", "--loss_function hinge",
                                  "--l1 0.0005 --l2 0.0001"])
def test_gpu_batch1_is_the_sequential_learner(args):
    """gpuBatchSize=1 runs VW's update rule example by example: on mixed-scale features (where the
    normalized update matters) the exported GPU model predicts like the exact host learner's."""
    rng = np.random.default_rng(5)
    n = 3000
    X = rng.normal(size=(n, 6)) * np.array([1e-2, 1.0, 30.0, 1.0, 5.0, 0.3])
    y = X @ np.array([20.0, -1.0, 0.05, 0.7, 0.2, 2.0]) + 0.05 * rng.normal(size=n)
    if "logistic" in args or "hinge" in args:
        y = np.where(y > 0, 1.0, -1.0)
    df = DataFrame({"features": X, "label": y})
    kw = dict(passThroughArgs=args, numPasses=1)
    g = VowpalWabbitRegressor(deviceType="gpu", gpuBatchSize=1, **kw).fit(df)
    c = VowpalWabbitRegressor(**kw).fit(df)
    pg, pc = g.transform(df)["prediction"], c.transform(df)["prediction"]
    np.testing.assert_allclose(pg, pc, rtol=1e-4, atol=1e-4 * np.abs(pc).max())


@pytest.mark.gpu
def test_gpu_oaa_multiclass():
    """--oaa K on the device (one wave per class per example): accuracy close to the host learner's."""
    rng = np.random.default_rng(7)
    n, d, K = 20000, 10, 4
    X = rng.normal(size=(n, d))
    W = rng.normal(size=(d, K))
    y = (np.argmax(X @ W, 1) + 1).astype(np.float64)
    df = DataFrame({"features": X, "label": y})
    kw = dict(passThroughArgs=f"--oaa {K}", numClasses=K, numPasses=3)
    g = VowpalWabbitClassifier(deviceType="gpu", gpuBatchSize=64, **kw).fit(df)
    c = VowpalWabbitClassifier(**kw).fit(df)
    acc = lambda m: float(np.mean(m.transform(df)["prediction"] == y))
    ag, ac = acc(g), acc(c)
    assert ag > 0.8 and ag > ac - 0.03, (ag, ac)


def _three_ns(n=3000, seed=11):
    rng = np.random.default_rng(seed)
    A = rng.normal(size=(n, 3))
    B = rng.normal(size=(n, 2)) * np.array([1.0, 4.0])
    C = rng.normal(size=(n, 2)) * 0.5
    y = A[:, 0] * B[:, 1] - 0.5 * A[:, 2] * C[:, 0] + 0.3 * B[:, 0] * C[:, 1] * A[:, 1] + 0.05 * rng.normal(size=n)
    return DataFrame({"a": A, "b": B, "c": C, "label": y})


def _host_scored(model, df):
    m = model.copy()
    m.set("deviceType", "cpu")
    return m.transform(df)["prediction"]


@pytest.mark.gpu
@pytest.mark.parametrize("args", ["-q ab", "-q ::", "-q a:", "--cubic abc", "--cubic abb", "--cubic :::",
                                  "-q :: --ignore b", "--interactions cab"])
def test_gpu_device_featurization_batch1_parity(args):
    """Device featurization (expand_count / expand_fill kernels: base namespaces, -q / --cubic incl. ':'
    wildcards with VW's combination semantics, ignored namespaces, the constant): at gpuBatchSize=1 the
    device learner equals the sequential host learner, and scoring the model on the device equals scoring
    it on the host."""
    df = _three_ns()
    kw = dict(featuresCol="a", additionalFeatures=["b", "c"], passThroughArgs=args, numPasses=1)
    g = VowpalWabbitRegressor(deviceType="gpu", gpuBatchSize=1, **kw).fit(df)
    c = VowpalWabbitRegressor(**kw).fit(df)
    p_dev = g.transform(df)["prediction"]            # device scoring of the device-trained model
    p_host = _host_scored(g, df)                      # the same model through the host learner
    p_cpu = c.transform(df)["prediction"]
    scale = np.abs(p_cpu).max()
    np.testing.assert_allclose(p_dev, p_host, rtol=1e-5, atol=1e-5 * scale)
    np.testing.assert_allclose(p_host, p_cpu, rtol=1e-4, atol=1e-4 * scale)


def _csoaa_lines(n=1500, seed=3):
    rng = np.random.default_rng(seed)
    lines = []
    for i in range(n):
        x = rng.normal(size=4)
        k = int(np.argmax([x[0], x[1] - x[2], 0.3 + x[3]]))
        costs = " ".join(f"{j + 1}:{0.0 if j == k else 1.0 + 0.1 * j}" for j in range(3))
        lines.append(f"{costs} |f x0:{x[0]:.4f} x1:{x[1]:.4f} x2:{x[2]:.4f} x3:{x[3]:.4f} |g t{i % 7}")
    return lines


@pytest.mark.gpu
def test_gpu_csoaa_generic_batch1_parity():
    """--csoaa on the device (csoaa_kernel): class scores at the oaa offsets, argmin prediction, the example's
    (class, cost) regressions applied in order. Text examples parsed on the host (VowpalWabbitGeneric
    deviceType='gpu'); batch 1 equals the host learner's weights."""
    from synapseml_amd.vw import VowpalWabbitGeneric

    lines = _csoaa_lines()
    df = DataFrame({"value": np.asarray(lines, dtype=object)})
    g = VowpalWabbitGeneric(passThroughArgs="--csoaa 3 -q fg", deviceType="gpu", gpuBatchSize=1).fit(df)
    c = VowpalWabbitGeneric(passThroughArgs="--csoaa 3 -q fg").fit(df)
    vw = native.load("_vw")
    wg = np.asarray(vw.VW("--testonly", g.getModel()).weights())
    wc = np.asarray(vw.VW("--testonly", c.getModel()).weights())
    np.testing.assert_allclose(wg, wc, rtol=1e-4, atol=1e-5 * np.abs(wc).max())
    pg, pc = g.transform(df)["prediction"], c.transform(df)["prediction"]
    assert np.mean(pg == pc) > 0.999


def _cb_frame(n=1200, A=4, seed=9):
    from synapseml_amd.core.linalg import DenseVector

    rng = np.random.default_rng(seed)
    shared = rng.normal(size=(n, 3))
    acts = np.empty(n, dtype=object)
    chosen = rng.integers(1, A + 1, size=n)
    cost = np.empty(n)
    for i in range(n):
        feats = [DenseVector(rng.normal(size=3)) for _ in range(A)]
        acts[i] = feats
        f = feats[chosen[i] - 1].values
        cost[i] = float(shared[i, 0] * f[0] - f[1] > 0)
    return DataFrame({"shared": shared, "features": acts, "chosenAction": chosen.astype(np.int32),
                      "label": cost, "probability": np.full(n, 1.0 / A)})


@pytest.mark.gpu
@pytest.mark.parametrize("cb_type", ["mtr", "dr", "ips"])
def test_gpu_contextual_bandit_batch1_parity(cb_type):
    """--cb_explore_adf on the device (cb_kernel): action rows featurized with their example's shared
    namespaces, epsilon-greedy pmf, --cb_type mtr / dr / ips updates. Batch 1 = the host learner: same
    weights, same action probabilities, same IPS / SNIPS estimates."""
    from synapseml_amd.vw.bandit import VowpalWabbitContextualBandit

    df = _cb_frame()
    kw = dict(epsilon=0.1, passThroughArgs=f"--cb_type {cb_type} -q sf")
    g = VowpalWabbitContextualBandit(deviceType="gpu", gpuBatchSize=1, **kw).fit(df)
    c = VowpalWabbitContextualBandit(**kw).fit(df)
    vw = native.load("_vw")
    wg = np.asarray(vw.VW("--testonly", g.getModel()).weights())
    wc = np.asarray(vw.VW("--testonly", c.getModel()).weights())
    np.testing.assert_allclose(wg, wc, rtol=1e-4, atol=1e-5 * max(np.abs(wc).max(), 1e-6))
    pg = np.stack(g.transform(df)["prediction"])
    pc = np.stack(c.transform(df)["prediction"])
    assert np.mean(np.all(np.abs(pg - pc) < 1e-6, axis=1)) > 0.99
    sg, sc = g.getPerformanceStatistics(), c.getPerformanceStatistics()
    np.testing.assert_allclose(sg["ipsEstimate"][0], sc["ipsEstimate"][0], rtol=1e-4)
    np.testing.assert_allclose(sg["snipsEstimate"][0], sc["snipsEstimate"][0], rtol=1e-4)


@pytest.mark.gpu
def test_gpu_scoring_b30_model_keeps_host_memory_flat():
    """A 2^30-slot model (16 GiB as a dense table) is transformed on the device from its nonzeros: host RSS
    stays flat (the host learner would allocate the dense table)."""
    import psutil

    rng = np.random.default_rng(2)
    X = rng.normal(size=(20000, 8))
    y = (X[:, 0] - X[:, 1] > 0).astype(np.float64)
    df = DataFrame({"features": X, "label": y})
    m = VowpalWabbitClassifier(deviceType="gpu", numBits=30, labelConversion=True,
                               passThroughArgs="--loss_function logistic", gpuBatchSize=64).fit(df)
    proc = psutil.Process()
    rss0 = proc.memory_info().rss
    out = m.transform(df)
    rss1 = proc.memory_info().rss
    assert rss1 - rss0 < (1 << 30), (rss0, rss1)
    acc = np.mean(out["prediction"] == y)
    assert acc > 0.95


@pytest.mark.gpu
@pytest.mark.parametrize("args,syncs", [("", 0), ("-q ab --loss_function logistic", 2), ("--oaa 3", 0)])
def test_gpu_fused_stage_learn_equals_stage_then_learn(monkeypatch, args, syncs):
    """The estimator learns pass 0's first sync segment while the pass's blocks upload (chunk by chunk, each
    chunk expanded and learned as it lands): at gpuBatchSize=1 the scalar learners (one wave per example,
    deterministic) give bitwise the model of staging everything first and learning after, with the pass cut
    into many chunks. --oaa runs one wave per class whose global-state atomics land in any order, so its
    models agree to rounding."""
    df = _three_ns(n=2500)
    y = df["label"]
    if "logistic" in args:
        df = DataFrame({"a": df["a"], "b": df["b"], "c": df["c"], "label": np.where(y > 0, 1.0, -1.0)})
    elif "oaa" in args:
        df = DataFrame({"a": df["a"], "b": df["b"], "c": df["c"], "label": (np.digitize(y, [-0.5, 0.5]) + 1.0)})
    kw = dict(featuresCol="a", additionalFeatures=["b", "c"], passThroughArgs=args, numPasses=2,
              numSyncsPerPass=syncs, deviceType="gpu", gpuBatchSize=1)
    if "oaa" in args:
        kw["numClasses"] = 3
    cls = VowpalWabbitClassifier if ("logistic" in args or "oaa" in args) else VowpalWabbitRegressor
    monkeypatch.setenv("SML_VW_STAGE_CHUNK_ROWS", "300")
    monkeypatch.setenv("SML_VW_STAGE_LEARN", "1")
    fused = cls(**kw).fit(df)
    monkeypatch.setenv("SML_VW_STAGE_LEARN", "0")
    plain = cls(**kw).fit(df)
    sf, sp = fused.getPerformanceStatistics(), plain.getPerformanceStatistics()
    if "oaa" in args:
        assert np.mean(fused.transform(df)["prediction"] == plain.transform(df)["prediction"]) > 0.99
        assert float(sf["averageLoss"][0]) == pytest.approx(float(sp["averageLoss"][0]), rel=1e-3)
        return
    assert fused.getNativeModel() == plain.getNativeModel()
    assert float(sf["averageLoss"][0]) == float(sp["averageLoss"][0])


@pytest.mark.gpu
def test_gpu_fused_stage_learn_non_power_of_two_batch(monkeypatch):
    """after the hogwild warm-up (launches of 1, 1, 2, 4, ... examples) the launch boundaries of a
    non-power-of-two batch are offset from the chunk boundaries (multiples of the batch); the fused staging
    now carries a straddling launch into the next chunk instead of cutting it, so both paths launch the same
    example ranges (batch > 1 is hogwild: models agree to rounding)."""
    df = _three_ns(n=2500)
    kw = dict(featuresCol="a", additionalFeatures=["b", "c"], numPasses=2, deviceType="gpu", gpuBatchSize=7)
    monkeypatch.setenv("SML_VW_STAGE_CHUNK_ROWS", "300")
    monkeypatch.setenv("SML_VW_STAGE_LEARN", "1")
    fused = VowpalWabbitRegressor(**kw).fit(df)
    monkeypatch.setenv("SML_VW_STAGE_LEARN", "0")
    plain = VowpalWabbitRegressor(**kw).fit(df)
    pf = np.asarray(fused.transform(df)["prediction"], dtype=np.float64)
    pp = np.asarray(plain.transform(df)["prediction"], dtype=np.float64)
    # hogwild at batch 7: concurrent examples' returning atomics land in any order, so the two fits differ
    # slightly (up to ~0.03 on a prediction) - they must learn the same function
    assert np.corrcoef(pf, pp)[0, 1] > 0.995
    assert np.max(np.abs(pf - pp)) < 0.15
    assert float(fused.getPerformanceStatistics()["averageLoss"][0]) == pytest.approx(
        float(plain.getPerformanceStatistics()["averageLoss"][0]), rel=0.05)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [12, 22])
def test_gpu_export_one_scan_regions_match_two_scans(monkeypatch, bits):
    """The model export's one-scan form (per-4096-slot record regions, then a compaction) writes the same
    bytes as the count-scan + write-scan form; a table too dense for the regions (2^12 slots) falls back."""
    vw = native.load("_vw")
    cfg = vw.GpuSgdConfig()
    cfg.bits = bits
    cfg.loss = 1
    sgd = vw.GpuSgd(cfg, 0)
    rng = np.random.default_rng(3)
    n, k = 20000, 16
    idx = rng.integers(0, 1 << 32, size=n * k, dtype=np.uint64).astype(np.uint32)
    val = rng.standard_normal(n * k).astype(np.float32)
    ip = np.arange(0, n * k + 1, k, dtype=np.int64)
    lab = (rng.random(n) > 0.5).astype(np.float32) * 2 - 1
    sgd.learn(ip, idx, val, lab, None, 256)
    args = f"--loss_function logistic -b {bits}"
    monkeypatch.setenv("SML_VW_EXPORT_REGIONS", "1")
    m1 = sgd.export_model(args)
    monkeypatch.setenv("SML_VW_EXPORT_REGIONS", "0")
    m0 = sgd.export_model(args)
    assert len(m1) > 200 and m1 == m0


def _cats_lines(n=2000, seed=0, x_informative=True):
    rng = np.random.default_rng(seed)
    lines = []
    for _ in range(n):
        a = rng.uniform(0, 20000)
        f = rng.integers(0, 2)
        lo, hi = (12000, 18000) if (f == 0 or not x_informative) else (2000, 8000)
        cost = 0.0 if lo < a < hi else 1.0
        lines.append(f"ca {a:.2f}:{cost}:{1 / 20000:.8f} | f{f} x")
    return DataFrame({"value": np.array(lines, dtype=object)})


@pytest.mark.gpu
@pytest.mark.parametrize("args", ["--cats_pdf 4 --bandwidth 2500 --min_value 0 --max_value 20000",
                                  "--cats_pdf 6 --bandwidth 1500 --min_value 0 --max_value 20000 --loss_function logistic",
                                  "--cats 8 --bandwidth 1000 --min_value 0 --max_value 20000"])
def test_gpu_cats_batch1_parity(args):
    """--cats_pdf / --cats on the device (filter tree of binary node learners, IPS leaf costs with the running-
    mean baseline, bottom-up tournament): at gpuBatchSize=1 the device-trained model routes like the host
    learner's - the same leaf for the examples (host scoring of both models, compared through the pdf's peak
    window or the sampled action's window) - and it learned the context-dependent cheap regions."""
    from synapseml_amd.vw import VowpalWabbitGeneric

    df = _cats_lines()
    g = VowpalWabbitGeneric(passThroughArgs=args, deviceType="gpu", gpuBatchSize=1).fit(df)
    c = VowpalWabbitGeneric(passThroughArgs=args).fit(df)
    og, oc = g.transform(df), c.transform(df)
    if "--cats_pdf" in args:
        peak = lambda seg: max(seg, key=lambda s: s["pdfValue"])["left"]  # noqa: E731
        pg = np.array([peak(s) for s in og["segments"]])
        pc = np.array([peak(s) for s in oc["segments"]])
        assert np.mean(pg == pc) > 0.97, np.mean(pg == pc)
        # context f0 -> cheap near 15000, f1 -> near 5000 (the peak window's centre)
        lines = df["value"].tolist()
        ctr = np.array([(max(s, key=lambda t: t["pdfValue"])["left"] + max(s, key=lambda t: t["pdfValue"])["right"]) / 2
                        for s in og["segments"]])
        f1 = np.array(["f1" in l for l in lines])
        assert np.median(ctr[~f1]) > 10000 and np.median(ctr[f1]) < 10000
    else:
        a = np.asarray(og["action"])
        assert ((a >= 0) & (a <= 20000)).all() and np.all(np.asarray(og["pdf"]) > 0)


@pytest.mark.gpu
def test_gpu_unit_values_cross_as_device_fill(monkeypatch):
    """Binary hashed features (every value 1.0): the stager sends such value pieces as a device fill instead of
    their bytes. Batch-1 fits with and without the fill give the same model bytes; a block with one other
    value is sent as bytes."""
    from synapseml_amd.core.linalg import CsrColumn

    vw = native.load("_vw")
    rng = np.random.default_rng(21)
    n, k = 6000, 12
    ip = np.arange(0, n * k + 1, k, dtype=np.int64)
    idx = rng.integers(0, 1 << 20, size=n * k, dtype=np.int64).astype(np.uint32)
    w = rng.standard_normal(1 << 20)
    y = np.where(w[idx.reshape(n, k)].sum(1) > 0, 1.0, -1.0)
    kw = dict(numBits=20, deviceType="gpu", gpuBatchSize=1, passThroughArgs="--loss_function logistic")
    monkeypatch.setenv("SML_VW_STAGE_CHUNK_ROWS", "1000")
    out = {}
    for fill in ("1", "0"):
        monkeypatch.setenv("SML_VW_UNIT_FILL", fill)
        before = vw._stager_unit_pieces()
        df = DataFrame({"features": CsrColumn(ip, idx, np.ones(n * k, np.float32), 1 << 32), "label": y})
        m = VowpalWabbitClassifier(**kw).fit(df)
        out[fill] = (m.getNativeModel(), vw._stager_unit_pieces() - before)
    assert out["1"][1] > 0 and out["0"][1] == 0
    assert bytes(out["1"][0]) == bytes(out["0"][0])
    val = np.ones(n * k, np.float32)
    val[-1] = 2.0  # the last piece is not all ones
    monkeypatch.setenv("SML_VW_UNIT_FILL", "1")
    df = DataFrame({"features": CsrColumn(ip, idx, val, 1 << 32), "label": y})
    a = VowpalWabbitClassifier(**kw).fit(df)
    monkeypatch.setenv("SML_VW_UNIT_FILL", "0")
    b = VowpalWabbitClassifier(**kw).fit(df)
    assert bytes(a.getNativeModel()) == bytes(b.getNativeModel())


@pytest.mark.gpu
def test_gpu_final_export_leaves_a_clean_table_for_the_next_fit(monkeypatch):
    """A fit's final export clears the exported components in place; the next learner of that size takes the
    table without its memset (SML_VW_CLEAN_TABLES=0: always zero a fresh one). Batch-1 fits in a row give the
    same model bytes either way, and a retired learner refuses further work."""
    from synapseml_amd.core.linalg import CsrColumn

    rng = np.random.default_rng(8)
    n, k = 5000, 10
    ip = np.arange(0, n * k + 1, k, dtype=np.int64)
    idx = rng.integers(0, 1 << 20, size=n * k, dtype=np.int64).astype(np.uint32)
    val = rng.standard_normal(n * k).astype(np.float32)
    y = np.where(rng.standard_normal(n) > 0, 1.0, -1.0)
    df = DataFrame({"features": CsrColumn(ip, idx, val, 1 << 32), "label": y})
    kw = dict(numBits=18, deviceType="gpu", gpuBatchSize=1, passThroughArgs="--loss_function logistic")
    models = {}
    for clean in ("1", "0"):
        monkeypatch.setenv("SML_VW_CLEAN_TABLES", clean)
        models[clean] = [VowpalWabbitClassifier(**kw).fit(df).getNativeModel() for _ in range(3)]
    assert len({bytes(m) for m in models["1"] + models["0"]}) == 1
    vw = native.load("_vw")
    cfg = vw.GpuSgdConfig()
    cfg.bits = 18
    cfg.loss = 1
    g = vw.GpuSgd(cfg, 0)
    g.learn(ip, idx, val, y.astype(np.float32), None, 1)
    assert len(g.export_model("--loss_function logistic -b 18", final=True)) > 100
    with pytest.raises(RuntimeError, match="cleared by the final export"):
        g.learn(ip, idx, val, y.astype(np.float32), None, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [14, 24])
def test_gpu_export_touch_map_skip_matches_full_scan(monkeypatch, bits):
    """The export scans only the 256-slot sub-blocks the touch map says were ever written: same bytes as the
    full scan (SML_VW_EXPORT_SKIP=0) after learning, after syncs (a world-1 communicator still runs them; the
    sync epochs advance and the touch map keeps every write) and for a warm-started learner (the import marks
    the sub-blocks it fills)."""
    vw = native.load("_vw")
    cfg = vw.GpuSgdConfig()
    cfg.bits = bits
    cfg.loss = 1
    rng = np.random.default_rng(5)
    n, k = 20000, 12
    idx = rng.integers(0, 1 << 32, size=n * k, dtype=np.uint64).astype(np.uint32)
    val = rng.standard_normal(n * k).astype(np.float32)
    ip = np.arange(0, n * k + 1, k, dtype=np.int64)
    lab = (rng.random(n) > 0.5).astype(np.float32) * 2 - 1
    args = f"--loss_function logistic -b {bits}"

    def both(g):
        monkeypatch.setenv("SML_VW_EXPORT_SKIP", "1")
        a = g.export_model(args)
        monkeypatch.setenv("SML_VW_EXPORT_SKIP", "0")
        b = g.export_model(args)
        assert a == b
        return a

    g = vw.GpuSgd(cfg, 0)
    g.learn(ip[: n // 2 + 1], idx[: ip[n // 2]], val[: ip[n // 2]], lab[: n // 2], None, 64)
    m_half = both(g)
    comm = vw.nccl_comm(vw.nccl_unique_id(), 0, 1, 60000.0)
    for _ in range(3):
        g.allreduce_average(comm)
    g.learn(ip[n // 2:] - ip[n // 2], idx[ip[n // 2]:], val[ip[n // 2]:], lab[n // 2:], None, 64)
    g.allreduce_average(comm)
    m_full = both(g)
    assert len(m_full) > len(m_half) > 200
    g2 = vw.GpuSgd(cfg, 0)
    g2.import_model(bytes(m_full))
    assert len(both(g2)) == len(m_full)  # every imported record found by the skipping scan
