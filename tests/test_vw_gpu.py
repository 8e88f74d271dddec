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


@pytest.mark.parametrize("args", ["--csoaa 3", "--cb_explore_adf", "--cats 4 --bandwidth 1 --min_value 0 --max_value 1",
                                  "--l1 0.001", "--ngram 2", "--ignore a", "--loss_function hinge",
                                  "--interactions abc"])
def test_gpu_rejects_reductions_it_does_not_run(args):
    """Reductions the device learner does not implement are refused by name before any GPU work,
    never silently run on the host."""
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
    from sklearn.metrics import roc_auc_score

    df, y = _binary()
    args = "--loss_function logistic"
    gpu = VowpalWabbitClassifier(deviceType="gpu", labelConversion=True, passThroughArgs=args, numPasses=3,
                                 gpuBatchSize=256).fit(df)
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
@pytest.mark.parametrize("args", ["", "--sgd", "--adaptive", "--normalized --invariant", "--loss_function logistic -l 0.3"])
def test_gpu_batch1_is_the_sequential_learner(args):
    """gpuBatchSize=1 runs VW's update rule example by example: on mixed-scale features (where the
    normalized update matters) the exported GPU model predicts like the exact host learner's."""
    rng = np.random.default_rng(5)
    n = 3000
    X = rng.normal(size=(n, 6)) * np.array([1e-2, 1.0, 30.0, 1.0, 5.0, 0.3])
    y = X @ np.array([20.0, -1.0, 0.05, 0.7, 0.2, 2.0]) + 0.05 * rng.normal(size=n)
    if "logistic" in args:
        y = np.where(y > 0, 1.0, -1.0)
    df = DataFrame({"features": X, "label": y})
    kw = dict(passThroughArgs=args, numPasses=1)
    g = VowpalWabbitRegressor(deviceType="gpu", gpuBatchSize=1, **kw).fit(df)
    c = VowpalWabbitRegressor(**kw).fit(df)
    pg, pc = g.transform(df)["prediction"], c.transform(df)["prediction"]
    np.testing.assert_allclose(pg, pc, rtol=2e-3, atol=2e-3 * np.abs(pc).max())


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
