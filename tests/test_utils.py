"""Utility modules (reference: core/src/test/scala/.../core/utils/*Suite.scala,
python downloader / plot / FluentAPI tests)."""
import hashlib
import os
import pickle
import threading
import time

import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.utils import (ModelDownloader, ModelSchema, SharedSingleton, SharedVariable, assert_stages_equal,
                                 buffered_map, cluster_info, retry)
from synapseml_amd.utils import fluent  # noqa: F401
from synapseml_amd.utils import platform, plot
from synapseml_amd.utils.cluster import rows_per_partition


def test_cluster_info_from_env(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    ci = cluster_info()
    assert ci.world_size == 8 and ci.rank == 3 and ci.num_nodes == 1 and not ci.is_driver
    assert rows_per_partition(10, 3) == [4, 3, 3]


def test_shared_variable_single_construction():
    calls = []
    sv = SharedVariable(lambda: calls.append(1) or object())
    vals = []
    ts = [threading.Thread(target=lambda: vals.append(sv.get())) for _ in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert len(calls) == 1 and all(v is vals[0] for v in vals)
    sv2 = pickle.loads(pickle.dumps(SharedSingleton(dict, key="k1")))
    assert sv2.key == "k1" and isinstance(sv2.instance, dict)


def test_buffered_map_order_and_retry():
    out = list(buffered_map(lambda x: (time.sleep(0.01 * (5 - x)), x * x)[1], range(6), concurrency=3))
    assert out == [0, 1, 4, 9, 16, 25]
    n = {"c": 0}

    def flaky():
        n["c"] += 1
        if n["c"] < 3:
            raise IOError("boom")
        return "ok"

    assert retry(flaky, backoffs_ms=(0, 1, 1, 1)) == "ok" and n["c"] == 3


def test_assert_stages_equal():
    from synapseml_amd.featurize.ml import HashingTF

    a = HashingTF(inputCol="w", outputCol="f", numFeatures=64)
    b = HashingTF(inputCol="w", outputCol="f", numFeatures=64)
    assert_stages_equal(a, b)
    with pytest.raises(AssertionError):
        assert_stages_equal(a, HashingTF(inputCol="w", outputCol="f", numFeatures=32))


def test_model_downloader_offline_repo(tmp_path):
    remote = tmp_path / "remote"
    remote.mkdir()
    blob = b"\x08\x01model-bytes"
    (remote / "tiny.onnx").write_bytes(blob)
    m = ModelSchema("tiny", "synthetic", "image", "tiny.onnx", hashlib.sha256(blob).hexdigest(), len(blob), 0, 1,
                    ["out"])
    (remote / "MANIFEST").write_text(m.to_json() + "\n")
    d = ModelDownloader(localPath=str(tmp_path / "local"), serverURL="file://" + str(remote))
    assert [x.name for x in d.remoteModels()] == ["tiny"]
    loc = d.downloadByName("tiny")
    assert loc.uri.startswith("file://") and os.path.exists(loc.uri[7:])
    assert [x.name for x in d.localModels()] == ["tiny"]
    bad = ModelSchema("bad", "d", "image", "tiny.onnx", "0" * 64, 1)
    with pytest.raises(IOError):
        d.downloadModel(bad)


def test_platform_and_secret(monkeypatch):
    assert platform.current_platform() in ("unknown", "databricks", "binder", "fabric")
    monkeypatch.setenv("MY_KEY", "s3cret")
    assert platform.find_secret("my-key", "vault") == "s3cret"
    with pytest.raises(RuntimeError):
        platform.find_secret("absent-secret-xyz", "vault")


def test_plots_and_fluent():
    rng = np.random.default_rng(0)
    y = rng.integers(0, 2, 200).astype(float)
    p = np.clip(y * 0.6 + rng.random(200) * 0.5, 0, 1)
    df = DataFrame({"y": y, "p": p, "yhat": (p > 0.5).astype(float)})
    fig, cm = plot.confusionMatrix(df, "y", "yhat", ["neg", "pos"])
    assert cm.sum() == 200
    fig2, (fpr, tpr, a) = plot.roc(df, "y", "p")
    assert 0.8 < a <= 1.0
    from synapseml_amd.stages.basic import DropColumns

    assert df.mlTransform(DropColumns(cols=["p"])).columns == ["y", "yhat"]
