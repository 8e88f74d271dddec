"""Behaviour of the reference-API methods added for parity (test_api_parity checks presence)."""
import numpy as np
import pytest

from synapseml_amd.core.dataframe import DataFrame


def test_conditional_ball_tree_save_load(tmp_path):
    from synapseml_amd.nn import ConditionalBallTree

    rng = np.random.default_rng(0)
    keys = rng.normal(size=(200, 4))
    t = ConditionalBallTree(keys, list(range(200)), [i % 3 for i in range(200)], leafSize=8)
    p = str(tmp_path / "cbt.json")
    t.save(p)
    t2 = ConditionalBallTree.load(p)
    q = rng.normal(size=4)
    a = t.findMaximumInnerProducts(q, {1, 2}, 5)
    b = t2.findMaximumInnerProducts(q, {1, 2}, 5)
    assert [(m.index, round(m.distance, 12)) for m in a] == [(m.index, round(m.distance, 12)) for m in b]


def test_hyperparam_get_and_space():
    from synapseml_amd.automl import DiscreteHyperParam, GridSpace, RandomSpace, RangeHyperParam
    from synapseml_amd.models import LogisticRegression

    d, r = DiscreteHyperParam([1, 2]), RangeHyperParam(0.1, 0.5)
    assert d.get() is d and r.get() is r
    lr = LogisticRegression()
    g = GridSpace([(lr, "regParam", d)])
    assert g.space() is g and len(list(g.paramMaps())) == 2
    rs = RandomSpace([(lr, "regParam", r)])
    assert rs.space() is rs


def test_onnx_model_inputs_outputs():
    from synapseml_amd.onnx import ONNXModel, proto as P
    from synapseml_amd.onnx.writer import GraphBuilder

    b = GraphBuilder("g")
    b.input("x", P.FLOAT32, ["N", 2])
    b.add("Relu", ["x"], out="y")
    b.output("y", P.FLOAT32, ["N", 2])
    m = ONNXModel().setModelPayload(b.to_bytes())
    assert list(m.getModelInputs()) == ["x"] and list(m.getModelOutputs()) == ["y"]


def test_vision_transform_fn_and_prediction_fn():
    from synapseml_amd.dl import DeepVisionClassifier
    from synapseml_amd.image import encode_png

    rng = np.random.default_rng(1)
    imgs = [encode_png(rng.integers(0, 255, (20, 20, 3), dtype=np.uint8)) for _ in range(8)]
    df = DataFrame({"image": np.array(imgs, dtype=object), "label": np.array([0, 1] * 4, np.float64)})
    calls = []

    def flip(t):
        calls.append(tuple(t.shape))
        return t.flip(-1)

    est = DeepVisionClassifier(backbone="resnet_tiny", num_classes=2, image_size=32, epochs=1, batch_size=4,
                               use_gpu=False, transform_fn=flip)
    est.setDropoutAUX(0.5)
    assert est.getDropoutAUX() == 0.5 and est.get_model_class().__name__ == "DeepVisionModel"
    m = est.fit(df)
    assert calls and calls[0] == (3, 32, 32)
    assert m.getTransformationFn() is flip and m.getOptimizer() == "adam"
    p = m.get_prediction_fn()(imgs[:3])
    assert p.shape == (3, 2) and np.allclose(p.sum(1), 1.0, atol=1e-5)


def test_text_train_from_scratch_requires_layers():
    from synapseml_amd.dl import DeepTextClassifier

    df = DataFrame({"text": np.array(["a b", "c d"], dtype=object), "label": np.array([0.0, 1.0])})
    with pytest.raises(ValueError, match="additional_layers_to_train"):
        DeepTextClassifier(checkpoint="tiny-bert", num_classes=2, train_from_scratch=False,
                           additional_layers_to_train=-1, use_gpu=False).fit(df)
    assert DeepTextClassifier().get_model_class().__name__ == "DeepTextModel"


def test_synapseml_logger_decorators():
    from synapseml_amd.core.logging import SynapseMLLogger, add_event_sink, remove_event_sink

    seen = []
    add_event_sink(seen.append)
    try:
        class Thing(SynapseMLLogger):
            @SynapseMLLogger.log_transform()
            def transform(self, df):
                return df

            @SynapseMLLogger.log_fit()
            def fit(self, df):
                raise ValueError("bad sig=" + "a" * 50 + "%3d")

        t = Thing(uid="thing_1")
        t.log_class("tests")
        t.transform(DataFrame({"a": np.arange(3), "b": np.arange(3)}))
        with pytest.raises(ValueError):
            t.fit(None)
    finally:
        remove_event_sink(seen.append)
    methods = [p.get("method") for p in seen]
    assert methods == ["constructor", "transform", "fit"]
    assert seen[1]["dfInfo"]["input"]["numCols"] == 2 and "executionSeconds" in seen[1]
    assert seen[2]["errorType"] == "ValueError" and "sig=####" in seen[2]["errorMessage"]
