"""CNTKModel shim API (reference deep-learning/src/main/python/synapse/ml/cntk/CNTKModel.py): node / column
setters rewrite the feed / fetch dictionaries; ONNX exports run on the executor; native CNTK bytes are refused."""
import numpy as np
import pytest

from synapseml_amd.cntk import CNTKModel
from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.onnx import proto as P
from synapseml_amd.onnx.writer import GraphBuilder


def _model(tmp_path):
    b = GraphBuilder("two_heads")
    b.input("feats", P.FLOAT32, ["N", 3])
    w = b.init("w", np.arange(6, dtype=np.float32).reshape(3, 2))
    y = b.add("MatMul", ["feats", w], out="logits")
    b.add("Relu", [y], out="act")
    b.output("logits", P.FLOAT32, ["N", 2])
    b.output("act", P.FLOAT32, ["N", 2])
    p = tmp_path / "m.onnx"
    p.write_bytes(b.to_bytes())
    return str(p)


def test_cntk_shim_api(tmp_path):
    path = _model(tmp_path)
    X = np.array([[1.0, -2.0, 0.5], [-1.0, 0.0, 3.0]])
    df = DataFrame({"x": X})
    m = CNTKModel().setModelLocation(path).setInputCol("x").setOutputCol("out").setMiniBatchSize(1)
    assert m.getFeedDict() == {"feats": "x"} and m.getFetchDict() == {"out": "logits"}
    assert m.getInputShapes() == [["N", 3]]
    ref = X.astype(np.float32) @ np.arange(6, dtype=np.float32).reshape(3, 2)
    np.testing.assert_allclose(np.stack(m.transform(df)["out"]), ref, rtol=1e-6)
    m.setOutputNode("act")
    assert m.getFetchDict() == {"out": "act"} and m.getOutputNode() == "act"
    np.testing.assert_allclose(np.stack(m.transform(df)["out"]), np.maximum(ref, 0), rtol=1e-6)
    m.setOutputNodeIndex(0)
    assert m.getFetchDict() == {"out": "logits"} and m.getOutputNodeIndex() == 0
    m.setInputNode("feats")
    assert m.getFeedDict() == {"feats": "x"} and m.getInputNodeIndex() == 0
    assert m.rebroadcastCNTKModel(None) is m
    with pytest.raises(ValueError, match="not in the model outputs"):
        m.setOutputNode("nope")
    native = tmp_path / "m.model"
    native.write_bytes(b"\x0a\x05CNTK2" + bytes(32))
    with pytest.raises(NotImplementedError, match="ONNX"):
        CNTKModel().setModelLocation(str(native))
