"""ONNX executor + ONNXModel tests (model: reference deep-learning/src/test/
scala/.../onnx/ONNXModelSuite.scala). The reference downloads its models;
here every model is produced by our own writer with the same topology/names
(random weights), so numerical parity is pinned against an unoptimised
reference execution of the same graph and against plain numpy/torch math."""
import numpy as np
import pytest
import torch

from synapseml_amd.core.dataframe import DataFrame
from synapseml_amd.core.linalg import DenseVector
from synapseml_amd.onnx import Graph, InferenceSession, ONNXModel, proto as P, writer
from synapseml_amd.onnx.writer import GraphBuilder


# ------------------------------------------------------------------ codec
def test_proto_roundtrip():
    b = GraphBuilder("g")
    b.input("x", P.FLOAT32, ["N", 3])
    w = b.init("w", np.arange(6, dtype=np.float32).reshape(3, 2))
    b.add("MatMul", ["x", w], out="y")
    b.add("Softmax", ["y"], {"axis": -1}, out="z")
    b.output("z", P.FLOAT32, ["N", 2])
    data = b.to_bytes()
    m = P.load_model(data)
    assert m.graph.node[0].op_type == "MatMul"
    assert m.graph.node[1].attribute[0].i == -1
    g = Graph.from_bytes(data)
    assert g.inputs[0].shape == ["N", 3]
    np.testing.assert_array_equal(g.initializers["w"], np.arange(6, dtype=np.float32).reshape(3, 2))
    # re-encode the decoded graph
    g2 = Graph.from_bytes(g.to_bytes())
    assert [n.op_type for n in g2.nodes] == ["MatMul", "Softmax"]
    assert P.encode(P.decode("TensorProto", P.encode(P.numpy_to_tensor(np.array([1, -2], np.int64))))) == \
        P.encode(P.numpy_to_tensor(np.array([1, -2], np.int64)))


def test_tensor_formats():
    t = P.Message("TensorProto", dims=[2], data_type=P.FLOAT32, float_data=[1.5, -2.0])
    np.testing.assert_array_equal(P.tensor_to_numpy(P.decode("TensorProto", P.encode(t))), [1.5, -2.0])
    t = P.Message("TensorProto", dims=[3], data_type=P.INT64, int64_data=[1, -5, 7])
    np.testing.assert_array_equal(P.tensor_to_numpy(P.decode("TensorProto", P.encode(t))), [1, -5, 7])
    s = P.numpy_to_tensor(np.array(["a", "bc"], dtype=object))
    assert P.tensor_to_numpy(P.decode("TensorProto", P.encode(s))).tolist() == ["a", "bc"]


# ------------------------------------------------------------------ executor numerics
def _conv_ref(x, w, b, stride, pad):
    return torch.nn.functional.conv2d(torch.from_numpy(x), torch.from_numpy(w),
                                      None if b is None else torch.from_numpy(b), stride=stride, padding=pad).numpy()


def test_conv_bn_relu_fusion_matches_unfused():
    rng = np.random.default_rng(0)
    b = GraphBuilder("cbr")
    b.input("x", P.FLOAT32, ["N", 4, 9, 9])
    w = b.init("w", rng.standard_normal((8, 4, 3, 3)).astype(np.float32))
    y = b.add("Conv", ["x", w], {"kernel_shape": [3, 3], "pads": [1, 1, 1, 1], "strides": [2, 2]})
    g = b.init("g", rng.random(8).astype(np.float32) + 0.5)
    be = b.init("be", rng.standard_normal(8).astype(np.float32))
    m = b.init("m", rng.standard_normal(8).astype(np.float32))
    v = b.init("v", rng.random(8).astype(np.float32) + 0.5)
    y = b.add("BatchNormalization", [y, g, be, m, v], {"epsilon": 1e-5})
    y = b.add("Relu", [y], out="out")
    b.output("out", P.FLOAT32, None)
    data = b.to_bytes()
    x = rng.standard_normal((2, 4, 9, 9)).astype(np.float32)
    s_opt = InferenceSession(data, device="cpu")
    assert [n.op_type for n in s_opt.nodes] == ["_FusedConv"]
    o1 = s_opt.run(None, {"x": x})[0]
    o0 = InferenceSession(data, device="cpu", optimization_level="NO_OPT").run(None, {"x": x})[0]
    np.testing.assert_allclose(o1, o0, rtol=1e-4, atol=1e-4)
    # independent numpy/torch reference
    ref = _conv_ref(x, b.inits["w"], None, 2, 1)
    sc = b.inits["g"] / np.sqrt(b.inits["v"] + 1e-5)
    ref = np.maximum(0, (ref - b.inits["m"][None, :, None, None]) * sc[None, :, None, None] +
                     b.inits["be"][None, :, None, None])
    np.testing.assert_allclose(o0, ref, rtol=1e-4, atol=1e-4)


def test_preact_add_bn_relu_pattern():
    rng = np.random.default_rng(1)
    b = GraphBuilder("preact")
    b.input("a", P.FLOAT32, ["N", 8, 4, 4])
    b.input("c", P.FLOAT32, ["N", 8, 4, 4])
    s = b.add("Add", ["a", "c"], out="sum")
    params = [b.init(n, (rng.random(8) + 0.5).astype(np.float32)) for n in ("g", "be", "m", "v")]
    y = b.add("BatchNormalization", [s] + params)
    b.add("Relu", [y], out="act")
    b.output("sum", P.FLOAT32, None)
    b.output("act", P.FLOAT32, None)
    data = b.to_bytes()
    sess = InferenceSession(data, device="cpu")
    assert [n.op_type for n in sess.nodes] == ["_AddAffineAct"]
    a = rng.standard_normal((2, 8, 4, 4)).astype(np.float32)
    c = rng.standard_normal((2, 8, 4, 4)).astype(np.float32)
    o_sum, o_act = sess.run(None, {"a": a, "c": c})
    r_sum, r_act = InferenceSession(data, device="cpu", optimization_level="NO_OPT").run(None, {"a": a, "c": c})
    np.testing.assert_allclose(o_sum, a + c, rtol=1e-6)
    np.testing.assert_allclose(o_act, r_act, rtol=1e-5, atol=1e-5)


def test_mnist_and_resnet_slices():
    m = writer.mnist_cnn()
    s = InferenceSession(m, device="cpu")
    x = np.random.default_rng(0).random((1, 1, 28, 28), dtype=np.float32)
    np.testing.assert_allclose(s.run(None, {"Input3": x})[0],
                               InferenceSession(m, device="cpu", optimization_level="NO_OPT").run(None, {"Input3": x})[0],
                               rtol=1e-4, atol=1e-4)
    r = writer.resnet50_v2(seed=1)
    g = Graph.from_bytes(r).slice_at(["resnetv24_pool1_fwd"])
    sess = InferenceSession.from_graph(g, device="cpu")
    xb = np.random.default_rng(2).random((1, 3, 224, 224), dtype=np.float32)
    feat = sess.run(None, {"data": xb})[0]
    assert feat.shape == (1, 2048, 1, 1)
    full = InferenceSession(r, device="cpu", optimization_level="NO_OPT")
    ref = full.run_values({"data": xb}, ["resnetv24_pool1_fwd"])[0].numpy()
    np.testing.assert_allclose(feat, ref, rtol=2e-3, atol=2e-3 * np.abs(ref).max())


def test_op_coverage_misc():
    b = GraphBuilder("misc")
    b.input("x", P.FLOAT32, ["N", 6])
    shp = b.add("Shape", ["x"])
    n = b.add("Gather", [shp, b.init("i0", np.array(0, np.int64))], {"axis": 0})
    n1 = b.add("Unsqueeze", [n, b.init("ax", np.array([0], np.int64))])
    tgt = b.add("Concat", [n1, b.init("c", np.array([2, 3], np.int64))], {"axis": 0})
    r = b.add("Reshape", ["x", tgt])
    t = b.add("Transpose", [r], {"perm": [0, 2, 1]})
    red = b.add("ReduceMean", [t], {"axes": [1], "keepdims": 0})
    sm = b.add("Softmax", [red], {"axis": -1})
    cl = b.add("Clip", [sm, b.init("lo", np.array(0.1, np.float32)), b.init("hi", np.array(0.9, np.float32))])
    w = b.add("Where", [b.add("Greater", [cl, b.init("h", np.array(0.5, np.float32))]), cl,
                        b.init("z", np.array(0.0, np.float32))], out="y")
    am = b.add("ArgMax", [red], {"axis": 1, "keepdims": 0}, out="am")
    sl = b.add("Slice", ["x", b.init("s0", np.array([1], np.int64)), b.init("e0", np.array([5], np.int64)),
                          b.init("a0", np.array([1], np.int64)), b.init("st", np.array([2], np.int64))], out="sl")
    b.output("y", P.FLOAT32, None)
    b.output("am", P.INT64, None)
    b.output("sl", P.FLOAT32, None)
    x = np.arange(12, dtype=np.float32).reshape(2, 6) / 10
    y, am, sl = InferenceSession(b.to_bytes(), device="cpu").run(None, {"x": x})
    ref_red = x.reshape(2, 2, 3).transpose(0, 2, 1).mean(1)
    e = np.exp(ref_red - ref_red.max(1, keepdims=True))
    ref_sm = np.clip(e / e.sum(1, keepdims=True), 0.1, 0.9)
    np.testing.assert_allclose(y, np.where(ref_sm > 0.5, ref_sm, 0), rtol=1e-5)
    np.testing.assert_array_equal(am, ref_red.argmax(1))
    np.testing.assert_array_equal(sl, x[:, 1:5:2])


# ------------------------------------------------------------------ ONNXModel stage
def _iris_model():
    coef = np.array([[-0.4, 0.8, -2.2, -0.9], [0.5, -0.3, -0.2, -0.9], [-0.1, -0.5, 2.4, 1.8]], np.float32)
    inter = np.array([9.0, 2.0, -11.0], np.float32)
    return writer.linear_classifier_zipmap(coef, inter, [0, 1, 2]), coef, inter


def test_onnx_model_iris_zipmap_and_argmax():
    data, coef, inter = _iris_model()
    feats = np.array([[6.7, 3.1, 4.7, 1.5], [4.9, 3.0, 1.4, 0.2], [5.8, 2.7, 5.1, 1.9]], np.float32)
    col = np.empty(3, dtype=object)
    for i in range(3):
        col[i] = feats[i].tolist()
    df = DataFrame({"features": col})
    m = (ONNXModel().setModelPayload(data).setFeedDict({"float_input": "features"})
         .setFetchDict({"prediction": "output_label", "rawProbability": "output_probability"})
         .setArgMaxDict({"rawProbability": "argmax"}).setSoftMaxDict({"rawProbability": "sm"}).setDeviceType("CPU"))
    out = m.transform(df)
    s = feats @ coef.T + inter
    p = np.exp(s - s.max(1, keepdims=True))
    p /= p.sum(1, keepdims=True)
    assert out["prediction"].tolist() == s.argmax(1).tolist()
    for i in range(3):
        d = out["rawProbability"][i]
        assert set(d) == {0, 1, 2}
        np.testing.assert_allclose([d[k] for k in range(3)], p[i], rtol=1e-5)
    assert out["argmax"].tolist() == s.argmax(1).astype(float).tolist()
    assert isinstance(out["sm"][0], DenseVector)
    # vector and double inputs coerce to the model's float input
    dv = DataFrame({"features": np.array([DenseVector(r.astype(np.float64)) for r in feats], dtype=object)})
    assert m.transform(dv)["prediction"].tolist() == s.argmax(1).tolist()
    assert m.transform(DataFrame({"features": feats.astype(np.float64)}))["prediction"].tolist() == \
        s.argmax(1).tolist()


def test_onnx_model_shape_errors():
    data, _, _ = _iris_model()
    m = (ONNXModel().setModelPayload(data).setFeedDict({"float_input": "features"})
         .setFetchDict({"prediction": "output_label"}).setDeviceType("CPU"))
    bad = np.empty(1, dtype=object)
    bad[0] = [6.7, 3.1, 4.7]
    with pytest.raises(ValueError, match="IllegalArgumentException"):
        m.transform(DataFrame({"features": bad}))
    bad2 = np.empty(2, dtype=object)
    bad2[0] = [6.7, 3.1, 4.7, 1.5]
    bad2[1] = [6.7, 3.1, 4.7]
    with pytest.raises(ValueError, match="IllegalArgumentException"):
        m.transform(DataFrame({"features": bad2}))
    empty = np.empty(1, dtype=object)
    empty[0] = []
    with pytest.raises(ValueError, match="IllegalArgumentException"):
        m.transform(DataFrame({"features": empty}))
    with pytest.raises(ValueError):
        m.setFetchDict({"features": "output_label"}).transform(DataFrame({"features": np.ones((1, 4))}))


def test_onnx_model_boolean_and_variable_length_text():
    m = (ONNXModel().setModelPayload(writer.boolean_and()).setFeedDict({"A": "i1", "B": "i2"})
         .setFetchDict({"Output": "Y"}).setMiniBatchSize(5).setDeviceType("CPU"))
    out = m.transform(DataFrame({"i1": [True, True, False], "i2": [True, False, False]}))
    assert out["Output"].tolist() == [True, False, False]
    t = ONNXModel().setModelPayload(writer.tfidf_counts()).setFeedDict({"text": "features"}) \
        .setFetchDict({"encoded": "result"}).setDeviceType("CPU")
    one = np.empty(1, dtype=object)
    one[0] = ["A", "B", "C"]
    r = t.setMiniBatchSize(10).transform(DataFrame({"features": one}))
    assert np.asarray(r["encoded"][0]).tolist() == [1.0, 1.0, 1.0]
    two = np.empty(2, dtype=object)
    two[0] = ["A", "B", "B", "C", "A"]
    two[1] = ["A", "B", "C"]
    r = t.setMiniBatchSize(1).transform(DataFrame({"features": two}))
    assert np.asarray(r["encoded"][0]).tolist() == [2.0, 2.0, 1.0]
    assert np.asarray(r["encoded"][1]).tolist() == [1.0, 1.0, 1.0]
    with pytest.raises(ValueError):
        t.setMiniBatchSize(10).transform(DataFrame({"features": two}))


def test_onnx_model_slicing_auto_and_manual():
    data = writer.resnet50_v2(seed=3)
    rng = np.random.default_rng(0)
    imgs = np.empty(2, dtype=object)
    for i in range(2):
        imgs[i] = rng.random((3, 224, 224), dtype=np.float32)
    df = DataFrame({"image": imgs})
    m = ONNXModel().setModelPayload(data).setFeedDict({"data": "image"}).setDeviceType("CPU")
    auto = m.copy().setFetchDict({"rawFeatures": "resnetv24_pool1_fwd"})
    assert "resnetv24_pool1_fwd" not in auto.modelOutput
    f = auto.transform(df)["rawFeatures"][0]
    assert np.asarray(f).shape == (2048, 1, 1)
    sliced = m.sliceAtOutput("resnetv24_pool1_fwd").setFetchDict({"rawFeatures": "resnetv24_pool1_fwd"})
    assert "resnetv24_pool1_fwd" in sliced.modelOutput
    np.testing.assert_allclose(np.asarray(sliced.transform(df)["rawFeatures"][1]),
                               np.asarray(auto.transform(df)["rawFeatures"][1]), rtol=1e-5)


def test_tree_ensemble_classifier():
    # two stumps: x0 <= 0.5 -> class weight
    b = GraphBuilder("trees")
    b.input("X", P.FLOAT32, [None, 2])
    b.add("TreeEnsembleClassifier", ["X"], {
        "nodes_treeids": [0, 0, 0, 1, 1, 1], "nodes_nodeids": [0, 1, 2, 0, 1, 2],
        "nodes_featureids": [0, 0, 0, 1, 0, 0], "nodes_values": [0.5, 0, 0, 1.0, 0, 0],
        "nodes_modes": ["BRANCH_LEQ", "LEAF", "LEAF", "BRANCH_LEQ", "LEAF", "LEAF"],
        "nodes_truenodeids": [1, 0, 0, 1, 0, 0], "nodes_falsenodeids": [2, 0, 0, 2, 0, 0],
        "class_treeids": [0, 0, 1, 1], "class_nodeids": [1, 2, 1, 2], "class_ids": [0, 0, 0, 0],
        "class_weights": [-1.0, 1.0, -0.5, 0.5], "classlabels_int64s": [0, 1], "post_transform": "LOGISTIC"},
        n_out=2, domain="ai.onnx.ml", out="te")
    b.nodes[-1].outputs = ["label", "probs"]
    b.output("label", P.INT64, [None])
    b.output("probs", P.FLOAT32, [None, 2])
    X = np.array([[0.0, 0.0], [1.0, 2.0], [0.0, 2.0]], np.float32)
    lab, pr = InferenceSession(b.to_bytes({"": 13, "ai.onnx.ml": 1}), device="cpu").run(None, {"X": X})
    s = np.array([-1.5, 1.5, -0.5])
    np.testing.assert_allclose(pr[:, 1], 1 / (1 + np.exp(-s)), rtol=1e-6)
    assert lab.tolist() == [0, 1, 0]


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_gpu_resnet_matches_cpu_and_graph_replay(monkeypatch):
    data = writer.resnet50_v2(seed=4)
    x = np.random.default_rng(5).random((4, 3, 224, 224), dtype=np.float32)
    cpu = InferenceSession(data, device="cpu").run(None, {"data": x})[0]
    gpu = InferenceSession(data, device="cuda", use_graph=True)
    # every conv (the 3-channel stem included) and the FC run on our MFMA kernels: no library conv / matmul
    lib = []
    for name in ("conv1d", "conv2d", "conv3d"):
        real = getattr(torch.nn.functional, name)
        monkeypatch.setattr(torch.nn.functional, name, lambda *a, _r=real, **k: lib.append(1) or _r(*a, **k))
    real_mm = torch.matmul
    monkeypatch.setattr(torch, "matmul", lambda *a, **k: lib.append(1) or real_mm(*a, **k))
    o1 = gpu.run(None, {"data": x})[0]
    o2 = gpu.run(None, {"data": x})[0]  # HIP graph replay path
    assert not lib, "a library conv / matmul ran on the GPU path"
    scale = np.abs(cpu).max()
    # exact-f32 MFMA convs and GEMM: fp32-level agreement with the CPU graph (was 2e-3 with library kernels)
    np.testing.assert_allclose(o1, cpu, rtol=0, atol=2e-5 * scale)
    # our kernels have no split-K atomics: replays are bitwise identical
    np.testing.assert_array_equal(o1, o2)
    assert any(v != "eager" for v in gpu._graphs.values()), "HIP graph capture fell back to eager"
    # fp32 graphs run the exact f32-input MFMA conv with the pre-activation BN+ReLU folded into its loader
    assert any(n.op_type == "_FusedConv" and len(n.inputs) > 5 and n.inputs[4] for n in gpu.nodes)
    half = InferenceSession(data, device="cuda", precision="fp16").run(None, {"data": x})[0].astype(np.float64)
    assert np.linalg.norm(half - cpu) / np.linalg.norm(cpu) < 3e-3


@pytest.mark.gpu
def test_gpu_epilogue_kernels_match_torch():
    from synapseml_amd.ops import native

    nn = native.load("_nn")
    dev = torch.device("cuda")
    for dtype in (torch.float32, torch.float16, torch.bfloat16):
        x = torch.randn(2, 64, 7, 7, device=dev).to(dtype).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x)
        sc = torch.rand(64, device=dev) + 0.5
        sh = torch.randn(64, device=dev)
        y = torch.empty_like(x)
        nn.affine_act(x.data_ptr(), x.numel(), 64, 49, 1, sc.data_ptr(), sh.data_ptr(), r.data_ptr(), 1, 0.0,
                      {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[dtype], y.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
        ref = torch.relu(x.float() * sc[None, :, None, None] + sh[None, :, None, None] + r.float())
        tol = 1e-5 if dtype == torch.float32 else 2e-2
        torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
        s = torch.empty_like(x)
        a = torch.empty_like(x)
        nn.add_affine_act(x.data_ptr(), r.data_ptr(), x.numel(), 64, 49, 1, sc.data_ptr(), sh.data_ptr(), 1,
                          {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[dtype], s.data_ptr(), a.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
        torch.testing.assert_close(s.float(), (x + r).float(), rtol=tol, atol=tol)
        ref2 = torch.relu((x + r).float() * sc[None, :, None, None] + sh[None, :, None, None])
        torch.testing.assert_close(a.float(), ref2, rtol=tol, atol=tol * 4)


@pytest.mark.gpu
def test_gpu_onnx_model_stage():
    data, coef, inter = _iris_model()
    feats = np.random.default_rng(0).random((37, 4)).astype(np.float32) * 5
    m = (ONNXModel().setModelPayload(data).setFeedDict({"float_input": "features"})
         .setFetchDict({"prediction": "output_label"}).setDeviceType("GPU"))
    out = m.transform(DataFrame({"features": feats}))
    assert out["prediction"].tolist() == (feats @ coef.T + inter).argmax(1).tolist()
    # many prefetch chunks through the pinned staging ring (wraps 3 slots), float64 column cast to the
    # model's float32 input while staging
    feats64 = np.random.default_rng(1).random((1001, 4)) * 5
    out = m.copy().setMiniBatchSize(7).transform(DataFrame({"features": feats64}))
    assert out["prediction"].tolist() == (feats64.astype(np.float32) @ coef.T + inter).argmax(1).tolist()


# ------------------------------------------------------------------ ImageFeaturizer
def _image_df(n=3, seed=0):
    from synapseml_amd.image import encode_png, make_image_row

    rng = np.random.default_rng(seed)
    col = np.empty(n, dtype=object)
    for i in range(n):
        a = rng.integers(0, 256, (60 + 7 * i, 80, 3), dtype=np.uint8)
        col[i] = make_image_row(a) if i % 2 == 0 else encode_png(a)
    return DataFrame({"image": col})


def test_image_featurizer_headless_cpu():
    from synapseml_amd.onnx import ImageFeaturizer

    data = writer.resnet50_v2(seed=7)
    f = (ImageFeaturizer(inputCol="image", outputCol="features", featureTensorName="resnetv24_pool1_fwd",
                         outputTensorName="resnetv24_dense0_fwd", imageTensorName="data")
         .setModel(data))
    f.getOnnxModel().setDeviceType("CPU")
    df = _image_df()
    out = f.transform(df)
    v = out["features"][0]
    assert isinstance(v, DenseVector) and len(v.toArray()) == 2048
    head = f.copy().setHeadless(False).transform(df)["features"][1]
    assert len(head.toArray()) == 1000


@pytest.mark.gpu
def test_image_featurizer_gpu_matches_cpu():
    from synapseml_amd.onnx import ImageFeaturizer

    data = writer.resnet50_v2(seed=8)
    df = _image_df(n=5, seed=1)

    def run(dev):
        f = ImageFeaturizer(inputCol="image", outputCol="features", featureTensorName="resnetv24_pool1_fwd",
                            imageTensorName="data").setModel(data)
        f.getOnnxModel().setDeviceType(dev)
        return np.stack([v.toArray() for v in f.transform(df)["features"]])

    g, c = run("GPU"), run("CPU")
    # fused preprocess is bit-exact with the host stages and the MFMA convs / GEMM are exact-f32 (measured
    # 1.6e-6 max relative error of the whole network on MI355X)
    np.testing.assert_allclose(g, c, rtol=0, atol=2e-5 * np.abs(c).max())


def test_prologue_fusion_pass_cpu_fallback():
    """The MFMA prologue/residual rewrite (normally GPU-only) applied on CPU: the fallback runtime path must give
    the same numbers, and the v2 pre-activations disappear from the graph."""
    data = writer.resnet50_v2(seed=11)
    x = np.random.default_rng(12).random((1, 3, 64, 64), dtype=np.float32)
    sess = InferenceSession(data, device="cpu")
    ref = sess.run(None, {"data": x})[0]
    before = [n.op_type for n in sess.nodes]
    sess.nodes = sess._fuse_prologues(sess.nodes)
    sess._plan_liveness()
    after = [n.op_type for n in sess.nodes]
    assert after.count("_AffineAct") < before.count("_AffineAct")
    assert after.count("_AddAffineAct") < before.count("_AddAffineAct")
    assert sum(1 for n in sess.nodes if n.op_type == "_FusedConv" and len(n.inputs) > 5) >= 16
    out = sess.run(None, {"data": x})[0]
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["fp16", "bf16"])
def test_gpu_mfma_fused_resnet_matches_cpu(prec):
    data = writer.resnet50_v2(seed=13)
    x = np.random.default_rng(14).random((8, 3, 224, 224), dtype=np.float32)
    cpu = InferenceSession(data, device="cpu").run(None, {"data": x})[0]
    sess = InferenceSession(data, device="cuda", precision=prec)
    fused = [n for n in sess.nodes if n.op_type == "_FusedConv" and len(n.inputs) > 5]
    assert len(fused) >= 16  # pre-activations folded into MFMA conv prologues
    # the input BatchNormalization rides the stem kernel's im2col (no separate affine pass over the images)
    stem = [n for n in sess.nodes if sess._stem_conv_node(n)]
    assert len(stem) == 1 and stem[0].inputs[0] == "data" and len(stem[0].inputs) == 6
    out = sess.run(None, {"data": x})[0].astype(np.float64)
    # relative L2 error of the logits vs the fp32 host graph: measured 7.3e-4 (fp16) / 5.4e-3 (bf16) on
    # MI355X, i.e. the rounding of the storage format; a wrong fusion (dropped bias, BN or residual) is O(1)
    rel = np.linalg.norm(out - cpu) / np.linalg.norm(cpu)
    assert rel < (3e-3 if prec == "fp16" else 2e-2), rel
    assert (out.argmax(1) == cpu.argmax(1)).mean() >= 7 / 8


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["float16", "bfloat16", "float32"])
def test_gpu_maxpool_nhwc_kernel_matches_torch(dtype):
    """K16: the NHWC max-pool kernel (ResNet stem 3x3/2 pad 1, and 2x2/2) against torch's max_pool2d."""
    import torch

    from synapseml_amd.ops import native

    nn = native.load("_nn")
    dt = getattr(torch, dtype)
    code = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[dt]
    for (n, c, h, w, k, s, p) in ((4, 64, 112, 112, 3, 2, 1), (2, 32, 15, 9, 2, 2, 0)):
        x = torch.randn(n, c, h, w, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        ref = torch.nn.functional.max_pool2d(x.float(), k, s, p)
        oh, ow = ref.shape[2:]
        y = torch.empty((n, c, oh, ow), dtype=dt, device="cuda", memory_format=torch.channels_last)
        nn.maxpool_nhwc(x.data_ptr(), n, h, w, c, k, k, s, s, p, p, oh, ow, code, y.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(y.float(), ref.to(dt).float())
        # fused epilogue (a stem conv's bias + ReLU moved past the pool): bitwise the unfused order, since
        # rounding x + b and ReLU are monotone and commute with max
        b = torch.randn(c, device="cuda")
        unfused = torch.nn.functional.max_pool2d(torch.relu(x.float() + b.view(1, -1, 1, 1)).to(dt).float(), k, s, p)
        y2 = torch.empty_like(y)
        nn.maxpool_nhwc(x.data_ptr(), n, h, w, c, k, k, s, s, p, p, oh, ow, code, y2.data_ptr(),
                        torch.cuda.current_stream().cuda_stream, b.data_ptr(), 1)
        torch.cuda.synchronize()
        assert torch.equal(y2.float(), unfused)


@pytest.mark.gpu
def test_gpu_stem_epilogue_moves_past_maxpool():
    """ResNet-50 v2 on the GPU: the library stem conv's bias + ReLU run inside the max-pool kernel, the last
    add + BN + ReLU is the final conv's dual output, and the session output still matches the unfused host
    execution (fp32 and fp16)."""
    data = writer.resnet50_v2(seed=7)
    x = np.random.default_rng(8).random((2, 3, 224, 224), dtype=np.float32)
    gpu = InferenceSession(data, device="cuda")
    pools = [n for n in gpu.nodes if n.op_type == "MaxPool"]
    stem = [n for n in gpu.nodes if gpu._stem_conv_node(n)]
    if stem:  # fp32 on bf16 planes: the stem kernel takes the input BN as its prologue, bias + ReLU in its epilogue
        assert len(stem) == 1 and stem[0].inputs[0] == "data" and len(stem[0].inputs) == 6
        assert stem[0].attrs.get("__act") == 1 and pools and len(pools[0].inputs) == 1
    else:
        assert pools and len(pools[0].inputs) == 2 and pools[0].attrs.get("__act") == 1
    # the last block's residual add + post-activation BN + ReLU: the final conv's second output
    assert any(n.op_type == "_FusedConv" and len(n.outputs) == 2 and len(n.inputs) == 8 for n in gpu.nodes)
    cpu = InferenceSession(data, device="cpu").run(None, {"data": x})[0]
    out = gpu.run(None, {"data": x})[0]
    np.testing.assert_allclose(out, cpu, rtol=0, atol=2e-5 * np.abs(cpu).max())
    half = InferenceSession(data, device="cuda", precision="fp16").run(None, {"data": x})[0].astype(np.float64)
    assert np.linalg.norm(half - cpu) / np.linalg.norm(cpu) < 3e-3


@pytest.mark.gpu
def test_gpu_featurizer_encoded_bytes_match_decoded_rows():
    """ImageFeaturizer on encoded PNG bytes (decoded in RGB order, the channel flip folded into the fused
    preprocess kernel's channel map) equals the features of the same images given as decoded OpenCV rows."""
    from synapseml_amd.core.dataframe import DataFrame
    from synapseml_amd.image import encode_png, make_image_row
    from synapseml_amd.onnx import ImageFeaturizer, writer

    rng = np.random.default_rng(4)
    imgs = [rng.integers(0, 256, (96 + 8 * i, 112, 3), dtype=np.uint8) for i in range(6)]
    rows = np.empty(6, dtype=object)
    pngs = np.empty(6, dtype=object)
    for i, a in enumerate(imgs):
        rows[i] = make_image_row(a)
        pngs[i] = encode_png(a)
    model = writer.resnet50_v2(seed=0)

    def feats(col):
        f = ImageFeaturizer(inputCol="image", outputCol="features", featureTensorName="resnetv24_pool1_fwd",
                            imageTensorName="data").setModel(model)
        f.getOnnxModel().setPrecision("fp32").setDeviceType("gpu")
        return np.stack([v.toArray() for v in f.transform(DataFrame({"image": col}))["features"]])

    np.testing.assert_allclose(feats(pngs), feats(rows), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_gpu_graph_capture_records_work_or_runs_eager():
    """HIP-graph replay (session._capture) is only kept when the captured graph has nodes; a plan whose work
    did not reach the capture stream runs eagerly, so a replay never returns stale capture-time buffers."""
    from synapseml_amd.onnx.session import _graph_num_nodes

    data, coef, inter = _iris_model()
    s = InferenceSession(data, device="cuda", use_graph=True)
    for seed in (0, 1, 2):
        x = np.random.default_rng(seed).random((64, 4)).astype(np.float32) * 5
        label = s.run(["output_label"], {"float_input": x})[0]
        assert np.asarray(label).tolist() == (x @ coef.T + inter).argmax(1).tolist()
    # the ZipMap output (a sequence of host dicts) makes the plan non-graphable: it never captures
    assert not s._graphable({"float_input": x}) and not s._graphs
    # LinearClassifier alone (integer labels gathered on the device, coefficients cached on the device)
    # captures a non-empty graph whose replays track new inputs
    b = GraphBuilder("lc")
    b.input("float_input", P.FLOAT32, [None, 4])
    b.add("LinearClassifier", ["float_input"], {"coefficients": [float(v) for v in np.ravel(coef)],
                                                "intercepts": [float(v) for v in inter],
                                                "classlabels_ints": [0, 1, 2], "post_transform": "SOFTMAX"},
          n_out=2, domain="ai.onnx.ml", out="lc")
    b.nodes[-1].outputs = ["output_label", "probabilities"]
    b.output("output_label", P.INT64, [None])
    b.output("probabilities", P.FLOAT32, [None, 3])
    s1 = InferenceSession(b.to_bytes({"": 13, "ai.onnx.ml": 1}), device="cuda", use_graph=True)
    for seed in (5, 6, 7):
        x = np.random.default_rng(seed).random((64, 4)).astype(np.float32) * 5
        label = s1.run(["output_label"], {"float_input": x})[0]
        label = label.cpu().numpy() if torch.is_tensor(label) else np.asarray(label)
        assert label.tolist() == (x @ coef.T + inter).argmax(1).tolist()
    entry = next(iter(s1._graphs.values()))
    assert entry != "eager" and _graph_num_nodes(entry[0]) > 0
    # a plain tensor graph is replayed from a non-empty capture with fresh results per batch
    b = GraphBuilder("lin")
    b.input("x", P.FLOAT32, ["N", 4])
    w = b.init("w", np.eye(4, dtype=np.float32) * 2)
    y = b.add("MatMul", ["x", w])
    b.add("Relu", [y], out="z")
    b.output("z", P.FLOAT32, ["N", 4])
    s2 = InferenceSession(b.to_bytes(), device="cuda", use_graph=True)
    for seed in (3, 4):
        x = np.random.default_rng(seed).standard_normal((32, 4)).astype(np.float32)
        out = s2.run(None, {"x": x})[0]
        out = out.cpu().numpy() if torch.is_tensor(out) else np.asarray(out)
        np.testing.assert_allclose(out, np.maximum(2 * x, 0), rtol=1e-6)
    entry = next(iter(s2._graphs.values()))
    assert entry != "eager" and _graph_num_nodes(entry[0]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.bfloat16])
def test_gpu_global_average_pool_kernel(dt):
    """GlobalAveragePool on channels-last device tensors runs the HIP kernel (fp32 accumulation, output in the
    input dtype) and equals an fp32 torch mean."""
    b = GraphBuilder("gap")
    b.input("x", P.FLOAT32, ["N", 64, 7, 7])
    b.add("GlobalAveragePool", ["x"], out="y")
    b.output("y", P.FLOAT32, ["N", 64, 1, 1])
    s = InferenceSession(b.to_bytes(), device="cuda", use_graph=False)
    x = torch.randn(16, 64, 7, 7, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    from synapseml_amd.onnx import ops

    class _RT:
        session = s
        node_outputs = ["y"]

    y = ops.OPS["GlobalAveragePool"](_RT(), {}, [x])[0]
    assert y.dtype == dt and y.shape == (16, 64, 1, 1)
    ref = x.float().mean(dim=(2, 3), keepdim=True)
    tol = 1e-6 if dt == torch.float32 else 1e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


def test_conv_split_k_plan():
    """Split-K planning (host side of csrc/nn/conv_mfma.hip ConvSplitPlan; opt-in, SML_CONV_SPLITK): the deep few-tile layers of
    ResNet-50 at batch 128 split K (>= 512 blocks, >= 4 K tiles per split, <= 8 splits), the early
    many-tile layers and forced tiles do not, and the workspace is one fp32 partial tile per split."""
    from synapseml_amd.ops import native

    nn = native.load("_nn")

    def plan(C, H, Co, k, B=128, dt=1, kernel=0, pro=True):  # prologue layers (the others stage by LDS-DMA)
        pd = k // 2
        g = [B, H, H, C, Co, k, k, 1, 1, pd, pd, 1, 1, H, H]
        return nn.conv_split_plan(g, dt, pro, kernel)

    assert plan(64, 56, 256, 1) == (1, 0, 0)             # 6272 tiles, one K tile
    assert plan(256, 14, 256, 3) == (2, 392 * 2 * 128 * 128, 392)
    assert plan(512, 7, 512, 3) == (3, 196 * 3 * 128 * 128, 196)
    assert plan(512, 7, 512, 3, kernel=128128)[0] == 1  # forced tiles never split
    assert plan(512, 7, 2048, 1)[0] == 1                 # 784 tiles
    sk, wsf, cnt = plan(512, 7, 512, 3, B=1)            # batch 1: 4 tiles, 72 K tiles -> 8 splits
    assert (sk, cnt) == (8, 4) and wsf == 4 * 8 * 128 * 128
    sk, wsf, cnt = plan(128, 7, 64, 3, B=1)              # Cout <= 64: 64x64 tiles, 18 K tiles -> 4 splits
    assert (sk, cnt) == (4, 1) and wsf == 4 * 64 * 64
    assert plan(64, 7, 64, 1, B=1)[0] == 1               # too short a K loop
    assert plan(256, 14, 256, 3, dt=4)[0] == 2           # fp32 on bf16 planes: 32-wide K tiles
    assert plan(256, 14, 256, 3, pro=False)[0] == 1      # f16 without a prologue: the LDS-DMA form, no split


def test_stem_weight_packing_order():
    """pack_stem_weight: k = (r * S + s) * C + c, zero tail to 160 (the stem kernel's im2col order); the
    3-channel row-run form: k = r * 24 + s * 3 + c, zero in the slots past S * 3 and past R * 24."""
    from synapseml_amd.ops.conv import STEM_KP, STEM_WIDE_KP, pack_stem_weight, stem_wide

    w = torch.arange(2 * 4 * 5 * 5, dtype=torch.float32).reshape(2, 4, 5, 5)
    assert not stem_wide(w)
    wk = pack_stem_weight(w)
    assert wk.shape == (2, STEM_KP)
    r, s_, c = 4, 3, 2
    assert wk[1, (r * 5 + s_) * 4 + c] == w[1, c, r, s_]
    assert torch.all(wk[:, 100:] == 0)
    w7 = torch.arange(2 * 3 * 7 * 7, dtype=torch.float32).reshape(2, 3, 7, 7) + 1
    assert stem_wide(w7)
    assert pack_stem_weight(w7).shape == (2, STEM_KP)  # the gather form unless SML_STEM_ROWRUN=1
    wk7 = pack_stem_weight(w7, wide=True)
    assert wk7.shape == (2, STEM_WIDE_KP)
    for (r, s_, c) in ((0, 0, 0), (4, 5, 2), (6, 6, 1)):
        assert wk7[1, r * 24 + s_ * 3 + c] == w7[1, c, r, s_]
    lay = wk7.reshape(2, 8, 24)
    assert torch.all(lay[:, :7, 21:] == 0) and torch.all(lay[:, 7:] == 0)
    assert int((wk7 != 0).sum()) == w7.numel()


def test_onnx_model_transform_fans_out_over_partitions(monkeypatch):
    """ONNXModel.transform maps the partitions, one task per executor (ONNXModel.scala:242-251): with two
    executor tasks a 3-partition DataFrame is transformed in 2 processes, rows in order, same outputs."""
    data, coef, inter = _iris_model()
    rng = np.random.default_rng(3)
    feats = rng.normal(4, 2, (60, 4)).astype(np.float32)
    df = DataFrame({"features": feats, "id": np.arange(60.0)}, num_partitions=3)
    m = (ONNXModel().setModelPayload(data).setFeedDict({"float_input": "features"})
         .setFetchDict({"prediction": "output_label"}).setDeviceType("CPU"))
    single = m.transform(df)
    from synapseml_amd.parallel import runtime as R

    monkeypatch.setenv("SML_EXECUTOR_TASKS", "2")
    calls = []
    real = R.fan_out_transform
    monkeypatch.setattr(R, "fan_out_transform", lambda *a, **k: calls.append(a[2]) or real(*a, **k))
    m.transform(df)
    assert calls == []  # 60 rows: below the per-task row threshold, scored in this process
    with pytest.raises(ValueError, match="not in the DataFrame"):  # validated before any fan-out
        m.copy().setFeedDict({next(iter(m.modelInput)): "nope"}).transform(df)
    monkeypatch.setenv("SML_TRANSFORM_MIN_ROWS", "1")
    out = m.transform(df)
    assert calls == [2]
    assert out["id"].tolist() == list(range(60))
    assert out["prediction"].tolist() == single["prediction"].tolist() == (feats @ coef.T + inter).argmax(1).tolist()
