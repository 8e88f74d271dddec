"""ONNX model builder (our own writer — no ``onnx`` package here) and a
small synthetic model zoo with random-init weights for tests and benchmarks:

* ``resnet50_v2`` — the topology and tensor names of the ONNX model zoo's
  ``resnet50-v2-7`` (pre-activation bottlenecks, ``resnetv24_*`` names, input
  ``data`` [N,3,224,224], ``resnetv24_pool1_fwd`` [N,2048,1,1],
  ``resnetv24_dense0_fwd`` [N,1000]); the reference's north-star model
  (deep-learning/src/test/.../onnx/ONNXModelSuite.scala:352-407).
* ``mnist_cnn`` — the mnist-8 layout (Conv/Relu/MaxPool ×2 → Reshape → MatMul).
* ``linear_classifier_zipmap`` — sklearn-onnx style ``LinearClassifier`` +
  ``ZipMap`` (iris / adults-income style outputs ``output_label``,
  ``output_probability``).
* ``boolean_and`` — GH1996 (bool in → bool out).
* ``tfidf_counts`` — ``TfIdfVectorizer`` over string tokens (variable length).
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Sequence

import numpy as np

from . import proto as P
from .graph import Node, ValueInfo


def make_attr(name: str, v: Any) -> P.Message:
    a = P.Message("AttributeProto", name=name)
    if isinstance(v, bool):
        v = int(v)
    if isinstance(v, float) or isinstance(v, np.floating):
        a.type, a.f = P.A_FLOAT, float(v)
    elif isinstance(v, (int, np.integer)):
        a.type, a.i = P.A_INT, int(v)
    elif isinstance(v, str):
        a.type, a.s = P.A_STRING, v.encode("utf-8")
    elif isinstance(v, bytes):
        a.type, a.s = P.A_STRING, v
    elif isinstance(v, np.ndarray):
        a.type, a.t = P.A_TENSOR, P.numpy_to_tensor(v)
    elif isinstance(v, (list, tuple)):
        if all(isinstance(x, (int, np.integer)) and not isinstance(x, bool) for x in v):
            a.type, a.ints = P.A_INTS, [int(x) for x in v]
        elif all(isinstance(x, (int, float, np.number)) for x in v):
            a.type, a.floats = P.A_FLOATS, [float(x) for x in v]
        elif all(isinstance(x, str) for x in v):
            a.type, a.strings = P.A_STRINGS, [x.encode("utf-8") for x in v]
        else:
            raise TypeError(f"unsupported list attribute {name}")
    else:
        from .graph import Graph

        if isinstance(v, Graph):
            a.type = P.A_GRAPH
            a.g = make_graph(v.nodes, v.name or name, v.inputs, v.outputs, v.initializers)
        else:
            raise TypeError(f"unsupported attribute {name}: {type(v)}")
    return a


def make_value_info(vi: ValueInfo) -> P.Message:
    def tensor_type(elem, shape):
        tt = P.Message("TypeProto.Tensor", elem_type=elem)
        if shape is not None:
            dims = []
            for s in shape:
                d = P.Message("TensorShapeProto.Dimension")
                if isinstance(s, str):
                    d.dim_param = s
                elif s is not None:
                    d.dim_value = int(s)
                dims.append(d)
            tt.shape = P.Message("TensorShapeProto", dim=dims)
        return P.Message("TypeProto", tensor_type=tt)

    if vi.kind == "tensor":
        tp = tensor_type(vi.elem_type, vi.shape)
    elif vi.kind == "map":
        tp = P.Message("TypeProto", map_type=P.Message("TypeProto.Map", key_type=vi.key_type,
                                                       value_type=tensor_type(vi.elem_type, None)))
    else:
        if vi.seq_of_maps:
            inner = P.Message("TypeProto", map_type=P.Message("TypeProto.Map", key_type=vi.key_type,
                                                              value_type=tensor_type(vi.elem_type, None)))
        else:
            inner = tensor_type(vi.elem_type, None)
        tp = P.Message("TypeProto", sequence_type=P.Message("TypeProto.Sequence", elem_type=inner))
    return P.Message("ValueInfoProto", name=vi.name, type=tp)


def make_graph(nodes: Iterable[Node], name: str, inputs: Sequence[ValueInfo], outputs: Sequence[ValueInfo],
               initializers: Optional[Dict[str, np.ndarray]] = None, value_info: Sequence[ValueInfo] = ()) -> P.Message:
    g = P.Message("GraphProto", name=name)
    for n in nodes:
        g.node.append(P.Message("NodeProto", input=list(n.inputs), output=list(n.outputs), name=n.name,
                                op_type=n.op_type, domain=n.domain,
                                attribute=[make_attr(k, v) for k, v in n.attrs.items() if not k.startswith("__")]))
    for k, v in (initializers or {}).items():
        g.initializer.append(P.numpy_to_tensor(v, k))
    g.input = [make_value_info(v) for v in inputs]
    g.output = [make_value_info(v) for v in outputs]
    g.value_info = [make_value_info(v) for v in value_info]
    return g


def make_model(graph: P.Message, opset: Optional[Dict[str, int]] = None, ir_version: int = 7,
               producer: str = "synapseml_amd") -> P.Message:
    opset = opset or {"": 13}
    return P.Message("ModelProto", ir_version=ir_version, producer_name=producer, graph=graph,
                     opset_import=[P.Message("OperatorSetIdProto", domain=d, version=v) for d, v in opset.items()])


class GraphBuilder:
    """Tiny imperative builder: ``b.add("Conv", [x, w], attrs) -> out name``."""

    def __init__(self, name: str = "graph"):
        self.name = name
        self.nodes: List[Node] = []
        self.inits: Dict[str, np.ndarray] = {}
        self.inputs: List[ValueInfo] = []
        self.outputs: List[ValueInfo] = []
        self._n = 0

    def input(self, name: str, elem_type: int = P.FLOAT32, shape=None, kind: str = "tensor") -> str:
        self.inputs.append(ValueInfo(name, kind=kind, elem_type=elem_type, shape=shape))
        return name

    def init(self, name: str, arr: np.ndarray) -> str:
        self.inits[name] = np.asarray(arr)
        return name

    def add(self, op: str, inputs: Sequence[str], attrs: Optional[dict] = None, out: Optional[str] = None,
            n_out: int = 1, domain: str = "", name: Optional[str] = None):
        self._n += 1
        outs = [out] if out and n_out == 1 else [f"{out or op.lower()}_{self._n}_{i}" for i in range(n_out)]
        self.nodes.append(Node(op, list(inputs), outs, dict(attrs or {}), name or f"{op}_{self._n}", domain))
        return outs[0] if n_out == 1 else outs

    def output(self, name: str, elem_type: int = P.FLOAT32, shape=None, kind: str = "tensor", key_type: int = 0,
               seq_of_maps: bool = False) -> None:
        self.outputs.append(ValueInfo(name, kind=kind, elem_type=elem_type, shape=shape, key_type=key_type,
                                      seq_of_maps=seq_of_maps))

    def to_bytes(self, opset: Optional[Dict[str, int]] = None) -> bytes:
        g = make_graph(self.nodes, self.name, self.inputs, self.outputs, self.inits)
        return P.encode(make_model(g, opset=opset))


# ------------------------------------------------------------------ zoo
def _he(rng, shape):
    fan_in = int(np.prod(shape[1:]))
    return (rng.standard_normal(shape) * np.sqrt(2.0 / fan_in)).astype(np.float32)


def _bn(b: GraphBuilder, rng, x: str, c: int, name: str, out: str) -> str:
    gamma = b.init(f"{name}_gamma", (1.0 + 0.1 * rng.standard_normal(c)).astype(np.float32))
    beta = b.init(f"{name}_beta", (0.1 * rng.standard_normal(c)).astype(np.float32))
    mean = b.init(f"{name}_running_mean", (0.1 * rng.standard_normal(c)).astype(np.float32))
    var = b.init(f"{name}_running_var", (1.0 + 0.1 * rng.random(c)).astype(np.float32))
    return b.add("BatchNormalization", [x, gamma, beta, mean, var], {"epsilon": 1e-5}, out=out, name=name)


def _conv(b: GraphBuilder, rng, x: str, cin: int, cout: int, k: int, s: int, name: str, out: str) -> str:
    w = b.init(f"{name}_weight", _he(rng, (cout, cin, k, k)))
    return b.add("Conv", [x, w], {"kernel_shape": [k, k], "strides": [s, s], "pads": [k // 2] * 4,
                                  "dilations": [1, 1], "group": 1}, out=out, name=name)


def resnet50_v2(seed: int = 0, num_classes: int = 1000) -> bytes:
    """ResNet-50 v2 (pre-activation) with the model zoo's tensor names."""
    rng = np.random.default_rng(seed)
    b = GraphBuilder("resnet50_v2")
    p = "resnetv24"
    x = b.input("data", P.FLOAT32, ["N", 3, 224, 224])
    x = _bn(b, rng, x, 3, f"{p}_batchnorm0", f"{p}_batchnorm0_fwd")
    x = _conv(b, rng, x, 3, 64, 7, 2, f"{p}_conv0", f"{p}_conv0_fwd")
    x = _bn(b, rng, x, 64, f"{p}_batchnorm1", f"{p}_batchnorm1_fwd")
    x = b.add("Relu", [x], out=f"{p}_relu0_fwd")
    x = b.add("MaxPool", [x], {"kernel_shape": [3, 3], "strides": [2, 2], "pads": [1, 1, 1, 1]},
              out=f"{p}_pool0_fwd")
    cin = 64
    for si, (nblk, cout) in enumerate(zip([3, 4, 6, 3], [256, 512, 1024, 2048])):
        mid = cout // 4
        for bi in range(nblk):
            stride = 2 if (bi == 0 and si > 0) else 1
            sp = f"{p}_stage{si + 1}"
            bn1 = _bn(b, rng, x, cin, f"{sp}_batchnorm{3 * bi}", f"{sp}_batchnorm{3 * bi}_fwd")
            a1 = b.add("Relu", [bn1], out=f"{sp}_activation{3 * bi}")
            if bi == 0:
                sc = _conv(b, rng, a1, cin, cout, 1, stride, f"{sp}_downsample", f"{sp}_downsample_fwd")
            else:
                sc = x
            c1 = _conv(b, rng, a1, cin, mid, 1, 1, f"{sp}_conv{3 * bi}", f"{sp}_conv{3 * bi}_fwd")
            bn2 = _bn(b, rng, c1, mid, f"{sp}_batchnorm{3 * bi + 1}", f"{sp}_batchnorm{3 * bi + 1}_fwd")
            a2 = b.add("Relu", [bn2], out=f"{sp}_activation{3 * bi + 1}")
            c2 = _conv(b, rng, a2, mid, mid, 3, stride, f"{sp}_conv{3 * bi + 1}", f"{sp}_conv{3 * bi + 1}_fwd")
            bn3 = _bn(b, rng, c2, mid, f"{sp}_batchnorm{3 * bi + 2}", f"{sp}_batchnorm{3 * bi + 2}_fwd")
            a3 = b.add("Relu", [bn3], out=f"{sp}_activation{3 * bi + 2}")
            c3 = _conv(b, rng, a3, mid, cout, 1, 1, f"{sp}_conv{3 * bi + 2}", f"{sp}_conv{3 * bi + 2}_fwd")
            x = b.add("Add", [c3, sc], out=f"{sp}__plus{bi}")
            cin = cout
    x = _bn(b, rng, x, cin, f"{p}_batchnorm2", f"{p}_batchnorm2_fwd")
    x = b.add("Relu", [x], out=f"{p}_relu1_fwd")
    x = b.add("GlobalAveragePool", [x], out=f"{p}_pool1_fwd")
    shape = b.init("flatten_shape", np.array([0, -1], dtype=np.int64))
    x = b.add("Reshape", [x, shape], out=f"{p}_flatten0_reshape0")
    w = b.init(f"{p}_dense0_weight", (rng.standard_normal((num_classes, 2048)) * 0.02).astype(np.float32))
    bias = b.init(f"{p}_dense0_bias", np.zeros(num_classes, np.float32))
    b.add("Gemm", [x, w, bias], {"alpha": 1.0, "beta": 1.0, "transA": 0, "transB": 1}, out=f"{p}_dense0_fwd")
    b.output(f"{p}_dense0_fwd", P.FLOAT32, ["N", num_classes])
    return b.to_bytes({"": 7})


def mnist_cnn(seed: int = 0) -> bytes:
    rng = np.random.default_rng(seed)
    b = GraphBuilder("mnist")
    x = b.input("Input3", P.FLOAT32, [1, 1, 28, 28])
    w1 = b.init("Parameter5", _he(rng, (8, 1, 5, 5)))
    b1 = b.init("Parameter6", np.zeros((8, 1, 1), np.float32))
    x = b.add("Conv", [x, w1], {"kernel_shape": [5, 5], "strides": [1, 1], "auto_pad": "SAME_UPPER"}, out="Conv26")
    x = b.add("Add", [x, b1], out="Plus28")
    x = b.add("Relu", [x], out="ReLU32")
    x = b.add("MaxPool", [x], {"kernel_shape": [2, 2], "strides": [2, 2]}, out="Pooling66")
    w2 = b.init("Parameter87", _he(rng, (16, 8, 5, 5)))
    b2 = b.init("Parameter88", np.zeros((16, 1, 1), np.float32))
    x = b.add("Conv", [x, w2], {"kernel_shape": [5, 5], "strides": [1, 1], "auto_pad": "SAME_UPPER"}, out="Conv110")
    x = b.add("Add", [x, b2], out="Plus112")
    x = b.add("Relu", [x], out="ReLU114")
    x = b.add("MaxPool", [x], {"kernel_shape": [3, 3], "strides": [3, 3]}, out="Pooling160")
    shp = b.init("Pooling160_Output_0_reshape0_shape", np.array([1, 256], np.int64))
    x = b.add("Reshape", [x, shp], out="Pooling160_Output_0_reshape0")
    w3 = b.init("Parameter193_reshape1", (rng.standard_normal((256, 10)) * 0.05).astype(np.float32))
    x = b.add("MatMul", [x, w3], out="Times212")
    b3 = b.init("Parameter194", np.zeros((1, 10), np.float32))
    b.add("Add", [x, b3], out="Plus214_Output_0")
    b.output("Plus214_Output_0", P.FLOAT32, [1, 10])
    return b.to_bytes({"": 8})


def linear_classifier_zipmap(coef: np.ndarray, intercept: np.ndarray, classes: Sequence[int],
                             input_name: str = "float_input", post_transform: str = "SOFTMAX") -> bytes:
    """sklearn-onnx LogisticRegression export shape: LinearClassifier + ZipMap."""
    b = GraphBuilder("linear_classifier")
    nf = coef.shape[1]
    x = b.input(input_name, P.FLOAT32, [None, nf])
    lab, prob = b.add("LinearClassifier", [x], {"coefficients": [float(v) for v in np.ravel(coef)],
                                                "intercepts": [float(v) for v in np.ravel(intercept)],
                                                "classlabels_ints": [int(c) for c in classes], "multi_class": 1,
                                                "post_transform": post_transform},
                      n_out=2, domain="ai.onnx.ml", out="lc")
    b.nodes[-1].outputs = ["output_label", "probabilities"]
    b.add("ZipMap", ["probabilities"], {"classlabels_int64s": [int(c) for c in classes]}, out="output_probability",
          domain="ai.onnx.ml")
    b.output("output_label", P.INT64, [None])
    b.output("output_probability", P.FLOAT32, None, kind="sequence", key_type=P.INT64, seq_of_maps=True)
    return b.to_bytes({"": 13, "ai.onnx.ml": 1})


def boolean_and() -> bytes:
    b = GraphBuilder("gh1996")
    b.input("A", P.BOOL, [None])
    b.input("B", P.BOOL, [None])
    b.add("And", ["A", "B"], out="Y")
    b.output("Y", P.BOOL, [None])
    return b.to_bytes({"": 13})


def tfidf_counts(vocab: Sequence[str] = ("A", "B", "C")) -> bytes:
    b = GraphBuilder("tfidf")
    b.input("text", P.STRING_T, [None])
    b.add("TfIdfVectorizer", ["text"], {"mode": "TF", "min_gram_length": 1, "max_gram_length": 1,
                                        "max_skip_count": 0, "ngram_counts": [0],
                                        "ngram_indexes": list(range(len(vocab))), "pool_strings": list(vocab)},
          out="result", domain="")
    b.output("result", P.FLOAT32, [len(vocab)])
    return b.to_bytes({"": 13})
