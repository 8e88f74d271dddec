"""ONNX inference on the MI355X (reference: deep-learning/ onnx package):
own protobuf codec + graph IR, an optimizing executor (constant folding,
Conv/BN folding, fused HIP epilogues, hipGraph replay) standing in for ONNX
Runtime, and the ONNXModel / ImageFeaturizer / ONNXHub stages."""
from .graph import Graph, Node, ValueInfo
from .model import ImageFeaturizer, ONNXHub, ONNXModel, ONNXModelInfo, get_session
from .session import InferenceSession
from . import writer

__all__ = ["Graph", "Node", "ValueInfo", "ImageFeaturizer", "ONNXHub", "ONNXModel", "ONNXModelInfo",
           "InferenceSession", "get_session", "writer"]
