"""synapseml_amd: an MI355X-native distributed ML-on-DataFrame framework with
the capabilities and API surface of SynapseML (LightGBM-style boosting, Vowpal
Wabbit-style hashed learning, ONNX inference, image transforms, pipeline
stages), built on hand-written HIP/CDNA4 kernels and RCCL over xGMI."""

__version__ = "0.1.0"

from .core import (DataFrame, DenseVector, Estimator, Model, Pipeline, PipelineModel, Row, SparseVector, Transformer,
                   Vectors, createDataFrame)

__all__ = [
    "DataFrame", "DenseVector", "Estimator", "Model", "Pipeline", "PipelineModel", "Row", "SparseVector",
    "Transformer", "Vectors", "createDataFrame", "__version__",
]
