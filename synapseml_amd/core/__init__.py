from .dataframe import DataFrame, GroupedData, Row, createDataFrame
from .linalg import DenseVector, SparseVector, Vector, Vectors
from .params import Param, Params, TypeConverters
from .pipeline import Estimator, Evaluator, Model, Pipeline, PipelineModel, PipelineStage, Transformer

__all__ = [
    "DataFrame", "GroupedData", "Row", "createDataFrame", "DenseVector", "SparseVector", "Vector", "Vectors",
    "Param", "Params", "TypeConverters", "Estimator", "Evaluator", "Model", "Pipeline", "PipelineModel",
    "PipelineStage", "Transformer",
]
