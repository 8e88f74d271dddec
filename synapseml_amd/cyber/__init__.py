"""Cyber-security analytics (reference: core/src/main/python/synapse/ml/cyber/**)."""
from .anomaly import (AccessAnomaly, AccessAnomalyConfig, AccessAnomalyModel, ComplementAccessTransformer,
                      ConnectedComponents)
from .dataset import DataFactory
from .feature import (IdIndexer, IdIndexerModel, LinearScalarScaler, LinearScalarScalerModel, MultiIndexer,
                      MultiIndexerModel, StandardScalarScaler, StandardScalarScalerModel)

__all__ = [n for n in dir() if not n.startswith("_")]
