"""Fluent DataFrame helpers (reference: core/src/main/python/synapse/ml/core/spark/
FluentAPI.py): ``df.mlTransform(stage, ...)`` applies transformers in order,
``df.mlFit(estimator)`` fits. Installed on import of this module."""
from __future__ import annotations

from ..core.dataframe import DataFrame


def _ml_transform(self, *stages):
    df = self
    for t in stages:
        df = t.transform(df)
    return df


def _ml_fit(self, estimator):
    return estimator.fit(self)


DataFrame.mlTransform = _ml_transform  # type: ignore[attr-defined]
DataFrame.mlFit = _ml_fit  # type: ignore[attr-defined]

__all__ = []
