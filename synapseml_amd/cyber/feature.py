"""Cyber feature engineering: per-partition id indexers and scalar scalers
(reference: core/src/main/python/synapse/ml/cyber/feature/{indexers,
scalers}.py).

``partitionKey`` (e.g. the tenant) makes every statistic / index local to a
partition value; ``None`` computes them over the whole frame."""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from ..core.dataframe import DataFrame
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Estimator, Model, Transformer


def _keys(df: DataFrame, partition_key: Optional[str]) -> list:
    return df[partition_key].tolist() if partition_key else [None] * df.count()


class _Cols(Params):
    inputCol = Param("The name of the input column", None, T.toString)
    outputCol = Param("The name of the output column", None, T.toString)
    partitionKey = Param("The name of the column to partition by", None, T.toString)

    # snake-case properties used throughout the reference's cyber code
    input_col = property(lambda self: self.getInputCol())
    output_col = property(lambda self: self.getOutputCol())
    partition_key = property(lambda self: self.getPartitionKey())


# ---------------------------------------------------------------------- indexers
class IdIndexerModel(Model, _Cols):
    vocab = Param("(partition, value) -> index", None, complex=True)

    def __init__(self, input_col=None, partition_key=None, output_col=None, vocab=None, **kw):
        super().__init__(**kw)
        self.setParams(inputCol=input_col, partitionKey=partition_key, outputCol=output_col)
        if vocab is not None:
            self.set("vocab", vocab)

    def _transform(self, df):
        voc = self.getVocab()
        ks = _keys(df, self.getPartitionKey())
        out = np.asarray([voc.get((k, v), 0) for k, v in zip(ks, df[self.getInputCol()].tolist())], dtype=np.int64)
        return df.withColumn(self.getOutputCol(), out).drop(self.getInputCol())

    def undo_transform(self, df: DataFrame) -> DataFrame:
        inv = {(k, i): v for (k, v), i in self.getVocab().items()}
        ks = _keys(df, self.getPartitionKey())
        vals = np.empty(df.count(), dtype=object)
        for j, (k, i) in enumerate(zip(ks, df[self.getOutputCol()].tolist())):
            vals[j] = inv.get((k, int(i)))
        return df.withColumn(self.getInputCol(), vals)


class IdIndexer(Estimator, _Cols):
    """Distinct (partition, value) pairs sorted, numbered from 1 (0 = unseen). ``resetPerPartition``
    restarts numbering in every partition."""

    resetPerPartition = Param("When True indexing is consecutive from [1..n] for each partition value", False,
                              T.toBoolean)

    def __init__(self, input_col=None, partition_key=None, output_col=None, reset_per_partition=False, **kw):
        super().__init__(**kw)
        self.setParams(inputCol=input_col, partitionKey=partition_key, outputCol=output_col,
                       resetPerPartition=reset_per_partition)

    def _fit(self, df):
        pairs = sorted(set(zip(_keys(df, self.getPartitionKey()), df[self.getInputCol()].tolist())),
                       key=lambda kv: (str(kv[0]), str(kv[1])))
        vocab: Dict[Tuple, int] = {}
        counters: Dict = {}
        for k, v in pairs:
            key = k if self.getResetPerPartition() else None
            counters[key] = counters.get(key, 0) + 1
            vocab[(k, v)] = counters[key]
        return IdIndexerModel(self.getInputCol(), self.getPartitionKey(), self.getOutputCol(), vocab)


class MultiIndexerModel(Transformer):
    def __init__(self, models: List[IdIndexerModel] = None, **kw):
        super().__init__(**kw)
        self.models = list(models or [])

    def get_model_by_input_col(self, input_col: str) -> Optional[IdIndexerModel]:
        return next((m for m in self.models if m.getInputCol() == input_col), None)

    def get_model_by_output_col(self, output_col: str) -> Optional[IdIndexerModel]:
        return next((m for m in self.models if m.getOutputCol() == output_col), None)

    def undo_transform(self, df):
        for m in self.models:
            df = m.undo_transform(df)
        return df

    def _transform(self, df):
        for m in self.models:
            # keep the input columns (the reference drops them per model; keep them for the next indexers)
            out = m.transform(df)
            df = out.withColumn(m.getInputCol(), df[m.getInputCol()])
        return df


class MultiIndexer(Estimator):
    def __init__(self, indexers: List[IdIndexer] = None, **kw):
        super().__init__(**kw)
        self.indexers = list(indexers or [])

    def _fit(self, df):
        return MultiIndexerModel([ix.fit(df) for ix in self.indexers])


# ---------------------------------------------------------------------- scalers
class _ScalerModel(Model, _Cols):
    stats = Param("per-partition statistics", None, complex=True)

    def _norm(self, x: np.ndarray, st: Dict[str, float]) -> np.ndarray:
        raise NotImplementedError

    @property
    def per_group_stats(self):
        return self.getStats()

    @property
    def use_pandas(self) -> bool:
        return False  # columnar numpy transform (the reference's pandas-UDF switch)

    def is_partitioned(self) -> bool:
        """statistics are kept per partition-key group (reference scalers.py is_partitioned)"""
        return self.getPartitionKey() is not None

    def _transform(self, df):
        x = np.asarray(df[self.getInputCol()], dtype=np.float64)
        ks = _keys(df, self.getPartitionKey())
        out = np.empty_like(x)
        groups: Dict = {}
        for i, k in enumerate(ks):
            groups.setdefault(k, []).append(i)
        for k, idx in groups.items():
            st = self.getStats().get(k)
            idx = np.asarray(idx)
            out[idx] = np.nan if st is None else self._norm(x[idx], st)
        return df.withColumn(self.getOutputCol(), out)


class _ScalerEstimator(Estimator, _Cols):
    @property
    def use_pandas(self) -> bool:
        return False

    def _stats(self, x: np.ndarray) -> Dict[str, float]:
        raise NotImplementedError

    def _model(self, stats) -> _ScalerModel:
        raise NotImplementedError

    def _fit(self, df):
        x = np.asarray(df[self.getInputCol()], dtype=np.float64)
        ks = _keys(df, self.getPartitionKey())
        groups: Dict = {}
        for i, k in enumerate(ks):
            groups.setdefault(k, []).append(i)
        return self._model({k: self._stats(x[np.asarray(idx)]) for k, idx in groups.items()})


class StandardScalarScalerModel(_ScalerModel):
    coefficientFactor = Param("After scaling values of outputCol are multiplied by coefficient", 1.0, T.toFloat)

    def _norm(self, x, st):
        c = self.getCoefficientFactor()
        return c * (x - st["mean"]) / st["std"] if st["std"] != 0 else x - st["mean"]


class StandardScalarScaler(_ScalerEstimator):
    """(x - mean) / std_pop per partition, times ``coefficientFactor``."""

    coefficientFactor = Param("After scaling values of outputCol are multiplied by coefficient", 1.0, T.toFloat)

    def __init__(self, input_col=None, partition_key=None, output_col=None, coefficient_factor=1.0, **kw):
        super().__init__(**kw)
        self.setParams(inputCol=input_col, partitionKey=partition_key, outputCol=output_col,
                       coefficientFactor=coefficient_factor)

    def _stats(self, x):
        return {"mean": float(x.mean()), "std": float(x.std())}

    def _model(self, stats):
        m = StandardScalarScalerModel(inputCol=self.getInputCol(), partitionKey=self.getPartitionKey(),
                                      outputCol=self.getOutputCol(), coefficientFactor=self.getCoefficientFactor())
        return m.set("stats", stats)


class LinearScalarScalerModel(_ScalerModel):
    minRequiredValue = Param("Scale the outputCol to have a value between [minRequiredValue, maxRequiredValue]",
                             0.0, T.toFloat)
    maxRequiredValue = Param("Scale the outputCol to have a value between [minRequiredValue, maxRequiredValue]",
                             1.0, T.toFloat)

    def _norm(self, x, st):
        lo, hi = self.getMinRequiredValue(), self.getMaxRequiredValue()
        delta = st["max"] - st["min"]
        if delta == 0:
            return np.full_like(x, (lo + hi) / 2.0)
        a = (hi - lo) / delta
        return a * x + (hi - a * st["max"])


class LinearScalarScaler(_ScalerEstimator):
    """Per-partition min/max linear map onto [minRequiredValue, maxRequiredValue] (constant partitions map to
    the midpoint)."""

    minRequiredValue = Param("Scale the outputCol to have a value between [minRequiredValue, maxRequiredValue]",
                             0.0, T.toFloat)
    maxRequiredValue = Param("Scale the outputCol to have a value between [minRequiredValue, maxRequiredValue]",
                             1.0, T.toFloat)

    def __init__(self, input_col=None, partition_key=None, output_col=None, min_required_value=0.0,
                 max_required_value=1.0, **kw):
        super().__init__(**kw)
        self.setParams(inputCol=input_col, partitionKey=partition_key, outputCol=output_col,
                       minRequiredValue=min_required_value, maxRequiredValue=max_required_value)

    def _stats(self, x):
        return {"min": float(x.min()), "max": float(x.max())}

    def _model(self, stats):
        m = LinearScalarScalerModel(inputCol=self.getInputCol(), partitionKey=self.getPartitionKey(),
                                    outputCol=self.getOutputCol(), minRequiredValue=self.getMinRequiredValue(),
                                    maxRequiredValue=self.getMaxRequiredValue())
        return m.set("stats", stats)


__all__ = ["IdIndexer", "IdIndexerModel", "MultiIndexer", "MultiIndexerModel", "StandardScalarScaler",
           "StandardScalarScalerModel", "LinearScalarScaler", "LinearScalarScalerModel"]


# reference cyber/feature/scalers.py names of the per-partition scaler bases
PerPartitionScalarScalerEstimator = _ScalerEstimator
PerPartitionScalarScalerModel = _ScalerModel
