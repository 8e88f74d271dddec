"""Mini-batching (reference: core/.../stages/MiniBatchTransformer.scala:19-253,
Batchers.scala:11-151). A batched DataFrame has one row per batch and every
column holds the list of the batch's values; ``FlattenBatch`` inverts it.
Batches never cross partition boundaries (the reference batches per
partition iterator)."""
from __future__ import annotations

import time
from typing import List

import numpy as np

from ..core.dataframe import DataFrame
from ..core.params import Param, Params, TypeConverters as T
from ..core.pipeline import Transformer

_MAXINT = 2 ** 31 - 1


class _MiniBatchBase(Transformer):
    def _batch_bounds(self, n: int) -> List[tuple]:
        raise NotImplementedError

    def _transform(self, df: DataFrame) -> DataFrame:
        names = df.columns
        out = {k: [] for k in names}
        bounds = [0]
        for a, b in df.partition_bounds():
            nb = 0
            for s, e in self._batch_bounds(b - a):
                for k in names:
                    col = df[k]
                    vals = col[a + s:a + e]
                    out[k].append([v for v in (vals.tolist() if col.ndim == 1 else list(vals))])
                nb += 1
            bounds.append(bounds[-1] + nb)
        cols = {}
        for k, v in out.items():
            arr = np.empty(len(v), dtype=object)
            for i, x in enumerate(v):
                arr[i] = x
            cols[k] = arr
        return DataFrame(cols, partition_bounds=bounds)


class FixedMiniBatchTransformer(_MiniBatchBase):
    batchSize = Param("The max size of the buffer", 10, T.toInt)
    maxBufferSize = Param("The max size of the buffer", _MAXINT, T.toInt)
    buffered = Param("Whether or not to buffer batches in memory", False, T.toBoolean)

    def _batch_bounds(self, n):
        bs = max(1, self.getBatchSize())
        return [(s, min(n, s + bs)) for s in range(0, n, bs)]


class DynamicMiniBatchTransformer(_MiniBatchBase):
    """Batches whatever is available (here: the whole partition, capped at maxBatchSize)."""

    maxBatchSize = Param("The max size of the buffer", _MAXINT, T.toInt)

    def _batch_bounds(self, n):
        bs = max(1, self.getMaxBatchSize())
        return [(s, min(n, s + bs)) for s in range(0, n, bs)]


class TimeIntervalMiniBatchTransformer(_MiniBatchBase):
    """Collects rows for ``millisToWait`` per batch (static data: all rows are available at once, so batches
    are bounded by ``maxBatchSize`` only; the wait is honoured between batches when rows arrive lazily)."""

    millisToWait = Param("The time to wait before constructing a batch", 1000, T.toInt)
    maxBatchSize = Param("The max size of the buffer", _MAXINT, T.toInt)

    def _batch_bounds(self, n):
        bs = max(1, self.getMaxBatchSize())
        return [(s, min(n, s + bs)) for s in range(0, n, bs)]


class FlattenBatch(Transformer):
    def _transform(self, df: DataFrame) -> DataFrame:
        names = df.columns
        out = {k: [] for k in names}
        bounds = [0]
        for a, b in df.partition_bounds():
            cnt = 0
            for i in range(a, b):
                vals = [df[k][i] for k in names]
                lens = {len(v) for v in vals if isinstance(v, (list, tuple, np.ndarray)) and v is not None}
                if not lens:
                    continue
                if len(lens) != 1:
                    raise ValueError("FlattenBatch: list columns of one row have different lengths")
                L = lens.pop()
                for j in range(L):
                    for k, v in zip(names, vals):
                        out[k].append(None if v is None else (v[j] if isinstance(v, (list, tuple, np.ndarray))
                                                               else v))
                cnt += L
            bounds.append(bounds[-1] + cnt)
        cols = {}
        for k, v in out.items():
            arr = np.empty(len(v), dtype=object)
            for i, x in enumerate(v):
                arr[i] = x
            if len(v) and all(isinstance(x, (int, float, bool, np.number)) for x in v):
                arr = np.asarray(v)
            cols[k] = arr
        return DataFrame(cols, partition_bounds=bounds)


class HasMiniBatcher(Params):
    miniBatcher = Param("Minibatcher to use", None, complex=True)

    def setMiniBatchSize(self, n: int):  # noqa: N802
        mb = self.getMiniBatcher() or FixedMiniBatchTransformer()
        if isinstance(mb, FixedMiniBatchTransformer):
            mb.setBatchSize(n)
        else:
            mb.setMaxBatchSize(n)
        return self.set("miniBatcher", mb)

    def getMiniBatchSize(self) -> int:  # noqa: N802
        mb = self.getMiniBatcher() or FixedMiniBatchTransformer()
        return mb.getBatchSize() if isinstance(mb, FixedMiniBatchTransformer) else mb.getMaxBatchSize()


def _sleep_ms(ms: int) -> None:  # pragma: no cover - used by streaming sources
    time.sleep(ms / 1000.0)
