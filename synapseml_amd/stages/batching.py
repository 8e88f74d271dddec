"""Mini-batching (reference: core/.../stages/MiniBatchTransformer.scala:19-253,
Batchers.scala:11-151: FixedBatcher, FixedBufferedBatcher, DynamicBufferedBatcher,
TimeIntervalBatcher below). A batched DataFrame has one row per batch and every
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


# ------------------------------------------------------------------ iterator batchers (Batchers.scala)
# Batch a (possibly lazy, possibly slow) row iterator: what the mini-batch transformers do to a partition
# iterator in the reference, and what streaming sources (serving) use directly.
class FixedBatcher:
    """Consecutive lists of ``batch_size`` items (the last may be shorter)."""

    def __init__(self, it, batch_size: int):
        self._it = iter(it)
        self._bs = max(1, int(batch_size))

    def __iter__(self):
        return self

    def __next__(self) -> list:
        out = []
        for x in self._it:
            out.append(x)
            if len(out) == self._bs:
                break
        if not out:
            raise StopIteration
        return out


class TimeIntervalBatcher:
    """Each batch takes the first available item, then keeps taking items until ``millis`` have passed
    since the batch started or it holds ``max_buffer_size`` items."""

    def __init__(self, it, millis: int, max_buffer_size: int = _MAXINT):
        self._it = iter(it)
        self._ms = millis
        self._cap = max(1, int(max_buffer_size))
        self._peek = []

    def __iter__(self):
        return self

    def __next__(self) -> list:
        first = next(self._it)  # StopIteration ends the stream
        start = time.monotonic()
        out = [first]
        while len(out) < self._cap and (time.monotonic() - start) * 1000.0 < self._ms:
            try:
                out.append(next(self._it))
            except StopIteration:
                break
        return out


class _BufferedBatcher:
    """A producer thread drains the source into a bounded queue while batches are consumed."""

    _DONE = object()

    def __init__(self, it, max_buffer_size: int, item_fn):
        import queue
        import threading

        self._it = iter(it)
        self._q = queue.Queue(maxsize=0 if max_buffer_size >= _MAXINT else max(1, int(max_buffer_size)))
        self._item_fn = item_fn
        self._started = False
        self._finished = False
        self._error = None
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._stop = threading.Event()

    def _run(self):
        try:
            while not self._stop.is_set():
                item = self._item_fn(self._it)
                if item is self._DONE:
                    break
                self._q.put(item)
        except BaseException as e:  # surfaced to the consumer
            self._error = e
        finally:
            self._q.put(self._DONE)

    def start(self):
        if not self._started:
            self._started = True
            self._thread.start()
        return self

    def close(self):
        self._stop.set()

    def __iter__(self):
        return self


class FixedBufferedBatcher(_BufferedBatcher):
    """Fixed-size batches produced ahead of the consumer (at most ``max_buffer_size`` batches queued)."""

    def __init__(self, it, batch_size: int, max_buffer_size: int = _MAXINT):
        bs = max(1, int(batch_size))

        def take(src):
            out = []
            for x in src:
                out.append(x)
                if len(out) == bs:
                    break
            return out or self._DONE

        super().__init__(it, max_buffer_size, take)

    def __next__(self) -> list:
        self.start()
        if self._finished:
            raise StopIteration
        b = self._q.get()
        if b is self._DONE:
            self._finished = True
            if self._error is not None:
                raise self._error
            raise StopIteration
        return b


class DynamicBufferedBatcher(_BufferedBatcher):
    """Each batch is everything the producer has buffered so far (at least one item): batch sizes adapt
    to how fast the consumer is relative to the source."""

    def __init__(self, it, max_buffer_size: int = _MAXINT):
        super().__init__(it, max_buffer_size, lambda src: next(src, self._DONE))

    def __next__(self) -> list:
        import queue

        self.start()
        if self._finished:
            raise StopIteration
        out = []
        x = self._q.get()  # block for the first item
        while True:
            if x is self._DONE:
                self._finished = True
                break
            out.append(x)
            try:
                x = self._q.get_nowait()
            except queue.Empty:
                break
        if self._error is not None and self._finished:
            raise self._error
        if not out:
            raise StopIteration
        return out
