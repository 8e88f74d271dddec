"""PowerBI streaming-dataset writer (reference: CORE/io/powerbi/PowerBIWriter.scala).

Rows are mini-batched (fixed/dynamic/timed) and POSTed as JSON arrays to the
dataset's push URL through SimpleHTTPTransformer; HTTP errors raise."""
from __future__ import annotations

from typing import Dict, Optional

from ..core.dataframe import DataFrame
from ..stages.basic import PartitionConsolidator
from ..stages.batching import (DynamicMiniBatchTransformer, FixedMiniBatchTransformer,
                               TimeIntervalMiniBatchTransformer)
from .http import SimpleHTTPTransformer

_OPTIONS = {"consolidate", "concurrency", "concurrentTimeout", "minibatcher", "maxBatchSize", "batchSize",
            "buffered", "maxBufferSize", "millisToWait"}


def _prepare(df: DataFrame, url: str, options: Optional[Dict[str, str]] = None) -> DataFrame:
    options = dict(options or {})
    for k in options:
        if k not in _OPTIONS:
            raise ValueError(f"{k} not an applicable option {sorted(_OPTIONS)}")
    kind = options.get("minibatcher", "fixed")
    max_bs = int(options.get("maxBatchSize", 2 ** 31 - 1))
    if kind == "dynamic":
        mb = DynamicMiniBatchTransformer(maxBatchSize=max_bs)
    elif kind == "fixed":
        mb = FixedMiniBatchTransformer(batchSize=int(options.get("batchSize", 10)))
    elif kind == "timed":
        mb = TimeIntervalMiniBatchTransformer(millisToWait=int(options.get("millisToWait", 1000)),
                                              maxBatchSize=max_bs)
    else:
        raise ValueError(f"unknown minibatcher {kind}")
    if str(options.get("consolidate", "false")).lower() == "true":
        df = PartitionConsolidator().transform(df)
    rows = df.collect()
    packed = DataFrame({"input": _rows(rows)})
    t = SimpleHTTPTransformer(inputCol="input", outputCol="output", errorCol="errors",
                              concurrency=int(options.get("concurrency", 1)),
                              concurrentTimeout=float(options.get("concurrentTimeout", 30.0)),
                              flattenOutputBatches=False)
    t.setUrl(url)
    t.set("miniBatcher", mb)
    return t.transform(packed)


def _rows(rows):
    import numpy as np

    col = np.empty(len(rows), dtype=object)
    for i, r in enumerate(rows):
        col[i] = dict(r)
    return col


def write(df: DataFrame, url: str, options: Optional[Dict[str, str]] = None) -> None:
    out = _prepare(df, url, options)
    errs = [e for e in out["errors"].tolist() if e is not None]
    if errs:
        raise RuntimeError(f"PowerBI write failed: {errs[0]}")


class PowerBIWriter:
    write = staticmethod(write)
    prepareDF = staticmethod(_prepare)  # noqa: N815


__all__ = ["PowerBIWriter", "write"]
