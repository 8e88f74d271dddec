"""PySpark partition runtime: Spark stays the orchestrator.

The reference trains inside Spark barrier stages (LightGBMBase.scala:608-628,
``useBarrierExecutionMode``) and infers with ``mapPartitions``
(ONNXModel.scala:242-251). This adapter runs the framework's estimators and
models the same way when ``pyspark`` is importable:

* ``fit_on_spark(estimator, spark_df)``: one barrier task per partition; task 0
  publishes a free port through ``BarrierTaskContext.allGather``, every task
  joins ``torch.distributed`` (RCCL when the task owns a GPU — the address
  Spark assigned in ``resources()["gpu"]`` is pinned — gloo otherwise), turns its
  rows into a columnar partition and calls ``estimator.fit`` exactly as the
  local multi-process runtime (runtime.py) does; the model comes back from
  task 0 (BasePartitionTask.scala:450-461).
* ``transform_on_spark(model, spark_df, schema)``: ``mapInArrow`` over the
  partitions; each Arrow batch becomes a DataFrame, is transformed on the
  executor's device and goes back as Arrow.

The executor-side code is the same code the local runtime runs; pyspark is an
optional dependency (not installed in this image: ``tests/test_spark_adapter.py``
drives the adapter through a minimal stand-in of the pyspark API surface).
"""
from __future__ import annotations

import os
import pickle
import socket
from typing import Any, Iterable, Iterator, List

import numpy as np

from ..core.dataframe import DataFrame


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("", 0))
        return s.getsockname()[1]


def _rows_to_frame(rows: List[Any]) -> DataFrame:
    """Spark Rows (with pyspark.ml vectors) -> columnar partition."""
    if not rows:
        return DataFrame({})
    names = list(rows[0].asDict().keys()) if hasattr(rows[0], "asDict") else list(rows[0].keys())
    cols = {}
    for k in names:
        vals = [r[k] for r in rows]
        if vals and hasattr(vals[0], "toArray"):
            cols[k] = np.stack([np.asarray(v.toArray(), dtype=np.float64) for v in vals])
        else:
            cols[k] = vals
    return DataFrame(cols)


def _barrier_fit_task(est_bytes: bytes, use_gpu: bool):
    def run(iterator: Iterable[Any]) -> Iterator[bytes]:
        import torch
        import torch.distributed as dist
        from pyspark import BarrierTaskContext

        ctx = BarrierTaskContext.get()
        rank = ctx.partitionId()
        infos = ctx.getTaskInfos()
        world = len(infos)
        host = infos[0].address.split(":")[0]
        port = ctx.allGather(str(_free_port()) if rank == 0 else "")[0]
        if use_gpu and torch.cuda.is_available():
            gpus = (ctx.resources() or {}).get("gpu")
            dev = int(gpus.addresses[0]) if gpus is not None and gpus.addresses else rank % torch.cuda.device_count()
            torch.cuda.set_device(dev)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR=host,
                          MASTER_PORT=str(port))
        backend = "nccl" if use_gpu and torch.cuda.is_available() else "gloo"
        if world > 1:
            dist.init_process_group(backend=backend, init_method=f"tcp://{host}:{port}", rank=rank, world_size=world)
        try:
            est = pickle.loads(est_bytes)  # produced by fit_on_spark on the driver (our own object)
            model = est.fit(_rows_to_frame(list(iterator)))
            if world > 1:
                ctx.barrier()
        finally:
            if world > 1 and dist.is_initialized():
                dist.destroy_process_group()
        yield pickle.dumps(model) if rank == 0 else b""

    return run


def fit_on_spark(estimator, spark_df, use_gpu: bool = True):
    """Data-parallel ``fit`` with one barrier task per partition of ``spark_df``."""
    est_bytes = pickle.dumps(estimator)
    out = spark_df.rdd.barrier().mapPartitions(_barrier_fit_task(est_bytes, use_gpu)).collect()
    models = [b for b in out if b]
    if not models:
        raise RuntimeError("no model was returned by the barrier stage")
    return pickle.loads(models[0])  # written by task 0 of our own barrier stage


def transform_on_spark(model, spark_df, schema):
    """``model.transform`` per partition through ``mapInArrow`` (Arrow in, Arrow out)."""
    model_bytes = pickle.dumps(model)

    def run(batches):
        m = pickle.loads(model_bytes)  # our own object, shipped by the driver
        for b in batches:
            out = m.transform(DataFrame.fromArrow(b))
            for rb in out.toArrow().to_batches():
                yield rb

    return spark_df.mapInArrow(run, schema)


__all__ = ["fit_on_spark", "transform_on_spark"]
