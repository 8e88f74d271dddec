"""PySpark partition runtime: Spark stays the orchestrator.

The reference trains inside Spark barrier stages (LightGBMBase.scala:608-628,
``useBarrierExecutionMode``) and infers with ``mapPartitions``
(ONNXModel.scala:242-251). This adapter runs the framework's estimators and
models the same way when ``pyspark`` is importable:

* ``fit_on_spark(estimator, spark_df)``: one barrier task per partition
  (``mapInArrow(barrier=True)``: the partition arrives as Arrow batches, no Row
  objects; Rows only on Spark < 3.5); task 0 publishes a free port through
  ``BarrierTaskContext.allGather``, every task pins the GPU Spark assigned in
  ``resources()["gpu"]``, joins ``torch.distributed`` (gloo control plane; the
  engines' data plane is their own RCCL communicator) and calls
  ``estimator.fit`` exactly as the local multi-process runtime (runtime.py)
  does; the model comes back from task 0 (BasePartitionTask.scala:450-461).
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
        import torch.distributed as dist

        ctx, rank, world = _join(use_gpu)
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


def _join(use_gpu: bool):
    """Barrier-task rendezvous shared by both fit paths: task 0 publishes a free port through allGather,
    every task pins its GPU (Spark's resource address) and joins torch.distributed. Returns (ctx, rank, world)."""
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
    if world > 1:
        # gloo control plane; the engines build their own RCCL communicators for the data plane
        dist.init_process_group(backend="gloo", init_method=f"tcp://{host}:{port}", rank=rank, world_size=world)
    return ctx, rank, world


def _arrow_barrier_fit_task(est_bytes: bytes, use_gpu: bool):
    """mapInArrow(barrier=True) task: the partition arrives as Arrow record batches and becomes a columnar
    DataFrame without touching a Row (vector columns were turned into array<double> on the driver side of the
    plan, and fixed-width lists become 2-D arrays in DataFrame.fromArrow)."""
    def run(batches):
        import pyarrow as pa
        import torch.distributed as dist

        ctx, rank, world = _join(use_gpu)
        try:
            bl = [b for b in batches if b.num_rows]
            part = DataFrame.fromArrow(bl) if bl else DataFrame({})
            est = pickle.loads(est_bytes)  # produced by fit_on_spark on the driver (our own object)
            model = est.fit(part)
            if world > 1:
                ctx.barrier()
        finally:
            if world > 1 and dist.is_initialized():
                dist.destroy_process_group()
        yield pa.RecordBatch.from_pydict({"model": [pickle.dumps(model) if rank == 0 else b""]},
                                         schema=pa.schema([("model", pa.binary())]))

    return run


def _vectors_as_arrays(spark_df):
    """ML vector columns -> array<double> (``vector_to_array``), so the partition can travel as Arrow."""
    try:
        from pyspark.ml.functions import vector_to_array
        from pyspark.sql.functions import col
    except Exception:  # noqa: BLE001 - stand-ins / minimal installs: columns are already Arrow-encodable
        return spark_df
    for f in getattr(getattr(spark_df, "schema", None), "fields", []) or []:
        if getattr(f.dataType, "typeName", lambda: "")() == "vector" or type(f.dataType).__name__ == "VectorUDT":
            spark_df = spark_df.withColumn(f.name, vector_to_array(col(f.name)))
    return spark_df


def fit_on_spark(estimator, spark_df, use_gpu: bool = True):
    """Data-parallel ``fit`` with one barrier task per partition of ``spark_df``.

    Spark >= 3.5: ``mapInArrow(..., barrier=True)`` - partitions reach the executors' engines as Arrow
    batches (the reference's per-row JNI copy loop, StreamingPartitionTask.scala:280-299, has no
    counterpart). Older Spark (no barrier mode for mapInArrow): ``rdd.barrier().mapPartitions`` over Rows."""
    est_bytes = pickle.dumps(estimator)
    sdf = _vectors_as_arrays(spark_df)
    try:
        res = sdf.mapInArrow(_arrow_barrier_fit_task(est_bytes, use_gpu), "model binary", barrier=True)
    except TypeError:  # mapInArrow() got an unexpected keyword argument 'barrier'
        res = None
    if res is not None:
        models = [bytes(r["model"]) for r in res.collect() if r["model"]]
    else:
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
