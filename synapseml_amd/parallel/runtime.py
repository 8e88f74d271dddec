"""Local multi-process partition runtime.

Plays the role Spark plays for the reference: a driver splits a DataFrame into
partitions, starts one executor process per partition group (one per GPU on
an MI355X node, pinned with ``torch.cuda.set_device``), the executors
rendezvous (TCPStore on 127.0.0.1 - the reference's NetworkManager driver
socket, LightGBM/NetworkManager.scala:59-84) and run the same partition task;
results are collected on the driver (C6 in SURVEY §2.5).

``barrier=True`` mirrors Spark barrier execution: all ranks initialise the
process group before any runs its task; ranks whose partition is empty still
join the collectives with zero rows (the reference's "ignore" status, so
nothing hangs, BasePartitionTask.scala:134-137).
"""
from __future__ import annotations

import os
import pickle
import socket
import traceback
from typing import Any, Callable, List, Optional

from ..core.dataframe import DataFrame


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _injected_fault(rank: int) -> Optional[str]:
    """Test-only fault injection: ``SML_FAULT_INJECT="<rank>:<kind>"`` with kind in
    raise | crash_before | crash_after_init | empty (the rank sees an empty partition)."""
    spec = os.environ.get("SML_FAULT_INJECT", "")
    for item in filter(None, spec.split(",")):
        r, _, kind = item.partition(":")
        if r.strip() == str(rank):
            return kind.strip()
    return None


def _worker(rank: int, world: int, port: int, backend: str, fn_bytes: bytes, parts_bytes: bytes, out_dir: str,
            use_gpu: bool) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    result: Any
    fault = _injected_fault(rank)
    if fault == "crash_before":
        os._exit(17)  # hard crash before the rendezvous (test-only, SML_FAULT_INJECT)
    try:
        import torch
        import torch.distributed as dist

        if use_gpu:
            torch.cuda.set_device(rank % max(1, torch.cuda.device_count()))
        dist.init_process_group(backend=backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        fn = pickle.loads(fn_bytes)
        part = pickle.loads(parts_bytes)
        if fault == "raise":
            raise RuntimeError(f"injected fault on rank {rank}")
        if fault == "crash_after_init":
            os._exit(18)  # dies while the other ranks wait in collectives
        if fault == "empty":
            part = part.slice(0, 0)
        result = ("ok", fn(part, rank, world))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - report to the driver
        result = ("err", f"{type(e).__name__}: {e}\n{traceback.format_exc()}")
    with open(os.path.join(out_dir, f"result_{rank}.pkl"), "wb") as f:
        pickle.dump(result, f)


def run_partitions(fn: Callable[[DataFrame, int, int], Any], df: DataFrame, num_workers: Optional[int] = None,
                   backend: Optional[str] = None, use_gpu: bool = False, timeout_s: float = 1200.0,
                   fail_fast: bool = True) -> List[Any]:
    """Run ``fn(partition_df, rank, world)`` in ``num_workers`` processes.

    Partitions are grouped contiguously onto workers (coalesce). Returns the
    per-rank results in rank order.
    """
    import tempfile

    import torch.multiprocessing as mp

    world = num_workers or df.getNumPartitions()
    parts = df.coalesce(world).partitions() if df.getNumPartitions() >= world else df.repartition(world).partitions()
    while len(parts) < world:
        parts.append(df.slice(0, 0))
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    port = _free_port()
    fn_bytes = pickle.dumps(fn)
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        procs = []
        for r in range(world):
            p = ctx.Process(target=_worker, args=(r, world, port, backend, fn_bytes, pickle.dumps(parts[r]), d, use_gpu))
            p.start()
            procs.append(p)
        # fail fast: a rank that exits with an error (or dies) aborts the job instead of leaving the others
        # blocked in collectives until the timeout (the reference waits for the Spark task timeout)
        import time as _time

        deadline = _time.monotonic() + timeout_s
        failed = None
        while any(p.is_alive() for p in procs):
            for r, p in enumerate(procs):
                if p.is_alive():
                    continue
                path = os.path.join(d, f"result_{r}.pkl")
                if p.exitcode != 0 or not os.path.exists(path):
                    failed = failed or (r, f"exit code {p.exitcode}")
                else:
                    with open(path, "rb") as f:
                        st = pickle.load(f)[0]  # written by our own worker process
                    if st != "ok":
                        failed = failed or (r, "task error")
            if (failed and fail_fast) or _time.monotonic() > deadline:
                break
            _time.sleep(0.05)
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(10)
                if p.is_alive():
                    p.kill()
                    p.join()
        if failed is not None and not fail_fast:
            # every rank ran to its own end: report what each one saw
            errs = []
            for r in range(world):
                path = os.path.join(d, f"result_{r}.pkl")
                if not os.path.exists(path):
                    errs.append(f"worker {r}: exit code {procs[r].exitcode}, no result")
                    continue
                with open(path, "rb") as f:
                    st, val = pickle.load(f)  # written by our own worker process
                if st != "ok":
                    errs.append(f"worker {r}: {val}")
            raise RuntimeError("partition tasks failed: " + " | ".join(errs))
        if failed is not None:
            r, why = failed
            path = os.path.join(d, f"result_{r}.pkl")
            if os.path.exists(path):
                with open(path, "rb") as f:
                    st, val = pickle.load(f)  # written by our own worker process
                if st != "ok":
                    why = val
            raise RuntimeError(f"worker {r} failed ({why}); the job was aborted on the remaining ranks")
        if _time.monotonic() > deadline:
            raise TimeoutError(f"partition tasks did not finish within {timeout_s}s")
        results = []
        for r in range(world):
            path = os.path.join(d, f"result_{r}.pkl")
            if not os.path.exists(path):
                raise RuntimeError(f"worker {r} produced no result (exit code {procs[r].exitcode})")
            with open(path, "rb") as f:
                # written by our own worker process above
                status, val = pickle.load(f)
            if status != "ok":
                raise RuntimeError(f"worker {r} failed: {val}")
            results.append(val)
    return results


class _FitTask:
    def __init__(self, estimator):
        self.estimator = estimator

    def __call__(self, part: DataFrame, rank: int, world: int):
        model = self.estimator.fit(part)
        return model if rank == 0 else None


def distributed_fit(estimator, df: DataFrame, num_workers: Optional[int] = None, use_gpu: bool = False,
                    **kw):
    """Data-parallel ``fit`` across worker processes; returns rank 0's model
    (only the main worker returns the model, BasePartitionTask.scala:450-461).
    Extra keyword arguments go to :func:`run_partitions` (timeout_s, fail_fast)."""
    return run_partitions(_FitTask(estimator), df, num_workers=num_workers, use_gpu=use_gpu, **kw)[0]
