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

import numpy as np

from ..core.dataframe import DataFrame


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


MAX_PORT = 65535
NETWORK_RETRIES = 3          # LightGBMConstants.NetworkRetries
INITIAL_DELAY_S = 1.0        # LightGBMConstants.InitialDelay (ms 1000), doubled per retry


def _bindable(port: int) -> bool:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        try:
            s.bind(("127.0.0.1", port))
            return True
        except OSError:
            return False


def find_open_port(base: int, max_tries: int = 1000) -> int:
    """First bindable port at or above ``base`` (NetworkManager.findOpenPort, NetworkManager.scala:240-271):
    at most ``max_tries`` ports are probed and none above 65535."""
    if base <= 0:
        return _free_port()
    if base > MAX_PORT:
        raise ValueError(f"port {base} out of range")
    for port in range(base, min(MAX_PORT, base + max_tries - 1) + 1):
        if _bindable(port):
            return port
    raise RuntimeError(f"could not find an open port in [{base}, {min(MAX_PORT, base + max_tries - 1)}]")


def rendezvous_port(driver_listen_port: int = 0, default_listen_port: int = 0) -> int:
    """The rank-0 rendezvous (TCPStore) port for a job this runtime launches - the role of the reference
    driver's listen socket and the workers' LightGBM listen ports (LightGBMParams.scala:39-49):
    ``driverListenPort > 0`` is used as given (an error if it is taken, as the driver's bind would fail);
    otherwise the first open port at or above ``defaultListenPort`` (12400 by default); otherwise any
    free port."""
    if driver_listen_port and driver_listen_port > 0:
        if driver_listen_port > MAX_PORT:
            raise ValueError(f"driverListenPort {driver_listen_port} out of range")
        if not _bindable(driver_listen_port):
            raise RuntimeError(f"driverListenPort {driver_listen_port} is already in use")
        return driver_listen_port
    return find_open_port(default_listen_port) if default_listen_port and default_listen_port > 0 else _free_port()


def _injected_fault(rank: int) -> Optional[str]:
    """Test-only fault injection: ``SML_FAULT_INJECT="<rank>:<kind>"`` with kind in
    raise | crash_before | crash_after_init | empty (the rank sees an empty partition) | netinit_fail (the
    rank's first rendezvous attempt fails)."""
    spec = os.environ.get("SML_FAULT_INJECT", "")
    for item in filter(None, spec.split(",")):
        r, _, kind = item.partition(":")
        if r.strip() == str(rank):
            return kind.strip()
    return None



# ---------------------------------------------------------------- partition hand-off
# Partitions reach the spawned workers through POSIX shared memory instead of pickled process arguments: the
# driver copies every numeric column (and the CSR arrays of sparse vector columns) of a partition into one
# /dev/shm segment once, and the worker maps them as numpy views - no serialisation, no pipe transfer, and
# no second copy on the worker side (an 11M x 28 float32 partition was a 1.2 GB pickle per rank). Object
# columns (strings, vector objects) still travel pickled inside the small descriptor.
_SHM_ALIGN = 64
_SHM_DIR = "/dev/shm"


def _shm_fits(nbytes: int) -> bool:
    """True when /dev/shm has room for a segment of ``nbytes`` (plus 64 MiB of headroom for the other
    segments of this job and the rest of the host); ``SML_SHM_HANDOFF=0`` forces the pickled hand-off."""
    if os.environ.get("SML_SHM_HANDOFF", "1") == "0":
        return False
    try:
        st = os.statvfs(_SHM_DIR)
    except OSError:
        return False
    return st.f_bavail * st.f_frsize >= nbytes + (64 << 20)


def _share_partition(df: DataFrame):
    from multiprocessing import shared_memory

    from ..core.linalg import CsrColumn

    plan, arrays, total = [], [], 0

    def place(a: np.ndarray):
        nonlocal total
        a = np.ascontiguousarray(a)
        off = total
        total += (a.nbytes + _SHM_ALIGN - 1) // _SHM_ALIGN * _SHM_ALIGN
        arrays.append((off, a))
        return (off, a.dtype.str, a.shape)

    for name in df.columns:
        col = df[name]
        if isinstance(col, CsrColumn):
            ip, ind, val = col.csr()
            plan.append((name, "csr", (place(ip), place(ind), place(val), col.size)))
        elif isinstance(col, np.ndarray) and col.dtype != object:
            plan.append((name, "shm", place(col)))
        else:
            plan.append((name, "pickle", pickle.dumps(col)))
    if total and not _shm_fits(total):
        # a small /dev/shm (Docker's 64 MB default, k8s without a Memory emptyDir): filling a segment past its
        # free space raises SIGBUS inside the driver, so the partition travels pickled instead
        desc = {"n": df.count(), "meta": {k: df.metadata(k) for k in df.columns}, "shm": None,
                "cols": [(name, "pickle", pickle.dumps(df[name])) for name in df.columns]}
        return pickle.dumps(desc), None
    shm = shared_memory.SharedMemory(create=True, size=max(total, 1)) if total else None
    if shm is not None:
        for off, a in arrays:
            np.ndarray(a.shape, dtype=a.dtype, buffer=shm.buf, offset=off)[...] = a
    desc = {"n": df.count(), "meta": {k: df.metadata(k) for k in df.columns}, "cols": plan,
            "shm": shm.name if shm is not None else None}
    return pickle.dumps(desc), shm


def _attach_partition(desc_bytes: bytes):
    from ..core.linalg import CsrColumn
    from .executor import attach_shm

    desc = pickle.loads(desc_bytes)  # built by a process of this job (_share_partition)
    shm = None
    if desc["shm"]:
        # the creator owns (and unlinks) the segment: attached without a resource-tracker registration (the
        # tracker is shared with the driver; an attach + unregister here dropped the driver's own entry and its
        # unlink then failed inside the tracker with KeyError '/psm_...')
        shm = attach_shm(desc["shm"])

    def view(spec):
        off, dt, shape = spec
        return np.ndarray(shape, dtype=np.dtype(dt), buffer=shm.buf, offset=off)

    cols = {}
    for name, kind, info in desc["cols"]:
        if kind == "shm":
            cols[name] = view(info)
        elif kind == "csr":
            cols[name] = CsrColumn(view(info[0]), view(info[1]), view(info[2]), info[3])
        else:
            cols[name] = pickle.loads(info)  # serialized by the driver of this job
    df = DataFrame(cols, metadata={k: v for k, v in desc["meta"].items() if v})
    if not cols:
        df = DataFrame({})
    return df, shm

def _worker(rank: int, world: int, port: int, backend: str, fn_bytes: bytes, parts_bytes: bytes, out_dir: str,
            use_gpu: bool, attempt: int = 0, env: Optional[dict] = None) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), SML_PARTITION_TASK="1")
    if env:
        os.environ.update({k: str(v) for k, v in env.items()})
    result: Any
    fault = _injected_fault(rank)
    if fault == "crash_before":
        os._exit(17)  # hard crash before the rendezvous (test-only, SML_FAULT_INJECT)
    try:
        import torch
        import torch.distributed as dist

        if use_gpu:
            torch.cuda.set_device(rank % max(1, torch.cuda.device_count()))
        try:
            if fault == "netinit_fail" and attempt == 0:
                raise OSError("injected network-init failure")
            dist.init_process_group(backend=backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                    world_size=world, timeout=_init_timeout())
        except Exception as e:  # noqa: BLE001 - the driver retries the rendezvous (NetworkManager retry)
            result = ("netinit", f"{type(e).__name__}: {e}")
            with open(os.path.join(out_dir, f"result_{rank}.pkl"), "wb") as f:
                pickle.dump(result, f)
            return
        fn = pickle.loads(fn_bytes)
        part, shm = _attach_partition(parts_bytes)
        if fault == "raise":
            raise RuntimeError(f"injected fault on rank {rank}")
        if fault == "crash_after_init":
            os._exit(18)  # dies while the other ranks wait in collectives
        if fault == "empty":
            part = part.slice(0, 0)
        # serialised while the partition is still mapped: a result may view the shared-memory columns (a
        # transformed partition keeps its input columns), and numpy views do not pin the mapping - closing it
        # first left them dangling (the pickling then read unmapped memory)
        payload = pickle.dumps(("ok", fn(part, rank, world)))
        del part
        dist.barrier()
        from . import distributed as D

        D.close_shm_reducer()
        dist.destroy_process_group()
        if shm is not None:
            try:
                shm.close()
            except BufferError:
                pass
    except BaseException as e:  # noqa: BLE001 - report to the driver
        payload = pickle.dumps(("err", f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))
    tmp = os.path.join(out_dir, f"result_{rank}.pkl.tmp")
    with open(tmp, "wb") as f:
        f.write(payload)
    os.replace(tmp, os.path.join(out_dir, f"result_{rank}.pkl"))  # the driver never sees a partial file


def _init_timeout():
    import datetime

    return datetime.timedelta(seconds=float(os.environ.get("SML_RENDEZVOUS_TIMEOUT_S", "120")))


def run_partitions(fn: Callable[[DataFrame, int, int], Any], df: DataFrame, num_workers: Optional[int] = None,
                   backend: Optional[str] = None, use_gpu: bool = False, timeout_s: float = 1200.0,
                   fail_fast: bool = True, port: Optional[int] = None, default_listen_port: int = 0,
                   network_retries: int = NETWORK_RETRIES, initial_delay_s: float = INITIAL_DELAY_S,
                   env: Optional[dict] = None) -> List[Any]:
    """Run ``fn(partition_df, rank, world)`` in ``num_workers`` processes.

    Partitions are grouped contiguously onto workers (coalesce). Returns the
    per-rank results in rank order. ``env`` is exported in every worker before
    it imports anything (e.g. ``SML_GBDT_SHARED_DEVICE``).

    Network initialisation follows the reference's NetworkInit retry (NetworkManager.scala:195-218): when
    any rank fails to join the rendezvous, every rank of that attempt is stopped and the job is relaunched
    on the next open port, up to ``network_retries`` times, sleeping ``initial_delay_s`` doubled per retry.
    ``port`` pins the rendezvous port (driverListenPort); otherwise the first open port at or above
    ``default_listen_port`` (defaultListenPort), or any free port.
    """
    import time as _time

    delay = initial_delay_s
    pinned = port
    for attempt in range(network_retries + 1):
        p = pinned if pinned else (find_open_port(default_listen_port) if default_listen_port > 0 else _free_port())
        try:
            return _run_once(fn, df, num_workers, backend, use_gpu, timeout_s, fail_fast, p, attempt, env)
        except _NetworkInitError as e:
            if attempt == network_retries:
                raise RuntimeError(f"network init failed after {network_retries} retries: {e}") from None
            _time.sleep(delay)
            delay *= 2
            if default_listen_port > 0 and not pinned:
                default_listen_port = p + 1  # the next open port, as findOpenPort walks upward
    raise AssertionError("unreachable")


class _NetworkInitError(RuntimeError):
    pass


def _run_once(fn, df, num_workers, backend, use_gpu, timeout_s, fail_fast, port, attempt, env=None) -> List[Any]:
    import tempfile

    import torch.multiprocessing as mp

    world = num_workers or df.getNumPartitions()
    parts = _task_partitions(df, world)
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    fn_bytes = pickle.dumps(fn)
    ctx = mp.get_context("spawn")
    shared = []
    try:
        # every partition is placed before any worker starts: a hand-off that fails leaves no started worker
        # waiting in the rendezvous
        descs = []
        for r in range(world):
            desc, shm = _share_partition(parts[r])
            if shm is not None:
                shared.append(shm)
            descs.append(desc)
        with tempfile.TemporaryDirectory() as d:
            return _run_procs(ctx, fn_bytes, descs, world, port, backend, use_gpu, attempt, timeout_s, fail_fast, d,
                              env)
    finally:
        for shm in shared:
            try:
                shm.close()
                shm.unlink()
            except Exception:  # noqa: BLE001 - already gone
                pass


def _run_procs(ctx, fn_bytes, descs, world, port, backend, use_gpu, attempt, timeout_s, fail_fast, d, env):
    procs = []
    try:
        for r in range(world):
            p = ctx.Process(target=_worker,
                            args=(r, world, port, backend, fn_bytes, descs[r], d, use_gpu, attempt, env))
            p.start()
            procs.append(p)
    except BaseException:
        for p in procs:  # a worker that failed to start: the started ones would wait in the rendezvous
            p.terminate()
            p.join(10)
        raise
    # fail fast: a rank that exits with an error (or dies) aborts the job instead of leaving the others
    # blocked in collectives until the timeout (the reference waits for the Spark task timeout)
    import time as _time

    deadline = _time.monotonic() + timeout_s
    failed = None
    timed_out = False
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
                if st == "netinit":
                    failed = failed or (r, "netinit")
                elif st != "ok":
                    failed = failed or (r, "task error")
        if failed and (fail_fast or failed[1] == "netinit"):
            break
        if _time.monotonic() > deadline:
            timed_out = True
            break
        _time.sleep(0.05)
    for p in procs:
        if p.is_alive():
            p.terminate()
            p.join(10)
            if p.is_alive():
                p.kill()
                p.join()
    if timed_out and failed is None:
        # the ranks still running at the deadline were terminated (exit code -15): a timeout, not a task failure
        raise TimeoutError(f"partition tasks did not finish within {timeout_s}s")
    if failed is None:
        # every worker had exited by the last poll: a crash after its result file (or a missing file) is a failure
        for r, p in enumerate(procs):
            if p.exitcode != 0 or not os.path.exists(os.path.join(d, f"result_{r}.pkl")):
                failed = (r, f"exit code {p.exitcode}")
                break
    if failed is not None and failed[1] == "netinit":
        with open(os.path.join(d, f"result_{failed[0]}.pkl"), "rb") as f:
            msg = pickle.load(f)[1]  # written by our own worker process
        raise _NetworkInitError(f"rank {failed[0]} on port {port}: {msg}")
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
    def __init__(self, estimator, barrier: bool = False, with_measures: bool = False):
        self.estimator = estimator
        self.barrier = barrier
        self.with_measures = with_measures

    def __call__(self, part: DataFrame, rank: int, world: int):
        if self.barrier:
            from . import distributed as D

            D.barrier()  # barrier execution mode: every task starts its fit together
        model = self.estimator.fit(part)
        if self.with_measures:
            get = getattr(self.estimator, "getPerformanceMeasures", None)
            return (model if rank == 0 else None, get() if get else None)
        return model if rank == 0 else None


# ---------------------------------------------------------------- estimator-driven fan-out
def in_partition_task() -> bool:
    """True inside a distributed task: a worker this runtime started, a torchrun rank, or any process whose
    default process group is up. A fit there trains its own partition and joins the group's collectives;
    it never fans out again."""
    from . import distributed as D

    return os.environ.get("SML_PARTITION_TASK") == "1" or D.is_initialized()


def executor_tasks(use_gpu: bool) -> int:
    """Tasks the local "cluster" runs at once (ClusterUtil.getNumExecutorTasks, ClusterUtil.scala:92-140):
    one per visible MI355X for a GPU job; a CPU job runs one task unless ``SML_EXECUTOR_TASKS`` says how many
    CPU executors to use (the reference's executor cores)."""
    env = os.environ.get("SML_EXECUTOR_TASKS")
    if env:
        return max(1, int(env))
    if use_gpu:
        from ..utils.cluster import _device_count

        return max(1, _device_count())
    return 1


def determine_num_tasks(config_num_tasks: int, df: DataFrame, use_gpu: bool) -> int:
    """LightGBMBase.determineNumTasks (LightGBMBase.scala:449-456): ``numTasks > 0`` wins, otherwise
    min(executor tasks, the DataFrame's partitions)."""
    if config_num_tasks and int(config_num_tasks) > 0:
        return int(config_num_tasks)
    return max(1, min(executor_tasks(use_gpu), df.getNumPartitions()))


def fan_out(fn: Callable[[DataFrame, int, int], Any], df: DataFrame, num_tasks: int, use_gpu: bool, **kw) -> List[Any]:
    """Run ``fn`` over ``num_tasks`` partition tasks, one process each (Spark's mapPartitions over the
    coalesced / repartitioned DataFrame, LightGBMBase.scala:608-628). GPU tasks take one MI355X each over
    RCCL; with more tasks than visible devices the ranks share devices (gloo control plane, the engines'
    shared-device communicators - a rehearsal mode, not a scaling configuration)."""
    env = dict(kw.pop("env", None) or {})
    backend = kw.pop("backend", None)
    if use_gpu:
        from ..utils.cluster import _device_count

        ndev = _device_count()
        if num_tasks > max(1, ndev):
            backend = backend or "gloo"
            env.setdefault("SML_GBDT_SHARED_DEVICE", "1")
    from . import executor as X

    if not X.pool_enabled():
        return run_partitions(fn, df, num_workers=num_tasks, backend=backend, use_gpu=use_gpu, env=env, **kw)
    # the persistent executors (executor.py): started on the first call, reused by the later ones
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    run_kw = {k: kw.pop(k) for k in ("timeout_s", "fail_fast") if k in kw}
    start_kw = {k: kw.pop(k) for k in ("port", "default_listen_port", "network_retries", "initial_delay_s")
                if k in kw}
    if kw:
        raise TypeError(f"fan_out: unexpected arguments {sorted(kw)}")
    parts = _task_partitions(df, num_tasks)
    pool = X.get_pool(num_tasks, use_gpu, backend, env, **start_kw)
    return pool.run(fn, parts, **run_kw)


def _task_partitions(df: DataFrame, world: int) -> List[DataFrame]:
    """The DataFrame cut into ``world`` task partitions (coalesced or repartitioned; empty ones padded)."""
    parts = df.coalesce(world).partitions() if df.getNumPartitions() >= world else df.repartition(world).partitions()
    while len(parts) < world:
        parts.append(df.slice(0, 0))
    return parts


class _TransformTask:
    # kept by a persistent executor between calls (by the digest of its bytes): the transformer's session,
    # graphs and device buffers are built once per executor, as the reference's per-executor ONNX sessions
    cacheable = True

    def __init__(self, transformer):
        self.transformer = transformer

    def __call__(self, part: DataFrame, rank: int, world: int):
        return self.transformer.transform(part)


TRANSFORM_MIN_ROWS_PER_TASK = 1024


def transform_tasks(df: DataFrame, use_gpu: bool) -> int:
    """Partition tasks of a model's transform (ONNXModel.scala:242-251 maps the partitions, each task on its
    executor's device): min(executor tasks, partitions, rows / SML_TRANSFORM_MIN_ROWS (default 1024) per task);
    1 inside a task. A small DataFrame stays in this process: handing it to the executors costs more than
    scoring it here."""
    if in_partition_task():
        return 1
    min_rows = int(os.environ.get("SML_TRANSFORM_MIN_ROWS", str(TRANSFORM_MIN_ROWS_PER_TASK)))
    by_rows = max(1, df.count() // max(1, min_rows))
    return max(1, min(executor_tasks(use_gpu), df.getNumPartitions(), by_rows))


def fan_out_transform(transformer, df: DataFrame, num_tasks: int, use_gpu: bool) -> DataFrame:
    """``transformer.transform`` of every partition in its own task (one MI355X each), the results
    concatenated in partition order."""
    parts = fan_out(_TransformTask(transformer), df, num_tasks, use_gpu)
    return DataFrame.union_all(parts, keep_partitions=True)


def distributed_fit(estimator, df: DataFrame, num_workers: Optional[int] = None, use_gpu: bool = False,
                    **kw):
    """Data-parallel ``fit`` across worker processes; returns rank 0's model
    (only the main worker returns the model, BasePartitionTask.scala:450-461).
    Extra keyword arguments go to :func:`run_partitions` (timeout_s, fail_fast, ...). An estimator with
    driverListenPort / defaultListenPort params (LightGBM) sets the rendezvous port from them."""
    if "port" not in kw and hasattr(estimator, "getDriverListenPort"):
        dp = int(estimator.getDriverListenPort() or 0)
        if dp > 0:
            kw["port"] = rendezvous_port(dp)
        elif hasattr(estimator, "getDefaultListenPort"):
            kw.setdefault("default_listen_port", int(estimator.getDefaultListenPort() or 0))
    return run_partitions(_FitTask(estimator), df, num_workers=num_workers, use_gpu=use_gpu, **kw)[0]
