"""Persistent per-GPU executor pool behind ``fan_out``.

The reference's Spark executors are long-lived JVMs: the native LightGBM library is loaded once per executor
(``LightGBMUtils.scala:31-35``), state shared by the tasks of an executor lives in ``SharedSingleton``s
(``SharedVariable.scala:36-63``) and ``ONNXModel`` keeps one session per executor fed from broadcast bytes
(``ONNXModel.scala:192-196,239-251``). ``run_partitions`` (runtime.py) starts fresh processes per call - every
fit paid process start, ``import torch``, the native modules' load, HIP / RCCL initialisation and (for ONNX) the
session and hipGraph build again: ~5 s per ``numTasks=2`` fit that takes 0.03 s in-process (round-5 verdict).

Here the driver starts N workers ONCE per (world, device use, backend, environment) and keeps them:

* each worker pins its MI355X (``torch.cuda.set_device(rank % devices)``) before any other GPU call, joins the
  process group once (TCPStore rendezvous on 127.0.0.1, the NetworkManager retry on a fresh port when a rank
  fails to join), and then serves tasks from a pipe until it is told to stop;
* the process-wide caches of a worker survive between tasks: the native communicators
  (``distributed.gbdt_comm``), pinned stagers, device pools, and the task objects themselves - a task whose
  callable sets ``cacheable = True`` (transforms) is unpickled once per worker and kept by the digest of its
  bytes, so an ``ONNXModel`` keeps its session / hipGraph from one ``transform`` to the next; the driver mirrors
  each worker's LRU and sends the bytes only when the worker does not hold them;
* partitions go in through POSIX shared memory (the ``_share_partition`` hand-off of runtime.py) and DataFrame
  results come back the same way (the worker writes its result's numeric columns into a segment, the driver
  copies them out and unlinks it); other results are pickled over the pipe - no temp files;
* a worker that dies or a task that raises aborts the job on every rank (the others may be blocked in
  collectives) and retires the pool: the next call starts fresh child processes (never an exec);
* shutdown is explicit (``shutdown()``, the pool as a context manager) and registered with ``atexit``.

Shared-memory attach never registers the segment with the (shared) resource tracker, so a worker can no longer
drop the driver's registration (the round-5 ``KeyError: '/psm_...'`` tracker tracebacks).
``SML_EXECUTOR_POOL=0`` makes ``fan_out`` spawn per call as before.
"""
from __future__ import annotations

import atexit
import hashlib
import os
import pickle
import threading
import time
import traceback
from collections import OrderedDict
from typing import Any, Callable, List, Optional

import numpy as np

from ..core.dataframe import DataFrame

_CACHE_SLOTS = 8  # cacheable task objects kept per worker (LRU, mirrored by the driver)


def pool_enabled() -> bool:
    return os.environ.get("SML_EXECUTOR_POOL", "1") != "0"


# ---------------------------------------------------------------- shared-memory helpers
def attach_shm(name: str):
    """Map an existing segment without registering it with the resource tracker (the creator owns it and
    unlinks it; a registration here would be dropped by whoever unlinks first - on Python 3.10 the tracker
    keeps one entry per name, so an attach + unregister removed the creator's entry)."""
    from multiprocessing import resource_tracker, shared_memory

    reg = resource_tracker.register
    resource_tracker.register = lambda *a, **k: None
    try:
        return shared_memory.SharedMemory(name=name)
    finally:
        resource_tracker.register = reg


def _pack_result(out: Any):
    """A task's result for the pipe: DataFrames travel as a shared-memory descriptor, anything else pickled."""
    if isinstance(out, DataFrame):
        from .runtime import _share_partition

        parts = out.partitions() if out.getNumPartitions() > 1 else [out]
        descs = []
        for p in parts:
            desc, shm = _share_partition(p)
            if shm is not None:
                shm.close()  # the segment outlives the mapping; the driver unlinks it after copying
            descs.append(desc)
        return ("df", descs)
    return ("obj", pickle.dumps(out))


def _unpack_result(packed) -> Any:
    kind, val = packed
    if kind == "obj":
        return pickle.loads(val)  # written by this job's own worker process
    from .runtime import _attach_partition

    parts = []
    for desc in val:
        df, shm = _attach_partition(desc)
        if shm is not None:
            # own copies of the columns, then the segment goes (the worker closed its mapping already)
            from ..core.linalg import CsrColumn

            cols = {}
            for k in df.columns:
                c = df[k]
                if isinstance(c, CsrColumn):
                    ip, ind, v = c.csr()
                    c = CsrColumn(np.array(ip), np.array(ind), np.array(v), c.size)
                elif isinstance(c, np.ndarray) and c.dtype != object:
                    c = np.array(c)
                cols[k] = c
            meta = {k: df.metadata(k) for k in df.columns}
            del df
            df = DataFrame(cols, metadata={k: v for k, v in meta.items() if v})
            try:
                shm.close()
            except BufferError:
                pass
            try:
                shm.unlink()
            except FileNotFoundError:
                pass
        parts.append(df)
    return parts[0] if len(parts) == 1 else DataFrame.union_all(parts, keep_partitions=True)


# ---------------------------------------------------------------- worker
def _pool_worker(rank: int, world: int, port: int, backend: str, use_gpu: bool, env: Optional[dict], conn,
                 attempt: int) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), SML_PARTITION_TASK="1", SML_EXECUTOR_POOL_WORKER="1")
    if env:
        os.environ.update({k: str(v) for k, v in env.items()})
    from .runtime import _attach_partition, _init_timeout, _injected_fault

    fault = _injected_fault(rank)
    try:
        import torch
        import torch.distributed as dist

        if use_gpu:
            # the device is pinned before anything else touches the GPU in this process
            torch.cuda.set_device(rank % max(1, torch.cuda.device_count()))
        if fault == "netinit_fail" and attempt == 0:
            raise OSError("injected network-init failure")
        dist.init_process_group(backend=backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world, timeout=_init_timeout())
    except BaseException as e:  # noqa: BLE001 - the driver retries the rendezvous on a fresh port
        try:
            conn.send(("netinit", f"{type(e).__name__}: {e}"))
        finally:
            return
    conn.send(("ready", os.getpid()))
    cache: "OrderedDict[str, Any]" = OrderedDict()
    while True:
        try:
            msg = conn.recv()
        except (EOFError, OSError):
            break
        if msg[0] == "stop":
            break
        _, task_id, digest, fn_bytes, desc = msg
        shm = None
        try:
            if digest is not None and digest in cache:
                fn = cache[digest]
                cache.move_to_end(digest)
            else:
                fn = pickle.loads(fn_bytes)  # serialized by this pool's driver
                if digest is not None:
                    cache[digest] = fn
                    while len(cache) > _CACHE_SLOTS:
                        cache.popitem(last=False)
            part, shm = _attach_partition(desc)
            if fault == "raise":
                raise RuntimeError(f"injected fault on rank {rank}")
            if fault == "crash_after_init":
                os._exit(18)
            if fault == "empty":
                part = part.slice(0, 0)
            # packed while the partition is still mapped (a transformed partition may view its input columns)
            reply = ("ok", task_id, _pack_result(fn(part, rank, world)))
            del part
        except BaseException as e:  # noqa: BLE001 - reported to the driver, which aborts the job
            reply = ("err", task_id, f"{type(e).__name__}: {e}\n{traceback.format_exc()}")
        finally:
            if shm is not None:
                try:
                    shm.close()
                except BufferError:
                    pass
        try:
            conn.send(reply)
        except (BrokenPipeError, OSError):
            break
    try:
        import torch.distributed as dist

        from . import distributed as D

        D.close_shm_reducer()
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - exiting anyway
        pass


# ---------------------------------------------------------------- driver side
class PoolBroken(RuntimeError):
    pass


class ExecutorPool:
    """N long-lived task processes, one per rank (one MI355X each for a GPU pool)."""

    def __init__(self, world: int, use_gpu: bool, backend: str, env: Optional[dict] = None,
                 port: Optional[int] = None, default_listen_port: int = 0, network_retries: int = 3,
                 initial_delay_s: float = 1.0, start_timeout_s: float = 600.0):
        from . import runtime as R

        self.world, self.use_gpu, self.backend = world, use_gpu, backend
        self.env = dict(env or {})
        self.procs: list = []
        self.conns: list = []
        self._lru: List["OrderedDict[str, None]"] = []
        self._task_seq = 0
        self._lock = threading.Lock()
        self.closed = False
        self.tasks_run = 0
        delay = initial_delay_s
        pinned = port
        for attempt in range(network_retries + 1):
            p = pinned if pinned else (R.find_open_port(default_listen_port) if default_listen_port > 0
                                       else R._free_port())
            err = self._start(p, attempt, start_timeout_s)
            if err is None:
                self.port = p
                return
            self._kill()
            if attempt == network_retries:
                raise RuntimeError(f"network init failed after {network_retries} retries: {err}")
            time.sleep(delay)
            delay *= 2
            if default_listen_port > 0 and not pinned:
                default_listen_port = p + 1

    def _start(self, port: int, attempt: int, timeout_s: float) -> Optional[str]:
        import torch.multiprocessing as mp

        ctx = mp.get_context("spawn")
        self.procs, self.conns, self._lru = [], [], []
        for r in range(self.world):
            parent, child = ctx.Pipe()
            p = ctx.Process(target=_pool_worker, args=(r, self.world, port, self.backend, self.use_gpu, self.env,
                                                       child, attempt), daemon=True)
            p.start()
            child.close()
            self.procs.append(p)
            self.conns.append(parent)
            self._lru.append(OrderedDict())
        deadline = time.monotonic() + timeout_s
        ready = [False] * self.world
        while not all(ready):
            for r, c in enumerate(self.conns):
                if ready[r]:
                    continue
                if c.poll(0.02):
                    try:
                        st, val = c.recv()
                    except (EOFError, OSError):
                        return f"rank {r} exited during start (exit code {self.procs[r].exitcode})"
                    if st == "netinit":
                        return f"rank {r} on port {port}: {val}"
                    ready[r] = True
                elif not self.procs[r].is_alive():
                    return f"rank {r} exited during start (exit code {self.procs[r].exitcode})"
            if time.monotonic() > deadline:
                return f"executors did not start within {timeout_s}s"
        return None

    def alive(self) -> bool:
        return not self.closed and all(p.is_alive() for p in self.procs)

    def run(self, fn: Callable[[DataFrame, int, int], Any], parts: List[DataFrame], timeout_s: float = 1200.0,
            fail_fast: bool = True) -> List[Any]:
        """``fn(parts[r], r, world)`` on every worker; results in rank order. Any failure aborts the job on all
        ranks, retires the pool and raises (RuntimeError / TimeoutError)."""
        from .runtime import _share_partition

        if len(parts) != self.world:
            raise ValueError(f"{len(parts)} partitions for a pool of {self.world}")
        with self._lock:
            if not self.alive():
                raise PoolBroken("executor pool is not running")
            fn_bytes = pickle.dumps(fn)
            digest = hashlib.sha1(fn_bytes).hexdigest() if getattr(fn, "cacheable", False) else None
            self._task_seq += 1
            tid = self._task_seq
            shared = []
            try:
                descs = []
                for p in parts:  # every partition is placed before any task is sent
                    desc, shm = _share_partition(p)
                    if shm is not None:
                        shared.append(shm)
                    descs.append(desc)
                for r, c in enumerate(self.conns):
                    send = fn_bytes
                    if digest is not None:
                        lru = self._lru[r]
                        if digest in lru:
                            lru.move_to_end(digest)
                            send = None
                        else:
                            lru[digest] = None
                            while len(lru) > _CACHE_SLOTS:
                                lru.popitem(last=False)
                    c.send(("task", tid, digest, send, descs[r]))
                return self._collect(tid, timeout_s, fail_fast)
            except BaseException:
                self.close(kill=True)
                raise
            finally:
                for shm in shared:
                    try:
                        shm.close()
                        shm.unlink()
                    except Exception:  # noqa: BLE001 - already gone
                        pass

    def _collect(self, tid: int, timeout_s: float, fail_fast: bool) -> List[Any]:
        deadline = time.monotonic() + timeout_s
        out: List[Any] = [None] * self.world
        done = [False] * self.world
        errs: List[Optional[str]] = [None] * self.world
        while not all(done):
            for r, c in enumerate(self.conns):
                if done[r]:
                    continue
                if c.poll(0.01):
                    try:
                        st, t, val = c.recv()
                    except (EOFError, OSError):
                        errs[r] = f"exit code {self.procs[r].exitcode}"
                        done[r] = True
                        continue
                    if t != tid:
                        continue  # a stale reply (cannot happen while the pool is serial; ignored)
                    done[r] = True
                    if st == "ok":
                        out[r] = val
                    else:
                        errs[r] = val
                elif not self.procs[r].is_alive():
                    errs[r] = f"exit code {self.procs[r].exitcode}"
                    done[r] = True
            failed = [r for r in range(self.world) if errs[r] is not None]
            if failed and fail_fast:
                r = failed[0]
                raise RuntimeError(f"worker {r} failed ({errs[r]}); the job was aborted on the remaining ranks")
            if time.monotonic() > deadline:
                raise TimeoutError(f"partition tasks did not finish within {timeout_s}s")
        failed = [r for r in range(self.world) if errs[r] is not None]
        if failed:
            raise RuntimeError("partition tasks failed: " + " | ".join(f"worker {r}: {errs[r]}" for r in failed))
        self.tasks_run += 1
        return [_unpack_result(v) for v in out]

    def _kill(self) -> None:
        for p in self.procs:
            if p.is_alive():
                p.terminate()
        for p in self.procs:
            p.join(10)
            if p.is_alive():
                p.kill()
                p.join()
        for c in self.conns:
            try:
                c.close()
            except OSError:
                pass

    def close(self, kill: bool = False) -> None:
        if self.closed:
            return
        self.closed = True
        if not kill:
            for c in self.conns:
                try:
                    c.send(("stop",))
                except (BrokenPipeError, OSError):
                    pass
            for p in self.procs:
                p.join(15)
        self._kill()

    def __enter__(self) -> "ExecutorPool":
        return self

    def __exit__(self, *exc) -> None:
        close_pool(self)


_pool: Optional[ExecutorPool] = None
_pool_key = None
_pool_lock = threading.Lock()


def get_pool(world: int, use_gpu: bool, backend: str, env: Optional[dict] = None, **start_kw) -> ExecutorPool:
    """The process-wide pool for this (world, device use, backend, environment); a pool with another key is
    shut down first (one set of executors holds the devices at a time)."""
    global _pool, _pool_key
    key = (world, bool(use_gpu), backend, tuple(sorted((env or {}).items())))
    with _pool_lock:
        if _pool is not None and (_pool_key != key or not _pool.alive()):
            _pool.close(kill=not _pool.alive())
            _pool = None
        if _pool is None:
            _pool = ExecutorPool(world, use_gpu, backend, env, **start_kw)
            _pool_key = key
        return _pool


def current_pool() -> Optional[ExecutorPool]:
    return _pool


def close_pool(pool: ExecutorPool) -> None:
    global _pool, _pool_key
    with _pool_lock:
        pool.close()
        if _pool is pool:
            _pool, _pool_key = None, None


def shutdown() -> None:
    """Stop the executors (also registered with atexit)."""
    global _pool, _pool_key
    with _pool_lock:
        if _pool is not None:
            _pool.close()
        _pool, _pool_key = None, None


atexit.register(shutdown)
