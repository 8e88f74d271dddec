"""Continuous-mode serving with epochs, task recovery and a restart-safe checkpoint (reference:
core/src/main/scala/org/apache/spark/sql/execution/streaming/continuous/HTTPSourceV2.scala:54-750 and
HTTPSinkV2.scala; the DataStreamReader/Writer helpers of IOImplicits.scala:22-64).

The micro-batch server (``serving.ServingServer``) answers whatever is queued as one DataFrame per batch.
Continuous mode instead hands every request to a long-running *partition task* the moment it arrives
(no batch formation, no trigger wait) - the reference's "as low as 1 ms" path:

* the HTTP front (one asyncio loop) appends each request to the queue of the current **epoch**;
  ``numPartitions`` partition tasks (threads of this process - one process per GPU, as everywhere in this
  framework) take requests one at a time, run the user's transform on a 1-row DataFrame(id, request) and
  reply;
* an epoch coordinator advances the epoch every ``epochLength`` ms (the continuous trigger interval); a
  partition task moves to the next epoch once it has drained the previous one, and an epoch is
  **committed** when every task has moved past it with all its requests answered: ``offsets/<epoch>`` is
  written when the epoch opens and ``commits/<epoch>`` when it commits (write-to-temp + rename, so a crash
  never leaves a torn file);
* every request a task takes is kept in the history of (epoch, partition) until that epoch commits. A task
  whose transform raises is **restarted** (attempt + 1) and re-registers at the same epoch; the requests of
  its epoch that have no reply yet are replayed to it first (HTTPSourceV2 ``registerPartition`` /
  ``recoveredPartitions``), so a crashed task loses no client request. A request that fails
  ``maxTaskFailures`` times is answered with 500;
* a query restarted on the same ``checkpointLocation`` resumes at the epoch after the last committed one,
  so epoch ids are never reused across restarts.

Builder API (the reference's ``readStream.continuousServer()...load()`` / ``writeStream...replyTo``)::

    q = (read_stream().continuous_server().address("0.0.0.0", 8888, "api").option("numPartitions", 2).load()
         .map(transform)
         .write_stream().continuous_server().reply_to("api")
         .option("checkpointLocation", "/tmp/ckpt").trigger(continuous="1 second").start())
"""
from __future__ import annotations

import collections
import json
import os
import re
import threading
import time
import uuid
from typing import Callable, Dict, List, Optional

from ..core.dataframe import DataFrame
from .serving import ServingServer, _obj, make_response


def _atomic_write(path: str, payload: dict) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    tmp = f"{path}.tmp-{uuid.uuid4().hex}"
    with open(tmp, "w") as f:
        json.dump(payload, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def _last_committed(ckpt: Optional[str]) -> int:
    if not ckpt:
        return -1
    d = os.path.join(ckpt, "commits")
    if not os.path.isdir(d):
        return -1
    eps = [int(n) for n in os.listdir(d) if n.isdigit()]
    return max(eps) if eps else -1


class ContinuousServingServer(ServingServer):
    """HTTP serving in continuous mode (see the module docstring)."""

    def __init__(self, transform: Callable[[DataFrame], DataFrame], host: str = "127.0.0.1", port: int = 0,
                 api: str = "", num_partitions: int = 2, epoch_length_ms: float = 30000.0,
                 checkpoint_location: Optional[str] = None, reply_col: str = "reply", request_timeout: float = 60.0,
                 max_task_failures: int = 4, name: Optional[str] = None):
        super().__init__(transform, host, port, api, max_batch_size=1, reply_col=reply_col,
                         request_timeout=request_timeout)
        if num_partitions < 1:
            raise ValueError("numPartitions must be >= 1")
        self.name = name or self.api or "continuous"
        self.num_partitions = num_partitions
        self.epoch_length_ms = float(epoch_length_ms)
        self.checkpoint_location = checkpoint_location
        self.max_task_failures = max_task_failures
        self._cond = threading.Condition()
        self.start_epoch = _last_committed(checkpoint_location) + 1
        self._epoch = self.start_epoch
        self._queues: Dict[int, collections.deque] = {self._epoch: collections.deque()}
        self._history: Dict[tuple, List[tuple]] = collections.defaultdict(list)
        self._answered: set = set()
        self._failures: collections.Counter = collections.Counter()
        self._task_epoch: Dict[int, int] = {}
        self._received: collections.Counter = collections.Counter()
        self.task_attempts: collections.Counter = collections.Counter()
        self.committed: List[int] = []
        self.progress: List[dict] = []
        self._halt = threading.Event()
        self._open_epoch(self._epoch)
        self._threads = [threading.Thread(target=self._partition_task, args=(p,), daemon=True, name=f"part-{p}")
                         for p in range(num_partitions)]
        self._threads.append(threading.Thread(target=self._coordinator, daemon=True, name="epochs"))

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "ContinuousServingServer":
        super().start()
        for t in self._threads:
            if not t.is_alive():
                t.start()
        return self

    def stop(self) -> None:
        self._halt.set()
        with self._cond:
            self._cond.notify_all()
        for t in self._threads:
            if t.is_alive():
                t.join(10)
        super().stop()

    # ------------------------------------------------------------------ front end (event-loop thread)
    async def _submit(self, req: dict) -> dict:
        fut = self._loop.create_future()
        with self._cond:
            e = self._epoch
            rid = f"{e}-{uuid.uuid4().hex[:12]}"
            self._pending[rid] = (fut, time.perf_counter())
            self._queues[e].append((rid, req))
            self._received[e] += 1
            self._cond.notify_all()  # the coordinator waits on the same condition: wake a task for sure
        import asyncio

        try:
            return await asyncio.wait_for(fut, self.request_timeout)
        except asyncio.TimeoutError:
            self._pending.pop(rid, None)
            return make_response("request timed out", 504, "Gateway Timeout")

    # ------------------------------------------------------------------ epochs
    def _open_epoch(self, e: int) -> None:
        if self.checkpoint_location:
            _atomic_write(os.path.join(self.checkpoint_location, "offsets", str(e)),
                          {"epoch": e, "name": self.name, "partitions": self.num_partitions, "opened": time.time()})

    def _coordinator(self) -> None:
        t0 = time.monotonic()
        while not self._halt.is_set():
            with self._cond:
                self._cond.wait(timeout=min(0.05, self.epoch_length_ms / 1e3))
                if time.monotonic() - t0 >= self.epoch_length_ms / 1e3:
                    t0 = time.monotonic()
                    self._epoch += 1
                    self._queues[self._epoch] = collections.deque()
                    self._open_epoch(self._epoch)
                    self._cond.notify_all()
                self._try_commit()

    def _try_commit(self) -> None:
        """Commit every epoch all tasks have moved past with all its requests answered (caller holds _cond)."""
        for e in sorted(k for k in self._queues if k < self._epoch):
            if self._queues[e] or any(self._task_epoch.get(p, e) <= e for p in range(self.num_partitions)):
                return
            if any(rid not in self._answered for p in range(self.num_partitions) for rid, _ in self._history.get((e, p), ())):
                return
            n = self._received.pop(e, 0)
            del self._queues[e]
            for p in range(self.num_partitions):
                for rid, _ in self._history.pop((e, p), ()):
                    self._answered.discard(rid)
                    self._failures.pop(rid, None)
            if self.checkpoint_location:
                _atomic_write(os.path.join(self.checkpoint_location, "commits", str(e)),
                              {"epoch": e, "requests": n, "committed": time.time()})
            self.committed.append(e)
            self.progress.append({"epoch": e, "numInputRows": n, "name": self.name, "timestamp": time.time()})

    # ------------------------------------------------------------------ partition tasks
    def _next(self, pid: int, replay: collections.deque):
        """Next request for task pid: replayed history first, then its epoch's queue; moves the task to the
        next epoch once its epoch is drained and closed. None when stopping."""
        if replay:
            return replay.popleft()
        with self._cond:
            while not self._halt.is_set():
                e = self._task_epoch[pid]
                q = self._queues.get(e)
                if q:
                    item = q.popleft()
                    self._history[(e, pid)].append(item)
                    return item
                if e < self._epoch:
                    self._task_epoch[pid] = e + 1  # epoch e drained by this task
                    self._try_commit()
                    continue
                self._cond.wait(timeout=0.05)
        return None

    def _partition_task(self, pid: int) -> None:
        with self._cond:
            self._task_epoch[pid] = self._epoch
        replay: collections.deque = collections.deque()
        while not self._halt.is_set():
            item = self._next(pid, replay)
            if item is None:
                return
            rid, req = item
            if rid in self._answered:
                continue
            try:
                out = self.transform_fn(DataFrame({"id": _obj([rid]), "request": _obj([req])}))
                reps = dict(zip(out["id"].tolist(), out[self.reply_col].tolist()))
                rep = reps.get(rid, make_response("no reply produced", 500, "Internal Server Error"))
                self._finish(rid, rep if isinstance(rep, dict) and "statusLine" in rep else make_response(rep))
            except Exception as e:  # noqa: BLE001 - the task "crashes" and is restarted at the same epoch
                self._failures[rid] += 1
                # counted before the reply: a client that sees the 500 also sees every attempt
                self.task_attempts[pid] += 1
                if self._failures[rid] >= self.max_task_failures:
                    self._finish(rid, make_response(f"{type(e).__name__}: {e}", 500, "Internal Server Error"))
                with self._cond:
                    e_now = self._task_epoch[pid]
                    replay = collections.deque(x for x in self._history.get((e_now, pid), ())
                                               if x[0] not in self._answered)

    def _finish(self, rid: str, rep: dict) -> None:
        with self._cond:
            self._answered.add(rid)
            self._cond.notify_all()
        self.reply(rid, rep)

    # ------------------------------------------------------------------ status
    @property
    def epoch(self) -> int:
        return self._epoch


# ====================================================================== builder API
_TRIGGER = re.compile(r"^\s*([\d.]+)\s*([a-z]*)\s*$")
_UNIT_MS = {"": 1.0, "ms": 1.0, "millisecond": 1.0, "milliseconds": 1.0, "s": 1000.0, "second": 1000.0,
            "seconds": 1000.0, "m": 60000.0, "min": 60000.0, "minute": 60000.0, "minutes": 60000.0}


def _interval_ms(v) -> float:
    """Trigger interval in ms: a number (ms) or "<x> milliseconds|seconds|minutes" (Spark's spelling)."""
    if isinstance(v, (int, float)):
        return float(v)
    m = _TRIGGER.match(str(v).lower())
    if not m or m.group(2) not in _UNIT_MS:
        raise ValueError(f"cannot parse trigger interval {v!r}")
    return float(m.group(1)) * _UNIT_MS[m.group(2)]


class ServingQuery:
    """A running serving query (the reference's StreamingQuery surface)."""

    def __init__(self, server: ServingServer, name: Optional[str]):
        self.server = server
        self.name = name
        self.id = uuid.uuid4().hex
        self._stopped = threading.Event()

    @property
    def address(self) -> str:
        return self.server.address

    @property
    def isActive(self) -> bool:  # noqa: N802 - Spark name
        return not self._stopped.is_set()

    @property
    def lastProgress(self) -> Optional[dict]:  # noqa: N802
        p = getattr(self.server, "progress", None)
        return p[-1] if p else None

    @property
    def recentProgress(self) -> List[dict]:  # noqa: N802
        return list(getattr(self.server, "progress", []))

    def stop(self) -> None:
        if not self._stopped.is_set():
            self.server.stop()
            self._stopped.set()

    def awaitTermination(self, timeout: Optional[float] = None) -> bool:  # noqa: N802
        return self._stopped.wait(timeout)


class ServingStreamWriter:
    def __init__(self, stream: "ServingStream"):
        self._stream = stream
        self._opts: Dict[str, object] = {}
        self._continuous: Optional[bool] = None
        self._trigger_ms: Optional[float] = None
        self._trigger_continuous = False
        self._name: Optional[str] = None

    def server(self) -> "ServingStreamWriter":
        self._continuous = False
        return self

    def continuous_server(self) -> "ServingStreamWriter":
        self._continuous = True
        return self

    continuousServer = continuous_server  # noqa: N815

    def reply_to(self, name: str) -> "ServingStreamWriter":
        self._opts["name"] = name
        return self

    replyTo = reply_to  # noqa: N815

    def option(self, key: str, value) -> "ServingStreamWriter":
        self._opts[key] = value
        return self

    def queryName(self, name: str) -> "ServingStreamWriter":  # noqa: N802
        self._name = name
        return self

    def trigger(self, processingTime=None, continuous=None) -> "ServingStreamWriter":  # noqa: N803
        if continuous is not None:
            self._trigger_ms, self._trigger_continuous = _interval_ms(continuous), True
        elif processingTime is not None:
            self._trigger_ms, self._trigger_continuous = _interval_ms(processingTime), False
        return self

    def start(self) -> ServingQuery:
        r = self._stream.reader
        if self._opts.get("name") not in (None, r.api):
            raise ValueError(f"replyTo({self._opts.get('name')!r}) does not name the source api {r.api!r}")
        continuous = r.continuous if self._continuous is None else self._continuous
        if continuous != r.continuous:
            raise ValueError("the source and the sink must both be continuous or both micro-batch servers")
        if continuous and self._trigger_ms is not None and not self._trigger_continuous:
            raise ValueError("a continuous server needs trigger(continuous=...), not processingTime")
        fn = self._stream.fn
        ck = self._opts.get("checkpointLocation")
        if continuous:
            srv = ContinuousServingServer(fn, r.host, r.port, r.api, num_partitions=int(r.opts.get("numPartitions", 2)),
                                          epoch_length_ms=self._trigger_ms or float(r.opts.get("epochLength", 30000)),
                                          checkpoint_location=ck, reply_col=str(self._opts.get("replyCol", "reply")),
                                          name=self._name)
        else:
            srv = ServingServer(fn, r.host, r.port, r.api, max_batch_size=int(r.opts.get("maxBatchSize", 64)),
                                max_wait_ms=self._trigger_ms or 0.0, reply_col=str(self._opts.get("replyCol", "reply")))
        return ServingQuery(srv.start(), self._name)


class ServingStream:
    """load() result: the request stream plus the transform applied to it."""

    def __init__(self, reader: "ServingStreamReader", fn: Callable[[DataFrame], DataFrame]):
        self.reader = reader
        self.fn = fn

    def map(self, fn: Callable[[DataFrame], DataFrame]) -> "ServingStream":
        prev = self.fn
        return ServingStream(self.reader, lambda df: fn(prev(df)))

    transform = map

    def write_stream(self) -> ServingStreamWriter:
        return ServingStreamWriter(self)

    writeStream = property(write_stream)  # noqa: N815 - Spark spelling: stream.writeStream.server()...


class ServingStreamReader:
    def __init__(self):
        self.continuous = False
        self.host, self.port, self.api = "127.0.0.1", 8888, ""
        self.opts: Dict[str, object] = {}

    def server(self) -> "ServingStreamReader":
        self.continuous = False
        return self

    def continuous_server(self) -> "ServingStreamReader":
        self.continuous = True
        return self

    continuousServer = continuous_server  # noqa: N815

    def address(self, host: str, port: int, api: str) -> "ServingStreamReader":
        self.host, self.port, self.api = host, int(port), api.strip("/")
        return self

    def option(self, key: str, value) -> "ServingStreamReader":
        self.opts[key] = value
        return self

    def load(self) -> ServingStream:
        return ServingStream(self, lambda df: df)


def read_stream() -> ServingStreamReader:
    return ServingStreamReader()


__all__ = ["ContinuousServingServer", "ServingQuery", "ServingStream", "ServingStreamReader", "ServingStreamWriter",
           "read_stream"]
